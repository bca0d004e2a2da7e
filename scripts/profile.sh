#!/bin/bash
# Profiles bench.py on one MI355X with rocprofv3: a kernel-trace/stats pass, then PMC passes, each
# in its own run (counters never combined with other trace domains).  Raw outputs go to
# gpurun_out/prof_<tag>/; scripts/rocprof_summary.py condenses them for profiles/.
# usage: scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 10 --warmup 3 --no-cpu-baseline}
PROG=${PROG:-bench.py}  # or e.g. PROG=scripts/bench_config.py for the non-bench configurations
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {  # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 200 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 $PROG $ARGS \
    > $OUT/${name}_bench.json 2> $OUT/${name}.err
}
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run rdreq --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_BUBBLE_sum || exit $?
run rd128 --pmc TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit $?
run hit --pmc TCC_HIT_sum TCC_MISS_sum || exit $?
if [ -n "${SQ_PASS:-}" ]; then  # where the waves' time goes (parked on s_waitcnt / issue / active)
  run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
fi
echo done
