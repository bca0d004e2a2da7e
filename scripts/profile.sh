#!/bin/bash
# Profiles bench.py on one MI355X: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in their own
# passes (gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads).
# usage: scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 10 --warmup 3 --no-cpu-baseline}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch_bench.json 2> $OUT/fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write_bench.json 2> $OUT/write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- python3 bench.py $ARGS > $OUT/hit_bench.json 2> $OUT/hit.err || exit $?
echo done
