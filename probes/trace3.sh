#!/bin/bash
# Kernel-trace (rocprofv3 --kernel-trace --stats) of bench.py for several configs, one run each.
# usage: probes/trace3.sh <tag> <config>...
set -u
TAG=$1; shift
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for c in "$@"; do
  OUT=gpurun_out/trace_${TAG}_$c
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
done
