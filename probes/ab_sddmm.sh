#!/bin/bash
# A/B of SDDMM builds (probes/ab_build.sh tags) through OFX_SPMM_LIB, interleaved, two rounds:
# bash probes/ab_sddmm.sh <out.jsonl> "<config:n> ..." "<tag> ..."   (tag "base" = the default build)
set -e
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=of-spmm_amd/oneflow_spmm
for round in 1 2; do
  for tag in $3; do
    if [ $tag = base ]; then lib=$PWD/$L/libofx_spmm.so; else lib=$PWD/$L/libofx_spmm_$tag.so; fi
    for cn in $2; do
      cfg=${cn%%:*}; n=${cn##*:}
      r=$(OFX_SPMM_LIB=$lib timeout -k 10 200 python scripts/bench_backward.py --config $cfg --n $n --only sddmm 2>/dev/null)
      echo "{\"round\": $round, \"tag\": \"$tag\", \"result\": $r}" >> $1
    done
  done
done
