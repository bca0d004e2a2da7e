# round 4, GPU call ab: the fp32 N = 16 narrow form of mid-size launches with the in-kernel hub
# reduce (automatic: 113 VGPRs, 4 waves per SIMD) against the same configuration with the reduce
# launch (tuning entry 10031: 96 VGPRs in round 3, 5 waves), graph replay, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SPECS="arxiv:16:0 arxiv:16:10031 g60k:16:0 g60k:16:10031 p2m:16:0 p2m:16:10031 u169k7:16:0 u169k7:16:10031"
for r in 1 2 3; do
  timeout -k 10 150 python -u scripts/probe_graph.py $SPECS >> gpurun_out/r04ab_lr_n16.jsonl 2>> gpurun_out/r04ab.err || { tail -20 gpurun_out/r04ab.err; exit 1; }
done
echo all done
