# round 4, GPU call ac: the fp32 N = 16 narrow form of mid-size launches -- loads in flight of the
# light rows (U) and of the wave items (HU) with the in-kernel reduce: tuning entries 10082-10084
# against the automatic pick (U = 4, HU = 16), graph replay, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SPECS="arxiv:16:0 arxiv:16:10082 arxiv:16:10083 arxiv:16:10084 g60k:16:0 g60k:16:10082 g60k:16:10083 g60k:16:10084 p2m:16:0 p2m:16:10082 p2m:16:10083 p2m:16:10084"
for r in 1 2 3; do
  timeout -k 10 150 python -u scripts/probe_graph.py $SPECS >> gpurun_out/r04ac_n16_u.jsonl 2>> gpurun_out/r04ac.err || { tail -20 gpurun_out/r04ac.err; exit 1; }
done
echo all done
