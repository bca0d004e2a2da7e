# round 3, GPU call k: light-row throughput of the narrow-N configurations on uniform-degree graphs
# (no hubs, no heavy rows) against the power-law arxiv-shaped graph
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=""
for g in u169k2 u169k7 u169k28 arxiv; do for v in 0 10021 10022 10026 10027 10028 10030 404 416 30003; do S="$S $g:16:$v"; done; done
for v in 0 10021 10022 10026 10028 404; do S="$S u1m20:16:$v"; done
timeout -k 10 600 python -u scripts/probe_graph.py $S > gpurun_out/r03k_graph.jsonl 2> gpurun_out/r03k_graph.err || { tail -20 gpurun_out/r03k_graph.err; exit 1; }
cat gpurun_out/r03k_graph.jsonl
echo all done
