# round 3, GPU call q: same-box A/B against the start-of-round build on the BASELINE configs, the
# tuning-table parity of variants 39-44, and N = 32 / 64 timing of the float4 + HL configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k tuning_table --timeout 120 --timeout-method thread > gpurun_out/r03q_tests.txt 2>&1 || { tail -30 gpurun_out/r03q_tests.txt; exit 1; }
tail -1 gpurun_out/r03q_tests.txt
S=""
for g in arxiv g60k p2m p5m p8m plaw1m; do
  for v in 0 30004 30005 10039 10040 10043; do S="$S $g:32:$v"; done
  for v in 0 30004 30005 10041 10042 10044; do S="$S $g:64:$v"; done
done
timeout -k 10 600 python -u scripts/probe_graph.py $S > gpurun_out/r03q_graph.jsonl 2> gpurun_out/r03q_graph.err || { tail -20 gpurun_out/r03q_graph.err; exit 1; }
cat gpurun_out/r03q_graph.jsonl
bash scripts/gpu_r03p.sh
