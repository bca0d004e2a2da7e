# round 3, GPU call o: the narrow form (fp32 N = 16) in the automatic pick: full GPU suite, N = 16
# sweep of the automatic pick, then call g (bench line, other configs, 8-rank rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03o_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03o_gpu_tests.txt
S=""
for g in pubmed small20k arxiv g60k p2m p5m p8m p11m p15m plaw1m u1m20; do S="$S $g:16:0"; done
timeout -k 10 300 python -u scripts/probe_graph.py $S > gpurun_out/r03o_auto16.jsonl 2> gpurun_out/r03o_auto16.err || { tail -20 gpurun_out/r03o_auto16.err; exit 1; }
cat gpurun_out/r03o_auto16.jsonl
bash scripts/gpu_r03g.sh
