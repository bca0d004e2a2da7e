# round 3, GPU call l: the HL wave-item mapping (tuning variants 31-36): parity of the tuning
# table, then N = 16 timing against the current automatic pick
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k tuning_table --timeout 120 --timeout-method thread > gpurun_out/r03l_tests.txt 2>&1 || { tail -30 gpurun_out/r03l_tests.txt; exit 1; }
tail -1 gpurun_out/r03l_tests.txt
S=""
for g in pubmed arxiv g60k p2m u169k7 p5m plaw1m; do for v in 0 10022 10031 10032 10033 10034 10035 10031h16 10031h64 10033h16; do S="$S $g:16:$v"; done; done
timeout -k 10 600 python -u scripts/probe_graph.py $S > gpurun_out/r03l_graph.jsonl 2> gpurun_out/r03l_graph.err || { tail -20 gpurun_out/r03l_graph.err; exit 1; }
cat gpurun_out/r03l_graph.jsonl
echo all done
