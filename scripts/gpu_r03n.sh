# round 3, GPU call n: wave items stride over a capped block count, light rows sized to the rows:
# WH parity (forms + tuning table), then N = 16 / 32 / 64 timing of the WH configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_out_of_range.py tests/test_gpu_configs.py -m gpu -x -q -k "tuning_table or form or zero_fill or wave" --timeout 200 --timeout-method thread > gpurun_out/r03n_tests.txt 2>&1 || { tail -30 gpurun_out/r03n_tests.txt; exit 1; }
tail -1 gpurun_out/r03n_tests.txt
S=""
for g in arxiv p2m p5m p8m p11m plaw1m u1m20 products; do for v in 0 10028 10031 10033 10034 10037 10038; do S="$S $g:16:$v"; done; done
for g in arxiv g60k p2m p5m; do for v in 0 30004 30005; do S="$S $g:32:$v $g:64:$v"; done; done
timeout -k 10 900 python -u scripts/probe_graph.py $S > gpurun_out/r03n_graph.jsonl 2> gpurun_out/r03n_graph.err || { tail -20 gpurun_out/r03n_graph.err; exit 1; }
cat gpurun_out/r03n_graph.jsonl
echo all done
