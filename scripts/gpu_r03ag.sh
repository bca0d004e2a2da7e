# round 3, GPU call ag: final fresh-box validation of the round's tree — full GPU suite, smoke,
# bench line, tiny-width check of the 8-lane rule
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ag_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ag_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ag_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ag_smoke.txt 2>&1 || { tail -20 gpurun_out/r03ag_smoke.txt; exit 1; }
cat gpurun_out/r03ag_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03ag_bench.json 2> gpurun_out/r03ag_bench.err || { tail -20 gpurun_out/r03ag_bench.err; exit 1; }
cat gpurun_out/r03ag_bench.json
timeout -k 10 400 python -u scripts/width_sweep.py --config plaw1m --widths 1,4 --dtypes f32 > gpurun_out/r03ag_tiny.jsonl 2> gpurun_out/r03ag.err || { tail -20 gpurun_out/r03ag.err; exit 1; }
cat gpurun_out/r03ag_tiny.jsonl
echo all done
