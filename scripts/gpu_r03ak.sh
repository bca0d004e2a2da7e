# round 3, GPU call ak: the final tree — full GPU suite and the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ak_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ak_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ak_gpu_tests.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03ak_bench.json 2> gpurun_out/r03ak_bench.err || { tail -20 gpurun_out/r03ak_bench.err; exit 1; }
cat gpurun_out/r03ak_bench.json
echo all done
