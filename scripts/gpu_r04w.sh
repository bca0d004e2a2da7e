# round 4, GPU call w: final fresh-box validation of the round-4 tree -- the full GPU suite, smoke,
# the bench line (products N=128, 1 GPU), rocprofv3 kernel trace + PMC of the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04w_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04w_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04w_smoke.txt 2>&1 || { tail -20 gpurun_out/r04w_smoke.txt; exit 1; }
cat gpurun_out/r04w_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || { tail -20 gpurun_out/r04w_bench.err; exit 1; }
cat gpurun_out/r04w_bench.json
bash scripts/profile.sh r04w_products --steps 10 --warmup 3 --no-cpu-baseline || exit 1
echo all done
