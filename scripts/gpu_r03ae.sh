# round 3, GPU call ae: fresh-box validation of the tree after the 16-bit load fix, the 16-bit
# lane layout, the 64-lane readlane path and the shifted window — full GPU suite, smoke, bench
# line, the other single-GPU BASELINE configs, rocprofv3 trace + PMC of the bench workload
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ae_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ae_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ae_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ae_smoke.txt 2>&1 || { tail -20 gpurun_out/r03ae_smoke.txt; exit 1; }
cat gpurun_out/r03ae_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03ae_bench.json 2> gpurun_out/r03ae_bench.err || { tail -20 gpurun_out/r03ae_bench.err; exit 1; }
cat gpurun_out/r03ae_bench.json
for c in plaw1m reddit; do
  timeout -k 10 600 python -u scripts/bench_config.py --config $c > gpurun_out/r03ae_$c.json 2> gpurun_out/r03ae_$c.err || { tail -20 gpurun_out/r03ae_$c.err; exit 1; }
  cat gpurun_out/r03ae_$c.json
done
bash scripts/profile.sh r03ae_products --steps 10 --warmup 3 --no-cpu-baseline || exit 1
echo all done
