# round 3, GPU call g: the fresh-box bench line (cpu_baseline = the kCPU kernel), the other
# single-GPU configs, and the products-scale 8-rank rehearsal of the bench's N>1 path on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err || { tail -20 gpurun_out/r03g_bench.err; exit 1; }
cat gpurun_out/r03g_bench.json
for c in plaw1m reddit; do
  timeout -k 10 600 python -u scripts/bench_config.py --config $c > gpurun_out/r03g_$c.json 2> gpurun_out/r03g_$c.err || { tail -20 gpurun_out/r03g_$c.err; exit 1; }
  cat gpurun_out/r03g_$c.json
done
T0=$SECONDS
timeout -k 10 900 python -u bench.py --gpus 8 --backend gloo --steps 3 --warmup 1 --tune-budget 150 > gpurun_out/r03g_rehearsal8_products.json 2> gpurun_out/r03g_rehearsal8_products.err || { tail -40 gpurun_out/r03g_rehearsal8_products.err; exit 1; }
echo "rehearsal wall seconds: $((SECONDS - T0))" | tee -a gpurun_out/r03g_rehearsal8_products.err
tail -30 gpurun_out/r03g_rehearsal8_products.err
echo all done
