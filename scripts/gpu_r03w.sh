# round 3, GPU call w: dense-width sweep (N = 1..512, fp32 and bf16) of the op on the products,
# Reddit and 1M power-law graphs, sampled rows bit-exact against the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/width_sweep.py --config products > gpurun_out/r03w_width_products.jsonl 2> gpurun_out/r03w.err || { tail -20 gpurun_out/r03w.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 16,32,64,128,256,512 > gpurun_out/r03w_width_reddit.jsonl 2>> gpurun_out/r03w.err || { tail -20 gpurun_out/r03w.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config plaw1m > gpurun_out/r03w_width_plaw1m.jsonl 2>> gpurun_out/r03w.err || { tail -20 gpurun_out/r03w.err; exit 1; }
cat gpurun_out/r03w_width_*.jsonl
echo all done
