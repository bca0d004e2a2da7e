# round 3, GPU call y: lane layout of narrow 16-bit rows (bf16 N = 8..64: VEC x LPR forced against
# the automatic widest-vector choice) on the products and Reddit graphs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/width_sweep.py --config products --widths 8,16,32,64 --dtypes bf16 --variants 0,804,808,404,408,416,204,208,216,232,108,116,132 > gpurun_out/r03y_lanes_products.jsonl 2> gpurun_out/r03y.err || { tail -20 gpurun_out/r03y.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 16,32,64 --dtypes bf16 --variants 0,804,808,404,408,416,204,208,216,116,132 > gpurun_out/r03y_lanes_reddit.jsonl 2>> gpurun_out/r03y.err || { tail -20 gpurun_out/r03y.err; exit 1; }
cat gpurun_out/r03y_lanes_*.jsonl
echo all done
