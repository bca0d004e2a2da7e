# round 3, GPU call ab: odd and wide dense widths (GNN classifier widths: 47 products, 41 Reddit, 40
# arxiv classes) — forced lane layouts against the automatic one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ab_odd.jsonl
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 47,41,17 --dtypes f32,bf16 --variants 0,116,132,164 > $O 2> gpurun_out/r03ab.err || { tail -20 gpurun_out/r03ab.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 3 --dtypes f32,bf16 --variants 0,104,108,116 >> $O 2>> gpurun_out/r03ab.err || { tail -20 gpurun_out/r03ab.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 40,100,200,300 --dtypes f32,bf16 --variants 0,216,232,264,416,432,464,816,832,864 >> $O 2>> gpurun_out/r03ab.err || { tail -20 gpurun_out/r03ab.err; exit 1; }
cat $O
echo all done
