# round 3, GPU call ah: the width sweep on mid-size and small graphs (arxiv-shaped 169k x 1.17M,
# 60k x 1.5M, PubMed-shaped 19.7k x 89k), f32 / bf16 / f16 and odd widths: the small, mid and
# prefetching forms at the widths the BASELINE configs do not cover
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ah_sweep.jsonl
for g in 169343:1166243 60000:1500000 19717:88648; do
  timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,41,47,64,128,256 --dtypes f32,bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r03ah.err || { tail -20 gpurun_out/r03ah.err; exit 1; }
done
cat $O
echo all done
