# round 4, GPU call p: fp32 N = 17-32 of mid-size launches -- tuning entries 10069-10072
# (one-element 16 / 32-lane groups with column passes; the shifted window with 16-lane wave items)
# against the automatic pick, on the arxiv-shaped and 60k x 1.5M graphs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04s_f32mid.jsonl
for g in 169343:1166243 60000:1500000; do
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 17,24,25,32,33,41 --dtypes f32 --rounds 3 --reps 20 \
    --variants 0,10069,10070,10071,10072 >> $O 2>> gpurun_out/r04s_p.err || { tail -20 gpurun_out/r04s_p.err; exit 1; }
done
echo all done
