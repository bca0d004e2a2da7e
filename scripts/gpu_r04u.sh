# round 4, GPU call u: 16-bit rows of 20-32 columns on mid-size graphs (bf16 N = 32: 220 us on the
# arxiv-shaped graph, the 2-element lanes' wave items at 259 VGPRs) -- tuning entries 10051 /
# 10059 / 10067 / 10073-10077 (8 / 16-B lanes or one-element passes, 16-lane wave items) against
# the automatic pick; every line bit-compared with it and sampled against the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04u_16bit_mid.jsonl
for g in 169343:1166243 60000:1500000; do
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 20,24,28,32 --dtypes bf16 --rounds 3 --reps 20 \
    --variants 0,10051,10059,10067,10073,10074,10075,10076,10077 >> $O 2>> gpurun_out/r04u.err || { tail -20 gpurun_out/r04u.err; exit 1; }
done
timeout -k 10 300 python -u scripts/width_sweep.py --graph 169343:1166243 --widths 32 --dtypes f16 --rounds 3 --reps 20 \
  --variants 0,10073,10074,10075,10076 >> $O 2>> gpurun_out/r04u.err || { tail -20 gpurun_out/r04u.err; exit 1; }
echo all done
