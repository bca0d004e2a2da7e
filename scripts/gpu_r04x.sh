# round 4, GPU call x: rows of 33-64 columns on mid-size graphs -- tuning entries 10078 / 10079
# (16-bit: 16 / 8-B lanes with 16-lane wave items) and 10080 / 10081 (fp32: 16-B lanes with 16-lane
# wave items, U = 8 / 4) against the automatic pick (wave items in the light rows' own lane
# mapping); every line bit-compared with it and sampled against the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04x_mid64.jsonl
for g in 169343:1166243 60000:1500000; do
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 40,48,64 --dtypes bf16 --rounds 3 --reps 20 \
    --variants 0,10078,10079 >> $O 2>> gpurun_out/r04x.err || { tail -20 gpurun_out/r04x.err; exit 1; }
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 36,48,64 --dtypes f32 --rounds 3 --reps 20 \
    --variants 0,10080,10081 >> $O 2>> gpurun_out/r04x.err || { tail -20 gpurun_out/r04x.err; exit 1; }
done
echo all done
