# round 4, GPU call aa: 64-lane rows (bf16 N >= 512, fp32 N >= 256) with col/val through the
# scalar cache (OFX_AB_LPR64_SCALAR build, the round-2 path) against the readlane path (round 3),
# Reddit-shaped (B in the Infinity Cache) and products-shaped (B in HBM) graphs, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for lib in new sc64 new sc64; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 300 python -u scripts/width_sweep.py --config reddit --widths 256,512,1024 --dtypes bf16,f32 --rounds 3 --reps 5 \
    2>> gpurun_out/r04aa.err | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04aa_lpr64.jsonl || { tail -20 gpurun_out/r04aa.err; exit 1; }
  OFX_SPMM_LIB=$f timeout -k 10 300 python -u scripts/width_sweep.py --config products --widths 512 --dtypes bf16 --rounds 3 --reps 5 \
    2>> gpurun_out/r04aa.err | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04aa_lpr64.jsonl || { tail -20 gpurun_out/r04aa.err; exit 1; }
done
echo all done
