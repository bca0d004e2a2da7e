# round 4, GPU call y: 16-bit rows of <= 64 columns in the small and mid forms (one launch for
# <= 2^20 products; block items) with N / 16 elements per lane, as the larger forms take them
# (OFX_AB_NARROW16_SMALL build), against this tree's widest-vector lanes: Cora-, PubMed-shaped
# and 20k-row graphs, bf16 / f16 N = 8-64, interleaved, each line sampled against the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for lib in new n16s new n16s; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  for g in 2708:10556 19717:88648 20000:400000; do
    OFX_SPMM_LIB=$f timeout -k 10 200 python -u scripts/width_sweep.py --graph $g --widths 8,16,32,64 --dtypes bf16,f16 --rounds 3 --reps 50 \
      2>> gpurun_out/r04y.err | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04y_small16.jsonl || { tail -20 gpurun_out/r04y.err; exit 1; }
  done
done
echo all done
