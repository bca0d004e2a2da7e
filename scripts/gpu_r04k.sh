# round 4, GPU call k: planner rows per thread by launch size (4 up to 2^18 rows, 16 above) and
# the narrow-row tuning entries 50-63 (16-bit N = 8 / 16, fp32 N = 8 on mid-size graphs).
# Parity selection; A/B against the round-3 library; then the variants on the arxiv-shaped,
# 60k x 1.5M and 2M-nonzero graphs (each line bit-compared with the automatic pick and sampled
# against the oracle).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04k_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04k_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04k_sel.txt | head -60; exit 1; }
SPECS="small20k:16:0 arxiv:16:0 arxiv:64:0 g60k:16:0 p2m:16:0 p5m:16:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04k_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04k_ab.jsonl || { tail -20 gpurun_out/r04k_ab.err; exit 1; }
done
echo "A/B done"
O=gpurun_out/r04k_variants.jsonl
for g in 169343:1166243 60000:1500000 169343:2000000; do
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 8,16 --dtypes bf16 --rounds 3 --reps 20 \
    --variants 0,10050,10051,10052,10053,10054,10055,10056,10057,10058,10059 >> $O 2>> gpurun_out/r04k.err || { tail -20 gpurun_out/r04k.err; exit 1; }
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 8 --dtypes f32 --rounds 3 --reps 20 \
    --variants 0,10060,10061,10062,10063 >> $O 2>> gpurun_out/r04k.err || { tail -20 gpurun_out/r04k.err; exit 1; }
done
echo all done
