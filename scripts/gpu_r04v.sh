# round 4, GPU call v: 16-bit rows of 17-32 even columns of mid-size launches in the narrow shape
# (launch_narrow_pf: 8-B lanes over 8 lanes or 4-B lanes over 16, 16-lane wave items).  Parity
# selection under the bounds-checked build and the release build (test_gpu_forms: bf16 N = 32,
# f16 N = 24 on both sides of kPrefetchNnz), an A/B against the round-3 library, the width sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition or reused"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04v_sel_dbg.txt 2>&1
rc=$?; echo "parity selection, bounds-checked: rc=$rc"; tail -2 gpurun_out/r04v_sel_dbg.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04v_sel_dbg.txt | head -60; exit 1; }
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04v_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04v_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04v_sel.txt | head -60; exit 1; }
SPECS="small20k:16:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 plaw1m:16:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04v_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04v_ab.jsonl || { tail -20 gpurun_out/r04v_ab.err; exit 1; }
done
echo "A/B done"
O=gpurun_out/r04v_sweep.jsonl
for g in 169343:1166243 60000:1500000 19717:88648; do
  timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,17,20,24,32,41,47,63,64,128,256 --dtypes f32,bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r04v.err || { tail -20 gpurun_out/r04v.err; exit 1; }
done
echo all done
