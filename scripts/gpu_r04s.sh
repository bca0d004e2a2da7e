# round 4, GPU call s: the tree with the fused plan reverted (three cuts measured slower) and the
# look-back's spins bounded.  Parity selection under the bounds-checked build and the release
# build (test_plan_reused_workspace: three graphs through one workspace), an A/B against the
# round-3 library, then the fp32 N = 17-41 mid-size tuning entries without the fused plan.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition or reused"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04s_sel_dbg.txt 2>&1
rc=$?; echo "parity selection, bounds-checked: rc=$rc"; tail -2 gpurun_out/r04s_sel_dbg.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04s_sel_dbg.txt | head -60; exit 1; }
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04s_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04s_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04s_sel.txt | head -60; exit 1; }
SPECS="small20k:16:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 plaw1m:16:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04s_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04s_ab.jsonl || { tail -20 gpurun_out/r04s_ab.err; exit 1; }
done
echo "A/B done"
bash scripts/gpu_r04p.sh
