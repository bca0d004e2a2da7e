# round 4, GPU call o: the fused plan (the mid-size wave-item forms plan inside spmm_main: one
# launch per call).  Parity selection under the bounds-checked build (every test's bounds record
# checked) and the release build; A/B of graph-replayed calls against the round-3 library and this
# tree without the fused plan (OFX_AB_NO_FUSED_PLAN); kernel trace of the arxiv-shaped calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04o_sel_dbg.txt 2>&1
rc=$?; echo "parity selection, bounds-checked: rc=$rc"; tail -2 gpurun_out/r04o_sel_dbg.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04o_sel_dbg.txt | head -60; exit 1; }
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04o_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04o_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04o_sel.txt | head -60; exit 1; }
SPECS="pubmed:16:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 plaw1m:16:0 products:128:0"
for lib in prev nofp new prev nofp new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04o_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04o_ab.jsonl || { tail -20 gpurun_out/r04o_ab.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_trace -o run \
  -- python3 scripts/probe_graph.py arxiv:16:0 arxiv:64:0 > gpurun_out/r04o_trace.txt 2>&1 \
  || { tail -20 gpurun_out/r04o_trace.txt; exit 1; }
echo all done
