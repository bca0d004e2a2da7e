# round 4, GPU call g: the one-launch planner's look-back was one lane per step (call e's A/B:
# products 8.53 -> 9.27 ms, 1M power-law N=16 351 -> 684 us, arxiv-shaped N=16 46 -> 72 us).
# Now 64 predecessors per step.  Parity selection (release), then an interleaved A/B of the
# round-3 library (prev), the tree before the planner change (ef1), this tree (new) and this tree
# without the in-kernel hub reduce (nolr), then a rocprofv3 kernel trace of this tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04g_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04g_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04g_sel.txt | head -60; exit 1; }
SPECS="pubmed:16:0 pubmed:64:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev ef1 new nolr prev ef1 new nolr; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04g_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04g_ab.jsonl || { tail -20 gpurun_out/r04g_ab.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04g_trace -o run \
  -- python3 scripts/probe_graph.py arxiv:16:0 plaw1m:16:0 products:128:0 > gpurun_out/r04g_trace.txt 2>&1 \
  || { tail -20 gpurun_out/r04g_trace.txt; exit 1; }
echo all done
