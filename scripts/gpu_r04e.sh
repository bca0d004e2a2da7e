# round 4, GPU call e: the current tree (parked prefetching-form layouts + one-launch planner +
# in-kernel hub reduce + forced global-load variant): the parity selection under the
# bounds-checked build (every test's bounds record checked), then under the release build; then an
# interleaved A/B of per-call time against the round-3 kernels (HIP graph replay).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04e_2a.txt 2>&1
rc=$?; echo "2a new tree, bounds-checked: rc=$rc"; tail -3 gpurun_out/r04e_2a.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04e_2a.txt | head -60; exit 1; }
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04e_2b.txt 2>&1
rc=$?; echo "2b new tree, release: rc=$rc"; tail -3 gpurun_out/r04e_2b.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04e_2b.txt | head -60; exit 1; }
SPECS="pubmed:16:0 pubmed:64:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_prev.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04e_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04e_ab.jsonl || { tail -20 gpurun_out/r04e_ab.err; exit 1; }
done
echo all done
