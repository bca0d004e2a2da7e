# round 4, GPU call c: the one-launch planner (decoupled look-back) and the in-kernel hub reduce of
# the mid-size forms (Cfg::LR): parity of every planned form, then an interleaved A/B of per-call
# time (HIP graph replay, scripts/probe_graph.py) against the round-3 library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose" \
  > gpurun_out/r04c_tests.txt 2>&1 || { tail -40 gpurun_out/r04c_tests.txt; exit 1; }
tail -3 gpurun_out/r04c_tests.txt
SPECS="pubmed:16:0 pubmed:64:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 p5m:64:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_prev.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 400 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04c_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04c_ab.jsonl || { tail -20 gpurun_out/r04c_ab.err; exit 1; }
done
echo all done
