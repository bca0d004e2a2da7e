# round 4, GPU call ad: the fp32 N = 16 narrow form of mid-size launches at U = 8 (call ac).
# Final tree: parity selection under the bounds-checked build, the full GPU suite, smoke, the
# bench line (release), a graph-replay A/B against the round-3 library, and the products profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition or reused"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04ad_sel_dbg.txt 2>&1
rc=$?; echo "parity selection, bounds-checked: rc=$rc"; tail -2 gpurun_out/r04ad_sel_dbg.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04ad_sel_dbg.txt | head -60; exit 1; }
timeout -k 10 900 $PT > gpurun_out/r04ad_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04ad_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04ad_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ad_smoke.txt 2>&1 || { tail -20 gpurun_out/r04ad_smoke.txt; exit 1; }
cat gpurun_out/r04ad_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r04ad_bench.json 2> gpurun_out/r04ad_bench.err || { tail -20 gpurun_out/r04ad_bench.err; exit 1; }
cat gpurun_out/r04ad_bench.json
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
SPECS="pubmed:16:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev new prev new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04ad_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04ad_ab.jsonl || { tail -20 gpurun_out/r04ad_ab.err; exit 1; }
done
bash scripts/profile.sh r04ad_products --steps 10 --warmup 3 --no-cpu-baseline || exit 1
echo all done
