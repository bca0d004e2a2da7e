# round 4, GPU call z: 16-bit rows of <= 64 columns in the small and mid forms with N / 16 elements
# per lane (call y).  Parity selection under the bounds-checked build, then the final tree's full
# GPU suite, smoke and bench line (release), and the small-graph width sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition or reused"
OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 400 $PT -k "$SEL2" > gpurun_out/r04z_sel_dbg.txt 2>&1
rc=$?; echo "parity selection, bounds-checked: rc=$rc"; tail -2 gpurun_out/r04z_sel_dbg.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04z_sel_dbg.txt | head -60; exit 1; }
timeout -k 10 900 $PT > gpurun_out/r04z_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r04z_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04z_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.txt 2>&1 || { tail -20 gpurun_out/r04z_smoke.txt; exit 1; }
cat gpurun_out/r04z_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || { tail -20 gpurun_out/r04z_bench.err; exit 1; }
cat gpurun_out/r04z_bench.json
for g in 2708:10556 19717:88648 20000:400000; do
  timeout -k 10 200 python -u scripts/width_sweep.py --graph $g --widths 8,16,32,64,128 --dtypes f32,bf16,f16 --rounds 3 --reps 50 \
    >> gpurun_out/r04z_small_sweep.jsonl 2>> gpurun_out/r04z.err || { tail -20 gpurun_out/r04z.err; exit 1; }
done
echo all done
