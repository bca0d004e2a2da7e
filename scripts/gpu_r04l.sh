# round 4, GPU call l: the narrow shape for 16-bit N = 8 / 16 and fp32 N = 8 in the prefetching
# form's size range (launch_narrow_pf).  Parity selection (test_gpu_forms runs these widths on both
# sides of kPrefetchNnz), then the mid-size width sweep of call i again on this tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04l_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04l_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04l_sel.txt | head -60; exit 1; }
O=gpurun_out/r04l_sweep.jsonl
for g in 169343:1166243 60000:1500000 19717:88648; do
  timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,41,47,64,128,256 --dtypes f32,bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r04l.err || { tail -20 gpurun_out/r04l.err; exit 1; }
done
echo all done
