# round 4, GPU call m: odd 16-bit widths 17-64 of mid-size launches in one-element 16 / 32-lane
# groups (launch_odd16_pf).  Parity selection (test_gpu_forms: bf16 N=41, f16 N=63 both sides of
# kPrefetchNnz), the mid-size width sweep on this tree, and a kernel trace of the arxiv-shaped
# N = 16 / 64 calls (plan and main separately).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04m_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04m_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04m_sel.txt | head -60; exit 1; }
O=gpurun_out/r04m_sweep.jsonl
for g in 169343:1166243 60000:1500000 19717:88648; do
  timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,17,41,47,63,64,128,256 --dtypes f32,bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r04m.err || { tail -20 gpurun_out/r04m.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_trace -o run \
  -- python3 scripts/probe_graph.py arxiv:16:0 arxiv:64:0 > gpurun_out/r04m_trace.txt 2>&1 \
  || { tail -20 gpurun_out/r04m_trace.txt; exit 1; }
echo all done
