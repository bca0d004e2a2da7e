# round 3, GPU call ai: 16-bit N <= 64 lanes (N / 16 per lane, >= 16 lanes) in the prefetching form
# too — parity subset, then the mid-size sweep with the new library and the previous one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefetch_form_lane or shifted_window or narrow_16bit or dtype_width or forced_variants or mid_form or small_form or walked or narrow_form or plan_once" > gpurun_out/r03ai_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ai_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ai_gpu_tests.txt
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
O=gpurun_out/r03ai_sweep.jsonl
for lib in new prev; do
  if [ $lib = new ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_prev.so; fi
  echo "== $lib" >> $O
  for g in 169343:1166243 60000:1500000 200000:2800000; do
    timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,32,48,64 --dtypes bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r03ai.err || { tail -20 gpurun_out/r03ai.err; exit 1; }
    timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 17,41,47,99 --dtypes f32 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r03ai.err || { tail -20 gpurun_out/r03ai.err; exit 1; }
  done
done
unset OFX_SPMM_LIB
echo all done
