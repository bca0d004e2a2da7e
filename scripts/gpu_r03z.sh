# round 3, GPU call z: the 16-bit narrow-row lane layout (>= 16 lanes per row up to N = 64 in the
# bandwidth configuration): parity tests, then the automatic choice against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "narrow_16bit or dtype_width or forced_variants or tuning_table or baseline_configs" > gpurun_out/r03z_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03z_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03z_gpu_tests.txt
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = new ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_prev.so; fi
    echo "== $lib" >> gpurun_out/r03z_sweep.jsonl
    timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 8,16,32,48,64,128 --dtypes bf16,f16 >> gpurun_out/r03z_sweep.jsonl 2>> gpurun_out/r03z.err || { tail -20 gpurun_out/r03z.err; exit 1; }
    timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 16,32,64,256 --dtypes bf16 >> gpurun_out/r03z_sweep.jsonl 2>> gpurun_out/r03z.err || { tail -20 gpurun_out/r03z.err; exit 1; }
  done
done
unset OFX_SPMM_LIB
echo all done
