# round 3, GPU call ac: the 64-lane path with coalesced (col, val) batches + v_readlane (new) against
# the scalar-cache form (lpr64old), odd and wide widths, forced 32- and 64-lane layouts; GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ac_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ac_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ac_gpu_tests.txt
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
O=gpurun_out/r03ac_sweep.jsonl
for lib in new old; do
  if [ $lib = new ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_lpr64old.so; fi
  echo "== $lib" >> $O
  timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 41,47 --dtypes f32,bf16 --variants 0,132,164 >> $O 2>> gpurun_out/r03ac.err || { tail -20 gpurun_out/r03ac.err; exit 1; }
  timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 200,256,300,512 --dtypes f32,bf16 --variants 0,432,464,832,864 >> $O 2>> gpurun_out/r03ac.err || { tail -20 gpurun_out/r03ac.err; exit 1; }
  timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 41,512 --dtypes bf16,f32 --variants 0 >> $O 2>> gpurun_out/r03ac.err || { tail -20 gpurun_out/r03ac.err; exit 1; }
done
unset OFX_SPMM_LIB
echo all done
