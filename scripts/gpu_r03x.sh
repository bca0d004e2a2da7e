# round 3, GPU call x: branch-free B-row loads in the bandwidth configurations (16-bit types had one
# row in flight per lane: hipcc waited vmcnt(0) before each load under its per-slot branch) —
# full GPU suite, then the width sweep with the previous library and the new one, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03x_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03x_gpu_tests.txt
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = new ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_prev.so; fi
    echo "== $lib" >> gpurun_out/r03x_sweep.jsonl
    timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 8,16,32,64,128,256 --dtypes bf16,f32 >> gpurun_out/r03x_sweep.jsonl 2>> gpurun_out/r03x.err || { tail -20 gpurun_out/r03x.err; exit 1; }
    timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 32,64,128,256 --dtypes bf16,f32 >> gpurun_out/r03x_sweep.jsonl 2>> gpurun_out/r03x.err || { tail -20 gpurun_out/r03x.err; exit 1; }
    timeout -k 10 400 python -u scripts/width_sweep.py --config plaw1m --widths 64,128 --dtypes bf16,f32 >> gpurun_out/r03x_sweep.jsonl 2>> gpurun_out/r03x.err || { tail -20 gpurun_out/r03x.err; exit 1; }
  done
done
unset OFX_SPMM_LIB
echo all done
