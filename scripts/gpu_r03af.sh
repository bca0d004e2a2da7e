# round 3, GPU call af: 16-lane groups for rows of fewer than 16 single-element lanes (N < 16) in the
# bandwidth configuration — parity tests, then automatic against the n-lane layouts
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shifted_window or narrow_16bit or dtype_width or forced_variants or edge_cases or unaligned" > gpurun_out/r03af_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03af_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03af_gpu_tests.txt
O=gpurun_out/r03af_sweep.jsonl
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 1,2,3,4,8 --dtypes f32,bf16 --variants 0,104,108,116 > $O 2> gpurun_out/r03af.err || { tail -20 gpurun_out/r03af.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config plaw1m --widths 1,4,8 --dtypes f32 --variants 0,104,108,116 >> $O 2>> gpurun_out/r03af.err || { tail -20 gpurun_out/r03af.err; exit 1; }
cat $O
echo all done
