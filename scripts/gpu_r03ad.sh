# round 3, GPU call ad: fp32 widths not a multiple of 4 (shifted last window, Cfg::SH) — parity
# tests, then the automatic choice against the one-element-per-lane layouts it replaces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shifted_window or unaligned or dtype_width or forced_variants or out_of_range or edge_cases" > gpurun_out/r03ad_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03ad_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03ad_gpu_tests.txt
O=gpurun_out/r03ad_sweep.jsonl
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 17,41,47,63,99,301 --dtypes f32 --variants 0,132,164 > $O 2> gpurun_out/r03ad.err || { tail -20 gpurun_out/r03ad.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config reddit --widths 41 --dtypes f32 --variants 0,164 >> $O 2>> gpurun_out/r03ad.err || { tail -20 gpurun_out/r03ad.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 16,48,64,128 --dtypes f32 >> $O 2>> gpurun_out/r03ad.err || { tail -20 gpurun_out/r03ad.err; exit 1; }
cat $O
echo all done
