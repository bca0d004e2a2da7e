# round 3, GPU call t: walked hubs (hubs of <= 4 chunks summed by one worker in launches of >= 2^26
# nonzeros): parity tests, then same-process A/B of walk settings on the BASELINE configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "walked_hubs or baseline_configs or products_scale or narrow_form or hub_rows or plan_once" > gpurun_out/r03t_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03t_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03t_gpu_tests.txt
for c in reddit products; do
  timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 4 --reps 5 --variants 0,0w-1,0w2,0w8 >> gpurun_out/r03t_ab.txt 2>&1 || { tail -5 gpurun_out/r03t_ab.txt; exit 1; }
done
timeout -k 10 300 python -u scripts/ab.py --config plaw1m --rounds 4 --reps 5 --variants 0,0w2,0w4 >> gpurun_out/r03t_ab.txt 2>&1 || { tail -5 gpurun_out/r03t_ab.txt; exit 1; }
timeout -k 10 300 python -u scripts/ab.py --config plaw1m --n 16 --rounds 4 --reps 5 --variants 0,0w2,0w4 >> gpurun_out/r03t_ab.txt 2>&1 || { tail -5 gpurun_out/r03t_ab.txt; exit 1; }
grep -E "median|identical" gpurun_out/r03t_ab.txt
echo all done
