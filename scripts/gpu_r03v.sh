# round 3, GPU call v: main-kernel occupancy A/B (amdgpu_waves_per_eu 8 / 7 against the default), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in main wpe8 wpe7; do
    if [ $lib = main ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_$lib.so; fi
    for c in products reddit plaw1m; do
      echo "== $lib $c" >> gpurun_out/r03v_ab.txt
      timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 3 --reps 5 --variants 0 2>&1 | grep "median" >> gpurun_out/r03v_ab.txt || { tail -5 gpurun_out/r03v_ab.txt; exit 1; }
    done
  done
done
unset OFX_SPMM_LIB
cat gpurun_out/r03v_ab.txt
echo all done
