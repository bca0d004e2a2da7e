# round 3, GPU call u: products regression hunt — the reverted tree (main) against buffer loads off
# (glob), light rows by order (order) and the round-2 library (base), same box, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in main glob order base; do
    if [ $lib = main ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_$lib.so; fi
    for c in products reddit plaw1m; do
      echo "== $lib $c" >> gpurun_out/r03u_ab.txt
      timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 3 --reps 5 --variants 0 2>&1 | grep "median" >> gpurun_out/r03u_ab.txt || { tail -5 gpurun_out/r03u_ab.txt; exit 1; }
    done
  done
done
unset OFX_SPMM_LIB
cat gpurun_out/r03u_ab.txt
echo all done
