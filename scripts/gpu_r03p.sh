# round 3, GPU call p: same-box A/B of the round-3 tree against the start-of-round build
# (8e123c2) on the BASELINE configs (Reddit bf16 N=256, products N=128, 1M power-law N=64)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm/libofx_spmm_base.so
for lib in base main base main; do
  if [ $lib = base ]; then export OFX_SPMM_LIB=$BASE; else unset OFX_SPMM_LIB; fi
  for c in reddit products plaw1m; do
    echo "== $lib $c" >> gpurun_out/r03p_ab.txt
    timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 4 --reps 5 --variants 0 >> gpurun_out/r03p_ab.txt 2>&1 || { tail -20 gpurun_out/r03p_ab.txt; exit 1; }
  done
done
unset OFX_SPMM_LIB
grep -A3 "==" gpurun_out/r03p_ab.txt | grep -v "^--" | head -80
echo all done
