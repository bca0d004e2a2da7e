# round 3, GPU call r: light rows by index / by order / runtime rule (default) / start-of-round
# build, same box, interleaved twice: BASELINE configs (ab.py) and mid-size launches (probe_graph)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in main order index base; do
    if [ $lib = main ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_$lib.so; fi
    for c in reddit products plaw1m; do
      echo "== $lib $c" >> gpurun_out/r03r_ab.txt
      timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 3 --reps 5 --variants 0 2>&1 | grep "median" >> gpurun_out/r03r_ab.txt || { tail -5 gpurun_out/r03r_ab.txt; exit 1; }
    done
    echo "== $lib mid" >> gpurun_out/r03r_ab.txt
    timeout -k 10 300 python -u scripts/probe_graph.py arxiv:16:0 arxiv:64:0 p2m:16:0 p2m:64:0 p5m:32:0 p5m:128:0 >> gpurun_out/r03r_ab.txt 2>> gpurun_out/r03r_graph.err || { tail -5 gpurun_out/r03r_graph.err; exit 1; }
  done
done
unset OFX_SPMM_LIB
cat gpurun_out/r03r_ab.txt
echo all done
