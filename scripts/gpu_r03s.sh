# round 3, GPU call s (re-entry): fresh-box validation of the tree at 70f22a4 — full GPU suite,
# smoke, bench line, same-box A/B against the round-2 library (BASELINE configs, mid-size N=16/64
# launches), rocprofv3 trace + PMC for products N=128 and the 1M power-law graph at N=16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03s_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03s_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s_smoke.txt 2>&1 || { tail -20 gpurun_out/r03s_smoke.txt; exit 1; }
cat gpurun_out/r03s_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03s_bench.json 2> gpurun_out/r03s_bench.err || { tail -20 gpurun_out/r03s_bench.err; exit 1; }
cat gpurun_out/r03s_bench.json
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
for r in 1 2; do
  for lib in main base; do
    if [ $lib = main ]; then unset OFX_SPMM_LIB; else export OFX_SPMM_LIB=$L/libofx_spmm_$lib.so; fi
    for c in reddit products plaw1m; do
      echo "== $lib $c" >> gpurun_out/r03s_ab.txt
      timeout -k 10 300 python -u scripts/ab.py --config $c --rounds 3 --reps 5 --variants 0 2>&1 | grep "median" >> gpurun_out/r03s_ab.txt || { tail -5 gpurun_out/r03s_ab.txt; exit 1; }
    done
    echo "== $lib mid" >> gpurun_out/r03s_ab.txt
    timeout -k 10 300 python -u scripts/probe_graph.py arxiv:16:0 arxiv:64:0 p2m:16:0 p2m:64:0 p5m:32:0 plaw1m:16:0 >> gpurun_out/r03s_ab.txt 2>> gpurun_out/r03s_graph.err || { tail -5 gpurun_out/r03s_graph.err; exit 1; }
  done
done
unset OFX_SPMM_LIB
cat gpurun_out/r03s_ab.txt
bash scripts/profile.sh r03s_products --steps 10 --warmup 3 --no-cpu-baseline || exit 1
PROG=scripts/bench_config.py bash scripts/profile.sh r03s_plaw1m_n16 --config plaw1m --n 16 --no-check --reps 10 || exit 1
echo all done
