# round 3, GPU call d: staged-offset zero fill: parity subset, forms sweep, zero-fill A/B, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_out_of_range.py tests/test_gpu_parity.py tests/test_fused.py tests/test_backward.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03d_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03d_gpu_tests.txt
timeout -k 10 600 python -u scripts/probe_split.py --no-old --graphs pubmed,small20k,arxiv,g60k,p2m,p5m,plaw1m,products --variants 0,30003,30004,30005 > gpurun_out/r03d_probe_forms.jsonl 2> gpurun_out/r03d_probe_forms.err || { tail -20 gpurun_out/r03d_probe_forms.err; exit 1; }
for lib in nozf main nozf; do
  if [ $lib = nozf ]; then export OFX_SPMM_LIB=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm/libofx_spmm_nozf.so; else unset OFX_SPMM_LIB; fi
  timeout -k 10 300 python -u scripts/probe_split.py --no-old --graphs arxiv,p2m,plaw1m,products --widths 16,128 --variants 0 --rounds 5 >> gpurun_out/r03d_ab_zero_fill_$lib.jsonl 2>> gpurun_out/r03d_ab.err || { tail -20 gpurun_out/r03d_ab.err; exit 1; }
done
unset OFX_SPMM_LIB
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || { tail -20 gpurun_out/r03d_bench.err; exit 1; }
cat gpurun_out/r03d_bench.json
timeout -k 10 300 python -u scripts/bench_config.py --config reddit > gpurun_out/r03d_reddit.json 2> gpurun_out/r03d_reddit.err || { tail -20 gpurun_out/r03d_reddit.err; exit 1; }
cat gpurun_out/r03d_reddit.json
echo all done
