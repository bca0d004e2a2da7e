# round 3, GPU call c: full GPU suite (zero-fill, new forms), forms sweep, bench, other configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03c_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r03c_gpu_tests.txt
timeout -k 10 900 python -u scripts/probe_split.py --no-old --variants 0,10022,30000,30001,30002,30003,30004,30005 > gpurun_out/r03c_probe_forms.jsonl 2> gpurun_out/r03c_probe_forms.err || { tail -20 gpurun_out/r03c_probe_forms.err; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err || { tail -20 gpurun_out/r03c_bench.err; exit 1; }
cat gpurun_out/r03c_bench.json
for c in reddit plaw1m; do
  timeout -k 10 600 python -u scripts/bench_config.py --config $c > gpurun_out/r03c_$c.json 2> gpurun_out/r03c_$c.err || { tail -20 gpurun_out/r03c_$c.err; exit 1; }
done
echo all done
