set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r03a_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r03a_gpu_tests.txt
timeout -k 10 600 python -u scripts/probe_split.py > gpurun_out/r03a_probe_split.jsonl 2> gpurun_out/r03a_probe_split.err || { tail -20 gpurun_out/r03a_probe_split.err; exit 1; }
echo probe done
