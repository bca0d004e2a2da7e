# round 3, GPU call i: mid-size N=16 configurations (rows per wave, prefetch, wave items, heavy cut)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k tuning_table --timeout 120 --timeout-method thread > gpurun_out/r03i_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r03i_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r03i_gpu_tests.txt
timeout -k 10 600 python -u scripts/probe_split.py --no-old --graphs pubmed,small20k,arxiv,g60k,p2m,p5m,plaw1m --widths 16 --variants 0,10021,10022,10026,10027,10028,10029,10030,10029h-1,10029h128,30004h-1,30005h-1,404 > gpurun_out/r03i_probe_n16.jsonl 2> gpurun_out/r03i_probe_n16.err || { tail -20 gpurun_out/r03i_probe_n16.err; exit 1; }
echo all done
