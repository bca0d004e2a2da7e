# round 3, GPU call f: buffer-load B rows + light rows by index: full GPU suite, same-box A/B
# against the previous commit's kernels, N=16 mid-size configurations, forms sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03f_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03f_gpu_tests.txt
BASE=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm/libofx_spmm_base.so
for lib in base main base main; do
  if [ $lib = base ]; then export OFX_SPMM_LIB=$BASE; else unset OFX_SPMM_LIB; fi
  timeout -k 10 300 python -u scripts/probe_split.py --no-old --graphs arxiv,p2m,plaw1m,products --widths 16 --variants 10021,10022 --rounds 3 >> gpurun_out/r03f_ab_$lib.jsonl 2>> gpurun_out/r03f_ab.err || { tail -20 gpurun_out/r03f_ab.err; exit 1; }
  timeout -k 10 300 python -u scripts/probe_split.py --no-old --graphs p2m,plaw1m,products --widths 64,128 --variants 416,432 --rounds 3 >> gpurun_out/r03f_ab_$lib.jsonl 2>> gpurun_out/r03f_ab.err || { tail -20 gpurun_out/r03f_ab.err; exit 1; }
done
unset OFX_SPMM_LIB
timeout -k 10 600 python -u scripts/probe_split.py --no-old --graphs pubmed,small20k,arxiv,g60k,p2m,p5m,plaw1m --widths 16 --variants 0,10021,10022,10026,10027,10028,10029,10030,10029h-1,10029h128,30004h-1,30005h-1,404 > gpurun_out/r03f_probe_n16.jsonl 2> gpurun_out/r03f_probe_n16.err || { tail -20 gpurun_out/r03f_probe_n16.err; exit 1; }
timeout -k 10 600 python -u scripts/probe_split.py --no-old --variants 0,30003,30004,30005 > gpurun_out/r03f_probe_forms.jsonl 2> gpurun_out/r03f_probe_forms.err || { tail -20 gpurun_out/r03f_probe_forms.err; exit 1; }
echo all done
