# round 3, GPU call e: same-box A/B of the staged-offset zero fill against the previous commit's
# kernels (forced configurations present in both), and a kernel trace of mid-size launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm/libofx_spmm_base.so
for lib in base main base main; do
  if [ $lib = base ]; then export OFX_SPMM_LIB=$BASE; else unset OFX_SPMM_LIB; fi
  timeout -k 10 300 python -u scripts/probe_split.py --no-old --graphs arxiv,p2m,plaw1m,products --widths 16 --variants 10021,10022 --rounds 3 >> gpurun_out/r03e_ab_$lib.jsonl 2>> gpurun_out/r03e_ab.err || { tail -20 gpurun_out/r03e_ab.err; exit 1; }
  timeout -k 10 300 python -u scripts/probe_split.py --no-old --graphs p2m,plaw1m,products --widths 128 --variants 432 --rounds 3 >> gpurun_out/r03e_ab_$lib.jsonl 2>> gpurun_out/r03e_ab.err || { tail -20 gpurun_out/r03e_ab.err; exit 1; }
done
unset OFX_SPMM_LIB
mkdir -p gpurun_out/r03e_trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03e_trace -o run -- python3 scripts/trace_forms.py arxiv:16:0 arxiv:16:30003 arxiv:64:0 arxiv:128:0 pubmed:16:0 pubmed:128:0 p2m:16:0 p2m:128:0 > gpurun_out/r03e_trace.log 2>&1 || { tail -20 gpurun_out/r03e_trace.log; exit 1; }
echo all done
