# round 3, GPU call j: device (graph replay) against eager time per call, and the kernel trace of
# the same mid-size launches (which kernels the per-call time goes to)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SPECS="pubmed:16:0 pubmed:64:0 arxiv:16:0 arxiv:16:10022 arxiv:16:10028 arxiv:16:10029h128 arxiv:64:0 g60k:16:0 p2m:16:0 p2m:64:0 plaw1m:16:0 plaw1m:16:10028"
timeout -k 10 400 python -u scripts/probe_graph.py $SPECS > gpurun_out/r03j_graph.jsonl 2> gpurun_out/r03j_graph.err || { tail -20 gpurun_out/r03j_graph.err; exit 1; }
cat gpurun_out/r03j_graph.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03j_trace -o run -- python3 scripts/trace_forms.py $SPECS > gpurun_out/r03j_trace.log 2>&1 || { tail -20 gpurun_out/r03j_trace.log; exit 1; }
python3 scripts/trace_segments.py $(ls gpurun_out/r03j_trace/*/*kernel_trace.csv 2>/dev/null || ls gpurun_out/r03j_trace/*kernel_trace.csv) > gpurun_out/r03j_segments.txt
cat gpurun_out/r03j_segments.txt
echo all done
