# round 3, GPU call m: N = 16 over the size range (mid form to products) for the narrow-row
# configurations with HL wave items, against the automatic pick
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=""
for g in small20k u169k2 p8m p11m p15m plaw1m u1m20 products; do for v in 0 10021 10028 10031 10033 10034 10033h64 10034h64; do S="$S $g:16:$v"; done; done
timeout -k 10 900 python -u scripts/probe_graph.py $S > gpurun_out/r03m_graph.jsonl 2> gpurun_out/r03m_graph.err || { tail -20 gpurun_out/r03m_graph.err; exit 1; }
cat gpurun_out/r03m_graph.jsonl
echo all done
