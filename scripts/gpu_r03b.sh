# round 3, GPU call b: every launch form over power-law graphs (new split), for the form rules
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/probe_split.py --no-old > gpurun_out/r03b_probe_forms.jsonl 2> gpurun_out/r03b_probe_forms.err || { tail -20 gpurun_out/r03b_probe_forms.err; exit 1; }
echo probe done
