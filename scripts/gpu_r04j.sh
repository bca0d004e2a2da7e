# round 4, GPU call j: papers100M-scale on one GPU (111M rows, 1.62B nonzeros, N=128 fp32):
# re-timed on the round-4 tree with the sampled oracle check, then rocprofv3 kernel trace + PMC
# passes of bench.py --config papers (the lowest-fraction BASELINE workload,
# no PMC summary before).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/bench_config.py --config papers > gpurun_out/r04j_papers.json 2> gpurun_out/r04j_papers.err \
  || { tail -20 gpurun_out/r04j_papers.err; exit 1; }
cat gpurun_out/r04j_papers.json
bash scripts/profile.sh r04j_papers --config papers --steps 5 --warmup 2 --no-cpu-baseline || exit 1
cat gpurun_out/prof_r04j_papers/trace_bench.json
echo all done
