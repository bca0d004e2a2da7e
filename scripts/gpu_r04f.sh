# round 4, GPU call f: the rank-local SpMM phase on the round-4 kernels (VERDICT r3 item 5:
# products N=128 at G = 2 / 4 / 8, Reddit bf16 N=256 at G = 4), then rocprofv3 kernel trace + PMC
# passes of bench.py for the 1M power-law (N=64) and Reddit-shaped (bf16 N=256) configurations
# (VERDICT r3 item 3).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for g in 2 4 8; do
  timeout -k 10 240 python -u scripts/rank_local.py --config products --world $g \
    > gpurun_out/r04f_rank_local_products_g$g.json 2> gpurun_out/r04f_rank_local.err \
    || { tail -20 gpurun_out/r04f_rank_local.err; exit 1; }
  tail -c 300 gpurun_out/r04f_rank_local_products_g$g.json; echo
done
timeout -k 10 240 python -u scripts/rank_local.py --config reddit --world 4 \
  > gpurun_out/r04f_rank_local_reddit_g4.json 2>> gpurun_out/r04f_rank_local.err \
  || { tail -20 gpurun_out/r04f_rank_local.err; exit 1; }
tail -c 300 gpurun_out/r04f_rank_local_reddit_g4.json; echo
bash scripts/profile.sh r04f_plaw1m --config plaw1m --steps 10 --warmup 3 --no-cpu-baseline || exit 1
bash scripts/profile.sh r04f_reddit --config reddit --steps 10 --warmup 3 --no-cpu-baseline || exit 1
cat gpurun_out/prof_r04f_plaw1m/trace_bench.json gpurun_out/prof_r04f_reddit/trace_bench.json
# the 8-rank products rehearsal (gloo, ranks sharing this GPU): tune() must
# report the plain row split + all-gather (torch/p1 here, rccl/p1 on the node) as measured
T0=$SECONDS
timeout -k 10 900 python -u bench.py --gpus 8 --backend gloo --steps 3 --warmup 1 --tune-budget 150 \
  --deadline 850 > gpurun_out/r04f_rehearsal8_products.json 2> gpurun_out/r04f_rehearsal8_products.err \
  || { tail -40 gpurun_out/r04f_rehearsal8_products.err; exit 1; }
echo "rehearsal wall seconds: $((SECONDS - T0))" | tee -a gpurun_out/r04f_rehearsal8_products.err
grep "tune\]" gpurun_out/r04f_rehearsal8_products.err | head -20
echo all done
