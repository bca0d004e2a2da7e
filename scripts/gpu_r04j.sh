# round 4, GPU call j: (1) bench.py lines for the 1M power-law and Reddit-shaped configurations,
# now carrying roofline.traffic from the round-4 PMC summaries (profiles/{plaw1m,reddit}_rocprof);
# (2) odd 16-bit widths on mid-size graphs: tuning entries 10064-10068 (one element per lane in
# 16 / 32-lane groups, several column passes) against the automatic 64-lane rows; (3)
# papers100M-scale on one GPU (111M rows, 1.62B nonzeros, N=128 fp32): re-timed with the sampled
# oracle check, then rocprofv3 kernel trace + PMC passes of bench.py --config papers (VERDICT r3
# item 3).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in plaw1m reddit; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/r04j_bench_$c.json 2> gpurun_out/r04j_bench_$c.err \
    || { tail -20 gpurun_out/r04j_bench_$c.err; exit 1; }
  cat gpurun_out/r04j_bench_$c.json
done
O=gpurun_out/r04j_odd16.jsonl
for g in 169343:1166243 60000:1500000; do
  timeout -k 10 300 python -u scripts/width_sweep.py --graph $g --widths 17,41,47,63 --dtypes bf16 --rounds 3 --reps 20 \
    --variants 0,10064,10065,10066,10067,10068 >> $O 2>> gpurun_out/r04j.err || { tail -20 gpurun_out/r04j.err; exit 1; }
done
echo "odd widths done"
timeout -k 10 600 python -u scripts/bench_config.py --config papers > gpurun_out/r04j_papers.json 2> gpurun_out/r04j_papers.err \
  || { tail -20 gpurun_out/r04j_papers.err; exit 1; }
cat gpurun_out/r04j_papers.json
bash scripts/profile.sh r04j_papers --config papers --steps 5 --warmup 2 --no-cpu-baseline || exit 1
cat gpurun_out/prof_r04j_papers/trace_bench.json
echo all done
