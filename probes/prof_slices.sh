set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_slices
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for n in 64 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_n$n -o run -- python3 scripts/bench_config.py --config products --n $n --no-check --reps 10 > $OUT/trace_n$n.json 2> $OUT/trace_n$n.err || exit 1
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit_n$n -o run -- python3 scripts/bench_config.py --config products --n $n --no-check --reps 3 > $OUT/hit_n$n.json 2> $OUT/hit_n$n.err || exit 1
  timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B_sum --output-format csv -d $OUT/rd_n$n -o run -- python3 scripts/bench_config.py --config products --n $n --no-check --reps 3 > $OUT/rd_n$n.json 2> $OUT/rd_n$n.err || exit 1
done
echo done
