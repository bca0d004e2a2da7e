# round 3, GPU call aa: wider sweep for hidden weak spots — odd widths (fp32 / bf16), f64, int64
# indices, on the products graph; every line carries a sampled bit-exact check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03aa_sweep.jsonl
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 3,17,47,100,200,300 --dtypes f32,bf16 > $O 2> gpurun_out/r03aa.err || { tail -20 gpurun_out/r03aa.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config products --widths 16,64,128 --dtypes f64 >> $O 2>> gpurun_out/r03aa.err || { tail -20 gpurun_out/r03aa.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config products --idx int64 --widths 16,64,128 --dtypes f32,bf16 >> $O 2>> gpurun_out/r03aa.err || { tail -20 gpurun_out/r03aa.err; exit 1; }
timeout -k 10 400 python -u scripts/width_sweep.py --config plaw1m --widths 3,17,47,100 --dtypes f32,bf16 >> $O 2>> gpurun_out/r03aa.err || { tail -20 gpurun_out/r03aa.err; exit 1; }
cat $O
echo all done
