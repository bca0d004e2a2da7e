# round 4, GPU call i: (1) planner rows per thread 4 / 8 / 16 (OFX_PLAN_RPT A/B builds: fewer plan
# blocks, shorter look-back) against the round-3 library, graph replay; (2) the mid-size width
# sweep of round 3 (profiles/r03ah_width_sweep_midsize.jsonl) on this tree: arxiv-shaped,
# 60k x 1.5M and PubMed-shaped graphs, f32 / bf16 / f16, N = 8 / 16 / 41 / 47 / 64 / 128 / 256,
# each line with the sampled oracle check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
SPECS="small20k:16:0 arxiv:16:0 arxiv:64:0 g60k:16:0 p2m:16:0 p5m:16:0 plaw1m:16:0 plaw1m:64:0 products:128:0"
for lib in prev new rpt8 rpt16 prev new rpt8 rpt16; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04i_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04i_ab.jsonl || { tail -20 gpurun_out/r04i_ab.err; exit 1; }
done
echo "A/B done"
O=gpurun_out/r04i_sweep.jsonl
for g in 169343:1166243 60000:1500000 19717:88648; do
  timeout -k 10 400 python -u scripts/width_sweep.py --graph $g --widths 8,16,41,47,64,128,256 --dtypes f32,bf16,f16 --rounds 5 --reps 20 >> $O 2>> gpurun_out/r04i.err || { tail -20 gpurun_out/r04i.err; exit 1; }
done
echo all done
