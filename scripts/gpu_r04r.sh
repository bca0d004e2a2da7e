# round 4, GPU call r: the fused plan, third cut
# -- plan block 0 tags the done word with the launch epoch before its status, every plan block
# adds 1 after writing its rows, one lane per waiting wave polls it (call q: a compare-and-swap
# count serialised the plan blocks on one address, arxiv-shaped N=16 579 us), light-row blocks
# dispatched before the item blocks.  Parity selection (release), A/B against the round-3 library
# and this tree without the fused plan, then the fp32 N = 17-32 mid-size tuning entries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SEL2="forms or prefetch_form_lane or mid_form or small_form or narrow or plan_once or forced_variants or dtype_width or golden or hub or sddmm or backward or gathered or epilogue or fused or out_of_range or transpose or shifted or zero_fill or partition"
timeout -k 10 300 $PT -k "$SEL2" > gpurun_out/r04r_sel.txt 2>&1
rc=$?; echo "parity selection, release: rc=$rc"; tail -2 gpurun_out/r04r_sel.txt
[ $rc -eq 0 ] || { grep -B2 -A12 "Error\|assert" gpurun_out/r04r_sel.txt | head -60; exit 1; }
SPECS="pubmed:16:0 small20k:16:0 small20k:64:0 arxiv:16:0 arxiv:64:0 arxiv:128:0 g60k:16:0 g60k:64:0 p2m:16:0 p2m:64:0 p5m:16:0 plaw1m:16:0 products:128:0"
for lib in prev nofp new prev nofp new; do
  f=$L/libofx_spmm_$lib.so; [ $lib = new ] && f=$L/libofx_spmm.so
  OFX_SPMM_LIB=$f timeout -k 10 150 python -u scripts/probe_graph.py $SPECS 2>> gpurun_out/r04r_ab.err \
    | sed "s/^/{\"lib\": \"$lib\", \"r\": /; s/$/}/" >> gpurun_out/r04r_ab.jsonl || { tail -20 gpurun_out/r04r_ab.err; exit 1; }
done
echo "A/B done"
bash scripts/gpu_r04p.sh
