# round 3, GPU call aj: the reverted (validated) tree after the faulting patch — smoke and a parity
# subset on a fresh box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aj_smoke.txt 2>&1 || { tail -20 gpurun_out/r03aj_smoke.txt; exit 1; }
cat gpurun_out/r03aj_smoke.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shifted_window or narrow_16bit or baseline_configs or small_form or mid_form or narrow_form" > gpurun_out/r03aj_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r03aj_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r03aj_gpu_tests.txt
echo all done
