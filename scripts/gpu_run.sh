#!/bin/bash
# One parameterised GPU call (replaces round 3-4's one-off scripts/gpu_r0*.sh).
#
# usage (through gpurun):  bash scripts/gpu_run.sh <tag> <step> [<step> ...]
# steps, run in order, each under its own time limit; the first failure ends the call:
#   tests                   the whole -m gpu suite (release library)
#   tests:<-k expression>   a selection of it
#   dbgtests:<-k expr>      a selection under the bounds-checked library (make -C of-spmm_amd debug)
#   smoke                   __graft_entry__.smoke()
#   bench[:<args>]          bench.py (default args: none -> the driver's default run)
#   profile:<name>[:<args>] scripts/profile.sh <tag>_<name> <args>  (trace + PMC passes)
#   py:<script args>        python -u <script args> (a probe under scripts/)
# Every log goes to gpurun_out/<tag>_<step>.txt.  stderr is kept: pytest captures only the Python
# level (--capture=tee-sys), so a message the HIP runtime, ROCr or glibc writes to fd 2 lands in the
# log, faulthandler dumps every thread to gpurun_out/<tag>_faulthandler.txt (tests/conftest.py;
# pytest's own faulthandler plugin is off so that it does not take the handler back), and
# AMD_LOG_LEVEL=1 makes the HIP runtime print its errors.
set -o pipefail
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export AMD_LOG_LEVEL=${AMD_LOG_LEVEL:-1}
export OFX_FAULTHANDLER_FILE=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_faulthandler.txt
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/of-spmm_amd/oneflow_spmm
PT="python -u -m pytest tests -m gpu -q -rs --capture=tee-sys --timeout 300 --timeout-method thread -p no:cacheprovider -p no:faulthandler"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  log=gpurun_out/${TAG}_${n}_${kind}.txt
  echo "== step $n: $step  (log $log)"
  case $kind in
    tests)
      if [ -n "$arg" ]; then timeout -k 10 900 $PT -x -k "$arg" > $log 2>&1
      else timeout -k 10 1000 $PT -x > $log 2>&1; fi ;;
    dbgtests)
      # the bounds-checked library exists only for these runs (make -C of-spmm_amd debug; delete
      # it after, so it is not pushed with every call) and must be newer than every kernel source
      stale=$(find of-spmm_amd/csrc of-spmm_amd/Makefile -newer $L/libofx_spmm_dbg.so 2>/dev/null | head -3)
      if [ ! -f $L/libofx_spmm_dbg.so ] || [ -n "$stale" ]; then
        echo "dbgtests: $L/libofx_spmm_dbg.so is missing or older than: $stale (make -C of-spmm_amd debug)" > $log
        false
      else
        OFX_DEBUG_BOUNDS_CHECK=1 OFX_SPMM_LIB=$L/libofx_spmm_dbg.so timeout -k 10 900 $PT -x -k "$arg" > $log 2>&1
      fi ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/${TAG}_${n}_bench.json 2> $log ;;
    profile)
      name=${arg%%:*}; pargs=""; [ "$name" != "$arg" ] && pargs=${arg#*:}
      bash scripts/profile.sh ${TAG}_${name} $pargs > $log 2>&1 ;;
    py)
      timeout -k 10 600 python -u $arg > $log 2>&1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "   rc=$rc"; tail -3 $log
  if [ $rc -ne 0 ]; then
    echo "---- step $n failed (rc=$rc); the call ends here ----"
    grep -n -B3 -A25 "Error\|error\|assert\|Fatal\|fault\|Abort" $log | head -120
    exit $rc
  fi
done
echo "all $n steps done"
