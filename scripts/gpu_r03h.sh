# round 3, GPU call h: rocprofv3 kernel trace + PMC passes (separate runs) of plaw1m at N=16 and of
# the bench workload (products N=128) with the round-3 kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PROG=scripts/bench_config.py bash scripts/profile.sh r03_plaw1m_n16 --config plaw1m --n 16 --no-check --reps 10 || exit 1
bash scripts/profile.sh r03_products || exit 1
echo all done
