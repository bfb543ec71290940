set -u
cd "${GRAFT_REPO_ROOT}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_c3* gpurun_out/pmc_c5* gpurun_out/pmc_d8*
PMC_PREFIX=pmc_c3 BENCH_ARGS="--config cfg3" bash scripts/pmc_stall.sh || exit $?
PMC_PREFIX=pmc_d8 BENCH_ARGS="--config d8" bash scripts/pmc_stall.sh || exit $?
PMC_PREFIX=pmc_c5 BENCH_ARGS="--config cfg5" bash scripts/pmc_stall.sh || exit $?
echo done
