#!/bin/bash
# Round 6, seventh GPU call: stall counters of the layered path's GEMMs
# (h512, two chunks of 131072 rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_lay*
PMC_PREFIX=pmc_lay PMC_CMD="python3 scripts/layered_bench.py --configs h512 --rows 262144 --steps 1" bash scripts/pmc_stall.sh || exit $?
echo done
