#!/bin/bash
# Counter passes (pmc_stall.sh's three + HBM traffic) over the layered h512 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
export PMC_CMD="python3 scripts/layered_bench.py --configs h512 --steps 2 --rows 524288" PMC_PREFIX=${PMC_PREFIX:-h2pmc}
bash scripts/pmc_stall.sh &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/${PMC_PREFIX}f" -o run --output-format csv -- $PMC_CMD > gpurun_out/${PMC_PREFIX}f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/${PMC_PREFIX}w" -o run --output-format csv -- $PMC_CMD > gpurun_out/${PMC_PREFIX}w.log 2>&1 && echo pmc-done
