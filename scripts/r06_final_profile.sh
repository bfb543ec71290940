#!/bin/bash
# Round-6 evidence run: smoke + GPU suite + the default bench under a
# rocprofv3 kernel trace (round_trace.sh), then the counter passes
# (round_pmc.sh: stall / pipe counters of cfg2 and cfg4, FETCH / WRITE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash scripts/round_trace.sh || exit $?
bash scripts/round_pmc.sh || exit $?
