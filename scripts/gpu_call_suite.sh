#!/bin/bash
# The whole GPU suite in one call (record in gpurun_out/suite.log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/strict_parity.jsonl gpurun_out/acts_tiny.jsonl
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/suite.log 2>&1
rc=$?; tail -12 gpurun_out/suite.log; exit $rc
