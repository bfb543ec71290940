#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for a in softplus sigmoid; do
  timeout -k 10 240 python scripts/diag_acts.py $a >> gpurun_out/diag_acts.jsonl 2>> gpurun_out/diag_acts.err || { tail -5 gpurun_out/diag_acts.err; exit 1; }
done
cat gpurun_out/diag_acts.jsonl
