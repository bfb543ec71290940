#!/bin/bash
# Round-end measurement in one gpurun call: rocprofv3 kernel trace + PMC
# passes of the headline bench, the stall counters, every config, the
# training-step sweep, and K1 kernel traces at K = 16 and K = 32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/round_profile.sh || exit $?
export TMPDIR=/tmp
for k in 16 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/k1prof$k" -o run --output-format csv -- python3 scripts/bench_rqs.py 20 $k > gpurun_out/k1prof$k.log 2>&1 || exit $?
  tail -1 gpurun_out/k1prof$k.log
done
