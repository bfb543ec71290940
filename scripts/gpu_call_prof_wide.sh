#!/bin/bash
# rocprofv3 kernel traces of the cfg5 and d8 bench workloads (last build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for c in cfg5 d8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$c" -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-spline-kernel --no-configs > gpurun_out/prof_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/prof_$c.log | tail -1 | cut -c1-200
done
