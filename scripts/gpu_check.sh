#!/bin/bash
# One gpurun call: smoke -> GPU tests -> short bench (+ optional rocprof).
# Stops at the first crash / abort / timeout (exit >= 124 or a signal); an
# ordinary test failure (pytest exit 1) still lets the bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
stage() {  # stage <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/stages.log
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/stages.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
stage smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || [ $? -lt 124 ] || exit 1
if [ "$MODE" = "all" ] || [ "$MODE" = "tests" ]; then
  stage pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -ra
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "bench" ]; then
  stage bench 600 python bench.py --steps 20 --warmup 3
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  cd "${GRAFT_REPO_ROOT}"
  stage rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline
fi
exit 0
