#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then the HBM
# counters in separate --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
run() {  # run <name> <timeout> <args...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/stages.log
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/stages.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run prof_trace 600 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/prof_trace" -o run --output-format csv -- $B
run prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_fetch" -o run --output-format csv -- $B
run prof_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_write" -o run --output-format csv -- $B
exit 0
