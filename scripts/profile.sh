#!/bin/bash
# rocprofv3 passes over the bench workload (one gpurun call):
#   prof_trace  --kernel-trace --stats
#   prof_fetch  --pmc FETCH_SIZE            (TCC: FETCH_SIZE uses 3 of 4 slots)
#   prof_write  --pmc WRITE_SIZE
#   prof_sq     --pmc 6 SQ + GRBM_GUI_ACTIVE (MFMA / VALU pipe utilisation)
# then: python scripts/summarize_profiles.py <tag>  (on the CPU side).
# BENCH_ARGS is appended to the bench command (e.g. "--config cfg5").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spline-kernel ${BENCH_ARGS:-}"
run() {  # run <name> <timeout> <args...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/stages.log
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/stages.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run prof_trace 300 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/prof_trace" -o run --output-format csv -- $B
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_fetch" -o run --output-format csv -- $B
run prof_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_write" -o run --output-format csv -- $B
run prof_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$REPO/gpurun_out/prof_sq" -o run --output-format csv -- $B
exit 0
