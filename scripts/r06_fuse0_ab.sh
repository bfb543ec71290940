#!/bin/bash
# Layered path: the first Dense folded into the second's A stage
# (default) vs its own kernel (ZF_LAYERED_FUSE0=0), two rounds, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260" > gpurun_out/fuse0_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fuse0_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "== unfused"; ZF_LAYERED_FUSE0=0 timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
  echo "== fused"; timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/fuse0prof" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --steps 3 > gpurun_out/fuse0prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/fuse0prof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
