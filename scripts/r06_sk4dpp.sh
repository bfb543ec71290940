#!/bin/bash
# small-K first Dense with a DPP row max: layered parity tests (h1024k5 runs
# it at 65,536-row chunks), layered bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260 or layered" > gpurun_out/sk4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sk4_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/sk4prof" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --steps 3 > gpurun_out/sk4prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/sk4prof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
