#!/bin/bash
# A/B of gemm_h2_kernel's LDS stage: single buffer (80-B rows, two barriers
# per k-tile) vs double buffer (swizzled 64-B rows, one barrier), two rounds;
# then the in-tree library (double buffer + preloaded small-K rows) with a
# kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260" > gpurun_out/h2db_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h2db_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in h2db0 h2db1; do
  echo "== $v"; ZF_LIB=tune/lib$v.so timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
done; done
echo "== main"; timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/h2dbprof" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --steps 3 > gpurun_out/h2dbprof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/h2dbprof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
