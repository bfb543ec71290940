#!/bin/bash
# gemm_h2_kernel with the swish-only epilogue (compact code) vs the generic
# one (tune/libh2db1.so), two rounds, then a kernel trace of the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260" > gpurun_out/h2sw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h2sw_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "== generic"; ZF_LIB=tune/libh2db1.so timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
  echo "== swish"; timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/h2swprof" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --steps 3 > gpurun_out/h2swprof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/h2swprof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
