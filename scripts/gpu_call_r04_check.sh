#!/bin/bash
# Round-4 last check of the committed tree: the whole GPU suite, smoke(),
# the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r04c
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 960 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r04c/suite.log 2>&1
rc=$?; tail -3 gpurun_out/r04c/suite.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c/smoke.log 2>&1 || { tail -5 gpurun_out/r04c/smoke.log; exit 1; }
tail -1 gpurun_out/r04c/smoke.log
timeout -k 10 200 python -u bench.py > gpurun_out/r04c/bench.log 2>&1 || { tail -5 gpurun_out/r04c/bench.log; exit 1; }
grep '^{' gpurun_out/r04c/bench.log | cut -c1-300
exit $rc
