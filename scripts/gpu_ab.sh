#!/bin/bash
# One gpurun call for kernel tuning: optional parity suite on one tuning
# library, then alternating bench rounds of several (scripts/ab_libs.sh).
#   TEST_LIB=fu TEST_K="expr" LIBS="base fu" ROUNDS=2 BENCH_ARGS="--config cfg2" scripts/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "${TEST_LIB:-}" ]; then
  ZF_LIB=tune/lib$TEST_LIB.so timeout -k 10 900 python -u -m pytest ${TEST_FILES:-tests/test_gpu_flow.py} -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log
  [ $rc -ne 0 ] && { echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc; [ "${STOP_ON_FAIL:-1}" = 1 ] && exit $rc; }
fi
if [ -n "${TRACE_LIB:-}" ]; then
  for cfg in ${TRACE_CFGS:-cfg2}; do
    ZF_LIB=tune/lib$TRACE_LIB.so timeout -k 10 200 python scripts/x3_trace.py $cfg > gpurun_out/trace_${TRACE_LIB}_$cfg.json 2> gpurun_out/trace_err.log
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/trace_err.log; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k:(round(v['mean']) if isinstance(v,dict) else v) for k,v in d.items()})" gpurun_out/trace_${TRACE_LIB}_$cfg.json
  done
fi
exec_ab() { LIBS="$LIBS" ROUNDS="${ROUNDS:-2}" BENCH_ARGS="${BENCH_ARGS:-}" bash scripts/ab_libs.sh; }
[ -n "${LIBS:-}" ] && exec_ab
exit 0
