#!/bin/bash
# Round 6, first GPU call: changed-code tests, K1 one-log A/B, the cfg2 mix
# ceiling probe, ASET A/B, cfg5 phase trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_rqs.py tests/test_gpu_api.py "tests/test_gpu_flow.py::test_knot_counts" -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c1_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tune/mix_ceiling_probe | tee gpurun_out/c1_mix_probe.txt || exit $?
LIBS="k1a k1b" KS="16 32" bash scripts/ab_rqs.sh | tee gpurun_out/c1_k1_ab.txt || exit $?
LIBS="k1a k1b" KS="16" bash scripts/ab_rqs.sh | tee -a gpurun_out/c1_k1_ab.txt || exit $?
for cfg in cfg2relu cfg2gelu; do
  LIBS="base aset0" ROUNDS=2 BENCH_ARGS="--config $cfg" bash scripts/ab_libs.sh | tee -a gpurun_out/c1_aset_ab.txt || exit $?
done
ZF_LIB=tune/libtr32.so timeout -k 10 200 python scripts/x3_trace.py cfg5 > gpurun_out/c1_trace_cfg5.json 2> gpurun_out/c1_trace_err.log || { tail -5 gpurun_out/c1_trace_err.log; exit 1; }
cat gpurun_out/c1_trace_cfg5.json
