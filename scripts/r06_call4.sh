#!/bin/bash
# Round 6, fourth GPU call: hidden-256 parity with the spread DMA issue,
# cfg5 A/B (spread vs burst), cfg4 phase trace, layered-path kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "cfg5 or h256 or k24h256 or cfg2 or d8" > gpurun_out/c4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c4_tests.log; [ $rc -ne 0 ] && exit $rc
LIBS="nospr cur" ROUNDS=2 BENCH_ARGS="--config cfg5" bash scripts/ab_libs.sh | tee gpurun_out/c4_cfg5_ab.txt || exit $?
ZF_LIB=tune/libtr16.so timeout -k 10 200 python scripts/x3_trace.py cfg4 > gpurun_out/c4_trace_cfg4.json 2> gpurun_out/c4_trace_err.log || { tail -5 gpurun_out/c4_trace_err.log; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k:(round(v['mean']) if isinstance(v,dict) else v) for k,v in d.items()})" gpurun_out/c4_trace_cfg4.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c4_lay" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --rows 262144 --steps 3 > gpurun_out/c4_lay.log 2>&1 || { tail -5 gpurun_out/c4_lay.log; exit 1; }
grep -v rocprofv3 gpurun_out/c4_lay.log | tail -2
