#!/bin/bash
# Round 6, third GPU call: full GPU suite (new centred activation forms, the
# layered eval path without the pre-activation store, the vectorised first
# Dense, the trained_cfg1 row test), centred-activation A/B, layered bench,
# cfg2 / cfg4 phase traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/acts_tiny.jsonl gpurun_out/strict_rows.jsonl gpurun_out/strict_parity.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -ra \
  > gpurun_out/c3_suite.log 2>&1
rc=$?; tail -5 gpurun_out/c3_suite.log; [ $rc -ge 124 ] && exit $rc
for cfg in cfg2sigmoid cfg2softplus; do
  LIBS="actr5 cur" ROUNDS=2 BENCH_ARGS="--config $cfg" bash scripts/ab_libs.sh | tee -a gpurun_out/c3_act_ab.txt || exit $?
done
timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024 > gpurun_out/c3_layered.jsonl 2> gpurun_out/c3_layered.err || { tail -5 gpurun_out/c3_layered.err; exit 1; }
cat gpurun_out/c3_layered.jsonl
for cfg in cfg2 cfg4; do
  ZF_LIB=tune/libtr16.so timeout -k 10 200 python scripts/x3_trace.py $cfg > gpurun_out/c3_trace_$cfg.json 2> gpurun_out/c3_trace_err.log || { tail -5 gpurun_out/c3_trace_err.log; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k:(round(v['mean']) if isinstance(v,dict) else v) for k,v in d.items()})" gpurun_out/c3_trace_$cfg.json
done
exit $rc
