#!/bin/bash
# Round 6, second GPU call: GPU suite on the round's changes (activation sets,
# bf16x3 swish-only, 1-knot chains, coalesced K1), K1 coalesced vs direct
# A/B, per-scheme row diagnostics (trained_cfg1, cfg4), a layered-path trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/c2_suite.log 2>&1
rc=$?; tail -3 gpurun_out/c2_suite.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in direct coal; do
  if [ $v = direct ]; then export ZF_K1_DIRECT=1; else unset ZF_K1_DIRECT; fi
  for K in 16 8; do
    timeout -k 10 200 python scripts/bench_rqs.py 20 $K > gpurun_out/c2_k1.log 2>&1 || { tail -5 gpurun_out/c2_k1.log; exit 1; }
    echo "$v K=$K $(tail -1 gpurun_out/c2_k1.log)" | tee -a gpurun_out/c2_k1_ab.txt
  done
done; done
unset ZF_K1_DIRECT
timeout -k 10 300 python scripts/diag_scheme_rows.py trained_cfg1 > gpurun_out/c2_rows_trained_cfg1.json || exit $?
timeout -k 10 300 python scripts/diag_scheme_rows.py cfg4 > gpurun_out/c2_rows_cfg4.json || exit $?
head -20 gpurun_out/c2_rows_trained_cfg1.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c2_lay" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --rows 262144 --steps 3 > gpurun_out/c2_lay.log 2>&1 || { tail -5 gpurun_out/c2_lay.log; exit 1; }
tail -2 gpurun_out/c2_lay.log
