#!/bin/bash
# K1 at K = 16: slope rows staged through LDS (ZF_K1_SLOPE_LDS=1) vs the
# per-lane loads: parity tests under the variant, then interleaved timing.
set -o pipefail
mkdir -p gpurun_out/k1l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ZF_K1_SLOPE_LDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rqs.py \
  > gpurun_out/k1l/tests.txt 2>&1 || { tail -30 gpurun_out/k1l/tests.txt; exit 1; }
tail -1 gpurun_out/k1l/tests.txt
for r in 1 2 3; do
  timeout -k 10 60 python -u scripts/bench_rqs.py 20 16 | sed 's/^/base /' | cut -c1-400
  ZF_K1_SLOPE_LDS=1 timeout -k 10 60 python -u scripts/bench_rqs.py 20 16 | sed 's/^/lds  /' | cut -c1-400
done > gpurun_out/k1l/ab.txt 2>&1
cat gpurun_out/k1l/ab.txt
