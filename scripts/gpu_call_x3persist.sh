#!/bin/bash
# Persistent bf16x3 training GEMM: probe, the GEMM parity tests, train bench.
set -o pipefail
mkdir -p gpurun_out/xp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tune/gemm_probe > gpurun_out/xp/probe.txt 2>&1 || { tail -5 gpurun_out/xp/probe.txt; exit 1; }
grep -E " x3 |transposed|K=760" gpurun_out/xp/probe.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  -k "x3_gemm or 65536 or 32768 or h512" > gpurun_out/xp/tests.txt 2>&1 || { tail -30 gpurun_out/xp/tests.txt; exit 1; }
tail -1 gpurun_out/xp/tests.txt
timeout -k 10 200 python -u scripts/train_bench.py --configs cfg2,cfg5 --batches 65536 > gpurun_out/xp/bench.jsonl 2>&1 || exit 1
cat gpurun_out/xp/bench.jsonl
timeout -k 10 200 python -u scripts/layered_bench.py --configs h512,h1024 > gpurun_out/xp/layered.jsonl 2>&1 || exit 1
cat gpurun_out/xp/layered.jsonl
