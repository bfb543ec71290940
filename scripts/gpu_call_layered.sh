#!/bin/bash
# Layered eval path (hidden > 256) parity, and the fused-kernel flow suite
# (the shared ShiftBounds / latent helpers moved).
set -o pipefail
mkdir -p gpurun_out/lay
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_flow.py \
  tests/test_gpu_sampling.py -k "h512 or h384 or h1024 or layered" > gpurun_out/lay/tests_layered.txt 2>&1 \
  || { tail -40 gpurun_out/lay/tests_layered.txt; exit 1; }
tail -2 gpurun_out/lay/tests_layered.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_api.py \
  tests/test_gpu_sampling.py > gpurun_out/lay/tests_flow.txt 2>&1 || { tail -40 gpurun_out/lay/tests_flow.txt; exit 1; }
tail -2 gpurun_out/lay/tests_flow.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py -k "h512 or h384" \
  > gpurun_out/lay/tests_train.txt 2>&1 || { tail -40 gpurun_out/lay/tests_train.txt; exit 1; }
tail -2 gpurun_out/lay/tests_train.txt
timeout -k 10 300 python -u scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/lay/bench.jsonl 2>gpurun_out/lay/bench.err && cat gpurun_out/lay/bench.jsonl
