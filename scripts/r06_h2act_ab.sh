#!/bin/bash
# gemm_h2_kernel epilogue swish: IEEE divide (tune/libh2ieee.so) vs hardware
# reciprocal (in-tree), two rounds, after the layered parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260 or layered" > gpurun_out/h2act_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h2act_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "== ieee"; ZF_LIB=tune/libh2ieee.so timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
  echo "== rcp+dpp"; timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
done
