#!/bin/bash
# K1 spline kernels: lane exchanges / log-det sums by DPP (in-tree) vs
# __shfl = ds_bpermute (tune/libx3bperm.so, the previous commit), K = 16 and
# 32, three interleaved rounds, after the K1 parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rqs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k1dpp_tests.log 2>&1; rc=$?; tail -2 gpurun_out/k1dpp_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in bperm dpp; do
  if [ $v = bperm ]; then L=tune/libx3bperm.so; else L=zenflow_amd/libzenflow_amd.so; fi
  for K in 16 32; do echo "== $v K=$K"; ZF_LIB=$L timeout -k 10 120 python scripts/bench_rqs.py 20 $K | tail -1 || exit $?; done
done; done
