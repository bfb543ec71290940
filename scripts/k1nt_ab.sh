#!/bin/bash
# A/B of ab/libbase.so vs ab/libnt.so (non-temporal dx/dy loads in rqs_kernel_direct,
# a retired variant: see DESIGN.md K1; the -DZF_K1_NT switch was removed with it).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for v in base nt; do for k in 16 8 32; do
  echo "$v K=$k rep=$rep" >> gpurun_out/k1nt.log
  ZF_LIB=$PWD/ab/lib$v.so timeout -k 10 120 python scripts/bench_rqs.py 20 $k >> gpurun_out/k1nt.log 2>&1 || exit $?
done; done; done
