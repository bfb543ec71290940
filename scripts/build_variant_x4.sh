#!/bin/bash
# Tuning: a library variant that differs from the in-tree build only in the
# K = 16 two-set translation unit, compiled with extra flags:
#   scripts/build_variant_x4.sh NAME [-DFLAG=V ...]  ->  tune/libNAME.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tune
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-result -I/opt/rocm/include -Iinclude -fno-slp-vectorize"
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o tune/x4k16_$NAME.o zenflow_amd/csrc/zf_flow_x4_k16.hip
OBJS=$(ls build/obj/*.o | grep -v zf_flow_x4_k16.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tune/lib$NAME.so $OBJS tune/x4k16_$NAME.o -ldl
echo tune/lib$NAME.so
