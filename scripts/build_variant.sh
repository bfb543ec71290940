#!/bin/bash
# Tuning: a library variant that differs from the in-tree build only in some
# split-MFMA translation units (TUS, default the K = 16 one), compiled with
# extra flags:
#   [TUS="k16 k16_act2"] scripts/build_variant.sh NAME [-DFLAG=V ...]  ->  tune/libNAME.so
# (links the other objects of the last default build, build/obj/*.o)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p tune
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-result -I/opt/rocm/include -Iinclude -fno-slp-vectorize"
OBJS=$(ls build/obj/*.o)
NEW=""
for tu in ${TUS:-k16}; do
  # a split-MFMA unit by its suffix (k16, k16_act2) or any unit by its name (zf_rqs)
  base=zf_flow_x3_$tu; [ -f zenflow_amd/csrc/$tu.hip ] && base=$tu
  /opt/rocm/bin/hipcc $FLAGS "$@" -c -o tune/${tu}_$NAME.o zenflow_amd/csrc/$base.hip &
  OBJS=$(echo "$OBJS" | grep -v "/$base.o")
  NEW="$NEW tune/${tu}_$NAME.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tune/lib$NAME.so $OBJS $NEW -ldl
echo tune/lib$NAME.so
