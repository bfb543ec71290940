#!/bin/bash
# Kernel-tuning builds: ab/lib<name>.so for each "name=extra hipcc flags" argument,
# all from the working tree (e.g. base= noslp=-fno-slp-vectorize).
set -eu
cd "$(dirname "$0")/.."
mkdir -p ab
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -I/opt/rocm/include -Iinclude"
for v in "$@"; do
  name=${v%%=*}; extra=${v#*=}
  /opt/rocm/bin/hipcc $FLAGS $extra -o ab/lib$name.so zenflow_amd/csrc/*.hip -ldl &
done
wait
ls ab/
