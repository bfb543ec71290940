#!/bin/bash
# A/B builds for kernel tuning: ab/libA.so from a git ref (default HEAD),
# ab/libB.so from the working tree.  Run both on the box with scripts/ab_bench.sh.
set -eu
cd "$(dirname "$0")/.."
REF=${1:-HEAD}
rm -rf /tmp/zf_ab_src && mkdir -p /tmp/zf_ab_src ab
git archive "$REF" zenflow_amd/csrc include | tar -x -C /tmp/zf_ab_src
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -I/opt/rocm/include"
/opt/rocm/bin/hipcc $FLAGS -I/tmp/zf_ab_src/include -o ab/libA.so /tmp/zf_ab_src/zenflow_amd/csrc/*.hip -ldl &
/opt/rocm/bin/hipcc $FLAGS -Iinclude -o ab/libB.so zenflow_amd/csrc/*.hip -ldl &
wait
ls -la ab/
