#!/bin/bash
# Two-set kernel ablations (tune/lib*.so) beside the in-tree build, cfg2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0 ZF_X4=1
for r in 1 2; do
  for v in ${LIBS:-base abl1 abl2 abl3 abl4}; do
    lib=zenflow_amd/libzenflow_amd.so; [ "$v" != base ] && lib=tune/lib$v.so
    ZF_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-cfg2} --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/x4/abl_$v.log 2>&1 || { tail -3 gpurun_out/x4/abl_$v.log; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
try:
    d = json.loads([l for l in open(f"gpurun_out/x4/abl_{v}.log") if l.startswith("{")][-1])
    print(f"{v}: kernel {d['roofline'].get('kernel_us', 0):8.1f} us  frac {d['roofline']['frac']:.3f}")
except Exception as e:
    print(v, "no line", e)
PY
  done
done
