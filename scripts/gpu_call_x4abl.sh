#!/bin/bash
# Two-set kernel variants (tune/lib*.so; "base" = in-tree) and flow_kernel_x3
# ("x3": in-tree with ZF_X4=0), cfg2 bench, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for v in ${LIBS:-x3 base v1 abl1 abl2 abl3 abl4}; do
    lib=zenflow_amd/libzenflow_amd.so; x4=1
    case $v in base) ;; x3) x4=0 ;; *) lib=tune/lib$v.so ;; esac
    ZF_X4=$x4 ZF_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-cfg2} --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/x4/abl_$v.log 2>&1 || { tail -3 gpurun_out/x4/abl_$v.log; }
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
