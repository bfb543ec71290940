#!/bin/bash
# A/B the bf16x3 launch variants (ZF_X3_VARIANT) and the fp32 kernel: bench
# lines + the x3 parity tests under each variant.  One gpurun call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in ${VARIANTS:-0 1}; do
  ZF_X3_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_flow.py -q -p no:cacheprovider -x \
    -k "selection or x3 or parity or golden" > gpurun_out/ab_test_$v.log 2>&1
  rc=$?; echo "variant $v tests rc=$rc: $(tail -1 gpurun_out/ab_test_$v.log)"
  [ $rc -ge 124 ] && exit $rc
  ZF_X3_VARIANT=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-spline-kernel \
    > gpurun_out/ab_bench_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_bench_$v.log; exit $rc; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_bench_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"variant {sys.argv[1]}: {d['value']/1e6:.1f} M samples/s  {d['roofline']['kernel']}  frac {d['roofline']['frac']:.3f}")
PY
done
