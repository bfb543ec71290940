#!/bin/bash
# Tuning A/B on the GPU box: alternate bench runs of tune/lib<NAME>.so
#   LIBS="base exp1" ROUNDS=2 BENCH_ARGS="--config cfg2" scripts/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-base}; do
    ZF_LIB=tune/lib$v.so timeout -k 10 200 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
      --no-spline-kernel --no-configs ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$v.log; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:8s}: {d['value']/1e6:8.1f} M/s  {d['ms_per_step']:.4f} ms  kernel {d['roofline']['kernel_us']:.1f} us  frac {d['roofline']['frac']:.3f}  {d['config'].get('workload')[:40]}", flush=True)
PY
  done
done
