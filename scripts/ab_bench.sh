#!/bin/bash
# Alternate bench runs of ab/libA.so and ab/libB.so on one box (BENCH_ARGS
# extra flags, ROUNDS repetitions).  Prints value / kernel / frac per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-A B}; do
    ZF_LIB=ab/lib$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      --no-spline-kernel ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_$v.log; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]}: {d['value']/1e6:8.1f} M/s  {d['ms_per_step']:.4f} ms  {d['config'].get('workload')}  frac {d['roofline']['frac']:.3f}")
PY
  done
done
