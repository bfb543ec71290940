#!/bin/bash
# Two-set kernel check: targeted parity first, the GPU suite, then an A/B of
# the bench (ZF_X4=0: flow_kernel_x3) on the configs it covers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_flow.py -k "test_log_prob_parity and (cfg2 or cfg4 or cfg1) and 4096" > gpurun_out/x4/pt_quick.log 2>&1
rc=$?; tail -5 gpurun_out/x4/pt_quick.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread tests -m gpu ${TESTK:+-k "$TESTK"} > gpurun_out/x4/pt_all.log 2>&1
rc=$?; tail -8 gpurun_out/x4/pt_all.log; [ $rc -ne 0 ] && [ -z "${CONTINUE:-}" ] && exit $rc
for r in 1 2; do
  for c in ${CONFIGS:-cfg2 cfg4 cfg3}; do
    for v in 0 1; do
      ZF_X4=$v timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-spline-kernel > gpurun_out/x4/b_${c}_$v.log 2>&1 || { tail -5 gpurun_out/x4/b_${c}_$v.log; exit 1; }
      python - "$c" "$v" <<'PY'
import json, sys
c, v = sys.argv[1:3]
d = json.loads([l for l in open(f"gpurun_out/x4/b_{c}_{v}.log") if l.startswith("{")][-1])
print(f"{c} ZF_X4={v}: {d['value']/1e6:8.1f} M/s  kernel {d['roofline'].get('kernel_us', 0):8.1f} us  frac {d['roofline']['frac']:.3f}")
PY
    done
  done
done
for c in ${ACT_CONFIGS:-cfg2sigmoid cfg2softplus cfg2relu}; do
  timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-spline-kernel > gpurun_out/x4/b_$c.log 2>&1 || { tail -5 gpurun_out/x4/b_$c.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/x4/b_$c.log') if l.startswith('{')][-1]); print('$c', round(d['value']/1e6,1), 'M/s', d['config'].get('kernel'))"
done
for r in 1 2; do
  for v in 0 1; do
    ZF_K1_STREAM=$v timeout -k 10 120 python scripts/bench_rqs.py 20 16 > gpurun_out/x4/k1_$v.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/x4/k1_$v.json')); print('K1 K=16 stream=$v', {k: (round(d[k]['frac'], 3), round(d[k]['us'], 1)) for k in ('forward', 'inverse', 'normalize') if k in d}, d.get('check'))"
  done
done
