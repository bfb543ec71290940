#!/bin/bash
# Split-scheme A/B on one box: GPU flow tests, then cfg2 / cfg5 benches for
# f16x2 (default) and bf16x3 (ZF_X3_SCHEME=bf16x3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_flow.py}
timeout -k 10 600 python -u -m pytest $T -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log
[ $rc -ge 124 ] && exit $rc
for cfg in ${CFGS:-cfg2 cfg5}; do
  for sch in f16x2 bf16x3; do
    ZF_X3_SCHEME=$sch timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline --no-spline-kernel > gpurun_out/ab_${cfg}_${sch}.json 2> gpurun_out/ab_${cfg}_${sch}.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${cfg}_${sch}.json')); print('$cfg $sch', round(d['value']/1e6,1), 'M/s', d['roofline']['kernel'], round(d['roofline']['frac'],3), d.get('nll'))"
  done
done
exit $rc
