set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wide_tests.log 2>&1
rc=$?; tail -5 gpurun_out/wide_tests.log; [ $rc -ge 124 ] && exit $rc
for c in cfg2 d8 d4k32 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/wide_bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/wide_bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['config']['kernel'], d['roofline']['frac'])"
done
