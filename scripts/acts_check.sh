set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py > gpurun_out/flow_tests.log 2>&1 || { tail -30 gpurun_out/flow_tests.log; exit 1; }
tail -2 gpurun_out/flow_tests.log
for c in cfg2 cfg2relu cfg2gelu; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/b_$c.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/b_$c.log').read().strip().splitlines()[-1]);print('$c',round(d['value']/1e6,1),'M/s',d['roofline']['kernel'][:40],round(d['roofline']['frac'],3),d['parity']['max_rel_err_vs_oracle32'] if d.get('parity') else '')"
done
for c in cfg2relu cfg2gelu; do
  ZF_DISABLE_X3=1 timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/b_k2_$c.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/b_k2_$c.log').read().strip().splitlines()[-1]);print('K2 $c',round(d['value']/1e6,1),'M/s',d['roofline']['kernel'][:40])"
done
