#!/bin/bash
# Fused kernel: wave-half exchanges by v_permlane32_swap (in-tree) vs
# __shfl_xor(x, 32) = ds_bpermute (tune/libx3bperm.so): GPU suite, then the
# bench (cfg2 + its configs block) interleaved, three rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pl_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in bperm permlane; do
  if [ $v = bperm ]; then L=tune/libx3bperm.so; else L=zenflow_amd/libzenflow_amd.so; fi
  ZF_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel > gpurun_out/pl_$v$r.json || exit $?
  python3 - "$v" "gpurun_out/pl_$v$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d.get("configs", {})
print(sys.argv[1], "cfg2 %.1f us frac %.4f" % (d["roofline"]["kernel_us"], d["roofline"]["frac"]),
      " ".join("%s %.4f" % (k, v["frac"]) for k, v in c.items()))
PY
done; done
