#!/bin/bash
# Headline only: v_permlane32_swap (in-tree) vs ds_bpermute (tune/libx3bperm.so), four interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2 3 4; do for v in bperm permlane; do
  if [ $v = bperm ]; then L=tune/libx3bperm.so; else L=zenflow_amd/libzenflow_amd.so; fi
  ZF_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-spline-kernel --no-configs > gpurun_out/pl2_$v$r.json || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.1f us frac %.4f' % (d['roofline']['kernel_us'], d['roofline']['frac']))" $v gpurun_out/pl2_$v$r.json
done; done
