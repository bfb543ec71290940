#!/bin/bash
# f16x2 layered GEMM: layered parity tests, then the layered bench with and
# without it, then a kernel trace of h512 log_prob.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 300 --timeout-method thread \
  -k "h512 or h384c2 or h1024k5" > gpurun_out/h2_tests.log 2>&1 && tail -3 gpurun_out/h2_tests.log &&
ZF_LAYERED_H2=0 timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/h2_bench_off.jsonl &&
timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/h2_bench_on.jsonl &&
cat gpurun_out/h2_bench_off.jsonl gpurun_out/h2_bench_on.jsonl &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/h2prof" -o h2 --output-format csv -- python3 scripts/layered_bench.py --configs h512 --steps 3 > gpurun_out/h2_prof.log 2>&1 &&
find gpurun_out/h2prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/h2_kernel_stats.csv \; && cut -d, -f1-5 gpurun_out/h2_kernel_stats.csv | cut -c1-40,200- 
exit 0
export PMC_CMD="python3 scripts/layered_bench.py --configs h512 --steps 2 --rows 524288" PMC_PREFIX=h2pmc
bash scripts/pmc_stall.sh &&
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/h2fetch" -o run --output-format csv -- $PMC_CMD > gpurun_out/h2fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/h2write" -o run --output-format csv -- $PMC_CMD > gpurun_out/h2write.log 2>&1 && echo pmc-done
