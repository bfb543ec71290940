# Trainer parity tests, then the training throughput sweep and a kernel trace
# of the small-batch step (cfg2, 1024 rows).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_dp.py > gpurun_out/train_tests.log 2>&1 || { tail -30 gpurun_out/train_tests.log; exit 1; }
tail -3 gpurun_out/train_tests.log
timeout -k 10 200 python scripts/train_bench.py --configs cfg2,cfg5 --batches 1024,65536 2>/dev/null || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tprof -o run --output-format csv -- python3 scripts/train_bench.py --configs cfg2 --batches 1024 > gpurun_out/tprof.log 2>&1 || exit $?
head -16 gpurun_out/tprof/run_kernel_stats.csv | cut -d, -f1-4
