set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rqs.py tests/test_golden_oracle.py -m gpu -p no:cacheprovider > gpurun_out/k1_tests.log 2>&1 || { tail -30 gpurun_out/k1_tests.log; exit 1; }
tail -1 gpurun_out/k1_tests.log
for K in 8 16 32; do timeout -k 10 200 python scripts/bench_rqs.py 20 $K || exit 1; done
bash scripts/train_check.sh
