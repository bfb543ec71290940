#!/bin/bash
# One gpurun call: A/B of tune/lib*.so variants, K1 one-lane vs two-lane at
# K = 32, then the targeted GPU tests on the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBS="${LIBS:-base noslp fin finslp}" ROUNDS=${ROUNDS:-2} bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/ab.txt || exit 1
for r in 1 2; do
  ZF_K1_ONE_LANE=1 timeout -k 10 120 python scripts/bench_rqs.py 20 32 > gpurun_out/k1_one.json || exit 1
  timeout -k 10 120 python scripts/bench_rqs.py 20 32 > gpurun_out/k1_pair.json || exit 1
  python - <<'PY'
import json
for n in ("one", "pair"):
    d = json.load(open(f"gpurun_out/k1_{n}.json"))
    print("K1 K=32", n, {k: (round(d[k]["frac"], 3), round(d[k]["us"], 1)) for k in ("forward", "inverse") if k in d}, d.get("check"))
PY
done
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread ${TESTS:-tests/test_gpu_train_dp.py tests/test_gpu_flow.py tests/test_gpu_rqs.py} -k "${TESTK:-train_dp or two_ranks or train_function or rccl or activation or kernel_selection or extremes_other or inverse_parity or rqs}" > gpurun_out/pt2.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/pt2.log
