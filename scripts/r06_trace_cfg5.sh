#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ZF_LIB=tune/libtr32.so timeout -k 10 200 python scripts/x3_trace.py cfg5 > gpurun_out/c11_trace_cfg5.json 2> gpurun_out/c11_err.log || { tail -5 gpurun_out/c11_err.log; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:(round(v['mean']) if isinstance(v,dict) else v) for k,v in d.items()})" gpurun_out/c11_trace_cfg5.json
