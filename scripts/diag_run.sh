set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in zenflow_amd/variants/*.so; do ZF_ALLOW_MISSING_SYMBOLS=1 ZF_LIB=$PWD/$v timeout -k 10 300 python scripts/diag_parity.py >> gpurun_out/diag.jsonl 2> gpurun_out/diag_err.log || exit $?; done
