set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in zenflow_amd/variants/*.so; do echo "$v" >> gpurun_out/k1var.log; ZF_LIB=$PWD/$v timeout -k 10 120 python scripts/bench_rqs.py >> gpurun_out/k1var.log 2>&1 || exit $?; done
