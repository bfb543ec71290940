set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in zenflow_amd/variants/*.so; do echo "$v" >> gpurun_out/abl.log; ZF_LIB=$PWD/$v timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-spline-kernel >> gpurun_out/abl.log 2>&1 || exit $?; done
