set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in A B main; do
  if [ $v = main ]; then L=zenflow_amd/libzenflow_amd.so; else L=ab/lib$v.so; fi
  echo "== $v"; ZF_LIB=$L timeout -k 10 200 python scripts/train_bench.py --configs cfg2,cfg5 --batches 1024,65536 2>/dev/null || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tprof -o run --output-format csv -- python3 scripts/train_bench.py --configs cfg2 --batches 1024 > gpurun_out/tprof.log 2>&1 || exit $?
head -25 gpurun_out/tprof/run_kernel_stats.csv | cut -d, -f1-4
