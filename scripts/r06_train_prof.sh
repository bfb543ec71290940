#!/bin/bash
# Kernel trace of the training step at 65,536 rows (cfg2, cfg5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in ${TC:-cfg2 cfg5}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/tprof_$c" -o run --output-format csv -- python3 scripts/train_bench.py --configs $c --batches ${TB:-65536} --steps 10 > gpurun_out/tprof_$c.log 2>&1 || exit $?
python3 - "$c" <<'PY'
import csv, sys
c = sys.argv[1]
rows = list(csv.DictReader(open(f'gpurun_out/tprof_{c}/run_kernel_stats.csv')))
print('==', c)
for r in rows[:16]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
PY
done
