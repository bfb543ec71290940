"""Print per-kernel PMC counters (median over launches of the largest grid)."""
import csv, glob, sys
from collections import defaultdict
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/pmc*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:] + f" grid={r['Grid_Size']}"
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals, key=lambda k: -max(max(v) for v in vals[k].values())):
    if "grid=" in k and int(k.split("grid=")[1]) < 100000: continue
    print(k)
    for c, v in sorted(vals[k].items()):
        v = sorted(v); print(f"   {c:32s} {v[len(v)//2]:.4g}")
