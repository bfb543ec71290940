"""Print the mean per-phase ticks of x3_trace.py outputs side by side."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f.split("/")[-1], {k: round(v["mean"]) for k, v in d.items() if isinstance(v, dict)})
