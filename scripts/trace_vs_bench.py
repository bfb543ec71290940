"""Roofline fractions recomputed from a rocprofv3 kernel trace of the exact
bench invocation, beside the fractions the bench line printed in the same run
(agreement within 3%).

    python scripts/trace_vs_bench.py <dir with bench_trace.log + bench_trace/> [out.json]

For each config of the bench line (the headline and its `configs` block) the
split-MFMA kernel instantiation that config runs is picked out of the trace
by its template arguments and grid; frac = alg flops per launch / average
trace duration / the f16x2 split peak (838.9 TFLOP/s).  cfg3 (inverse) and
cfg3s (sample) run the same instantiation at the same grid: their launches are
split by order (the bench runs cfg3 first)."""
import csv
import json
import sys
from pathlib import Path

PEAK = 2516.6 / 3  # TFLOP/s, fp16 dense / 3
# config -> (template args of flow_kernel_x3, alg flops per sample)
KERNELS = {
    "cfg2": ("<2, 16, 4, false, false, false, false, 0>", 229376),
    "cfg3": ("<2, 16, 4, false, false, true, false, 0>", 229376),
    "cfg3s": ("<2, 16, 4, false, false, true, false, 0>", 229376),
    "cfg4": ("<2, 16, 4, false, true, false, false, 0>", 91136),
    "cfg5": ("<2, 32, 8, true, false, false, false, 0>", 4194304),
    "d8": ("<2, 16, 4, true, false, false, false, 0>", 2 * 8 * (4 * 128 + 128 * 128 + 128 * 4 * 47)),
}
ROWS = 1 << 20


def main(src, out=None):
    src = Path(src)
    line = next(json.loads(l) for l in open(src / "bench_trace.log") if l.startswith("{"))
    trace = list(csv.DictReader(open(src / "bench_trace" / "run_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    bench = {"cfg2": line["roofline"]["kernel_us"]}
    for k, v in line.get("configs", {}).items():
        bench[k] = v["kernel_us"]
    res = {}
    used = {}
    for cfg in bench:
        if cfg not in KERNELS:
            continue
        targs, flops = KERNELS[cfg]
        launches = [r for r in trace if "flow_kernel_x3" in r["Kernel_Name"] and targs in r["Kernel_Name"].replace(" ", "").replace(",", ", ")
                    and int(r.get("Grid_Size") or r["Grid_Size_X"]) >= ROWS * 2]
        if cfg in ("cfg3", "cfg3s"):  # same kernel: split the sequence in two halves by order
            n = len(launches) // 2
            launches = launches[:n] if cfg == "cfg3" else launches[n:]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in launches]
        if not d:
            continue
        avg = sum(d) / len(d)
        med = sorted(d)[len(d) // 2]
        frac_tr = flops * ROWS / (avg * 1e-6) / 1e12 / PEAK
        frac_b = flops * ROWS / (bench[cfg] * 1e-6) / 1e12 / PEAK
        res[cfg] = {"kernel": "flow_kernel_x3" + targs, "launches": len(d), "trace_avg_us": round(avg, 2),
                    "trace_median_us": round(med, 2), "bench_events_us": round(bench[cfg], 2),
                    "frac_trace": round(frac_tr, 4), "frac_bench": round(frac_b, 4),
                    "rel_diff": round(frac_b / frac_tr - 1, 4)}
    rec = {"bench_line_value": line["value"], "bench_ms_per_step": line["ms_per_step"],
           "bench_frac": line["roofline"]["frac"], "configs": res}
    print(json.dumps(rec, indent=1))
    if out:
        Path(out).write_text(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:3])
