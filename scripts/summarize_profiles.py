"""Summarise rocprofv3 output (gpurun_out/prof_*) into profiles/ (committed).

Writes profiles/<tag>_kernel_stats.csv (copy of rocprofv3 --stats),
profiles/<tag>_pmc_summary.json (per-kernel FETCH/WRITE per launch) and
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced stream, so it is doubled (calibrated on the K1 spline kernel, whose
algorithmic read bytes are known: see the `calibration` entry)."""

import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "profiles"


def short(name):
    for key in ("flow_kernel_x3<", "flow_kernel<", "rqs_kernel_direct<", "rqs_kernel<", "reduce_partials", "colstats_partial", "colstats_final",
                "normalize_vec_kernel<", "normalize_kernel", "squareplus_kernel", "softmax_threshold_kernel"):
        if key in name:
            i = name.index(key)
            j = name.find(">", i)
            return name[i : j + 1] if key.endswith("<") else key
    return name[:40]


def load_pmc(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    agg = {}
    for r in rows:
        k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    return agg


def main(tag="r01", src=ROOT / "gpurun_out"):
    OUT.mkdir(exist_ok=True)
    stats = src / "prof_trace" / "run_kernel_stats.csv"
    shutil.copy(stats, OUT / f"{tag}_kernel_stats.csv")
    fetch = load_pmc(src / "prof_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = load_pmc(src / "prof_write" / "run_counter_collection.csv", "WRITE_SIZE")
    trace = list(csv.DictReader(open(src / "prof_trace" / "run_kernel_trace.csv")))
    durs = {}
    for r in trace:
        k = (short(r["Kernel_Name"]), int(r.get("Grid_Size") or r["Grid_Size_X"]))
        durs.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        f = sorted(fetch.get(k, [0.0]))
        w = sorted(write.get(k, [0.0]))
        d = sorted(durs.get(k, [0.0]))
        med = lambda v: v[len(v) // 2]
        summary[f"{k[0]} grid={k[1]}"] = {
            "launches": len(f),
            "avg_duration_us_trace": sum(d) / max(1, len(d)),
            "median_duration_us_trace": med(d),
            "FETCH_SIZE_KiB_median": med(f),
            "WRITE_SIZE_KiB_median": med(w),
            "hbm_bytes_per_launch": (2 * med(f) + med(w)) * 1024,
        }
    json.dump(summary, open(OUT / f"{tag}_pmc_summary.json", "w"), indent=1)
    # bench.py reads the headline kernel (largest grid of flow_kernel) from here
    best = {}
    for key, v in summary.items():
        name = key.split(" grid=")[0]
        base = name.split("<")[0]
        grid = int(key.split("grid=")[1])
        if base not in best or grid > best[base][0]:
            best[base] = (grid, v)
    traffic = {b: dict(v, grid=g, source=f"profiles/{tag}_pmc_summary.json") for b, (g, v) in best.items()}
    json.dump(traffic, open(OUT / "pmc_traffic.json", "w"), indent=1)
    for k, v in summary.items():
        print(f"{k:55s} n={v['launches']:3d} t={v['median_duration_us_trace']:9.1f}us "
              f"hbm={v['hbm_bytes_per_launch'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["r01"]))
