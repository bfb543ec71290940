"""Summarise rocprofv3 output (gpurun_out/prof_*) into profiles/ (committed).

    python scripts/summarize_profiles.py <tag> [src]

Writes
* profiles/<tag>_kernel_stats.csv — copy of rocprofv3 --stats (all launches);
* profiles/<tag>_kernel_grid_stats.csv — the same trace split per (kernel,
  grid), so the headline kernel's launches at the bench grid are averaged on
  their own (train-mode / warm-up launches of other sizes excluded);
* profiles/<tag>_pmc_summary.json — per (kernel, grid): trace durations, the
  median of every collected counter per launch, HBM bytes per launch and the
  pipe-utilisation fractions below;
* profiles/pmc_traffic.json — the headline entries bench.py reads.

Units (MI355X_MICROARCH.md §HBM, §Per-instruction cycle constants):
FETCH_SIZE / WRITE_SIZE are KiB, FETCH_SIZE doubled on gfx950 (it tallies
128-B requests at 64 B); GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the
kernel's cycles = GRBM_GUI_ACTIVE / 8; SQ_VALU_MFMA_BUSY_CYCLES counts SIMD
cycles summed over the 1024 SIMDs, so mfma_busy = it / (1024 x cycles);
SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves, so
valu_active = 4 x it / (1024 x cycles) (two co-resident waves of one SIMD
can both count: an upper bound of the VALU pipe's share)."""

import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "profiles"
N_SIMD = 256 * 4


def short(name):
    for key in ("flow_kernel_x3<", "flow_kernel<", "rqs_kernel_direct<", "rqs_kernel<", "reduce_partials",
                "colstats_partial", "colstats_final", "normalize_vec_kernel<", "normalize_kernel",
                "squareplus_kernel", "softmax_threshold_kernel"):
        if key in name:
            i = name.index(key)
            j = name.find(">", i)
            return name[i : j + 1] if key.endswith("<") else key
    return name[:40]


def grid_of(r):
    return int(r.get("Grid_Size") or r["Grid_Size_X"])


def load_counters(src):
    agg = {}
    for path in sorted(glob.glob(str(src / "prof_*" / "run_counter_collection.csv"))
                       + glob.glob(str(src / "pmc*" / "run_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            k = (short(r["Kernel_Name"]), grid_of(r))
            agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return agg


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else 0.0


def main(tag="r02", src=ROOT / "gpurun_out"):
    src = Path(src)
    OUT.mkdir(exist_ok=True)
    shutil.copy(src / "prof_trace" / "run_kernel_stats.csv", OUT / f"{tag}_kernel_stats.csv")
    trace = list(csv.DictReader(open(src / "prof_trace" / "run_kernel_trace.csv")))
    durs = {}
    for r in trace:
        k = (short(r["Kernel_Name"]), grid_of(r))
        durs.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    with open(OUT / f"{tag}_kernel_grid_stats.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel", "Grid", "Calls", "AverageUs", "MedianUs", "MinUs", "MaxUs", "TotalUs"])
        for (name, g), d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, g, len(d), f"{sum(d) / len(d):.3f}", f"{med(d):.3f}", f"{min(d):.3f}",
                        f"{max(d):.3f}", f"{sum(d):.3f}"])
    counters = load_counters(src)
    summary = {}
    for k in sorted(set(counters) | set(durs)):
        d = durs.get(k, [])
        e = {"launches_trace": len(d), "avg_duration_us_trace": sum(d) / max(1, len(d)),
             "median_duration_us_trace": med(d)}
        cs = {c: med(v) for c, v in counters.get(k, {}).items()}
        e.update({f"{c}_median": v for c, v in sorted(cs.items())})
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["hbm_bytes_per_launch"] = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
        cyc = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8
        if cyc > 0:
            e["kernel_cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                e["mfma_busy"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc)
            if "SQ_ACTIVE_INST_VALU" in cs:
                e["valu_active"] = 4 * cs["SQ_ACTIVE_INST_VALU"] / (N_SIMD * cyc)
        summary[f"{k[0]} grid={k[1]}"] = e
    json.dump(summary, open(OUT / f"{tag}_pmc_summary.json", "w"), indent=1)
    # bench.py reads the headline kernels (largest grid of each) from here
    best = {}
    for key, v in summary.items():
        name, grid = key.split(" grid=")
        base = name.split("<")[0]
        if "hbm_bytes_per_launch" in v and (base not in best or int(grid) > best[base][0]):
            best[base] = (int(grid), v)
    traffic = {b: dict(v, grid=g, source=f"profiles/{tag}_pmc_summary.json") for b, (g, v) in best.items()}
    json.dump(traffic, open(OUT / "pmc_traffic.json", "w"), indent=1)
    for k, v in summary.items():
        print(f"{k:55s} n={v['launches_trace']:3d} t={v['median_duration_us_trace']:9.1f}us "
              f"hbm={v.get('hbm_bytes_per_launch', 0) / 1e6:9.2f} MB mfma={v.get('mfma_busy', 0):.3f} "
              f"valu={v.get('valu_active', 0):.3f}")


if __name__ == "__main__":
    main(*(sys.argv[1:3] or ["r02"]))
