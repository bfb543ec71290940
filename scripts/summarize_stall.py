"""Stall / co-execution counters of the headline kernel (scripts/pmc_stall.sh
passes in gpurun_out/pmc_st*) -> profiles/<tag>_x3_stall_counters.json.

Derived (per launch of the 2^20-row grid; the kernel's cycles =
GRBM_GUI_ACTIVE / 8 XCDs; SIMD-cycle counters are summed over 1024 SIMDs;
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* are wave quad-cycles):
  mfma_busy     SQ_VALU_MFMA_BUSY_CYCLES / (1024 cycles)
  coexec        SQ_VALU_MFMA_COEXEC_CYCLES / (1024 cycles)  (VALU and MFMA at once)
  valu_issue    4 SQ_ACTIVE_INST_VALU / (1024 cycles)       (MFMA issue included)
  wave split    SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES"""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KNAME = __import__("os").environ.get("ZF_STALL_KERNEL", "flow_kernel_x3")
NCOUP = {"cfg2": 4, "cfg3": 4, "cfg3s": 4, "cfg4": 2, "cfg5": 8, "d8": 8, "cfg1": 2}  # NSC couplings per flow


def main(tag="r02", src=ROOT / "gpurun_out", prefix="pmc_st", label="cfg2"):
    """prefix: the pmc_stall.sh PMC_PREFIX of the passes; label: the config
    (cfg2 also refreshes the bench's pmc_traffic.json entry)."""
    agg = {}
    kname = None
    # the bench run also launches its configs block: keep the label's own
    # instantiation only (template arguments as in scripts/trace_vs_bench.py)
    sys.path.insert(0, str(ROOT / "scripts"))
    from trace_vs_bench import KERNELS
    want = KNAME + KERNELS[label][0] if KNAME == "flow_kernel_x3" and label in KERNELS else KNAME
    for path in glob.glob(str(Path(src) / f"{prefix}*" / "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            if want not in r["Kernel_Name"]:
                continue
            if int(r.get("Grid_Size") or r["Grid_Size_X"]) < (1 << 20):
                continue
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            kname = r["Kernel_Name"]
    med = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
    cyc = med["GRBM_GUI_ACTIVE"] / 8
    simd = 1024 * cyc
    waves = med["SQ_WAVE_CYCLES"]
    out = {
        "kernel": (kname[kname.index(KNAME):kname.index(">") + 1] if kname else KNAME)
        + f" ({label}), 2^20-row launches",
        "counters_median": med,
        "kernel_cycles": cyc,
        "mfma_busy": med["SQ_VALU_MFMA_BUSY_CYCLES"] / simd,
        "valu_mfma_coexec": med["SQ_VALU_MFMA_COEXEC_CYCLES"] / simd,
        "valu_issue": 4 * med["SQ_ACTIVE_INST_VALU"] / simd,
        "wave_active": med["SQ_ACTIVE_INST_ANY"] / waves,
        "wave_wait_inst_any": med["SQ_WAIT_INST_ANY"] / waves,
        "wave_wait_any": med["SQ_WAIT_ANY"] / waves,
        "couplings": NCOUP.get(label, 4),
        "per_wave_coupling": {k: med[c] / med.get("SQ_WAVES", 32768) / NCOUP.get(label, 4) for k, c in (
            ("valu_insts", "SQ_INSTS_VALU"), ("mfma_insts", "SQ_INSTS_MFMA"), ("trans_f32_insts", "SQ_INSTS_VALU_TRANS_F32"),
            ("salu_insts", "SQ_INSTS_SALU"), ("lds_insts", "SQ_INSTS_LDS"), ("branches", "SQ_INSTS_BRANCH"))},
        "lds_bank_conflicts": med.get("SQ_LDS_BANK_CONFLICT"),
    }
    out["simd_idle"] = 1 - out["mfma_busy"] - out["valu_issue"] + out["valu_mfma_coexec"]
    name = f"{tag}_x3_stall_counters.json" if label == "cfg2" else f"{tag}_x3_stall_counters_{label}.json"
    (ROOT / "profiles" / name).write_text(json.dumps(out, indent=1) + "\n")
    # the bench line's roofline.valu_mfma_coexec (profiles/pmc_traffic.json)
    tf = ROOT / "profiles" / "pmc_traffic.json"
    if label == "cfg2" and tf.exists():
        t = json.loads(tf.read_text())
        if "flow_kernel_x3" in t:
            t["flow_kernel_x3"]["valu_mfma_coexec"] = out["valu_mfma_coexec"]
            t["flow_kernel_x3"]["stall_source"] = f"profiles/{tag}_x3_stall_counters.json"
            tf.write_text(json.dumps(t, indent=1) + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "counters_median"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
