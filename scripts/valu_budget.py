"""Static per-phase instruction budget of one flow_kernel_x3 instantiation
(tuning aid).  Build the kernel's translation unit with -DZF_X3_MARK
(`;ZFMARK n` comments at the phase boundaries of the NSC body; every group
step is unrolled, so the static count of a phase is its count per
wave-coupling) and pass the .s file:
  valu_budget.py <file.s> <kernel-name-regex> [--json out.json]
Phases: 0-1 layer 0 (+ first scale/swish/split), 1-2 hidden layers,
2-3 last-layer setup, 3-4 last Dense, 4-11 parameter gather, 11-12 spline
normalisation, 12-13 bin search, 13-5 spline eval + log-det."""
import json
import re
import sys
from collections import Counter

PHASES = {"0": "layer0", "1": "hidden", "2": "last_setup", "3": "last_dense", "4": "gather",
          "11": "normalise", "12": "search", "13": "eval_logdet", "5": "after_nsc", "10": "shift_bounds"}
TRANS = ("v_exp_", "v_rcp_", "v_sqrt_", "v_rsq_", "v_log_", "v_sin_", "v_cos_")
# gfx950 issue cycles per instruction class at several waves per SIMD
# (tests/hip/valu_cost_probe.hip, profiles/r05 records in DESIGN.md)
CYC = {"trans": 8.1, "mix": 8.1, "quarter": 4.2, "valu": 2.4, "mfma": 8.0}
QUARTER = ("v_cvt_pk_", "v_max3_", "v_min3_", "v_ldexp_", "v_cvt_f32_f16", "v_cndmask_", "v_max_", "v_min_")


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_fma_mix"):
        return "mix"
    if op.startswith(QUARTER):
        return "quarter"
    if op.startswith(("v_accvgpr", "v_")):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_setprio", "sched_")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    src, pat = sys.argv[1], sys.argv[2]
    s = open(src).read()
    names = [m for m in re.findall(r"^(_Z\S+):", s, re.M) if re.search(pat, m)]
    if not names:
        sys.exit(f"no kernel matches {pat!r}")
    body = s[s.index(names[0] + ":"):]
    body = body[: body.index(".Lfunc_end")]
    phase, per = None, {}
    for line in body.splitlines():
        t = line.strip()
        if "ZFMARK" in t:
            phase = PHASES.get(t.split("ZFMARK")[1].strip(), "?")
            continue
        tok = t.split()
        if phase is None or not tok or tok[0].startswith((".", ";")) or tok[0].endswith(":"):
            continue
        per.setdefault(phase, Counter())[klass(tok[0])] += 1
    order = ["layer0", "hidden", "last_setup", "last_dense", "gather", "normalise", "search", "eval_logdet"]
    rows, tot = {}, Counter()
    print(f"{names[0][:90]}")
    print(f"{'phase':12s} {'valu':>5s} {'trans':>5s} {'mix':>4s} {'qrt':>4s} {'mfma':>4s} {'lds':>4s} {'salu':>4s}"
          f" {'VALU':>5s} {'issue cyc':>9s}")
    for ph in order:
        c = per.get(ph, Counter())
        nvalu = c["valu"] + c["trans"] + c["mix"] + c["quarter"]
        cyc = sum(CYC[k] * c[k] for k in ("valu", "trans", "mix", "quarter"))
        rows[ph] = dict(c, VALU=nvalu, valu_issue_cycles=round(cyc))
        tot.update(c)
        print(f"{ph:12s} {c['valu']:5d} {c['trans']:5d} {c['mix']:4d} {c['quarter']:4d} {c['mfma']:4d} {c['lds']:4d}"
              f" {c['salu']:4d} {nvalu:5d} {cyc:9.0f}")
    nvalu = tot["valu"] + tot["trans"] + tot["mix"] + tot["quarter"]
    cyc = sum(CYC[k] * tot[k] for k in ("valu", "trans", "mix", "quarter"))
    print(f"{'total':12s} {tot['valu']:5d} {tot['trans']:5d} {tot['mix']:4d} {tot['quarter']:4d} {tot['mfma']:4d}"
          f" {tot['lds']:4d} {tot['salu']:4d} {nvalu:5d} {cyc:9.0f}")
    if "--json" in sys.argv:
        rows["total"] = dict(tot, VALU=nvalu, valu_issue_cycles=round(cyc))
        json.dump({"kernel": names[0], "cycles_per_class": CYC, "phases": rows},
                  open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
