"""Where a kernel spills: scratch load/store sites in a --save-temps .s file
with the instruction mix around each (tuning aid).
usage: spill_sites.py <file.s> <kernel-name-regex>"""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
s = open(src).read()
names = [m for m in re.findall(r"^(_Z\S+):", s, re.M) if re.search(pat, m)]
if not names:
    sys.exit(f"no kernel matches {pat!r}")
body = s[s.index(names[0] + ":"):]
body = body[: body.index(".Lfunc_end")]
ins = [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", "."))]
mf = 0
for i, ln in enumerate(ins):
    if ln.startswith("v_mfma"):
        mf += 1
    if "scratch_" in ln:
        ctx = " ".join(x.split()[0] for x in ins[max(0, i - 4) : i + 4])
        print(f"{i:5d} (after {mf:3d} mfma) {ln[:48]:48s} | {ctx[:140]}")
