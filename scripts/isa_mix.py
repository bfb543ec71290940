"""Static instruction mix of one kernel in a hipcc --save-temps gfx950 .s file
(tuning aid).  usage: isa_mix.py <file.s> <kernel-name-regex> [max-count]"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 10**9
s = open(src).read()
names = [m for m in re.findall(r"^(_Z\S+):", s, re.M) if re.search(pat, m)]
if not names:
    sys.exit(f"no kernel matches {pat!r}")
body = s[s.index(names[0] + ":"):]
body = body[: body.index(".Lfunc_end")]
c = Counter()
for line in body.splitlines():
    t = line.strip().split()
    if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
        continue
    c[t[0]] += 1
print(names[0][:80], "total", sum(c.values()))
for k, v in sorted(c.items(), key=lambda kv: (-kv[1], kv[0])):
    if v <= cap:
        print(f"  {k:32s}{v}")
