"""Per-kernel register / spill / occupancy summary of one HIP source
(hipcc -Rpass-analysis=kernel-resource-usage), for tuning sessions."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "zenflow_amd/csrc/zf_flow.hip"
extra = sys.argv[2:]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude", "-c", src,
                      "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage", *extra],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if "error" in k:
        continue
    print(f"{k[:70]:70s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} spill={v.get('VGPRs Spill')} "
          f"occ={v.get('Occupancy [waves/SIMD]')} lds={v.get('LDS Size [bytes/block]')}")
if "error" in out:
    print(out[-3000:])
