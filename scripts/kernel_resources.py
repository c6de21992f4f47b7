"""Per-kernel register / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python scripts/kernel_resources.py wam_amd/csrc/dwt2_tile.hip [filter-substring]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude", "-Iwam_amd/csrc", "-c", src,
       "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        print(f'{dm[:90]:90s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} vspill={r.get("VGPRs Spill")} '
              f'sspill={r.get("SGPRs Spill")} occ={r.get("Occupancy [waves/SIMD]")} lds={r.get("LDS Size [bytes/block]")}')
