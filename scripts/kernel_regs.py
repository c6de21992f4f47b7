"""VGPR / SGPR / spill counts of the kernels in one .hip file (compiled for gfx950 with
--save-temps into a temp dir). usage: python scripts/kernel_regs.py wam_amd/csrc/dwt2_plane.hip [regex]"""
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
d = tempfile.mkdtemp()
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "--save-temps",
                       "-munsafe-fp-atomics", src, "-o", os.path.join(d, "x.o")], cwd=d,
                      stderr=subprocess.DEVNULL)
s = open([os.path.join(d, f) for f in os.listdir(d) if f.endswith("gfx950.s")][0]).read()
for b in re.split(r"\n\s+- \.agpr_count", s):
    n = re.search(r"\.name:\s+(\S+)", b)
    if not n or not pat.search(n.group(1)):
        continue
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, b) or [None, "?"])[1]
    print("%-90s vgpr %3s sgpr %3s sgpr_spill %3s vgpr_spill %3s lds %6s" % (
        n.group(1)[:90], g("vgpr_count"), g("sgpr_count"), g("sgpr_spill_count"), g("vgpr_spill_count"),
        g("group_segment_fixed_size")))
