"""Tiny driver for PMC passes: plane-resident vs per-level analysis on the c2 WAM-group shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

x = torch.randn(4800, 224, 224, device="cuda")
for flags in (0, P.PLAN_NO_PLANE):
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda", flags=flags)
    for _ in range(3):
        p.wavedec(x)
torch.cuda.synchronize()
print("done")
