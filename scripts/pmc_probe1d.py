"""Tiny driver for PMC passes over the 1D tile kernels at the c3 shape (6400 x 80000, db6 J=5)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

p = P.get_plan(1, (80000,), 5, "db6", "reflect", "cuda")
x = torch.randn(6400, 80000, device="cuda")
for _ in range(2):
    cf = p.wavedec(x)
    p.waverec(cf, 6400)
torch.cuda.synchronize()
print("done")
