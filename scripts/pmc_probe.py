"""Tiny driver for PMC passes over the plane-resident kernels on the c2 WAM-group shape
(25 samples x 64 images x 3 channels of 224^2, db4 J=3)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

S, N, C = 25, 64, 3
p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
x = torch.randn(N, C, 224, 224, device="cuda")
sigma = P.item_sigma(x, C * 224 * 224, C * 224 * 224, 0.25)
xs = torch.randn(S * N * C, 224, 224, device="cuda")
for _ in range(3):
    p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0)
    cf = p.wavedec(xs)
    p.waverec(cf, S * N * C)
    p.adjoint_maps(xs, S, N, C, full=False)
torch.cuda.synchronize()
print("done")
