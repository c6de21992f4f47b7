"""PMC driver: the c3 1D analysis group (256 clips x 80,000 samples, db6 J=5 reflect), noisy
(5 samples per launch, as the c3 bench groups them) and clean (1,280 signals), three launches each."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

S, N, n = 5, 256, 80000
x = torch.randn(N, n, device="cuda")
sigma = P.item_sigma(x, n, n, 0.25)
xs = torch.randn(S * N, n, device="cuda")
p = P.get_plan(1, (n,), 5, "db6", "reflect", "cuda")
for _ in range(3):
    p.wavedec_noisy(x, sigma, S, N, 1, seed=1, sample_base=0)
    p.wavedec(xs)
torch.cuda.synchronize()
print("done")
