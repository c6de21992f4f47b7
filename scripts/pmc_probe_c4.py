"""PMC driver: the c4 synthesis (512^2 sym8 J=5 reflect waverec with 2 IG alphas, 32 images x 3
channels), 3 calls, plus the library's algorithmic bytes per k_dwt2_syn launch on stdout."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

N, C, H = 32, 3, 512
p = P.get_plan(2, (H, H), 5, "sym8", "reflect", "cuda")
x = torch.randn(N, C, H, H, device="cuda")
cf = p.wavedec(x)
torch.cuda.synchronize()
P.timing_drain()
P.timing_enable(True)
for _ in range(3):
    p.waverec(cf, N * C, alphas=[0.5, 1.0])
torch.cuda.synchronize()
P.timing_enable(False)
recs = [r for r in P.timing_drain() if r[0] == "k_dwt2_syn"]
print("k_dwt2_syn launches %d, algorithmic bytes per launch %.0f, mean us %.1f" % (
    len(recs), sum(r[2] for r in recs) / len(recs), sum(r[1] for r in recs) / len(recs) * 1e3))
