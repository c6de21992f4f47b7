"""PMC / timing driver for the c4 row kernels (512^2 sym8 J=5 reflect): wavedec of 32 images x 3
channels (k_ana_rows / k_dwt2_ana), the adjoint maps of 2 groups x 16 images (k_adj_maps) and the
waverec with 2 IG alphas (k_dwt2_syn), 3 calls each; prints per kernel launches, mean us and the
library's algorithmic bytes per launch."""
import collections
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

N, C, H = 32, 3, 512
p = P.get_plan(2, (H, H), 5, "sym8", "reflect", "cuda")
x = torch.randn(N, C, H, H, device="cuda")
g = torch.randn(2 * 16, C, H, H, device="cuda")
cf = p.wavedec(x)
p.adjoint_maps(g, 2, 16, C)
p.waverec(cf, N * C, alphas=[0.5, 1.0])
torch.cuda.synchronize()
P.timing_drain()
P.timing_enable(True)
for _ in range(3):
    p.wavedec(x)
    p.adjoint_maps(g, 2, 16, C)
    p.waverec(cf, N * C, alphas=[0.5, 1.0])
torch.cuda.synchronize()
P.timing_enable(False)
acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
for name, ms, nb in P.timing_drain():
    a = acc[name]
    a[0] += 1
    a[1] += ms
    a[2] += nb
for k, (n, ms, nb) in sorted(acc.items()):
    print("%-22s launches %3d  mean %8.1f us  algorithmic %10.0f B/launch  %6.0f GB/s" % (
        k, n, ms / n * 1e3, nb / n, nb / ms / 1e6))
