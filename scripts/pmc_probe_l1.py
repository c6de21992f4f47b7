"""PMC driver: level-1-only (J=1) plane analysis on the c2 group shape, noisy haar, noisy db4 and
clean db4 (25 samples x 64 images x 3 channels of 224^2), three launches each."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import plan as P

S, N, C = 25, 64, 3
x = torch.randn(N, C, 224, 224, device="cuda")
sigma = P.item_sigma(x, C * 224 * 224, C * 224 * 224, 0.25)
xs = torch.randn(S * N * C, 224, 224, device="cuda")
for wl in ("haar", "db4"):
    p = P.get_plan(2, (224, 224), int(os.environ.get("PROBE_J", "1")), wl, "reflect", "cuda")
    for _ in range(3):
        p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0)
        if wl == "db4":
            p.wavedec(xs)
    torch.cuda.synchronize()
print("done")
