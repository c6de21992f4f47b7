"""Workgroup-round (tail) check of the c2 plane kernels: time k_plane_maps / k_plane_syn /
k_plane_ana<noise> at work sizes just below and at the c2 size (library HIP events). With one
workgroup per image (maps) or plane (syn, noisy analysis) and two workgroups per CU, 512
workgroups run at once: 1,536 images are 3 full rounds, 1,600 are 3.125.

usage: python scripts/ab_tail.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import plan as P  # noqa: E402
from scripts.kbench_levels import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--groups", default="24,25")
    args = ap.parse_args()
    torch.manual_seed(0)
    N, C, H = 64, 3, 224
    p = P.get_plan(2, (H, H), 3, "db4", "reflect", "cuda")
    x = torch.randn(N, C, H, H, device="cuda")
    sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
    for G in [int(v) for v in args.groups.split(",")]:
        g = torch.randn(G * N * C, H, H, device="cuda")
        coeffs = p.wavedec_noisy(x, sigma, G, N, C, seed=1, sample_base=0)
        for tag, fn in (("maps", lambda: p.adjoint_maps(g, G, N, C, full=False)),
                        ("syn", lambda: p.waverec(coeffs, G * N * C)),
                        ("noisy", lambda: p.wavedec_noisy(x, sigma, G, N, C, seed=1, sample_base=0))):
            r = timed(fn, args.iters)
            for name, (us, nb) in sorted(r.items()):
                print(f"G={G} {tag:5s} {name:22s} {us:8.1f} us  {nb / us / 1e3:7.0f} GB/s", flush=True)
        del g, coeffs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
