"""Workgroup-round quantisation of the c2 plane kernels: k_plane_ana<noise>, k_plane_syn and
k_plane_maps timed at several sample counts S of the c2 group (64 images x 3 channels of 224^2,
db4 J=3), so that a launch whose planes fill a partial last round of resident workgroups shows as
a step in the time per plane.

usage: python scripts/kbench_tail.py [--iters 10] [--samples 8,16,24,25,26,32]
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--samples", default="8,16,24,25,26,32")
    ap.add_argument("--flags", type=int, default=0)
    args = ap.parse_args()
    torch.manual_seed(0)
    N, C, H = 64, 3, 224
    p = P.get_plan(2, (H, H), 3, "db4", "reflect", "cuda", flags=args.flags)
    x = torch.randn(N, C, H, H, device="cuda")
    sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
    smax = max(int(v) for v in args.samples.split(","))
    g_all = torch.randn(smax * N * C, H, H, device="cuda")
    for S in [int(v) for v in args.samples.split(",")]:
        g = g_all[: S * N * C]
        cf = p.wavedec(g)
        for tag, fn in (("noisy", lambda: p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0)),
                        ("syn", lambda: p.waverec(cf, S * N * C)),
                        ("maps", lambda: p.adjoint_maps(g, S, N, C, full=False))):
            r = timed(fn, args.iters)
            for name, (us, nb) in sorted(r.items()):
                print(f"S={S:3d} {tag:5s} {name:22s} {us:8.1f} us  {us / (S * N):7.4f} us/item  "
                      f"{nb / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
