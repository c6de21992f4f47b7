"""Per-launch timing of the c4 WAM kernels (512^2 sym8 J=5 reflect, IG): the per-level adjoint +
channel-mean maps (k_adj_maps / k_ana_rows) and the alpha-fused synthesis (k_dwt2_syn).
usage: python scripts/kbench_c4.py [--groups 2] [--images 128] [--iters 5] [--syn-only]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import plan as P  # noqa: E402
from scripts.kbench import run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--syn-only", action="store_true", help="time the alpha-group synthesis only")
    a = ap.parse_args()
    G, N, C, H = a.groups, a.images, 3, 512
    p = P.get_plan(2, (H, H), 5, "sym8", "reflect", "cuda")
    if not a.syn_only:
        g = torch.randn(G * N, C, H, H, device="cuda")
        run("c4 adjoint maps G=%d N=%d" % (G, N), lambda: p.adjoint_maps(g, G, N, C), a.iters)
        del g
    x = torch.randn(N, C, H, H, device="cuda")
    cf = p.wavedec(x)
    if not a.syn_only:
        run("c4 wavedec N=%d" % N, lambda: p.wavedec(x), a.iters)
    run("c4 waverec alphas=%d" % G, lambda: p.waverec(cf, N * C, alphas=[0.25 * (i + 1) for i in range(G)]), a.iters)


if __name__ == "__main__":
    main()
