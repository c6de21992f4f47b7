"""Per-launch timing of the non-Haar 3D levels: the fused tile kernels (dwt3_tile.hip) against the
per-axis kernels (generic plan) at the c5 volume shape with db4 / sym8 (16 x 128^3, J = 2, reflect):
wavedec3, waverec3 (2 IG alphas) and the adjoint.

usage: python scripts/kbench_3d.py [--iters 10]
"""
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
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.manual_seed(0)
    B, D = 16, 128
    x = torch.randn(B, D, D, D, device="cuda")
    for wav in ("db4", "sym8"):
        for tag, generic in (("fused", False), ("per-axis", True)):
            p = P.get_plan(3, (D, D, D), 2, wav, "reflect", "cuda", generic=generic)
            cf = p.wavedec(x)
            g = torch.randn((B,) + p.rec_shape, device="cuda")
            run("%s %s wavedec3" % (wav, tag), lambda: p.wavedec(x), a.iters)
            run("%s %s waverec3 (2 alphas)" % (wav, tag), lambda: p.waverec(cf, B, alphas=[0.5, 1.0]), a.iters)
            run("%s %s adjoint" % (wav, tag), lambda: p.adjoint(g), a.iters)


if __name__ == "__main__":
    main()
