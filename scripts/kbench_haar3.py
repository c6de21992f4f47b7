"""Per-launch timing of the c5 WAM kernels at the bench's launch shape (haar J=2, 128^3 volumes,
2 samples x 16 volumes = 32 items per launch): k_haar3_ana, k_haar3_syn, k_subband_maps.

usage: python scripts/kbench_haar3.py [--iters 20] [--items 32]
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--items", type=int, default=32)
    a = ap.parse_args()
    torch.manual_seed(0)
    B, D = a.items, 128
    p = P.get_plan(3, (D, D, D), 2, "haar", "reflect", "cuda")
    x = torch.randn(B, D, D, D, device="cuda")
    cf = p.wavedec(x)
    run("c5 wavedec3 %d items" % B, lambda: p.wavedec(x), a.iters)
    run("c5 waverec3 %d items" % B, lambda: p.waverec(cf, B), a.iters)
    run("c5 subband maps %d items" % B, lambda: P.subband_maps(p, cf, B, 1, 1), a.iters)


if __name__ == "__main__":
    main()
