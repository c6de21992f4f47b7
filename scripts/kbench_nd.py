"""Per-launch timing of the 1D (c3) and 3D (c5) transforms at the BASELINE config shapes.

usage: python scripts/kbench_nd.py [--iters 5]
c3: 1D db6 J=5, 256 clips x 80000 samples x 25 noise samples per launch group (6400 signals)
c5: 3D haar J=2 symmetric, 16 volumes of 128^3 x 25 samples (400 volumes)
c4: 2D sym8 J=5 reflect at 512^2, 128 images x 3 channels x 2 IG steps per call (768 planes)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from scripts.kbench import run  # noqa: E402
from wam_amd import plan as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default=None, help="c3, c4 or c5")
    args = ap.parse_args()
    torch.manual_seed(0)
    for tag, dim, shape, J, wav, mode, B in [("c3 1D", 1, (80000,), 5, "db6", "reflect", 6400),
                                             ("c5 3D", 3, (128, 128, 128), 2, "haar", "symmetric", 400),
                                             ("c4 2D", 2, (512, 512), 5, "sym8", "reflect", 768)]:
        if args.only and not tag.startswith(args.only):
            continue
        p = P.get_plan(dim, shape, J, wav, mode, "cuda")
        if dim == 1:  # the c3 bench's noisy group: 256 clips x 5 samples per launch
            xc = torch.randn(256, shape[0], device="cuda")
            sig = P.item_sigma(xc, shape[0], shape[0], 0.25)
            run(f"{tag} wavedec_noisy 256x5", lambda: p.wavedec_noisy(xc, sig, 5, 256, 1, seed=1, sample_base=0),
                args.iters)
            del xc
        x = torch.randn((B,) + shape, device="cuda")
        run(f"{tag} wavedec B={B}", lambda: p.wavedec(x), args.iters)
        cf = p.wavedec(x)
        run(f"{tag} waverec", lambda: p.waverec(cf, B), args.iters)
        del cf
        g = torch.randn((B,) + p.rec_shape, device="cuda")
        run(f"{tag} adjoint", lambda: p.adjoint(g), args.iters)
        del g, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
