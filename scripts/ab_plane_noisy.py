"""A/B of the c2 SmoothGrad analysis (`k_plane_ana<noise>`) at several sample counts (4,800 planes =
c2; 4,032 = one round of 4 waves per SIMD) and plan flags (0; 8 = NO_COOP; 16 = FORCE_COOP), timed with
the library's HIP events. WAM_LIB_PATH selects a variant build (scripts/build_variants.py).

usage: python scripts/ab_plane_noisy.py [--iters 20] [--samples 25,21] [--flags 0]
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
    ap.add_argument("--samples", default="25,21")
    ap.add_argument("--flags", default="0")
    ap.add_argument("--wavelet", default="db4")
    ap.add_argument("--J", type=int, default=3)
    args = ap.parse_args()
    torch.manual_seed(0)
    N, C, H = 64, 3, 224
    x = torch.randn(N, C, H, H, device="cuda")
    sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
    tag = os.path.basename(os.environ.get("WAM_LIB_PATH", "") or "cur")
    for S in [int(v) for v in args.samples.split(",")]:
        for f in [int(v) for v in args.flags.split(",")]:
            p = P.get_plan(2, (H, H), args.J, args.wavelet, "reflect", "cuda", flags=f)
            r = timed(lambda: p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0), args.iters)
            for name, (us, nb) in sorted(r.items()):
                planes = S * N * C
                print(f"{tag:10s} S={S:3d} planes={planes:5d} f{f:<3d} {name:22s} {us:8.1f} us  "
                      f"{us * 4800 / planes:8.1f} us@4800  {nb / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
