"""Per-level timing of the 2D WAM kernels on the bench workload shapes (library HIP-event timing).

usage: python scripts/kbench.py [--iters 20]
Prints, for each kernel path (flags), each launch of one call with its mean time and GB/s.
"""
import argparse
import collections
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import plan as P  # noqa: E402


def run(label, fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    P.timing_drain()
    P.timing_enable(True)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    P.timing_enable(False)
    recs = P.timing_drain()
    per = len(recs) // iters
    acc = collections.defaultdict(lambda: [0.0, 0.0, ""])
    for i, (name, ms, nb) in enumerate(recs):
        a = acc[i % per]
        a[0] += ms / iters
        a[1] = nb
        a[2] = name
    tot = sum(v[0] for v in acc.values())
    print(f"{label}: total {tot * 1e3:.1f} us")
    for k in sorted(acc):
        ms, nb, name = acc[k]
        print(f"   [{k}] {name:22s} {ms * 1e3:8.1f} us  {nb / 1e6:8.1f} MB  {nb / ms / 1e6:7.0f} GB/s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--wavelet", default="db4")
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--samples", type=int, default=25, help="noise samples per WAM launch (bench: all 25)")
    args = ap.parse_args()
    torch.manual_seed(0)
    N, C, S, H = 64, 3, args.samples, args.size
    x = torch.randn(N, C, H, H, device="cuda")
    modes = [(0, "plane"), (P.PLAN_NO_PLANE, "rows")]
    if os.environ.get("KBENCH_PLANE_ONLY"):
        modes = modes[:1]
    for flags, tag in modes:
        p = P.get_plan(2, (H, H), args.levels, args.wavelet, "reflect", "cuda", flags=flags)
        sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
        if p.caps & P.CAP_NOISY_WAVEDEC:
            run(f"{tag} wavedec_noisy S={S}", lambda: p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0),
                args.iters)
            xb = torch.randn(S * N, C, H, H, device="cuda")
            sb = P.item_sigma(xb, C * H * H, C * H * H, 0.25)
            run(f"{tag} wavedec_noisy S=1 N={S * N} (no shared source)",
                lambda: p.wavedec_noisy(xb, sb, 1, S * N, C, seed=1, sample_base=0), args.iters)
            del xb
        xs = torch.randn(S * N * C, H, H, device="cuda")
        run(f"{tag} wavedec", lambda: p.wavedec(xs), args.iters)
        g = torch.randn((S * N * C,) + p.rec_shape, device="cuda")
        if p.caps & P.CAP_ADJOINT_MAPS:
            run(f"{tag} adjoint_maps", lambda: p.adjoint_maps(g, S, N, C, full=False), args.iters)
        run(f"{tag} adjoint", lambda: p.adjoint(g), args.iters)
        del g
        cf = p.wavedec(xs)
        run(f"{tag} waverec", lambda: p.waverec(cf, S * N * C), args.iters)


if __name__ == "__main__":
    main()
