"""Per-level cost of the c2 plane analysis: k_plane_ana (noisy and clean) and k_plane_maps at
J = 1, 2, 3 on the c2 group shape (64 images x 25 samples x 3 channels of 224^2, db4 reflect),
timed with the library's HIP events. The difference J=k - J=k-1 is level k's share.

usage: python scripts/kbench_levels.py [--iters 10] [--wavelet db4] [--size 224]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import plan as P  # noqa: E402


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    P.timing_drain()
    P.timing_enable(True)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    P.timing_enable(False)
    recs = P.timing_drain()
    per = {}
    for name, ms, nb in recs:
        a = per.setdefault(name, [0.0, 0, nb])
        a[0] += ms
        a[1] += 1
    return {k: (v[0] / v[1] * 1e3, v[2]) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--wavelet", default="db4")
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--levels", default="1,2,3")
    ap.add_argument("--flags", type=int, default=0)
    args = ap.parse_args()
    torch.manual_seed(0)
    N, C, S, H = 64, 3, 25, args.size
    x = torch.randn(N, C, H, H, device="cuda")
    g = torch.randn(S * N, C, H, H, device="cuda")
    xs = torch.randn(S * N * C, H, H, device="cuda")
    for J in [int(v) for v in args.levels.split(",")]:
        p = P.get_plan(2, (H, H), J, args.wavelet, "reflect", "cuda", flags=args.flags)
        sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
        for tag, fn in (("noisy", lambda: p.wavedec_noisy(x, sigma, S, N, C, seed=1, sample_base=0)),
                        ("clean", lambda: p.wavedec(xs)),
                        ("maps", lambda: p.adjoint_maps(g, S, N, C, full=False))):
            r = timed(fn, args.iters)
            for name, (us, nb) in sorted(r.items()):
                print(f"J={J} {tag:5s} {name:24s} {us:8.1f} us  {nb / 1e6:8.1f} MB  {nb / us / 1e3:7.0f} GB/s",
                      flush=True)
        del p
    from wam_amd._lib import check, lib, ptr, stream_of
    a = torch.empty(512 << 20, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    nb = a.numel() * 4
    r = timed(lambda: check(lib.wam_copy(nb, ptr(a), ptr(b), stream_of(a.device))), args.iters)
    for name, (us, nbytes) in r.items():
        print(f"copy {name:24s} {us:8.1f} us  {nbytes / 1e6:8.1f} MB  {nbytes / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
