"""PMC / timing driver for the mosaic epilogues on the bench shapes: the c2 SmoothGrad accumulation
(25 samples x 64 images, db4 J=3 224^2, coefficient order) and the c4 IG trapezoid (21 steps x 128
images, sym8 J=5 512^2) in coefficient order (wam_frame_trapz_coef, the classes' path) and in pixel
order (wam_frame_trapz), 3 calls each; prints per kernel launches, mean us and algorithmic bytes."""
import collections
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import wam_amd  # noqa: F401
from wam_amd import frames, plan as P
from wam_amd._lib import check, lib, ptr, stream_of


def c2():
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    S, n = 25, 64
    gmap, (rh, rw) = frames.smooth_frame(p, n, "native", "cuda")
    maps = torch.rand(S * n * p.coeff_numel, device="cuda")
    bmax = torch.rand(S, p.nbands, device="cuda") + 0.5
    frame = torch.zeros(n * rh * rw, dtype=torch.float64, device="cuda")
    return lambda: P.frame_accumulate(S, n, gmap, maps, p.coeff_numel, bmax, p.nbands, True, frame)


def c4():
    p = P.get_plan(2, (512, 512), 5, "sym8", "reflect", "cuda")
    G, n = 21, 128
    _, gmap, (rh, rw) = frames.ig_frames(p, n, "native", "cuda")
    src, band = gmap
    maps = torch.rand(G * n * p.coeff_numel, device="cuda")
    bmax = torch.rand(G, p.nbands, device="cuda") + 0.5
    acc = torch.zeros(n * rh * rw, device="cuda")
    prev = torch.zeros_like(acc)
    coef = lambda: P.frame_trapz(G, 0, n, gmap, maps, p.coeff_numel, bmax, p.nbands, True, prev, acc)
    pix = lambda: check(lib.wam_frame_trapz(G, 0, n, src.numel(), ptr(src), ptr(band), ptr(maps), p.coeff_numel,
                                            ptr(bmax), p.nbands, 1, None, ptr(prev), ptr(acc), stream_of(acc.device)))
    return coef, pix


fa = c2()
coef, pix = c4()
fns = [fa, coef, pix]
for f in fns:
    f()
torch.cuda.synchronize()
P.timing_drain()
P.timing_enable(True)
for _ in range(3):
    for f in fns:
        f()
torch.cuda.synchronize()
P.timing_enable(False)
acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
for name, ms, nb in P.timing_drain():
    a = acc[name]
    a[0] += 1
    a[1] += ms
    a[2] += nb
for k, (n_, ms, nb) in sorted(acc.items()):
    print("%-26s launches %3d  mean %8.1f us  algorithmic %12.0f B/launch  %6.0f GB/s" % (
        k, n_, ms / n_ * 1e3, nb / n_, nb / ms / 1e6))
