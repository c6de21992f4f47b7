"""Stem input-gradient variants at the c2 model batch (832 x 64 x 112 x 112 bf16, channels_last):
(a) polyphase with an explicit F.pad (model_opt._PolyphaseInputGrad), (b) polyphase with the
conv's own symmetric padding and a crop, (c) as (b) with the gradient in NCHW, (d) MIOpen
backward-data of the original 7x7/2 convolution, (e-g) as (b) with the 12 output channels
zero-padded to 16/32/64. Times (median of 7) and max |diff| vs (a)."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels  # noqa: E402
from wam_amd.model_opt import InputConv2d, _PolyphaseInputGrad, _phase_geometry  # noqa: E402


def timeit(fn, n=7):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return sorted(ts)[n // 2]


def main(batch=832):
    conv = testmodels.resnet50(seed=0).conv1.cuda().to(torch.bfloat16)
    ic = InputConv2d(conv).cuda().to(torch.bfloat16)
    go = torch.randn(batch, 64, 112, 112, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    H = W = 224
    oy, Ty, _, ny = _phase_geometry(ic.kh, ic.pad[0], H)
    ox, Tx, _, nx = _phase_geometry(ic.kw, ic.pad[1], W)

    class _C:
        saved_tensors = (ic.wpoly,)
        geom = ((oy, Ty, ny), (ox, Tx, nx))
        in_hw = (H, W)

    def a():
        return _PolyphaseInputGrad.backward(_C, go)[0]

    py0, px0 = -oy, -ox
    py1 = (ny - 1 + oy + Ty - 1) - (go.shape[-2] - 1)
    px1 = (nx - 1 + ox + Tx - 1) - (go.shape[-1] - 1)
    P, Q = max(py0, py1), max(px0, px1)

    def b(g=go):
        o = F.conv2d(g, ic.wpoly, padding=(P, Q))
        o = o[..., P - py0:P - py0 + ny, Q - px0:Q - px0 + nx]
        return F.pixel_shuffle(o, 2)[..., :H, :W]

    gn = go.contiguous()

    def c():
        return b(gn)

    x = torch.empty(batch, 3, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def d():
        return torch.ops.aten.convolution_backward(go, x, conv.weight, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]

    def padded(cout):
        wp = torch.zeros(cout, *ic.wpoly.shape[1:], dtype=ic.wpoly.dtype, device="cuda")
        wp[:ic.wpoly.shape[0]] = ic.wpoly

        def e():
            o = F.conv2d(go, wp, padding=(P, Q))
            o = o[:, :ic.wpoly.shape[0], P - py0:P - py0 + ny, Q - px0:Q - px0 + nx]
            return F.pixel_shuffle(o, 2)[..., :H, :W]
        return e

    ref = a().float()
    print("pads", (py0, py1, px0, px1))
    for name, fn in (("a pad+polyphase", a), ("b conv-pad+crop", b), ("c conv-pad NCHW", c), ("d miopen bwd-data", d),
                     ("e b, 16 out ch", padded(16)), ("f b, 32 out ch", padded(32)), ("g b, 64 out ch", padded(64))):
        t = timeit(fn)
        diff = (fn().float() - ref).abs().max().item()
        print("%-18s %8.3f ms  max|diff vs a| %.3e" % (name, t, diff))


if __name__ == "__main__":
    main()
