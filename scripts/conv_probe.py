"""GPU probe: ResNet-50 1x1 convolutions at the c2 model batch (832 = 13 samples x 64 images),
NHWC bf16 -- MIOpen convolution (forward and backward-data) vs the same contraction as a
hipBLASLt GEMM over the [N*H*W, C] view. Prints one JSON line per shape.

usage: python scripts/conv_probe.py [--batch 832]
"""
import argparse
import json

import torch
import torch.nn.functional as F


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=832)
    a = ap.parse_args()
    dev = "cuda"
    # (H, Cin, Cout) of the stride-1 1x1 convs in ResNet-50 bottlenecks
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (14, 1024, 256),
              (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]
    for h, ci, co in shapes:
        n = a.batch
        x = torch.randn(n, ci, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(n, co, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2, w2, g2 = x.permute(0, 2, 3, 1).reshape(-1, ci), w.view(co, ci), g.permute(0, 2, 3, 1).reshape(-1, co)
        t_cf = timed(lambda: F.conv2d(x, w))
        t_cb = timed(lambda: torch.ops.aten.convolution_backward(g, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0],
                                                                 1, [True, False, False]))
        t_mf = timed(lambda: torch.mm(x2, w2.t()))
        t_mb = timed(lambda: torch.mm(g2, w2))
        m = n * h * h
        flops = 2.0 * m * ci * co
        byts = 2.0 * m * (ci + co)
        rec = {"h": h, "cin": ci, "cout": co, "M": m, "conv_fwd_ms": round(t_cf, 3), "conv_bwd_ms": round(t_cb, 3),
               "mm_fwd_ms": round(t_mf, 3), "mm_bwd_ms": round(t_mb, 3),
               "min_ms_at_8TBs": round(byts / 8e12 * 1e3, 3), "tflops_conv_fwd": round(flops / t_cf / 1e9, 1),
               "tflops_mm_fwd": round(flops / t_mf / 1e9, 1)}
        print(json.dumps(rec), flush=True)
        # correctness of the GEMM form (same contraction)
        y1 = F.conv2d(x, w).permute(0, 2, 3, 1).reshape(-1, co).float()
        y2 = torch.mm(x2, w2.t()).float()
        assert (y1 - y2).abs().max().item() <= 2e-2 * y1.abs().max().item()


if __name__ == "__main__":
    main()
