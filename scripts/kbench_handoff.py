"""Per-launch timing of the c2 hand-off kernels (library HIP events): the plane synthesis writing fp32
planes vs the model's bf16 NHWC input, and the maps pass over an fp32 / bf16 NCHW / bf16 NHWC
gradient, at the c2 shapes (4,800 planes; two model groups of 13 + 12 samples x 64 images).
Run it under rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE for the traffic of each form.

usage: python scripts/kbench_handoff.py [--iters 20]
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
    a = ap.parse_args()
    torch.manual_seed(0)
    N, C, S, H = 64, 3, 25, 224
    p = P.get_plan(2, (H, H), 3, "db4", "reflect", "cuda")
    B = S * N * C
    cf = p.wavedec(torch.randn(B, H, H, device="cuda"))
    run("waverec fp32 planes", lambda: p.waverec(cf, B), a.iters)
    run("waverec bf16 NHWC", lambda: p.waverec_bf16_nhwc(cf, B, C), a.iters)
    g32 = torch.randn(13 * N * C, H, H, device="cuda") * 1e-3
    gb = g32.view(13 * N, C, H, H).to(torch.bfloat16)
    gbl = gb.contiguous(memory_format=torch.channels_last)
    run("maps fp32 (13 x 64 images)", lambda: p.adjoint_maps(g32, 13, N, C), a.iters)
    run("maps bf16 NCHW", lambda: p.adjoint_maps(gb, 13, N, C), a.iters)
    run("maps bf16 NHWC", lambda: p.adjoint_maps(gbl, 13, N, C), a.iters)


if __name__ == "__main__":
    main()
