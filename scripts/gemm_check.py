"""Diagnose the pointwise-GEMM path of the fused input-gradient model (fp32, channels_last):
single-op gradients vs float64, then the whole fused model with the GEMM path on and off."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels  # noqa: E402
from wam_amd import model_fuse as mf  # noqa: E402
from wam_amd.model_opt import optimize_for_input_grad  # noqa: E402


def rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm()).item()


def single_ops():
    torch.manual_seed(0)
    for cin, cout in ((64, 256), (256, 64), (512, 128)):
        x = torch.randn(4, cin, 24, 24).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 1, 1) / cin ** 0.5
        b = torch.randn(cout) * 0.1
        g = torch.randn(4, cout, 24, 24)
        x64 = x.double().requires_grad_(True)
        y64 = torch.relu(torch.nn.functional.conv2d(x64, w.double(), b.double()))
        (gx64,) = torch.autograd.grad(y64, x64, g.double())
        xc = x.cuda().requires_grad_(True)
        y = mf._ConvBiasReLUFn.apply(xc, w.cuda(), b.cuda(), ((1, 1), (0, 0), (1, 1), 1))
        for gl, name in ((g.cuda(), "g nchw"), (g.cuda().contiguous(memory_format=torch.channels_last), "g cl")):
            (gx,) = torch.autograd.grad(y, xc, gl, retain_graph=True)
            print("ConvBiasReLU %d->%d %s: fwd %.2e grad %.2e" % (cin, cout, name, rel(y, y64), rel(gx, gx64)))
        y64 = torch.nn.functional.conv2d(x64, w.double())
        (gx64,) = torch.autograd.grad(y64, x64, g.double())
        xc = x.cuda().requires_grad_(True)
        w2 = w.cuda().reshape(cout, cin)
        y = mf._PointwiseConvFn.apply(mf._rows(xc).detach(), xc, w2)
        for gl, name in ((g.cuda(), "g nchw"), (g.cuda().contiguous(memory_format=torch.channels_last), "g cl")):
            (gx,) = torch.autograd.grad(y, xc, gl, retain_graph=True)
            print("PointwiseConv %d->%d %s: fwd %.2e grad %.2e" % (cin, cout, name, rel(y, y64), rel(gx, gx64)))


def whole(gemm, xseed=1):
    from tests.test_model_opt import _randomise_bn
    m = _randomise_bn(testmodels.resnet50(seed=0))
    torch.manual_seed(xseed)
    x = torch.randn(4, 3, 96, 96)
    x64 = x.double().requires_grad_(True)
    o64 = m.double()(x64)
    (g64,) = torch.autograd.grad(o64[:, 7].sum(), x64)
    m = m.float().cuda()
    saved = mf._rows
    if not gemm:
        mf._rows = lambda t: None
    try:
        fus = optimize_for_input_grad(m, dtype=torch.float32, fuse=True).to(memory_format=torch.channels_last)
        xx = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        o = fus(xx)
        (g,) = torch.autograd.grad(o[:, 7].float().sum(), xx)
    finally:
        mf._rows = saved
    print("whole resnet50 fp32 CL gemm=%s xseed=%d: out %.2e grad %.2e" % (gemm, xseed, rel(o, o64), rel(g, g64)))


if __name__ == "__main__":
    for xs in range(1, 6):
        whole(False, xs)
        whole(True, xs)
