"""wam_amd/model_opt.py: the optimized input-gradient model computes the model's function.

CPU (float64): polyphase input-gradient of stride-2 convs against autograd for odd/even sizes,
kernel sizes and paddings; BN folding on ResNet-18/50 with randomised running statistics
(outputs and input gradients). GPU: WAM-2D maps with optimize_model=True vs the model as is.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

import testmodels
from wam_amd.model_opt import InputConv2d, optimize_for_input_grad


def _randomise_bn(model, seed=0):
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            n = m.num_features
            m.running_mean.copy_(torch.rand(n, generator=g) - 0.5)
            m.running_var.copy_(0.5 + 1.5 * torch.rand(n, generator=g))
            m.weight.data.copy_(0.5 + torch.rand(n, generator=g))
            m.bias.data.copy_(0.4 * torch.rand(n, generator=g) - 0.2)
    return model


@pytest.mark.parametrize("k,p,h,w", [(7, 3, 224, 224), (7, 3, 31, 30), (3, 1, 17, 16), (4, 1, 20, 21),
                                     (5, 2, 9, 9), (2, 0, 12, 13), (7, 0, 40, 41), (1, 0, 8, 7)])
def test_polyphase_input_grad(k, p, h, w):
    torch.manual_seed(k * 100 + p)
    conv = nn.Conv2d(3, 8, k, 2, p, bias=True).double()
    ic = InputConv2d(conv).double()
    x = torch.randn(2, 3, h, w, dtype=torch.float64, requires_grad=True)
    y1 = conv(x)
    go = torch.randn_like(y1)
    (g1,) = torch.autograd.grad(y1, x, go)
    x2 = x.detach().requires_grad_(True)
    y2 = ic(x2)
    (g2,) = torch.autograd.grad(y2, x2, go)
    assert torch.equal(y1, y2)
    assert g2.shape == g1.shape
    assert (g1 - g2).abs().max().item() <= 1e-13 * max(1.0, g1.abs().max().item())


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_fold_matches_model(arch):
    m = _randomise_bn(getattr(testmodels, arch)(seed=0)).double()
    gm = optimize_for_input_grad(m)
    assert not any(isinstance(q, nn.BatchNorm2d) for q in gm.modules())
    assert isinstance(gm.conv1, InputConv2d)
    assert not any(p.requires_grad for p in gm.parameters())
    x = torch.randn(2, 3, 64, 64, dtype=torch.float64, requires_grad=True)
    o1 = m(x)
    (g1,) = torch.autograd.grad(o1[:, 3].sum(), x)
    x2 = x.detach().requires_grad_(True)
    o2 = gm(x2)
    (g2,) = torch.autograd.grad(o2[:, 3].sum(), x2)
    assert (o1 - o2).abs().max().item() <= 1e-12 * o1.abs().max().item()
    assert (g1 - g2).abs().max().item() <= 1e-12 * g1.abs().max().item()


def test_rejects_training_mode():
    with pytest.raises(ValueError):
        optimize_for_input_grad(testmodels.resnet18(seed=0).train())


def test_dtype_cast_keeps_polyphase_table():
    gm = optimize_for_input_grad(testmodels.resnet18(seed=0), dtype=torch.bfloat16)
    assert gm.conv1.weight.dtype == torch.bfloat16 and gm.conv1.wpoly.dtype == torch.bfloat16


class _TinyBN(nn.Module):
    """Kink-free conv-BN-tanh model: optimized vs original differ only by fp rounding."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 7, 2, 3, bias=False)
        self.bn = nn.BatchNorm2d(8)
        self.conv2 = nn.Conv2d(8, 8, 3, 2, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8 * 4 * 4, 10)

    def forward(self, x):
        h = torch.tanh(self.bn(self.conv(x)))
        h = torch.tanh(self.bn2(self.conv2(h)))
        h = nn.functional.adaptive_avg_pool2d(h, 4)
        return self.fc(torch.flatten(h, 1))


@pytest.mark.gpu
def test_gpu_wam2d_optimize_model_matches():
    from wam_amd.wam_2D import WaveletAttribution2D
    torch.manual_seed(0)
    m = _TinyBN()
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
    m = m.eval().cuda()
    x = torch.tensor(np.random.RandomState(0).standard_normal((2, 3, 64, 64)).astype(np.float32))
    kw = dict(wavelet="db4", J=3, method="smooth", n_samples=4, noise="philox", frame="native")
    a = WaveletAttribution2D(m, **kw)(x, [1, 3])
    b = WaveletAttribution2D(m, optimize_model=True, **kw)(x, [1, 3])
    assert a.shape == b.shape
    assert np.abs(a - b).max() <= 1e-4, np.abs(a - b).max()


# ------------------------------------------------------------------ fused elementwise (model_fuse)
def test_fuse_rewrite_structure():
    """The graph rewrite (CPU, no compute): every conv->ReLU, the stem and every residual tail of
    ResNet-50 become fused modules; no ReLU, add or biased conv is left on the pattern."""
    import operator
    from wam_amd import model_fuse
    gm = optimize_for_input_grad(testmodels.resnet50(seed=0), fuse=False)
    gm, n = model_fuse.fuse_elementwise(gm)
    assert n == 1 + 16 * 2 + 16 + 1
    kinds = [type(m).__name__ for m in gm.modules()]
    assert kinds.count("ConvBiasReLU") == 32 and kinds.count("AddBiasReLU") == 16
    assert kinds.count("InputConvReLUPool") == 1 and kinds.count("ConvNoBias") == 16 + 4
    assert "MaxPool2d" not in kinds and "InputConvReLU" not in kinds
    assert "ReLU" not in kinds
    assert not any(nd.op == "call_function" and nd.target is operator.add for nd in gm.graph.nodes)
    # identity blocks (16 minus the 4 with a downsample) hand their skip gradient to the
    # producing block's ReLU mask
    assert sum(getattr(m, "link_in", None) is not None for m in gm.modules()) == 12
    assert sum(getattr(m, "link_out", None) is not None for m in gm.modules()) == 12
    gm18, n18 = model_fuse.fuse_elementwise(optimize_for_input_grad(testmodels.resnet18(seed=0), fuse=False))
    assert n18 == 1 + 8 + 8 + 1
    # resnet18: layer1.0 takes the max-pool output (no producing add), so 5 - 1 links
    assert sum(getattr(m, "link_in", None) is not None for m in gm18.modules()) == 4


class _AuxBranchNet(nn.Module):
    """Non-ResNet topology: the producer's output feeds the consumer add's skip operand AND an
    auxiliary head that does not lead to the add's other operand, plus a broadcast add."""

    def __init__(self):
        super().__init__()
        self.c0 = nn.Conv2d(3, 8, 3, padding=1)
        self.c1 = nn.Conv2d(8, 8, 3, padding=1)
        self.c2 = nn.Conv2d(8, 8, 3, padding=1)
        self.pos = nn.Parameter(torch.randn(1, 8, 1, 1))
        self.aux = nn.Conv2d(8, 8, 1)
        self.fc = nn.Linear(8, 4)

    def forward(self, x):
        h = self.c0(x)
        p = torch.relu(self.c1(h) + h)      # producer (residual add + ReLU)
        aux = self.aux(p)                   # side branch: never reaches c2(h)
        q = torch.relu(self.c2(h) + p)      # consumer: a = c2(h), skip operand s = p
        r = torch.relu(q + self.pos)        # broadcast operand [1, C, 1, 1]
        return self.fc((r + aux).mean((2, 3)))


def test_fuse_guards_non_resnet_patterns():
    """no skip-gradient link when the producer's other user does not reach the
    consumer's `a` operand; a broadcast residual add falls back to torch (same values)."""
    from wam_amd import model_fuse
    torch.manual_seed(0)
    gm, _ = model_fuse.fuse_elementwise(torch.fx.symbolic_trace(_AuxBranchNet().eval()))
    kinds = [type(m).__name__ for m in gm.modules()]
    assert kinds.count("AddBiasReLU") == 3
    assert sum(getattr(m, "link_in", None) is not None for m in gm.modules()) == 0
    assert sum(getattr(m, "link_out", None) is not None for m in gm.modules()) == 0
    # broadcast / mismatched operands take the torch path (and CPU tensors are never fused)
    abr = model_fuse.AddBiasReLU(torch.randn(8), None)
    a, s = torch.randn(2, 8, 4, 4), torch.randn(1, 8, 1, 1)
    assert not abr._fusable(a, s)
    assert torch.equal(abr(a, s), torch.relu(a + abr.bias_a.view(1, -1, 1, 1) + s))


@pytest.mark.gpu
def test_gpu_fuse_guards_non_resnet_patterns():
    """The rewritten aux-branch / broadcast-add network on the GPU: outputs and input gradients
    equal the original module's (fp32; kernels and torch compute the same adds)."""
    from wam_amd import model_fuse
    torch.manual_seed(0)
    net = _AuxBranchNet().eval().cuda()
    gm = model_fuse.fuse_elementwise(torch.fx.symbolic_trace(net))[0]
    x = torch.randn(3, 3, 16, 16, device="cuda")
    outs = []
    for m in (net, gm):
        xx = x.clone().requires_grad_(True)
        o = m(xx)
        (g,) = torch.autograd.grad(o[:, 1].sum(), xx)
        outs.append((o.detach(), g))
    assert torch.allclose(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-6)
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-4, atol=1e-6)


def test_fuse_not_applied_on_cpu():
    gm = optimize_for_input_grad(testmodels.resnet18(seed=0))
    assert not any(type(m).__name__ == "ConvBiasReLU" for m in gm.modules())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
def test_gpu_ew_kernels_match_torch(dtype, cl):
    from wam_amd import model_fuse as mf
    torch.manual_seed(0)
    for shape in [(3, 64, 14, 14), (2, 24, 7, 7), (2, 5, 3, 3), (4, 256, 8, 8)]:
        mk = lambda: torch.randn(shape, device="cuda").to(dtype)  # noqa: E731
        y, a, s, g, g2 = mk(), mk(), mk(), mk(), mk()
        if cl:
            y, a, s, g, g2 = (t.contiguous(memory_format=torch.channels_last) for t in (y, a, s, g, g2))
        b1 = torch.randn(shape[1], device="cuda").to(dtype)
        b2 = torch.randn(shape[1], device="cuda").to(dtype)
        bc = lambda b: b.float().view(1, -1, 1, 1)  # noqa: E731
        ref = torch.relu(y.float() + bc(b1)).to(dtype)
        out = mf.bias_act_(y.clone(memory_format=torch.preserve_format), b1, True)
        assert torch.equal(out, ref)
        ref = torch.relu((a.float() + bc(b1)) + (s.float() + bc(b2))).to(dtype)
        assert torch.equal(mf.add_bias_relu(a, b1, s, b2), ref)
        assert torch.equal(mf.add_bias_relu(a, None, s, None), torch.relu(a.float() + s.float()).to(dtype))
        assert torch.equal(mf.relu_mask(g, y), torch.where(y > 0, g, torch.zeros_like(g)))
        assert torch.equal(mf.relu_mask(g, y, g2), torch.where(y > 0, (g.float() + g2.float()).to(dtype),
                                                                 torch.zeros_like(g)))
        # mixed layouts: gradient NCHW, activation NHWC
        assert torch.equal(mf.relu_mask(g.contiguous(), y), torch.where(y > 0, g, torch.zeros_like(g)))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k,st,p,h,w,c", [(3, 2, 1, 112, 112, 64), (3, 2, 1, 17, 14, 16), (2, 2, 0, 9, 8, 8),
                                          (3, 1, 1, 7, 6, 24)])
def test_gpu_maxpool_nhwc_matches_torch(dtype, k, st, p, h, w, c):
    """Byte-index NHWC max pool vs torch max_pool2d(_with_indices) and its backward: pooled values
    bit-equal, input gradient bit-equal (fp32 sums of <= 4 window terms in the same order), and
    with relu=True equal to torch's backward followed by the ReLU mask of the pooled input.
    Ties and exact zeros (ReLU outputs) are forced by quantising half of the input to 0."""
    from wam_amd import model_fuse as mf
    torch.manual_seed(3)
    y = torch.relu(torch.randn(3, c, h, w, device="cuda")).to(dtype)
    y = torch.where(torch.rand_like(y, dtype=torch.float32) < 0.3, torch.zeros_like(y), y)
    y = y.contiguous(memory_format=torch.channels_last)
    out, idx = mf.maxpool_nhwc(y, k, st, p)
    ref, ridx = torch.nn.functional.max_pool2d(y.float(), k, st, p, return_indices=True)
    assert torch.equal(out.float(), ref)
    go = torch.randn_like(ref).to(dtype).contiguous(memory_format=torch.channels_last)
    gref = torch.ops.aten.max_pool2d_with_indices_backward(go.float(), y.float(), [k, k], [st, st], [p, p], [1, 1],
                                                           False, ridx)
    g0 = mf.maxpool_nhwc_backward(go, idx, y.shape, k, st, p, relu=False)
    assert torch.allclose(g0.float(), gref.to(dtype).float(), rtol=0, atol=0)
    g1 = mf.maxpool_nhwc_backward(go, idx, y.shape, k, st, p, relu=True)
    assert torch.equal(g1.float(), torch.where(y.float() > 0, gref, torch.zeros_like(gref)).to(dtype).float())


@pytest.mark.gpu
@pytest.mark.parametrize("arch,dtype,cl", [("resnet50", torch.float32, False), ("resnet50", torch.bfloat16, True),
                                           ("resnet18", torch.bfloat16, False), ("resnet50", torch.float32, True)])
def test_gpu_fused_model_matches_unfused(arch, dtype, cl):
    """Fused input-gradient model vs the same folded model op by op, both against the model in
    float64 on the CPU: the fused form must be as close to the exact gradient as the unfused one.
    ReLU masks flip on rounding-level differences (measured on MI355X, scripts/gemm_check.py: one
    96^2 batch of 4 in 5 flips a mask in the MIOpen path as well as in the GEMM path, moving that
    batch's gradient by ~4e-3 relative), so the gradients are compared per image by the median
    over 8 images, with a bound on the worst image that a real layout or indexing error exceeds."""
    m = _randomise_bn(getattr(testmodels, arch)(seed=0))
    torch.manual_seed(1)
    x = torch.randn(8, 3, 96, 96)
    x64 = x.double().requires_grad_(True)
    o64 = m.double()(x64)
    (g64,) = torch.autograd.grad(o64[:, 7].sum(), x64)
    m = m.float().cuda()
    ref = optimize_for_input_grad(m, dtype=dtype, fuse=False)
    fus = optimize_for_input_grad(m, dtype=dtype, fuse=True)
    assert any(type(q).__name__ == "AddBiasReLU" for q in fus.modules())
    fmt = torch.channels_last if cl else torch.contiguous_format
    ref, fus = ref.to(memory_format=fmt), fus.to(memory_format=fmt)
    xd = x.cuda().to(dtype).contiguous(memory_format=fmt)
    errs = []
    for net in (ref, fus):
        xx = xd.detach().requires_grad_(True)
        o = net(xx)
        (g,) = torch.autograd.grad(o[:, 7].float().sum(), xx)
        oe = ((o.double().cpu() - o64.detach()).abs().max() / o64.abs().max()).item()
        d = (g.double().cpu() - g64).flatten(1).norm(dim=1) / g64.flatten(1).norm(dim=1)
        errs.append((oe, d.median().item(), d.max().item()))
    (oe_r, ge_r, _), (oe_f, ge_f, gmax_f) = errs
    floor = 1e-5 if dtype == torch.float32 else 1e-2
    worst = 5e-2 if dtype == torch.float32 else 0.5
    assert oe_f <= 2 * oe_r + floor, errs
    assert ge_f <= 2 * ge_r + floor, errs
    assert gmax_f <= worst, errs


@pytest.mark.gpu
def test_gpu_skip_handoff_two_forwards_before_backward():
    """The skip-gradient boxes are per forward call: two forwards through the fused model
    followed by their two backwards (in reverse order) give the input gradients of
    forward+backward pairs, and those of the model with the hand-off links removed."""
    m = _randomise_bn(testmodels.resnet50(seed=0)).float().cuda()
    fus = optimize_for_input_grad(m, dtype=torch.float32, fuse=True).to(memory_format=torch.channels_last)
    torch.manual_seed(5)
    xs = [torch.randn(2, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last) for _ in range(2)]

    def grad_of(x):
        xx = x.detach().requires_grad_(True)
        o = fus(xx)
        return xx, o[:, 3].sum()

    pairs = []
    for x in xs:
        xx, loss = grad_of(x)
        pairs.append(torch.autograd.grad(loss, xx)[0])
    (x0, l0), (x1, l1) = grad_of(xs[0]), grad_of(xs[1])
    g1 = torch.autograd.grad(l1, x1)[0]
    g0 = torch.autograd.grad(l0, x0)[0]
    # MIOpen's backward-data solvers are not bit-deterministic from call to call, and a rounding
    # difference can flip a ReLU mask (a local change of ~1e-3 relative, see
    # test_gpu_fused_model_matches_unfused), so images are compared by relative L2 error; a box
    # handed to the wrong forward would carry another input's skip gradient, an O(1) error
    def close(a, b):
        d = (a - b).flatten(1).norm(dim=1) / b.flatten(1).norm(dim=1)
        return bool((d < 5e-2).all())
    assert close(g0, pairs[0]) and close(g1, pairs[1])
    linked = [q for q in fus.modules() if getattr(q, "link_in", None) is not None or
              getattr(q, "link_out", None) is not None]
    assert linked
    for q in linked:
        q.link_in = q.link_out = None
    for x, g in zip(xs, pairs):
        xx, loss = grad_of(x)
        ref = torch.autograd.grad(loss, xx)[0]
        assert close(g, ref)
