"""Fused elementwise execution of a BN-folded ReLU network's input-gradient pass.

After ``model_opt`` folds BatchNorm into the convolutions, a ResNet input-gradient step is
convolutions (MIOpen, MFMA) plus per-channel bias adds, ReLUs, residual adds and ReLU masks.
Executed op by op in torch these elementwise steps are separate HBM passes over activation
tensors -- on MI355X about half of the c2 step (profiles/r01f_bench_kernel_stats.csv: torch
add / clamp / threshold_backward kernels next to the convolutions). ``fuse_elementwise``
rewrites the traced graph so each chain is one HIP kernel (wam_amd/csrc/model_ew.hip):

* ``conv -> relu``            -> ``ConvBiasReLU``: the convolution without bias, then
  y = max(y + b, 0) in place; backward = ReLU mask (one pass) + convolution backward-data.
* ``relu(a + s)`` where a / s are biased convolutions (bottleneck tail, downsample shortcut)
  -> the convolutions without bias and ``AddBiasReLU``: out = max((a + b_a) + (s + b_s), 0) in
  one pass; backward = one ReLU-mask pass whose result feeds both branches.
* the polyphase input convolution (``model_opt.InputConv2d``) followed by a ReLU gets the same
  bias + ReLU epilogue and a masked polyphase backward.

Only the pattern's own nodes are touched; everything else runs as traced. The functions are the
same as the graph's up to fp rounding (the bf16 tail sum rounds once instead of three times);
tests/test_model_opt.py compares outputs and input gradients with the unfused model on the GPU.
There is no CPU path for the fused ops: on a CPU model the rewrite is not applied.
"""
import operator

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .model_opt import InputConv2d, _PolyphaseInputGrad  # noqa: F401

_DT = {torch.float32: 0, torch.bfloat16: 1}


def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError("wam_amd fused model ops support float32 / bfloat16 activations, got %s" % t.dtype)


def _layout(t):
    """(tensor in a dense layout, inner) where the channel of flat element i is (i // inner) % C."""
    if t.dim() == 4 and t.shape[1] > 1 and t.shape[2] * t.shape[3] > 1:
        if t.is_contiguous(memory_format=torch.channels_last):
            return t, 1
        t = t.contiguous()
        return t, t.shape[2] * t.shape[3]
    t = t.contiguous()
    inner = 1
    for d in t.shape[2:]:
        inner *= d
    return t, inner


def _like(t, ref):
    """t in ref's memory layout (dense), so flat elementwise indexing lines up."""
    if ref.dim() == 4 and ref.is_contiguous(memory_format=torch.channels_last) and not ref.is_contiguous():
        return t.contiguous(memory_format=torch.channels_last)
    return t.contiguous()


def _stream(t):
    return _lib.c_vp(torch.cuda.current_stream(t.device).cuda_stream)


def bias_act_(y, b, relu=True):
    y, inner = _layout(y)
    _lib.check(_lib.lib.wam_ew_bias_act(_dt(y), y.numel(), y.shape[1], inner, _lib.ptr(y),
                                        _lib.ptr(b.to(y.dtype).contiguous() if b is not None else None),
                                        int(relu), _stream(y)))
    return y


def add_bias_relu(a, ba, s, bs):
    a, inner = _layout(a)
    s = _like(s, a)
    out = torch.empty_like(a)
    cast = (lambda b: None if b is None else b.to(a.dtype).contiguous())
    _lib.check(_lib.lib.wam_ew_add_bias_relu(_dt(a), a.numel(), a.shape[1], inner, _lib.ptr(a), _lib.ptr(cast(ba)),
                                             _lib.ptr(s), _lib.ptr(cast(bs)), _lib.ptr(out), _stream(a)))
    return out


def relu_mask(g, y, g2=None):
    """y > 0 ? g (+ g2) : 0 in y's layout."""
    g = _like(g, y)
    g2 = None if g2 is None else _like(g2, y)
    out = torch.empty_like(y)
    _lib.check(_lib.lib.wam_ew_relu_mask(_dt(y), y.numel(), _lib.ptr(g), _lib.ptr(g2), _lib.ptr(y), _lib.ptr(out),
                                         _stream(y)))
    return out


def _pool_ok(y, k, s, p):
    v = 8 if y.dtype == torch.bfloat16 else 4
    return (y.is_cuda and y.dim() == 4 and y.dtype in _DT and y.shape[1] % v == 0 and 2 * p <= k and k * k <= 127
            and y.is_contiguous(memory_format=torch.channels_last) and y.shape[0] <= 65535 and y.shape[2] <= 65535
            and y.shape[3] * (y.shape[1] // v) < 2 ** 30)


def maxpool_nhwc(y, k, s, p):
    """max_pool2d(y, k, s, p) of a channels_last activation -> (out, byte window index)."""
    n, c, h, w = y.shape
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    out = torch.empty((n, c, ho, wo), dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
    idx = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=y.device)
    _lib.check(_lib.lib.wam_ew_maxpool_nhwc(_dt(y), n, h, w, c, k, s, p, _lib.ptr(y), _lib.ptr(out), _lib.ptr(idx),
                                            _stream(y)))
    return out, idx


def maxpool_nhwc_backward(gy, idx, in_shape, k, s, p, relu):
    """Input gradient of maxpool_nhwc (channels_last); relu also applies the mask of the ReLU
    that produced the pooled input."""
    n, c, h, w = in_shape
    gy = gy.contiguous(memory_format=torch.channels_last)
    gx = torch.empty((n, c, h, w), dtype=gy.dtype, device=gy.device, memory_format=torch.channels_last)
    _lib.check(_lib.lib.wam_ew_maxpool_nhwc_backward(_dt(gy), n, h, w, c, k, s, p, _lib.ptr(gy), _lib.ptr(idx),
                                                     int(relu), _lib.ptr(gx), _stream(gy)))
    return gx


def _conv_nd(x, w, stride, padding, dilation, groups):
    return torch.ops.aten.convolution(x, w, None, stride, padding, dilation, False, [0] * len(stride), groups)


def _conv_grad_input(g, x, w, stride, padding, dilation, groups):
    return torch.ops.aten.convolution_backward(g, x, w, None, stride, padding, dilation, False, [0] * len(stride),
                                               groups, [True, False, False])[0]


# ---- pointwise (1x1, stride 1, unpadded) convolutions on channels_last activations as GEMMs
# An NHWC activation is a row-major [N*H*W, C] matrix, so a pointwise convolution is one GEMM
# (hipBLASLt) on a zero-copy view, and its input gradient is the GEMM with the weight untransposed.
# The forward's bias + ReLU run in the GEMM epilogue (torch._addmm_activation), so the fused
# ConvBiasReLU is a single kernel. Measured on MI355X at the c2 shapes (batch 832, bf16;
# scripts/gemm_probe.py, profiles/r01g_gemm_probe.log): 1.2-3.2x faster than the MIOpen
# convolution + epilogue pass forward, 1.1-1.9x faster for the input gradient.
# bf16 only: fp32 models keep the MIOpen convolutions, because the fp32 GEMM solution hipBLASLt
# picks varies by box in accumulation precision (one MI355X box gave a 3.4e-3 median relative
# input-gradient error on ResNet-50 NHWC against 1e-6 for the convolution path, r02h).
def _pointwise(w, geom):
    stride, padding, dilation, groups = geom
    return (w.dtype == torch.bfloat16 and w.dim() == 4 and w.shape[2] == 1 and w.shape[3] == 1 and groups == 1 and list(stride) == [1, 1]
            and list(padding) == [0, 0])


def _rows(t):
    """[N*H*W, C] view of a dense channels_last 4D tensor, or None."""
    if t.dim() != 4 or not t.is_cuda:
        return None
    v = t.permute(0, 2, 3, 1)
    return v.reshape(-1, t.shape[1]) if v.is_contiguous() else None


def _unrows(y2, like):
    n, _, h, w = like.shape
    return y2.view(n, h, w, y2.shape[1]).permute(0, 3, 1, 2)


def _addmm_relu(b, x2, w2t):
    try:
        return torch._addmm_activation(b, x2, w2t)
    except (AttributeError, RuntimeError):  # private op missing / no fused epilogue for this dtype
        return torch.relu_(torch.addmm(b, x2, w2t))


class _SkipGrad:
    """Hand-off of a residual block's skip-path gradient to the block that produced its input.

    In a ResNet identity block the input x (the previous block's AddBiasReLU output) feeds both
    conv1 and the residual add, so autograd would sum the two gradients of x in a separate
    elementwise pass before the producer's ReLU mask (8 % of the c2 step). Instead the add
    receives x detached and parks its skip gradient here, and the producer's backward, which
    autograd runs later (it is upstream of both users), applies its mask to the sum in one kernel
    (relu_mask(g, y, g2)). One box per forward call: the producer's forward opens it and the
    consumer's forward takes it, so repeated forwards before a backward stay separate. Measured:
    adding the skip gradient as the C operand of conv1's input-gradient GEMM instead gains nothing
    (torch.addmm copies C into the output first; scripts/skip_ab.py)."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None


class _SkipLink:
    """Link between a producer AddBiasReLU and the consumer AddBiasReLU that takes its output as
    the skip operand."""

    def __init__(self):
        self.cur = None


class _ConvBiasReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, geom):
        x2 = _rows(x) if _pointwise(w, geom) else None
        ctx.gemm = x2 is not None
        if ctx.gemm:
            w2 = w.reshape(w.shape[0], w.shape[1])
            y = _unrows(_addmm_relu(b.to(x.dtype), x2, w2.t()), x)
            ctx.save_for_backward(w2, y)
            return y
        y = bias_act_(_conv_nd(x, w, *geom), b, True)
        ctx.save_for_backward(x, w, y)
        ctx.geom = geom
        return y

    @staticmethod
    def backward(ctx, g):
        if ctx.gemm:
            w2, y = ctx.saved_tensors
            gm = relu_mask(g, y)
            return _unrows(torch.mm(_rows(gm), w2), y), None, None, None
        x, w, y = ctx.saved_tensors
        return _conv_grad_input(relu_mask(g, y), x, w, *ctx.geom), None, None, None


class _PointwiseConvFn(torch.autograd.Function):
    """Bias-free pointwise convolution of a channels_last activation as a GEMM."""

    @staticmethod
    def forward(ctx, x2, x, w2):
        ctx.save_for_backward(w2)
        ctx.shape = x.shape
        y = torch.mm(x2, w2.t())
        n, _, h, ww = x.shape
        return y.view(n, h, ww, w2.shape[0]).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        (w2,) = ctx.saved_tensors
        g2 = _rows(g)
        if g2 is None:
            g2 = _rows(g.contiguous(memory_format=torch.channels_last))
        n, c, h, ww = ctx.shape
        dx = torch.mm(g2, w2).view(n, h, ww, c).permute(0, 3, 1, 2)
        return None, dx, None


class _AddBiasReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, ba, s, bs, park=None, take=None):
        out = add_bias_relu(a, ba, s, bs)
        ctx.save_for_backward(out)
        ctx.park, ctx.take = park, take
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        g2 = None
        if ctx.take is not None:  # skip gradient of the consumer block, summed under the mask
            g2, ctx.take.g = ctx.take.g, None
        gm = relu_mask(g, out, g2)
        if ctx.park is not None:  # s was passed detached: its gradient goes to s's producer
            ctx.park.g = gm
            return gm, None, None, None, None, None
        return gm, None, gm, None, None, None


class _PolyphaseReLUFn(torch.autograd.Function):
    """relu(InputConv2d(x)): conv without bias + fused bias/ReLU; backward = mask + polyphase."""

    @staticmethod
    def forward(ctx, x, weight, bias, wpoly, pad, geom):
        y = bias_act_(F.conv2d(x, weight, None, 2, pad), bias, True)
        ctx.save_for_backward(wpoly, y)
        ctx.geom = geom
        ctx.in_hw = x.shape[-2:]
        return y

    @staticmethod
    def backward(ctx, go):
        wpoly, y = ctx.saved_tensors
        gm = relu_mask(go, y)

        class _C:  # reuse the polyphase backward with its saved table
            saved_tensors = (wpoly,)
            geom = ctx.geom
            in_hw = ctx.in_hw
        return _PolyphaseInputGrad.backward(_C, gm)


class _PolyphaseReLUPoolFn(torch.autograd.Function):
    """maxpool(relu(InputConv2d(x))): the pooled input is not kept -- the byte window index
    carries the ReLU mask, so the backward is one gather kernel + the polyphase convolution."""

    @staticmethod
    def forward(ctx, x, weight, bias, wpoly, pad, geom, pool):
        y = bias_act_(F.conv2d(x, weight, None, 2, pad), bias, True)
        k, s, p = pool
        ctx.geom, ctx.in_hw, ctx.pool, ctx.y_shape = geom, x.shape[-2:], pool, y.shape
        if _pool_ok(y, k, s, p):
            out, idx = maxpool_nhwc(y, k, s, p)
            ctx.save_for_backward(wpoly, idx)
            ctx.hip = True
        else:
            out, idx = F.max_pool2d(y, k, s, p, return_indices=True)
            ctx.save_for_backward(wpoly, idx, y)
            ctx.hip = False
        return out

    @staticmethod
    def backward(ctx, go):
        k, s, p = ctx.pool
        if ctx.hip:
            wpoly, idx = ctx.saved_tensors
            gm = maxpool_nhwc_backward(go, idx, ctx.y_shape, k, s, p, relu=True)
        else:
            wpoly, idx, y = ctx.saved_tensors
            gy = torch.ops.aten.max_pool2d_with_indices_backward(go, y, [k, k], [s, s], [p, p], [1, 1], False, idx)
            gm = relu_mask(gy, y)

        class _C:  # reuse the polyphase backward with its saved table
            saved_tensors = (wpoly,)
            geom = ctx.geom
            in_hw = ctx.in_hw
        return _PolyphaseInputGrad.backward(_C, gm) + (None,)


def _geom(conv):
    return (list(conv.stride), list(conv.padding), list(conv.dilation), conv.groups)


class ConvBiasReLU(nn.Module):
    """relu(conv(x)) for a frozen, zero-padded Conv1d/2d/3d with bias (one fused epilogue)."""

    def __init__(self, conv):
        super().__init__()
        self.weight = nn.Parameter(conv.weight.detach().clone(), requires_grad=False)
        b = conv.bias.detach().clone() if conv.bias is not None else torch.zeros(conv.out_channels)
        self.bias = nn.Parameter(b, requires_grad=False)
        self.geom = _geom(conv)


    def forward(self, x):
        return _ConvBiasReLUFn.apply(x, self.weight, self.bias, self.geom)


class ConvNoBias(nn.Module):
    """conv(x) with its bias moved into the consumer (AddBiasReLU)."""

    def __init__(self, conv):
        super().__init__()
        self.weight = nn.Parameter(conv.weight.detach().clone(), requires_grad=False)
        self.geom = _geom(conv)

    def forward(self, x):
        if _pointwise(self.weight, self.geom):
            x2 = _rows(x)
            if x2 is not None:
                w2 = self.weight.reshape(self.weight.shape[0], self.weight.shape[1])
                return _PointwiseConvFn.apply(x2.detach(), x, w2)
        return _conv_nd(x, self.weight, *self.geom)


class AddBiasReLU(nn.Module):
    """relu((a + bias_a) + (s + bias_s)) -- residual tail; biases may be absent."""

    def __init__(self, bias_a=None, bias_s=None):
        super().__init__()
        self.bias_a = None if bias_a is None else nn.Parameter(bias_a.detach().clone(), requires_grad=False)
        self.bias_s = None if bias_s is None else nn.Parameter(bias_s.detach().clone(), requires_grad=False)

        self.link_in = None   # _SkipLink: operand s comes from a linked producer (park its gradient)
        self.link_out = None  # _SkipLink: this output is a linked consumer's skip operand (take it)

    def _fusable(self, a, s):
        """The HIP kernel indexes s with a's flat index: same shape, dtype, layout and device only."""
        if not (a.is_cuda and s.is_cuda and a.device == s.device and a.dtype == s.dtype and a.dtype in _DT
                and a.shape == s.shape and a.dim() >= 2):
            return False
        for b in (self.bias_a, self.bias_s):
            if b is not None and (b.dim() != 1 or b.numel() != a.shape[1]):
                return False
        return True

    def forward(self, a, s):
        if not self._fusable(a, s):
            # broadcast / mixed operands (e.g. relu(x + pos_embed)): plain torch, no skip hand-off
            if self.link_out is not None:
                self.link_out.cur = None
            if self.link_in is not None:
                self.link_in.cur = None
            bias = (lambda t, b: t if b is None else t + b.to(t.dtype).view((1, -1) + (1,) * (t.dim() - 2)))
            return torch.relu(bias(a, self.bias_a) + bias(s, self.bias_s))
        park = take = None
        if self.link_in is not None and self.link_in.cur is not None and torch.is_grad_enabled():
            park, self.link_in.cur = self.link_in.cur, None
            s = s.detach()
        if self.link_out is not None:
            grad = torch.is_grad_enabled() and (a.requires_grad or s.requires_grad)
            take = self.link_out.cur = _SkipGrad() if grad else None
        return _AddBiasReLUFn.apply(a, self.bias_a, s, self.bias_s, park, take)


class InputConvReLU(nn.Module):
    """relu(InputConv2d(x)) with the fused bias/ReLU epilogue and masked polyphase backward."""

    def __init__(self, ic):
        super().__init__()
        self.ic = ic

    def forward(self, x):
        from .model_opt import _phase_geometry
        ic = self.ic
        H, W = x.shape[-2:]
        oy, Ty, _, ny = _phase_geometry(ic.kh, ic.pad[0], H)
        ox, Tx, _, nx = _phase_geometry(ic.kw, ic.pad[1], W)
        b = ic.bias if ic.bias is not None else torch.zeros(ic.weight.shape[0], dtype=ic.weight.dtype,
                                                            device=ic.weight.device)
        return _PolyphaseReLUFn.apply(x, ic.weight, b, ic.wpoly, ic.pad, ((oy, Ty, ny), (ox, Tx, nx)))


class InputConvReLUPool(InputConvReLU):
    """maxpool(relu(InputConv2d(x))) for a square, undilated, floor-mode max pool."""

    def __init__(self, ic, pool):
        super().__init__(ic)
        self.pool = pool  # (k, stride, pad)

    def forward(self, x):
        from .model_opt import _phase_geometry
        ic = self.ic
        H, W = x.shape[-2:]
        oy, Ty, _, ny = _phase_geometry(ic.kh, ic.pad[0], H)
        ox, Tx, _, nx = _phase_geometry(ic.kw, ic.pad[1], W)
        b = ic.bias if ic.bias is not None else torch.zeros(ic.weight.shape[0], dtype=ic.weight.dtype,
                                                            device=ic.weight.device)
        return _PolyphaseReLUPoolFn.apply(x, ic.weight, b, ic.wpoly, ic.pad, ((oy, Ty, ny), (ox, Tx, nx)), self.pool)


def _square(v):
    if isinstance(v, (tuple, list)):
        return v[0] if len(set(v)) == 1 else None
    return v


def _simple_pool(m):
    """(k, stride, pad) of a MaxPool2d the fused kernels implement, or None."""
    if type(m) is not nn.MaxPool2d or m.ceil_mode or m.return_indices or _square(m.dilation) != 1:
        return None
    k, s, p = _square(m.kernel_size), _square(m.stride if m.stride is not None else m.kernel_size), _square(m.padding)
    if None in (k, s, p) or 2 * p > k or k * k > 127:
        return None
    return (int(k), int(s), int(p))


# --------------------------------------------------------------------------------- graph rewrite
_RELU_FN = (F.relu, torch.relu)


def _is_relu(node, mods):
    if node.op == "call_module":
        m = mods.get(node.target)
        return type(m) is nn.ReLU
    if node.op == "call_function":
        return node.target in _RELU_FN and len(node.args) == 1
    if node.op == "call_method":
        return node.target in ("relu", "relu_") and len(node.args) == 1
    return False


def _fusable_conv(node, mods):
    if node.op != "call_module" or len(node.users) != 1:
        return None
    m = mods.get(node.target)
    if type(m) in (nn.Conv1d, nn.Conv2d, nn.Conv3d) and m.padding_mode == "zeros" and not isinstance(m.padding, str):
        return m
    return None


def fuse_elementwise(gm):
    """Rewrite a traced (BN-folded, frozen) GraphModule in place; returns it and the fusion count."""
    mods = dict(gm.named_modules())
    g = gm.graph
    count = 0
    uid = [0]

    def add_mod(prefix, m):
        uid[0] += 1
        name = "%s_wamfuse%d" % (prefix.replace(".", "_"), uid[0])
        gm.add_submodule(name, m)
        mods[name] = m
        return name

    for node in list(g.nodes):
        if not _is_relu(node, mods):
            continue
        src = node.args[0]
        if not isinstance(src, fx.Node) or len(src.users) != 1:
            continue
        conv = _fusable_conv(src, mods)
        if conv is not None:  # conv -> relu
            name = add_mod(src.target, ConvBiasReLU(conv))
            with g.inserting_before(node):
                new = g.call_module(name, (src.args[0],))
            node.replace_all_uses_with(new)
            g.erase_node(node)
            g.erase_node(src)
            count += 1
            continue
        if src.op == "call_module" and isinstance(mods.get(src.target), InputConv2d):  # input conv -> relu
            name = add_mod(src.target, InputConvReLU(mods[src.target]))
            with g.inserting_before(node):
                new = g.call_module(name, (src.args[0],))
            node.replace_all_uses_with(new)
            g.erase_node(node)
            g.erase_node(src)
            count += 1
            continue
        if src.op == "call_function" and src.target in (operator.add, torch.add) and len(src.args) == 2 \
                and not src.kwargs and all(isinstance(a, fx.Node) for a in src.args):
            operands, biases, drop = [], [], []
            for a in src.args:
                c = _fusable_conv(a, mods)
                if c is not None and c.bias is not None:
                    cname = add_mod(a.target, ConvNoBias(c))
                    with g.inserting_before(a):
                        na = g.call_module(cname, (a.args[0],))
                    operands.append(na)
                    biases.append(c.bias)
                    drop.append(a)
                else:
                    operands.append(a)
                    biases.append(None)
            name = add_mod("add_relu", AddBiasReLU(*biases))
            with g.inserting_before(node):
                new = g.call_module(name, tuple(operands))
            node.replace_all_uses_with(new)
            g.erase_node(node)
            g.erase_node(src)
            for a in drop:
                g.erase_node(a)
            count += 1
    for node in list(g.nodes):  # stem relu -> max pool
        if node.op != "call_module" or _simple_pool(mods.get(node.target)) is None:
            continue
        src = node.args[0] if node.args else None
        if not isinstance(src, fx.Node) or src.op != "call_module" or len(src.users) != 1 \
                or type(mods.get(src.target)) is not InputConvReLU:
            continue
        name = add_mod(src.target, InputConvReLUPool(mods[src.target].ic, _simple_pool(mods[node.target])))
        with g.inserting_before(node):
            new = g.call_module(name, (src.args[0],))
        node.replace_all_uses_with(new)
        g.erase_node(node)
        g.erase_node(src)
        count += 1
    _link_skip_gradients(gm, mods)
    g.lint()
    gm.recompile()
    gm.delete_all_unused_submodules()
    return gm, count


def _reaches(src, dst):
    """True when fx node dst is src or one of its (transitive) users."""
    seen, stack = set(), [src]
    while stack:
        n = stack.pop()
        if n is dst:
            return True
        if n in seen:
            continue
        seen.add(n)
        stack.extend(n.users)
    return False


def _link_skip_gradients(gm, mods):
    """Link each identity residual block's AddBiasReLU with the AddBiasReLU that produced its skip
    operand, when that output has exactly two users: the block's conv1 and the add (_SkipGrad)."""
    links = 0
    for node in gm.graph.nodes:
        if node.op != "call_module" or type(mods.get(node.target)) is not AddBiasReLU:
            continue
        users = list(node.users)
        if len(users) != 2:
            continue
        add = [u for u in users if u.op == "call_module" and type(mods.get(u.target)) is AddBiasReLU]
        if len(add) != 1 or len(add[0].args) != 2 or add[0].args[1] is not node or add[0].args[0] is node:
            continue
        # the parked gradient is only complete if autograd runs the consumer before the producer:
        # true when the producer's other user feeds the consumer's `a` operand (then the
        # consumer's backward precedes every gradient that reaches the producer through it)
        other = [u for u in users if u is not add[0]]
        if len(other) != 1 or not _reaches(other[0], add[0].args[0]):
            continue
        link = _SkipLink()
        mods[node.target].link_out = link
        mods[add[0].target].link_in = link
        links += 1
    return links
