"""Input-gradient execution of the explained model.

WAM only needs d loss / d input of the explained model (lib/wam_2D.py:114-116: forward, diag-mean
loss, backward). For an eval-mode model that is the gradient of a fixed function, so the model
may be run in any form that computes the same function. ``optimize_for_input_grad`` builds such a
form once per explainer (opt-in, build-only keyword ``optimize_model=True`` of the WAM classes):

* eval-mode BatchNorm folded into the preceding convolution (BN in eval mode is a per-channel
  affine map, so conv∘BN is one convolution with scaled weights and a bias). This removes the BN
  forward and the BN backward elementwise kernels -- about a quarter of a ResNet-50 input-gradient
  pass on MI355X (profiles/r01e_model_probe.log).
* the input convolution (a stride-2 Conv2d reading the model input, e.g. the ResNet 7x7 stem)
  gets a polyphase input-gradient: its transposed convolution is rewritten as ONE stride-1
  convolution of the output gradient with 4·C_in output channels (one per input channel and
  output phase) followed by a pixel shuffle. MIOpen's backward-data path for a 3-channel input
  is a per-image GEMM + col2im loop (≈11 % of the c2 step, profiles/r01c_kernel_stats.csv).
* parameters detached from autograd (only the input gradient is computed) and cast once to
  ``dtype`` (e.g. bf16) instead of being cast by autocast on every call.

The function is the model's up to floating-point rounding (folding reassociates one multiply);
tests/test_model_opt.py checks outputs and input gradients against the original model.
Models that torch.fx cannot trace, or that are in training mode, are rejected with an error.
"""
import copy

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

_BN = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d)
_CONV = (nn.Conv1d, nn.Conv2d, nn.Conv3d)


def _fold_conv_bn(conv, bn):
    """conv followed by eval-mode bn -> one conv (weights scaled per output channel, bias added)."""
    fused = copy.deepcopy(conv)
    with torch.no_grad():
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps) if bn.affine else \
            1.0 / torch.sqrt(bn.running_var + bn.eps)
        shift = bn.bias if bn.affine else torch.zeros_like(bn.running_mean)
        w = conv.weight * scale.reshape((-1,) + (1,) * (conv.weight.dim() - 1))
        b0 = conv.bias if conv.bias is not None else torch.zeros_like(bn.running_mean)
        fused.weight = nn.Parameter(w.detach().clone())
        fused.bias = nn.Parameter(((b0 - bn.running_mean) * scale + shift).detach().clone())
    return fused


# ------------------------------------------------------------------------------ polyphase stem
def _phase_geometry(k, p, n_in):
    """1D geometry of the input gradient of a stride-2 correlation with k taps and padding p:
    gx[2Y + r] = sum_t Wp[r, t] * go[Y + o + t], t in [0, T). Returns (o, T, taps[r][t] = kernel
    tap or -1, n_half = number of Y)."""
    cs, ms, qs = [], [], []
    for r in (0, 1):
        q = (r + p) % 2                  # parity of the kernel taps that reach phase r
        c = (r + p - q) // 2             # go index offset of tap m = 0
        m = (k - q + 1) // 2             # number of such taps
        cs.append(c), ms.append(m), qs.append(q)
    o = min(cs[r] - ms[r] + 1 for r in (0, 1))
    T = max(cs) - o + 1
    taps = [[-1] * T for _ in (0, 1)]
    for r in (0, 1):
        for t in range(T):
            m = cs[r] - o - t
            if 0 <= m < ms[r]:
                taps[r][t] = 2 * m + qs[r]
    return o, T, taps, (n_in + 1) // 2


class _PolyphaseInputGrad(torch.autograd.Function):
    """y = conv2d(x, W, b, stride 2, padding p); dx by one stride-1 conv + pixel shuffle."""

    @staticmethod
    def forward(ctx, x, weight, bias, wpoly, pad, geom):
        ctx.save_for_backward(wpoly)
        ctx.geom = geom
        ctx.in_hw = x.shape[-2:]
        return F.conv2d(x, weight, bias, 2, pad)

    @staticmethod
    def backward(ctx, go):
        (wpoly,) = ctx.saved_tensors
        (oy, Ty, ny), (ox, Tx, nx) = ctx.geom
        H, W = ctx.in_hw
        # go_ext[Y + o + t]: pad before by -o, after so that Y covers [0, n)
        py0, px0 = -oy, -ox
        py1 = (ny - 1 + oy + Ty - 1) - (go.shape[-2] - 1)
        px1 = (nx - 1 + ox + Tx - 1) - (go.shape[-1] - 1)
        c4 = wpoly.shape[0]
        wp = wpoly.to(go.dtype)
        if c4 % 16:  # MIOpen picks a far better solver for 16 output channels than for 12 (3.1 vs
            # 4.3 ms per c2 model call, scripts/stem_probe.py); the zero channels are cropped
            wp = F.pad(wp, (0, 0, 0, 0, 0, 0, 0, 16 - c4 % 16))
        if min(py0, py1, px0, px1) >= 0:
            # the convolution's own (symmetric) zero padding and a crop of the surplus rows /
            # columns instead of an F.pad copy: 5.8 -> 4.3 ms per c2 model call, bit-identical
            # (scripts/stem_probe.py)
            P, Q = max(py0, py1), max(px0, px1)
            go_ = F.conv2d(go, wp, padding=(P, Q))
            go_ = go_[:, :c4, P - py0:P - py0 + ny, Q - px0:Q - px0 + nx]
        else:
            go_ = F.conv2d(F.pad(go, (px0, px1, py0, py1)), wp)[:, :c4]
        gx = F.pixel_shuffle(go_, 2)
        return gx[..., :H, :W], None, None, None, None, None


class InputConv2d(nn.Module):
    """Drop-in for a stride-2, zero-padded, ungrouped Conv2d on the model input (frozen weights)."""

    def __init__(self, conv, in_hw=None):
        super().__init__()
        kh, kw = conv.kernel_size
        ph, pw = conv.padding
        self.pad = (ph, pw)
        self.weight = nn.Parameter(conv.weight.detach().clone(), requires_grad=False)
        self.bias = None if conv.bias is None else nn.Parameter(conv.bias.detach().clone(), requires_grad=False)
        self.kh, self.kw, self.cin = kh, kw, conv.in_channels
        self.register_buffer("wpoly", self._poly(self.weight.detach()), persistent=False)

    def _poly(self, w):
        oy, Ty, tay, _ = _phase_geometry(self.kh, self.pad[0], 2)
        ox, Tx, tax, _ = _phase_geometry(self.kw, self.pad[1], 2)
        cout, cin = w.shape[:2]
        wp = torch.zeros(cin * 4, cout, Ty, Tx, dtype=w.dtype, device=w.device)
        for ry in (0, 1):
            for rx in (0, 1):
                for ty in range(Ty):
                    ky = tay[ry][ty]
                    if ky < 0:
                        continue
                    for tx in range(Tx):
                        kx = tax[rx][tx]
                        if kx < 0:
                            continue
                        # pixel_shuffle: channel c * 4 + ry * 2 + rx -> out[c, 2Y + ry, 2X + rx]
                        wp[ry * 2 + rx::4, :, ty, tx] = w[:, :, ky, kx].t()
        return wp

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        self.wpoly = self._poly(self.weight.detach())  # keep the polyphase table in the weights' dtype/device
        return self

    def forward(self, x):
        H, W = x.shape[-2:]
        oy, Ty, _, ny = _phase_geometry(self.kh, self.pad[0], H)
        ox, Tx, _, nx = _phase_geometry(self.kw, self.pad[1], W)
        return _PolyphaseInputGrad.apply(x, self.weight, self.bias, self.wpoly, self.pad,
                                         ((oy, Ty, ny), (ox, Tx, nx)))


def _input_conv_ok(m):
    return (type(m) is nn.Conv2d and m.stride == (2, 2) and m.dilation == (1, 1) and m.groups == 1
            and m.padding_mode == "zeros" and isinstance(m.padding, tuple))


def _set_module(root, target, new):
    parent, _, name = target.rpartition(".")
    setattr(root.get_submodule(parent) if parent else root, name, new)


def optimize_for_input_grad(model, dtype=None, fold_bn=True, input_conv=True, fuse=None):
    """A traced, frozen copy of an eval-mode `model` computing the same function (see module doc).
    fuse: rewrite conv/bias/ReLU/residual chains into the fused HIP epilogues (model_fuse.py);
    None = when the model lives on the GPU (and WAM_MODEL_FUSE is not 0)."""
    if model.training:
        raise ValueError("optimize_for_input_grad needs an eval-mode model (BatchNorm folding uses running stats)")
    try:
        gm = fx.symbolic_trace(copy.deepcopy(model))
    except Exception as e:  # dynamic control flow etc.
        raise ValueError("optimize_for_input_grad: torch.fx cannot trace this model (%s); "
                         "construct the explainer with optimize_model=False" % e) from e
    mods = dict(gm.named_modules())
    if fold_bn:
        for node in list(gm.graph.nodes):
            if node.op != "call_module" or not isinstance(mods.get(node.target), _BN):
                continue
            src = node.args[0]
            if not (isinstance(src, fx.Node) and src.op == "call_module" and isinstance(mods.get(src.target), _CONV)):
                continue
            bn, conv = mods[node.target], mods[src.target]
            if len(src.users) > 1 or not bn.track_running_stats or bn.running_mean is None:
                continue
            if conv.weight.dim() - 2 != {nn.BatchNorm1d: 1, nn.BatchNorm2d: 2, nn.BatchNorm3d: 3}[type(bn)]:
                continue
            fused = _fold_conv_bn(conv, bn)
            _set_module(gm, src.target, fused)
            mods[src.target] = fused
            node.replace_all_uses_with(src)
            gm.graph.erase_node(node)
    if input_conv:
        inputs = [n for n in gm.graph.nodes if n.op == "placeholder"]
        if inputs:
            for user in list(inputs[0].users):
                if user.op == "call_module" and _input_conv_ok(mods.get(user.target)):
                    new = InputConv2d(mods[user.target])
                    _set_module(gm, user.target, new)
                    mods[user.target] = new
    gm.graph.lint()
    gm.recompile()
    gm.delete_all_unused_submodules()
    if fuse is None:
        import os
        dev = next((p.device for p in gm.parameters()), torch.device("cpu"))
        fuse = dev.type == "cuda" and os.environ.get("WAM_MODEL_FUSE", "1") != "0"
    if fuse:
        from .model_fuse import fuse_elementwise
        gm, _ = fuse_elementwise(gm)
    gm.eval()
    if dtype is not None:
        gm = gm.to(dtype)
    for p in gm.parameters():
        p.requires_grad_(False)
    return gm
