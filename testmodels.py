"""Explained models used by the tests and by ``bench.py`` (architectures only, random init).

These are the *models being explained*, not part of the WAM path: WAM treats the model as an
opaque differentiable function (``lib/wam_2D.py:114-116``). There is no network access for
pretrained weights, so every model is random-init from an explicit seed.

* ``resnet18`` / ``resnet50``: torchvision-compatible ResNet definitions (configs c1, c2, c4).
* ``TinySmooth2D``: Conv-Tanh-AvgPool-Linear, kink-free, for tight glue goldens.
* ``TinyAudio``: Conv2d-Tanh head over [N,1,T,n_mels] melspecs (1D goldens).
* ``weak_mxh64_1024`` / ``FtEx``: the config-c3 audio CNN (``src/network_architectures.py:219-272``,
  ``src/helpers.py:290-305`` architecture), random init.
* ``Voxel3D``: VoxelModel-style 3D CNN (``src/network_architectures.py:190-215``) with an
  adaptive pool so it accepts 128^3 (config c5); ``TinyVoxel`` for goldens.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------------- ResNet
def _conv3x3(i, o, s=1):
    return nn.Conv2d(i, o, 3, s, 1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inp, planes, stride=1, down=None):
        super().__init__()
        self.conv1 = _conv3x3(inp, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inp, planes, stride=1, down=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inp, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, block, planes, n, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(seed=0, num_classes=1000):
    torch.manual_seed(seed)
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes).eval()


def resnet50(seed=0, num_classes=1000):
    torch.manual_seed(seed)
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes).eval()


# ------------------------------------------------------------------------------- tiny models
def _np_init(module, seed):
    """Deterministic numpy-RandomState weights (identical on every torch build)."""
    rs = np.random.RandomState(seed)
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.tensor(rs.standard_normal(p.shape) * (1.0 / np.sqrt(max(1, p[0].numel()))),
                                 dtype=p.dtype))
    return module


class TinySmooth2D(nn.Module):
    """Conv-Tanh-AvgPool-Linear: no ReLU/max-pool kinks, so tight end-to-end parity is meaningful."""

    def __init__(self, c_in=3, n_classes=10, seed=7):
        super().__init__()
        self.conv = nn.Conv2d(c_in, 8, 5, 2, 2)
        self.conv2 = nn.Conv2d(8, 8, 3, 2, 1)
        self.fc = nn.Linear(8 * 4 * 4, n_classes)
        _np_init(self, seed)

    def forward(self, x):
        h = torch.tanh(self.conv(x))
        h = torch.tanh(self.conv2(h))
        h = F.adaptive_avg_pool2d(h, 4)
        return self.fc(torch.flatten(h, 1))


class TinySmooth2DAux(TinySmooth2D):
    """TinySmooth2D with a trainable head that forward() never uses: loss.backward() leaves its
    .grad None, and so must a sharded call (engine.param_grad_sum)."""

    def __init__(self, c_in=3, n_classes=10, seed=7):
        super().__init__(c_in, n_classes, seed)
        self.aux = nn.Linear(4, 4)


class TinyAudio(nn.Module):
    def __init__(self, n_classes=10, seed=11):
        super().__init__()
        self.conv = nn.Conv2d(1, 4, 3, 1, 1)
        self.fc = nn.Linear(4 * 4 * 4, n_classes)
        _np_init(self, seed)

    def forward(self, x):
        h = torch.tanh(self.conv(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(h, 4), 1))


class TinyVoxel(nn.Module):
    def __init__(self, n_classes=10, seed=13):
        super().__init__()
        self.conv = nn.Conv3d(1, 4, 3, 1, 1)
        self.fc = nn.Linear(4 * 2 * 2 * 2, n_classes)
        _np_init(self, seed)

    def forward(self, x):
        h = torch.tanh(self.conv(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool3d(h, 2), 1))


# ------------------------------------------------------------------------------- c3 audio CNN
def _cbr(i, o, k=3, p=1):
    return nn.Sequential(nn.Conv2d(i, o, kernel_size=k, padding=p), nn.BatchNorm2d(o), nn.ReLU())


class weak_mxh64_1024(nn.Module):
    """Architecture of ``src/network_architectures.py:219-272`` (L2I audio backbone)."""

    def __init__(self, nclass=527, glplfn=F.avg_pool2d):
        super().__init__()
        self.globalpool = glplfn
        self.layer1, self.layer2, self.layer3 = _cbr(1, 16), _cbr(16, 16), nn.MaxPool2d(2)
        self.layer4, self.layer5, self.layer6 = _cbr(16, 32), _cbr(32, 32), nn.MaxPool2d(2)
        self.layer7, self.layer8, self.layer9 = _cbr(32, 64), _cbr(64, 64), nn.MaxPool2d(2)
        self.layer10, self.layer11, self.layer12 = _cbr(64, 128), _cbr(128, 128), nn.MaxPool2d(2)
        self.layer13, self.layer14, self.layer15 = _cbr(128, 256), _cbr(256, 256), nn.MaxPool2d(2)
        self.layer16, self.layer17 = _cbr(256, 512), nn.MaxPool2d(2)
        self.layer18 = _cbr(512, 1024, k=2, p=0)
        self.layer19 = nn.Sequential(nn.Conv2d(1024, nclass, kernel_size=1), nn.Sigmoid())

    def forward(self, x):
        out = self.layer3(self.layer2(self.layer1(x)))
        out = self.layer6(self.layer5(self.layer4(out)))
        out = self.layer9(self.layer8(self.layer7(out)))
        out0 = self.layer11(self.layer10(out))
        out = self.layer12(out0)
        out1 = self.layer14(self.layer13(out))
        out = self.layer15(out1)
        out2 = self.layer16(out)
        out3 = self.layer18(self.layer17(out2))
        out = self.layer19(out3)
        out = self.globalpool(out, kernel_size=out.size()[2:])
        return out.view(out.size(0), -1), [out3, out2, out1, out0]


class FtEx(nn.Module):
    """``src/helpers.py:290-305``: weak_mxh64_1024 backbone + 1x1 conv head on its layer-18 map."""

    def __init__(self, n_classes=50, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.netx = weak_mxh64_1024(527, F.avg_pool2d)
        self.layer = nn.Sequential(nn.Conv2d(1024, 256, kernel_size=1), nn.ReLU())
        self.fc = nn.Linear(256, n_classes, bias=True)
        self.reg = nn.Dropout(0.2)
        self.eval()

    def forward(self, inp):
        _, inter = self.netx(inp)
        out = self.layer(inter[0])
        out = torch.flatten(F.avg_pool2d(out, kernel_size=out.shape[2:]), 1)
        return self.fc(self.reg(out))


class Voxel3D(nn.Module):
    """VoxelModel (``src/network_architectures.py:190-215``) with AdaptiveAvgPool3d(2) before the
    Linear(1024, 256) so it accepts 128^3 volumes (the reference model is 16^3-only)."""

    def __init__(self, n_out_classes=10, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.model = nn.Sequential(
            nn.Conv3d(1, 32, kernel_size=3), nn.ReLU(), nn.Dropout(0.3), nn.MaxPool3d(2),
            nn.Conv3d(32, 128, kernel_size=3), nn.ReLU(), nn.Dropout(0.3), nn.MaxPool3d(2),
            nn.AdaptiveAvgPool3d(2), nn.Flatten(),
            nn.Linear(1024, 256), nn.ReLU(), nn.Dropout(0.3), nn.Linear(256, n_out_classes))
        self.eval()

    def forward(self, x):
        return self.model(x)


# ------------------------------------------------------------------------------- config inputs
def audio_clips(n, length=80000, sr=16000, seed=3):
    """SURVEY 8(d) c3 input: 3 random sinusoids (50-4000 Hz) + 0.1 N(0,1), peak-normalised."""
    rs = np.random.RandomState(seed)
    t = np.arange(length) / sr
    out = np.empty((n, length), dtype=np.float32)
    for i in range(n):
        f = rs.uniform(50, 4000, 3)
        a = rs.uniform(0.2, 1.0, 3)
        w = (a[:, None] * np.sin(2 * np.pi * f[:, None] * t[None])).sum(0) + 0.1 * rs.standard_normal(length)
        out[i] = (w / np.abs(w).max()).astype(np.float32)
    return torch.tensor(out)


def voxel_volumes(n, size=128, seed=5):
    """SURVEY 8(d) c5 input: Gaussian-smoothed N(0,1) thresholded to {0, 1}."""
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(n, 1, size, size, size, generator=g)
    k = torch.tensor([0.25, 0.5, 0.25])
    for ax in (2, 3, 4):
        shape = [1, 1, 1, 1, 1]
        shape[ax] = 3
        v = torch.nn.functional.conv3d(v, k.view(shape), padding=[1 if a == ax else 0 for a in (2, 3, 4)])
    return (v > 0).float()
