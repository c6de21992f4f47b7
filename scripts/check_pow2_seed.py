"""GPU check of the power-of-two loss seed (engine.seed_gradient): the bench's c2 model (ResNet-50,
BN-folded bf16 copy, channels_last) input gradient with the scale seeded directly vs the unit seed
then the fp32 scale. Prints the max |difference| and the count of differing elements; runs each
form twice to show the run-to-run spread of the model's own kernels."""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from wam_amd import engine  # noqa: E402
import testmodels  # noqa: E402

torch.manual_seed(0)
m = testmodels.resnet50(seed=0).cuda().eval().to(memory_format=torch.channels_last)
for p in m.parameters():
    p.requires_grad_(False)
gm = engine.GradModel(m, torch.bfloat16, True, True)
x = torch.randn(64, 3, 224, 224, device="cuda")
y = list(range(64))
outs = {}
for form in ("pow2", "unit", "pow2b", "unitb"):
    if form.startswith("unit"):
        orig = math.frexp
        math.frexp = lambda v: (0.75, 0)  # force the unit-seed branch
        try:
            g = gm(x, y, 1, 64)
        finally:
            math.frexp = orig
    else:
        g = gm(x, y, 1, 64)
    torch.cuda.synchronize()
    outs[form] = g.clone()
for a, b in (("pow2", "unit"), ("pow2", "pow2b"), ("unit", "unitb")):
    d = (outs[a] - outs[b]).abs()
    print(a, "vs", b, "max|diff| %.3e" % d.max().item(), "differing", int((d > 0).sum()), "of", d.numel(),
          "max|g| %.3e" % outs[a].abs().max().item())
