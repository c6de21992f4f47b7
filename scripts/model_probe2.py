"""Model-side probe 2: the input-gradient pass of ResNet-50 run as is (autocast) vs through
wam_amd.model_opt (BN folded, polyphase input conv, bf16 weights), NCHW / NHWC, and the c2
bench step at several sample_batch values with optimize_model on."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels  # noqa: E402
from wam_amd.model_opt import optimize_for_input_grad  # noqa: E402
from wam_amd.engine import input_gradient  # noqa: E402


def timeit(fn, iters=6):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    base = testmodels.resnet50(seed=0).cuda().eval()
    for p in base.parameters():
        p.requires_grad_(False)
    y = [int(v) for v in np.random.RandomState(2).randint(0, 1000, 64)]
    variants = {
        "autocast": (base, torch.bfloat16, None, False),
        "opt_bf16": (optimize_for_input_grad(base, dtype=torch.bfloat16), None, torch.bfloat16, False),
        "opt_bf16_nostem": (optimize_for_input_grad(base, dtype=torch.bfloat16, input_conv=False), None,
                            torch.bfloat16, False),
        "opt_bf16_cl": (optimize_for_input_grad(base, dtype=torch.bfloat16).to(memory_format=torch.channels_last),
                        None, torch.bfloat16, True),
    }
    for batch in (256, 320):
        x = torch.randn(batch, 3, 224, 224, device="cuda")
        for tag, (m, ac, idt, cl) in variants.items():
            dt = timeit(lambda: input_gradient(m, x, y, batch // 64, 64, ac, cl, input_dtype=idt))
            print(json.dumps({"tag": tag, "batch": batch, "ms": round(dt * 1e3, 2),
                              "us_per_img": round(dt / batch * 1e6, 2)}), flush=True)
    # stem input-gradient alone: MIOpen backward-data vs polyphase
    conv = base.conv1.to(torch.bfloat16)
    from wam_amd.model_opt import InputConv2d
    ic = InputConv2d(conv).cuda().to(torch.bfloat16)
    x = torch.randn(256, 3, 224, 224, device="cuda", dtype=torch.bfloat16)
    go = torch.randn(256, 64, 112, 112, device="cuda", dtype=torch.bfloat16)
    for tag, mod in (("stem_miopen", conv), ("stem_polyphase", ic)):
        def f():
            xi = x.detach().requires_grad_(True)
            (g,) = torch.autograd.grad(mod(xi), xi, go)
            return g
        dt = timeit(f)
        print(json.dumps({"tag": tag, "batch": 256, "ms": round(dt * 1e3, 3)}), flush=True)

    from wam_amd.wam_2D import WaveletAttribution2D
    xb = torch.tensor(np.random.RandomState(1).standard_normal((64, 3, 224, 224)).astype(np.float32)).cuda()
    for sb in (4, 5, 9, 13, 25):
        ex = WaveletAttribution2D(base, wavelet="db4", J=3, n_samples=25, noise="philox", frame="native",
                                  sample_batch=sb, autocast_dtype=torch.bfloat16, optimize_model=True)
        dt = timeit(lambda: ex(xb, y), iters=3)
        print(json.dumps({"tag": "c2_step_opt", "sample_batch": sb, "ms_per_step": round(dt * 1e3, 1),
                          "attr_s": round(64 / dt, 1)}), flush=True)
        del ex
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
