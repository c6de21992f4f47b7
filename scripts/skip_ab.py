"""A/B in one process: fused ResNet-50 input-gradient step (bf16, channels_last, c2 model batch)
with and without the skip-gradient hand-off to the producing block's ReLU mask (model_fuse._SkipGrad)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels  # noqa: E402
from wam_amd.model_opt import optimize_for_input_grad  # noqa: E402


def main(batch=832, iters=6):
    m = testmodels.resnet50(seed=0).cuda().eval()
    fus = optimize_for_input_grad(m, dtype=torch.bfloat16, fuse=True).to(memory_format=torch.channels_last)
    linked = [q for q in fus.modules() if getattr(q, "link_in", None) is not None
              or getattr(q, "link_out", None) is not None]
    links = [(q.link_in, q.link_out) for q in linked]
    x = torch.randn(batch, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda")

    def step():
        xx = x.detach().requires_grad_(True)
        o = fus(xx)
        (g,) = torch.autograd.grad(o.gather(1, y[:, None]).float().sum(), xx)
        return g

    def set_links(on):
        for q, (li, lo) in zip(linked, links):
            q.link_in, q.link_out = (li, lo) if on else (None, None)

    res = {True: [], False: []}
    for on in (True, False):
        set_links(on)
        for _ in range(2):
            step()
    torch.cuda.synchronize()
    for it in range(iters):
        for on in (True, False):
            set_links(on)
            torch.cuda.synchronize()
            t = time.perf_counter()
            step()
            torch.cuda.synchronize()
            res[on].append((time.perf_counter() - t) * 1e3)
    set_links(True)
    g1 = step()
    set_links(False)
    g0 = step()
    d = ((g1.float() - g0.float()).norm() / g0.float().norm()).item()
    for on in (True, False):
        v = sorted(res[on])
        print("skip hand-off %-5s: median %.2f ms  min %.2f ms  (%d linked modules)" % (on, v[len(v) // 2], v[0], len(linked)))
    print("rel diff of input gradients linked vs unlinked: %.3e" % d)


if __name__ == "__main__":
    main()
