"""Model-side probe for the c2 step: ResNet-50 forward + input-gradient backward per image under
different execution settings (batch, autocast vs bf16 weights, NHWC, BN folded, HIP graph)."""
import copy, json, os, sys, time
import torch
import torch.nn as nn
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels


def fold_bn(model):
    m = copy.deepcopy(model)
    def rec(mod):
        names = list(mod._modules.keys())
        for i, n in enumerate(names):
            c = mod._modules[n]
            if isinstance(c, nn.Conv2d) and i + 1 < len(names) and isinstance(mod._modules[names[i + 1]], nn.BatchNorm2d):
                bn = mod._modules[names[i + 1]]
                s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
                c.weight.data = c.weight.data * s[:, None, None, None]
                b = bn.bias - bn.running_mean * s
                c.bias = nn.Parameter(b.detach().clone())
                mod._modules[names[i + 1]] = nn.Identity()
            elif c is not None:
                rec(c)
    rec(m)
    return m


def run(tag, model, batch, dtype, cl, autocast, graph=False, iters=6):
    dev = "cuda"
    x = torch.randn(batch, 3, 224, 224, device=dev)
    go = torch.zeros(batch, 1000, device=dev, dtype=dtype if not autocast else torch.bfloat16)
    go[:, 3] = 1.0 / batch
    def step(xin):
        xi = xin.detach().requires_grad_(True)
        inp = xi.to(dtype) if not autocast else xi
        if cl:
            inp = inp.contiguous(memory_format=torch.channels_last)
        if autocast:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(inp)
        else:
            out = model(inp)
        (g,) = torch.autograd.grad(out, xi, grad_outputs=go.to(out.dtype))
        return g
    for _ in range(2):
        step(x)
    torch.cuda.synchronize()
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gout = step(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            g.replay()
        torch.cuda.synchronize()
    else:
        t0 = time.perf_counter()
        for _ in range(iters):
            step(x)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    print(json.dumps({"tag": tag, "batch": batch, "ms": round(dt * 1e3, 2), "img_per_s": round(batch / dt, 1),
                      "us_per_img": round(dt / batch * 1e6, 2)}), flush=True)


def main():
    base = testmodels.resnet50(seed=0).cuda().eval()
    for p in base.parameters():
        p.requires_grad_(False)
    bf = copy.deepcopy(base).to(torch.bfloat16)
    fb = fold_bn(base).to(torch.bfloat16)
    for p in list(bf.parameters()) + list(fb.parameters()):
        p.requires_grad_(False)
    bf_cl = copy.deepcopy(bf).to(memory_format=torch.channels_last)
    fb_cl = copy.deepcopy(fb).to(memory_format=torch.channels_last)
    for b in (256, 512):
        run("autocast", base, b, torch.float32, False, True)
        run("bf16w", bf, b, torch.bfloat16, False, False)
        run("bf16w_cl", bf_cl, b, torch.bfloat16, True, False)
        run("foldbn_bf16w", fb, b, torch.bfloat16, False, False)
        run("foldbn_bf16w_cl", fb_cl, b, torch.bfloat16, True, False)
    run("bf16w_graph", bf, 256, torch.bfloat16, False, False, graph=True)
    run("foldbn_graph", fb, 256, torch.bfloat16, False, False, graph=True)
    run("bf16w", bf, 1024, torch.bfloat16, False, False)


if __name__ == "__main__":
    main()
