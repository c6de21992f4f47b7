"""1x1 convolutions of the c2 ResNet-50 (NHWC bf16, batch 832) as MIOpen convs vs hipBLASLt GEMMs
(torch.mm / torch._addmm_activation on the [N*H*W, C] view): forward with bias+ReLU, and the
input-gradient. usage: python scripts/gemm_probe.py"""
import json
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = "cuda"
B = 832
shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (14, 1024, 256),
          (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]


def timeit(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for hw, cin, cout in shapes:
    x = torch.randn(B, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05
    w = w.contiguous(memory_format=torch.channels_last)
    b = torch.randn(cout, device=dev, dtype=torch.bfloat16)
    g = torch.randn(B, cout, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w2 = w.view(cout, cin)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
    g2 = g.permute(0, 2, 3, 1).reshape(-1, cout)
    r = {"hw": hw, "cin": cin, "cout": cout}
    r["miopen_fwd_relu"] = timeit(lambda: torch.relu_(F.conv2d(x, w, b)))
    r["mm_fwd_relu"] = timeit(lambda: torch.relu_(torch.addmm(b, x2, w2.t())))
    try:
        r["addmm_act"] = timeit(lambda: torch._addmm_activation(b, x2, w2.t()))
    except Exception as e:  # noqa
        r["addmm_act"] = str(e)[:80]
    r["miopen_bwd_data"] = timeit(lambda: torch.ops.aten.convolution_backward(
        g, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0])
    r["mm_bwd_data"] = timeit(lambda: torch.mm(g2, w2))
    yref = F.conv2d(x, w, b).permute(0, 2, 3, 1).reshape(-1, cout).float()
    r["maxdiff_fwd"] = float((torch.addmm(b, x2, w2.t()).float() - yref).abs().max())
    gb = (x.numel() + g.numel()) * 2 / 1e9
    r["GB"] = round(gb, 3)
    print(json.dumps(r), flush=True)
