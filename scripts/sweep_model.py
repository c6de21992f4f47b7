"""Sweep model-side settings of the c2 bench step (sample_batch, MIOpen benchmark, layout, dtype)."""
import itertools, json, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import testmodels
from wam_amd.wam_2D import WaveletAttribution2D

x = torch.tensor(np.random.RandomState(1).standard_normal((64, 3, 224, 224)).astype(np.float32)).cuda()
y = [int(v) for v in np.random.RandomState(2).randint(0, 1000, 64)]
configs = [dict(sb=4, bench=False, cl=True, dt="bf16"), dict(sb=8, bench=False, cl=True, dt="bf16"),
           dict(sb=13, bench=False, cl=True, dt="bf16"), dict(sb=4, bench=False, cl=False, dt="bf16"),
           dict(sb=4, bench=True, cl=True, dt="bf16"), dict(sb=8, bench=True, cl=True, dt="bf16"),
           dict(sb=4, bench=False, cl=False, dt="fp32"), dict(sb=4, bench=False, cl=True, dt="fp16")]
for c in configs:
    torch.backends.cudnn.benchmark = c["bench"]
    m = testmodels.resnet50(seed=0).cuda()
    if c["cl"]:
        m = m.to(memory_format=torch.channels_last)
    for p in m.parameters():
        p.requires_grad_(False)
    dt = {"bf16": torch.bfloat16, "fp32": None, "fp16": torch.float16}[c["dt"]]
    ex = WaveletAttribution2D(m, wavelet="db4", J=3, n_samples=25, noise="philox", frame="native",
                              sample_batch=c["sb"], autocast_dtype=dt, channels_last=c["cl"])
    t0 = time.perf_counter(); ex(x, y); torch.cuda.synchronize(); tw = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(3):
        ex(x, y)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / 3
    print(json.dumps(dict(c, warm_s=round(tw, 2), ms_per_step=round(t * 1e3, 1), attr_s=round(64 / t, 1))), flush=True)
    del ex, m
    torch.cuda.empty_cache()
