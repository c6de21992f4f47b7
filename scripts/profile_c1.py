"""Host-side profile of one c1 call (1 image, haar J=3, 25 numpy-noise samples, ResNet-18 fp32):
cProfile's top entries by cumulative time, after two warm-up calls."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

wl = bench.workload("c1")
args = bench.parse([])
dev = torch.device("cuda", 0)
ex = bench.build_explainer(wl, dev, args)
x = wl.make_x()
with torch.no_grad():
    y = int(wl.model()(x).argmax().item())
xd = x.to(dev)
for _ in range(2):
    ex(xd, y)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5):
    ex(xd, y)
torch.cuda.synchronize()
print("mean call %.1f ms" % ((time.perf_counter() - t) / 5 * 1e3))
pr = cProfile.Profile()
pr.enable()
ex(xd, y)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
