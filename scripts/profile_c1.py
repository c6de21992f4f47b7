"""Host-side profile of one bench call (default c1: 1 image, haar J=3, 25 numpy-noise samples,
ResNet-18 fp32): cProfile's top entries by cumulative and by own time, after two warm-up calls.
usage: python scripts/profile_c1.py [config]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
wl = bench.workload(cfg)
args = bench.parse([])
dev = torch.device("cuda", 0)
ex = bench.build_explainer(wl, dev, args)
x = wl.make_x()
y = wl.make_y() if wl.make_y else None
if y is None:
    with torch.no_grad():
        y = int(wl.model()(x).argmax().item())
xd = x.to(dev)
for _ in range(2):
    ex(xd, y)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    ex(xd, y)
torch.cuda.synchronize()
print("mean call %.1f ms" % ((time.perf_counter() - t) / 3 * 1e3))
pr = cProfile.Profile()
pr.enable()
ex(xd, y)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
