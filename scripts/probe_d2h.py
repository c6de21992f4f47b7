"""Host time of returning a device result as numpy (the classes' return path, lib/wam_2D.py returns
numpy arrays): pageable .cpu().numpy() against a copy into torch's caching pinned-host allocator,
for the c2 (64 x 224^2 float64) and c4 (128 x 512^2 float64) attribution shapes; the previous
result is dropped before each call, as in the bench loop.
usage: python scripts/probe_d2h.py"""
import time

import torch


def pinned_numpy(t):
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def main():
    for shape in ((64, 224, 224), (128, 512, 512)):
        x = torch.rand(shape, dtype=torch.float64, device="cuda")
        for name, fn in (("pageable .cpu().numpy()", lambda: x.cpu().numpy()), ("pinned (caching host allocator)", lambda: pinned_numpy(x))):
            out = None
            ts = []
            for i in range(12):
                torch.cuda.synchronize()
                out = None
                t0 = time.perf_counter()
                out = fn()
                ts.append(time.perf_counter() - t0)
            ts = sorted(ts[2:])
            assert float(out[0, 0, 0]) == float(x[0, 0, 0])
            print("%-16s %-32s median %.3f ms  min %.3f ms" % (str(shape), name, ts[len(ts) // 2] * 1e3, ts[0] * 1e3))


if __name__ == "__main__":
    main()
