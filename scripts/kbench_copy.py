"""The library's k_copy over a 2 GiB fp32 buffer (the copy ceiling the bench reports), HIP events.
usage: python scripts/kbench_copy.py [--iters 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = 2 << 30
    x = torch.empty(n // 4, device="cuda").uniform_()
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.lib.wam_copy(n, x.data_ptr(), y.data_ptr(), st)  # noqa: E731
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    assert torch.equal(x, y)
    print("k_copy 2 GiB: %.1f us, %.0f GB/s (read + write)" % (ms * 1e3, 2 * n / ms / 1e6))


if __name__ == "__main__":
    main()
