"""k_item_sigma (split reduction) at the c1/c2/c3/c5 shapes, from cold caches as in a WAM call: a
512 MiB buffer is rewritten between calls so the input is read from HBM (library HIP events).

usage: python scripts/kbench_sigma.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import wam_amd  # noqa: E402,F401
from wam_amd import plan as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--single-block", action="store_true")
    args = ap.parse_args()
    flush = torch.empty(128 << 20, dtype=torch.float32, device="cuda")
    for mode in ("dirty", "clean"):
        for items, n in ((1, 3 * 224 * 224), (64, 3 * 224 * 224), (256, 80000), (16, 128 ** 3)):
            x = torch.randn(items * n, device="cuda")
            P.item_sigma(x, n, n, 0.25)
            torch.cuda.synchronize()
            P.timing_drain()
            tot = 0.0
            for _ in range(args.iters):
                if mode == "dirty":
                    flush.fill_(1.0)     # 512 MiB of dirty lines to write back while x is read
                else:
                    flush.sum()          # 512 MiB read: x evicted, the caches clean
                P.timing_enable(True)
                P.item_sigma(x, n, n, 0.25)
                torch.cuda.synchronize()
                P.timing_enable(False)
                tot += sum(r[1] for r in P.timing_drain())
            us = tot / args.iters * 1e3
            print(f"sigma {'single' if args.single_block else 'split'} {mode} items={items} len={n} {us:.1f} us {items * n * 4 / us / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
