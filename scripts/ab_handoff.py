"""Same-process A/B of the c2 model hand-off: the bf16 NHWC hand-off
(bf16_handoff=True: k_plane_syn writes the model input as bf16 NHWC, the maps pass reads the model's
bf16 gradient) against the fp32 hand-off (cast / layout passes) on one box, in one process,
alternating rounds so that the bf16 model's run-to-run drift hits both sides alike. (A third arm,
the hand-off maps of model group k on a side stream beside group k+1's model pass, measured no gain
and was removed: profiles/r06g_ab_handoff.log.)

usage: python scripts/ab_handoff.py [--rounds 6] [--steps 5]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = bench.workload("c2")
    x, y = wl.make_x().to(dev), wl.make_y()
    exs = {}
    for tag, off in (("bf16_handoff", False), ("fp32_handoff", True)):
        args = bench.parse(["--config", "c2"] + (["--no-bf16-handoff"] if off else []))
        exs[tag] = bench.build_explainer(wl, dev, args, n_local=wl.n)
        for _ in range(2):
            exs[tag](x, y)
    torch.cuda.synchronize()
    res = {k: [] for k in exs}
    for r in range(a.rounds):
        for tag, ex in (exs.items() if r % 2 == 0 else reversed(list(exs.items()))):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ex(x, y)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            res[tag].append(ms)
            print("round %d %-15s %8.2f ms per step" % (r, tag, ms), flush=True)
    for tag, v in res.items():
        v = sorted(v)
        print("%-15s median %.2f  min %.2f  max %.2f ms per step" % (tag, v[len(v) // 2], v[0], v[-1]))


if __name__ == "__main__":
    main()
