"""Idle time of the GPU over the last WINDOW ms of a rocprofv3 kernel trace: the union of kernel
intervals against the window, and the largest gaps with the kernels either side of them.
usage: python scripts/trace_gaps.py <kernel_trace.csv> [window_ms] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
end = max(e for _, e, _ in iv)
t0 = end - int(win * 1e6)
iv = [x for x in iv if x[1] > t0]
gaps, cur_end, prev = [], t0, "(window start)"
for s, e, n in iv:
    if s > cur_end:
        gaps.append((s - cur_end, prev, n))
    if e > cur_end:
        cur_end, prev = e, n
idle = sum(g[0] for g in gaps)
print("window %.0f ms: GPU idle %.2f ms in %d gaps (%.2f ms in gaps > 20 us)" % (
    win, idle / 1e6, len(gaps), sum(g[0] for g in gaps if g[0] > 20000) / 1e6))
for g, a, b in sorted(gaps, reverse=True)[:top]:
    print("%8.1f us  after %-60s before %s" % (g / 1e3, a[:60], b[:60]))
# the kernel sequence around a call boundary (after the window's first k_reproject: the end of one
# explainer call and the start of the next), with the idle time before each kernel
idx = next((i for i, x in enumerate(iv) if "k_reproject" in x[2]), None)
if idx is not None:
    print("\nsequence after the first k_reproject of the window (idle before, duration, kernel):")
    prev_end = iv[idx][1]
    for s, e, n in iv[idx:idx + 45]:
        print("%8.1f us idle %8.1f us  %s" % (max(0, s - prev_end) / 1e3, (e - s) / 1e3, n[:90]))
        prev_end = max(prev_end, e)
