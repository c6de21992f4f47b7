"""Per-kernel busy time over the last WINDOW ms of a rocprofv3 kernel trace (steady-state step).
usage: python scripts/trace_window.py <bench_kernel_trace.csv> [window_ms] [out_stats.csv]
out_stats.csv: rocprofv3-style per-kernel stats (Calls, TotalDurationNs, AverageNs, ...) of the
window only -- the whole-run kernel_stats.csv also holds the warm-up, where the first call of the
folded model makes MIOpen search its convolution solvers (naive_conv_* dominates that file)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 130.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
end = int(rows[-1]["End_Timestamp"])
sel = [r for r in rows if int(r["Start_Timestamp"]) >= end - int(win * 1e6)]
agg = collections.defaultdict(lambda: [0, 0])
for r in sel:
    agg[r["Kernel_Name"]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r["Kernel_Name"]][1] += 1
tot = sum(v[0] for v in agg.values())
print("busy %.2f ms of a %.0f ms window, %d kernels" % (tot / 1e6, win, len(sel)))
for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
    print("%7.2fms %5.1f%% n=%4d %s" % (d / 1e6, 100.0 * d / tot, c, n[:110]))
if len(sys.argv) > 3:
    per = collections.defaultdict(list)
    for r in sel:
        per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / max(1, tot), min(d), max(d)])

