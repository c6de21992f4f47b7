"""Summarise SQ counter passes (rocprofv3 --pmc counter_collection.csv files) per kernel name:
mean per dispatch of every counter, plus derived per-wave and per-SIMD rates.

usage: python scripts/pmc_sq.py <dir with p*/.../*counter_collection.csv>
"""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            m = re.search(r"(k_\w+(<[^(]*>)?)\(", row["Kernel_Name"])
            k = m.group(1) if m else row["Kernel_Name"][:60]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
