"""Per-kernel mean of every PMC counter found in the rocprofv3 counter_collection.csv files under a
directory (one pass per subdirectory, as scripts/pmc_probe.sh writes them).

usage: python scripts/pmc_table.py gpurun_out/pmcp [more dirs...]
SQ_* wave/cycle counters are summed over the dispatch by rocprofv3; ratios printed:
  valu_busy  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of wave time issuing VALU)
  wait_any   = SQ_WAIT_ANY / SQ_WAVE_CYCLES            (parked on s_waitcnt / barrier)
  wait_inst  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES       (issue stalls)
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"]) or row["Kernel_Name"][:40]
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    for d in sys.argv[1:]:
        print("==", d)
        for k, cs in sorted(load(d).items()):
            m = {c: sum(v) / len(v) for c, v in cs.items()}
            print("  %s" % k)
            for c in sorted(m):
                print("    %-28s %16.1f" % (c, m[c]))
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                for lab, c in (("valu_busy", "SQ_ACTIVE_INST_VALU"), ("wait_any", "SQ_WAIT_ANY"),
                               ("wait_inst", "SQ_WAIT_INST_ANY"), ("active_any", "SQ_ACTIVE_INST_ANY"),
                               ("lds_busy", "SQ_ACTIVE_INST_LDS")):
                    if c in m:
                        print("    %-28s %16.3f" % (lab, m[c] / wc))


if __name__ == "__main__":
    main()
