"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per WAM kernel.

usage: python scripts/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>

Kernel names are shortened to the names libwam_hip.so's live timing uses (bench.py roofline keys):
k_ana_rows<..., true> -> "k_ana_rows<noise>". Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section),
FETCH_SIZE on gfx950 reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is taken as is. Both counters are in KiB.
"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"::(k_\w+)(<([^>]*)>)?\(", name)
    if not m:
        return None
    base = m.group(1)
    args = [a.strip() for a in m.group(3).split(",")] if m.group(3) else []
    if base in ("k_ana_rows", "k_haar3_ana", "k_dwt1_ana", "k_dwt1_ana_p", "k_dwt1_ana_int") and args and args[-1] == "true":
        return base + "<noise>"
    if base == "k_plane_ana" and len(args) >= 5:  # <L, CPL, NOISE, MC, MAPS, COOP, IN>
        if args[4] == "true":
            fmt = args[6] if len(args) >= 7 else "0"
            return {"1": "k_plane_maps<bf16nhwc>", "2": "k_plane_maps<bf16>"}.get(fmt, "k_plane_maps")
        return "k_plane_ana<noise>" if args[2] == "true" else "k_plane_ana"
    if base == "k_plane_syn" and len(args) >= 2 and args[1] != "0":  # <L, OC>: bf16 NHWC output
        return "k_plane_syn<bf16nhwc>"
    if base == "k_cube_accumulate4":  # the four-voxel forms time under the entry point's name
        return "k_cube_accumulate"
    return base


def load(path, counter):
    acc = collections.defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            if k is None:  # not a libwam_hip.so kernel
                continue
            acc[k][0] += 1
            acc[k][1] += float(row["Counter_Value"]) * 1024.0
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over bench.py",
           "fetch_correction": 2.0, "per_call_bytes": {}, "per_call": {}}
    for k in sorted(set(fetch) | set(write)):
        nf, bf = fetch.get(k, [0, 0.0])
        nw, bw = write.get(k, [0, 0.0])
        rd = 2.0 * bf / max(nf, 1)
        wr = bw / max(nw, 1)
        out["per_call"][k] = {"launches": max(nf, nw), "read_bytes": round(rd), "write_bytes": round(wr)}
        out["per_call_bytes"][k] = round(rd + wr)
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
