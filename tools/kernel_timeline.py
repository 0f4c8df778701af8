#!/usr/bin/env python3
"""Per-kernel durations and the gaps between kernels from a rocprofv3
--kernel-trace CSV of tools/iter_floor.py (one segment per system size: each
size starts with its k_gen_spd launch).  For every segment: the median
duration of each kernel and the median idle gap before it (end of the previous
kernel to its start), over the segment's fixed-count iterations.

  python tools/kernel_timeline.py gpurun_out/prof_small/small_kernel_trace.csv --sizes 512 2048 8192 \
      > profiles/r02_kernel_timeline_small_n.json
"""
import argparse
import collections
import csv
import json
import re
import statistics


def short(name):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--sizes", type=int, nargs="+", required=True)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], None
    for r in rows:
        if "k_gen_spd" in r["Kernel_Name"]:
            cur = []
            segs.append(cur)
        if cur is not None:
            cur.append(r)
    out = {"source": args.trace, "note": "medians over each size's fixed-count iterations; us", "sizes": {}}
    for n, seg in zip(args.sizes, segs):
        dur, gap = collections.defaultdict(list), collections.defaultdict(list)
        prev_end = None
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            k = short(r["Kernel_Name"])
            dur[k].append((e - s) / 1e3)
            if prev_end is not None:
                gap[k].append(max(0.0, (s - prev_end) / 1e3))
            prev_end = e
        main_kernels = [k for k in dur if len(dur[k]) >= 100]
        out["sizes"][str(n)] = {k: {"launches": len(dur[k]), "dur_us": round(statistics.median(dur[k]), 3),
                                    "gap_before_us": round(statistics.median(gap[k]), 3) if gap[k] else None}
                                for k in main_kernels}
        per_iter = sum(v["dur_us"] + (v["gap_before_us"] or 0) for v in out["sizes"][str(n)].values())
        out["sizes"][str(n)]["iteration_us_from_trace"] = round(per_iter, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
