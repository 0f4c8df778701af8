#!/usr/bin/env python3
"""Summarise the Poisson (configs[4]) rocprofv3 outputs into
profiles/<tag>_pmc_poisson_m<M>.json: per fused kernel, HBM bytes per grid
point (2*FETCH_SIZE + WRITE_SIZE, KiB; FETCH_SIZE doubled per the gfx950
correction) next to the algorithmic bytes, and the kernel-trace average.

  python tools/pmc_poisson.py --tag r01 --m 8192 --dir gpurun_out
"""
import argparse
import collections
import csv
import json
import re

ALG = {"k_poisson_xr_f64": 40, "k_poisson_p_f64": 24, "k_stencil5_strip_f64": 16}


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def counters(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--dir", default="gpurun_out")
    a = ap.parse_args()
    n = a.m * a.m
    fe = counters(f"{a.dir}/prof_pois_fetch/fetch_counter_collection.csv", "FETCH_SIZE")
    wr = counters(f"{a.dir}/prof_pois_write/write_counter_collection.csv", "WRITE_SIZE")
    kt = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(f"{a.dir}/prof_pois_kt/kt_kernel_stats.csv"))}
    out = {"workload": f"configs[4] Poisson m={a.m}, fused iteration", "points": n,
           "correction": "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B)",
           "note": "k_poisson_p_f64 averages include each solve's first launch (p_0 = r_0: 16 B/point read+write "
                   "instead of 24)", "kernels": {}}
    for k in fe:
        base = k.split("<")[0]
        if base not in ALG:
            continue
        fb = 2 * sum(fe[k]) / len(fe[k]) * 1024 / n
        wb = sum(wr[k]) / len(wr[k]) * 1024 / n if wr.get(k) else None
        us = kt.get(k, 0.0) / 1e3
        out["kernels"][k] = {"pmc_launches": len(fe[k]), "fetch_B_per_point": fb, "write_B_per_point": wb,
                             "hbm_B_per_point": fb + (wb or 0), "algorithmic_B_per_point": ALG[base],
                             "kernel_trace_avg_us": us,
                             "algorithmic_GBps": ALG[base] * n / (us * 1e3) if us else None}
    path = f"profiles/{a.tag}_pmc_poisson_m{a.m}.json"
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
