#!/usr/bin/env python3
"""Summarise rocprofv3 outputs for one bench workload into profiles/.

  python tools/pmc_summary.py --tag r01 --n 65536 --gpus 1 \
      --kt gpurun_out/prof_kt/kt_kernel_stats.csv \
      --fetch gpurun_out/prof_fetch/fetch_counter_collection.csv \
      --write gpurun_out/prof_write/write_counter_collection.csv

HBM bytes per matVec launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).
FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is
exact for streaming stores.  Each counter comes from its own --pmc pass.
Writes profiles/pmc_summary.json (merged, keyed "n<N>_g<G>") and copies the
kernel-stats CSV to profiles/<tag>_kernel_stats_n<N>_g<G>.csv.
"""
import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_matvec_f64"


def counter_values(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    args = ap.parse_args()
    fetch = counter_values(args.fetch, "FETCH_SIZE")
    write = counter_values(args.write, "WRITE_SIZE")
    n, g = args.n, args.gpus
    nloc = n // g
    alg = 8 * nloc * n + 8 * n + 8 * nloc
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    avg_ns = None
    with open(args.kt) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Name"]:
                avg_ns = float(row["AverageNs"])
    entry = {
        "kernel": KERNEL,
        "tag": args.tag,
        "fetch_size_kib_median": f_kib,
        "write_size_kib_median": w_kib,
        "launches_counted": [len(fetch), len(write)],
        "hbm_bytes_per_matvec": hbm,
        "algorithmic_bytes_per_matvec": alg,
        "traffic_over_algorithmic": hbm / alg,
        "rocprof_avg_duration_ns": avg_ns,
        "rocprof_gbps_algorithmic": alg / avg_ns if avg_ns else None,
        "correction": "HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE reads half of wide streaming loads)",
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = os.path.join(ROOT, "profiles", "pmc_summary.json")
    data = {}
    if os.path.exists(out):
        with open(out) as f:
            data = json.load(f)
    data[f"n{n}_g{g}"] = entry
    with open(out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    shutil.copy(args.kt, os.path.join(ROOT, "profiles", f"{args.tag}_kernel_stats_n{n}_g{g}.csv"))
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
