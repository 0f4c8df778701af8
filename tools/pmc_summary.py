#!/usr/bin/env python3
"""Summarise rocprofv3 outputs for one bench workload into profiles/.

  python tools/pmc_summary.py --tag r01 --n 65536 --gpus 1 \
      --kt gpurun_out/prof_kt/kt_kernel_stats.csv \
      --fetch gpurun_out/prof_fetch/fetch_counter_collection.csv \
      --write gpurun_out/prof_write/write_counter_collection.csv

  python tools/pmc_summary.py --tag r06 --workload poisson --m 8192 --kt ... --fetch ... --write ...
      (configs[4]: the roofline kernel is the xr kernel, k_poisson_xr_f64 and
      its pipelined x catch-up k_poisson_xr_pipe_f64; run the passes with
      --steps 6 --warmup 0 so the launches are two whole x cycles, 0 0 3)

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


def counter_values(path, name, kernel=KERNEL):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return vals


def poisson(args):
    """The configs[4] line's roofline kernel: every xr launch of the passes
    (the x cycle's 24, 24 and 56 B/point launches), averaged per launch, so
    the figure matches bench.py's algorithmic_bytes_per_launch (34.67 B/point
    + the two halo rows)."""
    kern = "k_poisson_xr"
    fetch = counter_values(args.fetch, "FETCH_SIZE", kern)
    write = counter_values(args.write, "WRITE_SIZE", kern)
    m = args.m
    n = m * m
    hbm = (2 * sum(fetch) / len(fetch) + sum(write) / len(write)) * 1024
    alg = 104.0 / 3 * n + 16 * m
    dur = []
    with open(args.kt) as f:
        for row in csv.DictReader(f):
            if kern in row["Name"]:
                dur.append((float(row["TotalDurationNs"]), int(row["Calls"])))
    avg_ns = sum(d for d, _ in dur) / sum(c for _, c in dur) if dur else None
    entry = {
        "kernel": "k_poisson_xr_f64 + k_poisson_xr_pipe_f64 (the x cycle: two 24-B/point launches, one 56)",
        "tag": args.tag,
        "launches_counted": [len(fetch), len(write)],
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": hbm / alg,
        "rocprof_avg_duration_ns": avg_ns,
        "rocprof_gbps_algorithmic": alg / avg_ns if avg_ns else None,
        "correction": "HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE reads half of wide streaming loads), "
                      "mean over the xr launches",
    }
    return f"poisson_m{m}_g{args.gpus}", entry


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--workload", choices=["dense", "poisson"], default="dense")
    ap.add_argument("--m", type=int, default=8192)
    args = ap.parse_args()
    if args.workload == "poisson":
        key, entry = poisson(args)
        return save(key, entry, args, f"{args.tag}_kernel_stats_poisson_m{args.m}_g{args.gpus}.csv")
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
    return save(f"n{n}_g{g}", entry, args, f"{args.tag}_kernel_stats_n{n}_g{g}.csv")


def save(key, entry, args, kt_name):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = os.path.join(ROOT, "profiles", "pmc_summary.json")
    data = {}
    if os.path.exists(out):
        with open(out) as f:
            data = json.load(f)
    data[key] = entry
    with open(out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    shutil.copy(args.kt, os.path.join(ROOT, "profiles", kt_name))
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
