#!/usr/bin/env python3
"""Summarise tools/pmc_dram_bytes.sh: per workload and kernel, the mean of
every counter over its launches and the bytes they imply, next to the
kernel's algorithmic bytes per launch (where this file knows them).

  python3 tools/pmc_sizes.py --dir gpurun_out/pmcsz > gpurun_out/r03_pmc_sizes.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    if not m:
        return name
    if m.group(1) == "k_poisson_xr_f64" and m.group(2) and m.group(2).count(",") == 3:
        # x every other iteration: the variants move different bytes (XM = last argument)
        return f"k_poisson_xr_f64<XM={m.group(2).strip('<>').split(',')[-1].strip()}>"
    if m.group(1) == "k_poisson_xr_pipe_f64" and m.group(2) and m.group(2).count(",") >= 2:
        # the software-pipelined form <RB, NS, XM[, variant flags]>
        return f"k_poisson_xr_pipe_f64<XM={m.group(2).strip('<>').split(',')[2].strip()}>"
    return m.group(1)


def algorithmic(w, kernel, n, m):
    """Bytes per launch (steady-state launch) of the kernels DESIGN prices.
    `w` may carry a variant suffix (poisson_et1): the part before '_' counts."""
    w = w.split("_")[0]
    if w == "dense" and kernel == "k_matvec_f64":
        return 8 * n * n + 16 * n
    if w == "symmetric" and kernel == "k_symv_f64":
        t = n // 128
        return 8 * 128 * 128 * t * (t + 1) // 2 + 16 * n  # tiles + p + y (partials are overhead)
    if w == "poisson" and kernel in ("k_poisson_p_f64", "k_poisson_p_pipe_f64"):
        return 24 * m * m
    xr = kernel.replace("_pipe", "")
    if w == "poisson" and xr in ("k_poisson_xr_f64", "k_poisson_xr_f64<XM=1>"):
        return 40 * m * m + 16 * m
    if w == "poisson" and xr == "k_poisson_xr_f64<XM=0>":  # p_k (+ halo rows), r -> r
        return 24 * m * m + 16 * m
    if w == "poisson" and xr == "k_poisson_xr_f64<XM=2>":  # p_{k-1}, p_k (+ halo), x, r -> x, r
        return 48 * m * m + 16 * m
    if w == "poisson" and xr == "k_poisson_xr_f64<XM=3>":  # p_{k-2}, p_{k-1}, p_k (+ halo), x, r -> x, r
        return 56 * m * m + 16 * m
    if w == "poisson" and kernel == "k_poisson_xflush_f64":
        return 24 * m * m
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    a = ap.parse_args()
    out = {"counters": "A: TCC_EA0_RDREQ_DRAM_32B_sum / TCC_EA0_WRREQ_WRITE_DRAM_32B_sum (x32 B); "
                       "B: TCC_EA0_RDREQ_{32B,64B,128B}_sum, TCC_EA0_RDREQ_sum; C: FETCH_SIZE (KiB)",
           "workloads": {}}
    for wdir in sorted(glob.glob(os.path.join(a.dir, "*_A"))):
        w = os.path.basename(wdir)[:-2]
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for p in ("A", "B", "C"):
            for f in glob.glob(os.path.join(a.dir, f"{w}_{p}", "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        cfg = {}
        try:
            cfg = json.load(open(os.path.join(a.dir, f"{w}_A.json")))["config"]
        except (OSError, ValueError, KeyError):
            pass
        n, m = cfg.get("n", 65536), cfg.get("m", 8192)
        ks = {}
        for k, cs in vals.items():
            mean = {c: sum(v) / len(v) for c, v in cs.items()}
            e = {"launches": {c: len(v) for c, v in cs.items()}, "mean": mean}
            rd = mean.get("TCC_EA0_RDREQ_DRAM_32B_sum")
            wr = mean.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
            if rd is not None:
                e["dram_read_B"] = 32 * rd
            if wr is not None:
                e["dram_write_B"] = 32 * wr
            if "TCC_EA0_RDREQ_128B_sum" in mean:
                e["req_read_B"] = (128 * mean["TCC_EA0_RDREQ_128B_sum"] + 64 * mean["TCC_EA0_RDREQ_64B_sum"]
                                   + 32 * mean["TCC_EA0_RDREQ_32B_sum"])
            if "FETCH_SIZE" in mean:
                e["fetch_size_x2_B"] = 2 * 1024 * mean["FETCH_SIZE"]
            alg = algorithmic(w, k, n, m)
            if alg:
                e["algorithmic_B"] = alg
                if rd is not None and wr is not None:
                    e["dram_over_algorithmic"] = 32 * (rd + wr) / alg
            ks[k] = e
        out["workloads"][w] = {"config": cfg, "kernels": ks}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
