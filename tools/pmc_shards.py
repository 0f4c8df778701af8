#!/usr/bin/env python3
"""HBM traffic per matVec for one rank of a P-GPU run, measured on one GPU.

A P-rank run at N gives each GPU an (N/P) x N row block whose matVec is two
k_matvec_f64 launches (own column block while p is exchanged, then the rest).
Multi-shard mode on one GPU runs exactly those kernels on exactly those
shapes, so under rocprofv3 --pmc its k_matvec_f64 counters, summed per
(own, rest) pair, are the per-rank figure.  Two steps:

  run  (under rocprofv3, once per counter):
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_g8_f -o f --output-format csv -- \\
        python tools/pmc_shards.py run --n 65536 --shards 8
  summarise (merges into profiles/pmc_summary.json as n<N>_g<P>):
    python tools/pmc_shards.py summarise --n 65536 --shards 8 \\
        --fetch gpurun_out/pmc_g8_f/f_counter_collection.csv \\
        --write gpurun_out/pmc_g8_w/w_counter_collection.csv
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNEL = "k_matvec_f64"


def run(n, shards, iters):
    import conjugate_gradient_amd as cg
    with cg.Solver(n, devices=[0] * shards) as s:
        assert s.info.flags & cg.CGX_OVERLAP_ACTIVE, "overlap (own block + rest) must be on"
        s.generate_spd(42)
        s.begin()  # x0 = 0: no initial matVec
        s.iterate(iters, eps=-1.0)
        s.synchronize()


def counters(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    return vals


def summarise(n, shards, fetch_csv, write_csv, tag):
    fe, wr = counters(fetch_csv, "FETCH_SIZE"), counters(write_csv, "WRITE_SIZE")
    assert len(fe) % 2 == 0 and len(fe) == len(wr), (len(fe), len(wr))
    pairs_f = [fe[i] + fe[i + 1] for i in range(0, len(fe), 2)]
    pairs_w = [wr[i] + wr[i + 1] for i in range(0, len(wr), 2)]
    nloc = n // shards
    alg = 8 * nloc * n + 8 * n + 8 * nloc
    f_kib, w_kib = statistics.median(pairs_f), statistics.median(pairs_w)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    entry = {
        "kernel": KERNEL,
        "tag": tag,
        "measured_as": f"{shards} row blocks of {nloc} rows on one MI355X (multi-shard mode): per rank, the "
                       f"own-column-block and remaining-columns launches of one matVec, summed",
        "fetch_size_kib_median": f_kib,
        "write_size_kib_median": w_kib,
        "launch_pairs_counted": [len(pairs_f), len(pairs_w)],
        "hbm_bytes_per_matvec": hbm,
        "algorithmic_bytes_per_matvec": alg,
        "traffic_over_algorithmic": hbm / alg,
        "correction": "HBM = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE reads half of wide streaming loads)",
    }
    out = os.path.join(ROOT, "profiles", "pmc_summary.json")
    data = {}
    if os.path.exists(out):
        with open(out) as f:
            data = json.load(f)
    data[f"n{n}_g{shards}"] = entry
    with open(out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(json.dumps(entry, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "summarise"])
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--tag", default="r02", help="round the counters were collected in")
    a = ap.parse_args()
    if a.mode == "run":
        run(a.n, a.shards, a.iters)
    else:
        summarise(a.n, a.shards, a.fetch, a.write, a.tag)


if __name__ == "__main__":
    main()
