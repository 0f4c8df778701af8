#!/usr/bin/env python3
"""Sweep the fp64 matVec plan (rows per wave R, chunks in flight U, non-temporal
A loads, resident blocks per CU) on one GPU, interleaved rounds in one process
(cdna_hip_programming.md s5.4 rule 24).  Prints one JSON line per config with
the median / min matVec kernel time (HIP events) and algorithmic GB/s.

  python tools/sweep_matvec.py [--n 65536] [--rounds 3] [--iters 4]
"""
import argparse
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--R", default="1,2,4,8")
    ap.add_argument("--U", default="2,4,8")
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--bpc", default="0")
    args = ap.parse_args()
    n = args.n
    s = cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_TIMING)
    s.generate_spd(42)
    s.begin()
    configs = list(itertools.product(*(map(int, v.split(",")) for v in (args.R, args.U, args.nt, args.bpc))))
    times = {c: [] for c in configs}
    plans = {}
    bytes_launch = 8 * n * n + 16 * n
    for _ in range(args.rounds):
        for c in configs:
            s.set_matvec_plan(*c)
            plans[c] = s.matvec_plan()
            s.iterate(1, eps=-1.0)  # warm this plan
            s.reset_timing()
            s.iterate(args.iters, eps=-1.0)
            st = s.stats()
            times[c].append(st.matvec_ms / st.matvec_count)
    rows = []
    for c in configs:
        med, mn = statistics.median(times[c]), min(times[c])
        rows.append({"R": c[0], "U": c[1], "nt": c[2], "bpc": c[3], "blocks": plans[c]["blocks"],
                     "ms_med": med, "ms_min": mn, "gbps_med": bytes_launch / med / 1e6, "gbps_best": bytes_launch / mn / 1e6})
    rows.sort(key=lambda r: r["ms_med"])
    for r in rows:
        print(json.dumps(r))
    s.close()


if __name__ == "__main__":
    main()
