#!/usr/bin/env python3
"""matVec plan sweep for a row block of given height (e.g. the 8192 x 65536
block one GPU owns at N=65536 over 8 GPUs), through the kernel-level entry
point cgx_matvec with the plan taken from CGX_MV_PLAN.
Wall-clock timing over `--reps` back-to-back launches (launch overhead is
included: a few us against ~0.6 ms), interleaved rounds in one process.

  python tools/sweep_rows.py --rows 8192 --cols 65536
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--cols", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--R", default="1,2,4,8")
    ap.add_argument("--U", default="2,4,8")
    ap.add_argument("--nt", default="1")
    ap.add_argument("--bpc", default="0")
    args = ap.parse_args()
    rows, cols = args.rows, args.cols
    A = cg.DeviceArray.from_host(np.full((rows, cols), 0.25))
    v = cg.DeviceArray.from_host(np.full(cols, 0.5))
    out = cg.DeviceArray(rows)
    configs = list(itertools.product(*(map(int, s.split(",")) for s in (args.R, args.U, args.nt, args.bpc))))
    t = {c: [] for c in configs}
    L = cg.lib()
    for _ in range(args.rounds):
        for c in configs:
            os.environ["CGX_MV_PLAN"] = f"R={c[0]},U={c[1]},nt={c[2]}" + (f",bpc={c[3]}" if c[3] > 0 else "")
            cg.matVec(A, v, out, rows, cols)
            L.cgx_dev_synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                cg.matVec(A, v, out, rows, cols)
            L.cgx_dev_synchronize()
            t[c].append((time.perf_counter() - t0) / args.reps)
    got = out.to_host()
    assert np.allclose(got, 0.125 * cols), got[:4]
    bytes_launch = 8 * rows * cols + 8 * cols + 8 * rows
    res = []
    for c in configs:
        med = statistics.median(t[c])
        res.append({"rows": rows, "cols": cols, "R": c[0], "U": c[1], "nt": c[2], "bpc": c[3],
                    "ms_med": med * 1e3, "gbps_med": bytes_launch / med / 1e9})
    res.sort(key=lambda r: r["ms_med"])
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
