#!/usr/bin/env python3
"""CGX_F32_REF matVec kernels (CGX_REF_MV 2/3/4) at the reference's sizes,
with the row pitch lda varied: rows 32 KiB apart (N=8192, lda=N) all start a
tile at the same column offset, so a pitch that is not a multiple of a large
power of two spreads the chip's simultaneous requests over more HBM
channels.  Wall clock over back-to-back launches, interleaved rounds; the
result must equal the oracle bit for bit in every configuration.

  python tools/sweep_ref_mv.py [--n 8192] [--pads 0,16,64,128,512]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--pads", default="0,16,64,128,512")
    ap.add_argument("--variants", default="2,3,4")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    rng = np.random.default_rng(5)
    A = (rng.random((n, n), dtype=np.float32) - 0.5)
    v = rng.random(n, dtype=np.float32)
    ref = oracle.matvec_f32ref(A, v)
    L = cg.lib()
    configs = [(int(p), vv) for p in a.pads.split(",") for vv in a.variants.split(",")]
    bufs = {}
    for pad in {c[0] for c in configs}:
        lda = n + pad
        Ap = np.zeros((n, lda), np.float32)
        Ap[:, :n] = A
        bufs[pad] = (cg.DeviceArray.from_host(Ap), lda)
    vd = cg.DeviceArray.from_host(v)
    out = cg.DeviceArray(n, np.float32)
    t = {c: [] for c in configs}
    for _ in range(a.rounds):
        for c in configs:
            Ad, lda = bufs[c[0]]
            os.environ["CGX_REF_MV"] = c[1]
            cg.matVec(Ad, vd, out, n, n, lda)
            L.cgx_dev_synchronize()
            assert np.array_equal(out.to_host().view(np.uint32), ref.view(np.uint32)), c
            t0 = time.perf_counter()
            for _ in range(a.reps):
                cg.matVec(Ad, vd, out, n, n, lda)
            L.cgx_dev_synchronize()
            t[c].append((time.perf_counter() - t0) / a.reps)
    for c in configs:
        med = statistics.median(t[c])
        print(json.dumps({"n": n, "lda": n + c[0], "variant": c[1], "us_med": med * 1e6,
                          "gbps": 4.0 * n * n / med / 1e9, "bit_identical": True}), flush=True)


if __name__ == "__main__":
    main()
