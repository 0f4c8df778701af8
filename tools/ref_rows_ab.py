#!/usr/bin/env python3
"""A/B of k_matvec_ref_f32_w5's rows per block (the CGX_F32_REF matVec):
CGX_REF_ROWS=32 (the default: one block per CU, 132 KiB of LDS) against 16
(66 KiB, two blocks per CU where the registers allow), in the two-launch
iteration (CGX_REF_FUSE=1: the matVec's last block runs vecVec(p, Ap)) and
the four-launch one (CGX_REF_FUSE=0: plain matVec).  Whole solves of
generateSPDmatrix(n) from x0 = 0 at EPSILON = 1e-6 and 200 fixed-count
iterations, interleaved in one process; every solve's x must be
serialConjugate.c's (the oracle's) bit for bit.

  python tools/ref_rows_ab.py [n ...]        (default 2048 4096 8192)
"""
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
    sizes = [int(a) for a in sys.argv[1:]] or [2048, 4096, 8192]
    for n in sizes:
        A, b = oracle.spd_matlab(n, np.float32)
        x0 = np.zeros(n, np.float32)
        xr, sr = oracle.cg_f32ref(A, b, x0, eps=1e-6)
        solvers = {}
        for fuse in ("1", "0"):
            os.environ["CGX_REF_FUSE"] = fuse
            s = cg.Solver(n, flags=cg.CGX_F32_REF)
            s.set_system(A, b, x0)
            solvers[fuse] = s
        res = {}
        for rnd in range(8):
            for fuse, s in solvers.items():
                for rows in ("32", "16"):
                    os.environ["CGX_REF_ROWS"] = rows
                    key = f"fuse{fuse}_rows{rows}"
                    x, st = s.solve(x0, eps=1e-6)
                    assert st.iterations == sr.iterations, (key, st.iterations, sr.iterations)
                    assert np.array_equal(x.view(np.uint32), xr.view(np.uint32)), key
                    s.set_x(x0)
                    s.begin()
                    s.synchronize()
                    t0 = time.perf_counter()
                    s.iterate(200, eps=-1.0)
                    s.synchronize()
                    t1 = time.perf_counter()
                    if rnd:
                        res.setdefault(key + "_solve_ms", []).append(st.solve_ms)
                        res.setdefault(key + "_iter_us", []).append((t1 - t0) / 200 * 1e6)
        for s in solvers.values():
            s.close()
        row = {"n": n, "iterations": int(sr.iterations), "x_bit_identical_to_reference": True}
        row.update({k + "_med": statistics.median(v) for k, v in res.items()})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
