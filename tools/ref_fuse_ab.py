#!/usr/bin/env python3
"""A/B of the CGX_F32_REF iteration on one GPU: two launches per iteration
(CGX_REF_FUSE=1, the default: the matVec whose last block runs vecVec(p, Ap),
then one block for x/r + r.r + the stopping test + p) against four (matVec,
vecVec, x/r + r.r, p).  Whole solves of generateSPDmatrix(n) from x0 = 0 at
EPSILON = 1e-6 (the reference's published measurement, serialConjugate.c:
208-251), interleaved in one process, plus fixed-count iterations for the
per-iteration time; every solve's x must be serialConjugate.c's (the
oracle's) bit for bit.

  python tools/ref_fuse_ab.py [n ...]        (default 512 1024 2048 4096 8192)
  CGX_AB_SHARDS=4 python tools/ref_fuse_ab.py 8192   (P row blocks on this GPU:
      the matVec + partial vecVec launch against two launches; x checked
      against parallel_cg.c's MPICH combine order)
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
    sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192]
    for n in sizes:
        A, b = oracle.spd_matlab(n, np.float32)
        x0 = np.zeros(n, np.float32)
        P = int(os.environ.get("CGX_AB_SHARDS", "1"))
        xr, sr = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=P, combine="mpich")
        solvers = {}
        for fuse in ("1", "0"):
            os.environ["CGX_REF_FUSE"] = fuse
            s = cg.Solver(n, flags=cg.CGX_F32_REF, devices=[0] * P if P > 1 else None)
            assert P > 1 or bool(s.info.flags & cg.CGX_FUSED_ACTIVE) == (fuse == "1")
            s.set_system(A, b, x0)
            solvers["two_launch" if fuse == "1" else "four_launch"] = s
        solve_ms = {k: [] for k in solvers}
        iter_us = {k: [] for k in solvers}
        for rnd in range(8):
            for name, s in solvers.items():
                x, st = s.solve(x0, eps=1e-6)
                assert st.iterations == sr.iterations, (name, st.iterations, sr.iterations)
                assert np.array_equal(x.view(np.uint32), xr.view(np.uint32)), name
                # fixed-count iterations (x0 = 0 each time): the per-iteration floor
                s.set_x(x0)
                s.begin()
                s.synchronize()
                t0 = time.perf_counter()
                s.iterate(200, eps=-1.0)
                s.synchronize()
                t1 = time.perf_counter()
                if rnd:
                    solve_ms[name].append(st.solve_ms)
                    iter_us[name].append((t1 - t0) / 200 * 1e6)
        for s in solvers.values():
            s.close()
        row = {"n": n, "shards": P, "iterations": int(sr.iterations), "x_bit_identical_to_reference": True}
        for name in solvers:
            row[name + "_solve_ms_med"] = statistics.median(solve_ms[name])
            row[name + "_solve_ms_min"] = min(solve_ms[name])
            row[name + "_iter_us_med"] = statistics.median(iter_us[name])
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
