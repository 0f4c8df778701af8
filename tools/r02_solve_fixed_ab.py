#!/usr/bin/env python3
"""Median wall time of convergence-tested fp64 solves (cgx_solve from x0 = 0,
eps 1e-10, x left on the device: the CG region cg_hip times) at small N, for
an A/B of two builds: run this script from each tree in turn
(tools/r02_solve_fixed_ab.sh).  Prints one JSON line per N."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.getcwd())
import conjugate_gradient_amd as cg  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [512, 2048, 8192]:
    with cg.Solver(n) as s:
        s.generate_spd(42)
        ms, its = [], set()
        for i in range(40):
            s.set_x(__import__("numpy").zeros(n))
            _, st = s.solve(None, eps=1e-10)
            its.add(st.iterations)
            if i >= 5:
                ms.append(st.solve_ms)
    print(json.dumps({"tree": os.path.basename(os.getcwd()) or ".", "n": n, "iterations": sorted(its),
                      "solve_ms_med": statistics.median(ms), "solve_ms_min": min(ms)}), flush=True)
