#!/usr/bin/env python3
"""Latency of one whole solve at the reference's own sizes, one GPU,
CGX_F32_REF (serialConjugate.c's arithmetic): cgx_solve's wall time
(solve_ms, the figure cg_hip prints as the CG-method time) for `reps`
solves from x0 = 0 in one context, per N.  Run it under
`rocprofv3 --hip-trace --kernel-trace` to see where a solve's time goes
(host API calls against the kernels); each solve is a roctx range
"cgx_solve" (`--marker-trace`).

  python tools/small_solve_trace.py [n,...] [reps] > profiles/rNN_small_solve.jsonl

CGX_AB_LIB=<path to another libcgx.so build> loads that build instead (A/B
runs of a kernel change, processes interleaved by the caller).
"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402


def main():
    if os.environ.get("CGX_AB_LIB"):
        cg.LIB_PATH = os.environ["CGX_AB_LIB"]
    sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [512, 2048, 8192]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    flags = int(os.environ.get("CGX_SMALL_FLAGS", cg.CGX_F32_REF))
    dt = np.float64 if flags & cg.CGX_F32_REF == 0 else np.float32
    for n in sizes:
        A, b = oracle.spd_matlab(n, dt)
        ms = []
        with cg.Solver(n, flags=flags) as s:
            s.set_system(A, b)
            for _ in range(reps):
                s.set_x(np.zeros(n, dt))
                _, st = s.solve(None, eps=1e-6)
                ms.append(st.solve_ms)
        print(json.dumps({"lib": os.path.basename(cg.LIB_PATH), "n": n, "flags": flags, "iterations": st.iterations,
                          "reps": reps, "solve_ms_median": round(statistics.median(ms), 4), "solve_ms_min": round(min(ms), 4),
                          "solve_ms_first": round(ms[0], 4)}), flush=True)


if __name__ == "__main__":
    main()
