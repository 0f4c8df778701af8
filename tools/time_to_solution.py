#!/usr/bin/env python3
"""Time to solution of whole convergence-tested solves (cgx_solve: x0 = 0,
fp64, eps = 1e-10 absolute, device-gated stop) on one GPU, as the reference's
"clock execution time" measures a conjugrad call (serialConjugate.c:208-251).
Median of --reps solves after one warm-up solve.

  python tools/time_to_solution.py [--n 16384,65536] [--reps 5] [--out profiles/r01_time_to_solution.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="16384,65536")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = []
    for n in map(int, args.n.split(",")):
        with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_TIMING) as s:
            s.generate_spd(42)
            zero = np.zeros(n)
            times, its = [], set()
            for r in range(args.reps + 1):
                s.set_x(zero)
                s.reset_timing()
                _, st = s.solve(None, eps=1e-10)
                if r:
                    times.append(st.solve_ms)
                its.add(st.iterations)
            st2 = s.stats()
            rn, bn = s.residual_norm()
        med = statistics.median(times)
        row = {"n": n, "iterations": sorted(its), "solve_ms_median": med, "solve_ms_all": times,
               "matvecs_per_solve": st2.matvec_count, "matvec_ms_avg": st2.matvec_ms / max(1, st2.matvec_count),
               "relres": rn / bn, "note": "x0 = 0: the initial A x0 is skipped (exactly zero)"}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
