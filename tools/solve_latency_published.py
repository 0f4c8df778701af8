#!/usr/bin/env python3
"""Wall time of a convergence-tested fp64 solve (cgx_solve from x0 = 0,
eps 1e-10, device-gated) at the reference's sizes, round 3's default
(folded iteration, LDS-staged matVec at 2048-8192 columns) against round 2's
form (CGX_FOLD_P=0 CGX_MV_SMALL=0), interleaved in one process: median of 9
solves each, the solve's own clock (cgx_stats.solve_ms).
  python tools/solve_latency_published.py [sizes...] > profiles/r03_solve_latency.jsonl"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

FORMS = {"r03": {}, "r02": {"CGX_FOLD_P": "0", "CGX_MV_SMALL": "0"}}


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192]
    for n in sizes:
        solvers = {}
        for f, env in FORMS.items():
            for k in ("CGX_FOLD_P", "CGX_MV_SMALL"):
                os.environ[k] = env.get(k, "")
            s = cg.Solver(n)
            s.generate_spd(42)
            solvers[f] = s
        t = {f: [] for f in FORMS}
        its = {}
        for _ in range(9):
            for f, s in solvers.items():
                s.set_x(np.zeros(n))
                _, st = s.solve(None, eps=1e-10)
                t[f].append(st.solve_ms)
                its[f] = st.iterations
        for s in solvers.values():
            s.close()
        print(json.dumps({"n": n, "iterations": its, "solve_ms_median": {f: statistics.median(v) for f, v in t.items()},
                          "solve_ms_min": {f: min(v) for f, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
