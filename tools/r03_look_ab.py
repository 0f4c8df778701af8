#!/usr/bin/env python3
"""Convergence-tested solves (device-gated, x0 = 0, eps 1e-10) with the
host's pacing events varied: the system-scope fence on them (CGX_LOOK_FENCE)
and an event after every E-th iteration instead of every one
(CGX_LOOK_EVERY).  Each setting its own context, interleaved; median of 9.
  python tools/r03_look_ab.py [sizes...]"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

SETTINGS = {"fence_e1": ("1", "1"), "nofence_e1": ("0", "1"), "nofence_e2": ("0", "2"), "nofence_e4": ("0", "4")}
if os.environ.get("R03_LOOK_EVERY_ONLY"):  # the event interval alone, more solves
    SETTINGS = {"e1": ("0", "1"), "e2": ("0", "2"), "e4": ("0", "4"), "e8": ("0", "8")}
REPS = int(os.environ.get("R03_LOOK_REPS", "9"))


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192]
    for n in sizes:
        solvers = {}
        for name, (fence, every) in SETTINGS.items():
            os.environ["CGX_LOOK_FENCE"] = fence
            s = cg.Solver(n)  # the fence flag is read at creation
            s.generate_spd(42)
            solvers[name] = (s, every)
        t = {k: [] for k in SETTINGS}
        its = {}
        x = {}
        for _ in range(REPS):
            for name, (s, every) in solvers.items():
                os.environ["CGX_LOOK_EVERY"] = every
                s.set_x(np.zeros(n))
                xs, st = s.solve(None, eps=1e-10)
                t[name].append(st.solve_ms)
                its[name] = st.iterations
                x[name] = s.get_x()
        for s, _ in solvers.values():
            s.close()
        first = next(iter(x))
        same = all(np.array_equal(x[k], x[first]) for k in x)
        print(json.dumps({"n": n, "iterations": its, "x_bitwise_same": same,
                          "solve_ms_median": {k: round(statistics.median(v), 4) for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
