#!/usr/bin/env python3
"""Per-iteration wall time of fixed-count CG iterations (no stopping test,
nothing read back) on small systems: the launch-rate floor of the loop; the
host's own enqueue time per iteration beside it (equal to the wall time =>
the loop is bound by the host's launches), and the wall time of a whole
convergence-tested solve from x0 = 0.

  python tools/iter_floor.py [n ...]    (default 64 512 2048 8192)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    for n in [int(a) for a in sys.argv[1:]] or [64, 512, 2048, 8192]:
        s = cg.Solver(n)
        s.generate_spd(42)
        s.begin()
        s.iterate(50, eps=-1.0)
        s.synchronize()
        iters = 2000
        t0 = time.perf_counter()
        s.iterate(iters, eps=-1.0)
        t1 = time.perf_counter()  # the host has enqueued every launch
        s.synchronize()
        dt = time.perf_counter() - t0
        # convergence-tested solves from x0 = 0 (device-gated stop): per-solve wall time
        reps = 50
        x0 = np.zeros(n)
        s.solve(x0, eps=1e-10)
        t2 = time.perf_counter()
        for _ in range(reps):
            _, st = s.solve(x0, eps=1e-10)
        solve_ms = 1e3 * (time.perf_counter() - t2) / reps
        s.close()
        print(json.dumps({"n": n, "iterations": iters, "us_per_iteration": 1e6 * dt / iters,
                          "host_enqueue_us_per_iteration": 1e6 * (t1 - t0) / iters,
                          "solve_ms": solve_ms, "solve_iterations": st.iterations,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("CGX_")}}), flush=True)


if __name__ == "__main__":
    main()
