#!/usr/bin/env python3
"""Per-iteration wall time of fixed-count CG iterations (no stopping test,
nothing read back) on small systems: the launch-rate floor of the loop.

  python tools/iter_floor.py [n ...]    (default 64 512 2048 8192)
"""
import json
import os
import sys
import time

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
        s.synchronize()
        dt = time.perf_counter() - t0
        s.close()
        print(json.dumps({"n": n, "iterations": iters, "us_per_iteration": 1e6 * dt / iters}), flush=True)


if __name__ == "__main__":
    main()
