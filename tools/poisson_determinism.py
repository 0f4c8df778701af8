#!/usr/bin/env python3
"""Run-to-run determinism of the Poisson CG path: the same fixed-count solve
repeated on one context must give x bit for bit.  Checks the fused and split
iterations, both item-walk directions, at a few grid sizes and counts.

  python tools/poisson_determinism.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    for env in ({"CGX_POISSON_FUSED": "1", "CGX_POISSON_PLAN": "reverse=1"},
                {"CGX_POISSON_FUSED": "1", "CGX_POISSON_PLAN": "reverse=0"},
                {"CGX_POISSON_FUSED": "0", "CGX_POISSON_PLAN": "reverse=1"}):
        os.environ.update(env)
        for m in (256, 1024):
            with cg.Solver(None, poisson_m=m) as s:
                s.fill(1.0, 0.0)
                for iters in (1, 2, 3, 20):
                    xs = []
                    for _ in range(3):
                        s.fill(1.0, 0.0)  # b = 1, x0 = 0 again (begin() starts from the current x)
                        s.begin()
                        s.iterate(iters)
                        s.synchronize()
                        xs.append(s.get_x())
                    same = [bool(np.array_equal(xs[0].view("u1"), x.view("u1"))) for x in xs[1:]]
                    print(json.dumps({**env, "m": m, "iters": iters, "bitwise_same": same,
                                      "max_abs_diff": float(max(np.abs(xs[0] - x).max() for x in xs[1:]))}),
                          flush=True)


if __name__ == "__main__":
    main()
