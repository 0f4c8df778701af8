#!/usr/bin/env python3
"""A/B of the Poisson iteration: fused two-kernel (default) vs the
stencil / r / x,p split (CGX_POISSON_FUSED=0), same fixed iteration count,
one process; prints max |dx| / max |x| and the true residual of each.

  python tools/poisson_ab.py --m 2048 --iters 30 [--shards 1]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def run(m, iters, shards, fused):
    os.environ["CGX_POISSON_FUSED"] = "1" if fused else "0"
    with cg.Solver(None, poisson_m=m, devices=[0] * shards if shards > 1 else None) as s:
        active = bool(s.info.flags & cg.CGX_FUSED_ACTIVE)
        s.fill(1.0, 0.0)
        s.begin()
        s.iterate(iters, eps=-1.0)
        x = s.get_x()
        rn, bn = s.residual_norm()
    return x, rn / bn, active


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shards", type=int, default=1)
    a = ap.parse_args()
    xf, rf, af = run(a.m, a.iters, a.shards, True)
    xs, rs, as_ = run(a.m, a.iters, a.shards, False)
    print(json.dumps({"m": a.m, "iters": a.iters, "shards": a.shards, "fused_active": af, "split_active": as_,
                      "max_dx_over_max_x": float(np.max(np.abs(xf - xs)) / np.max(np.abs(xs))),
                      "relres_fused": rf, "relres_split": rs}))


if __name__ == "__main__":
    main()
