"""Fused Poisson, x every other iteration vs every iteration: the first
iteration count at which x (or r.r) differs, for a few grid widths (GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def run(m, count, xdefer, extra=None):
    os.environ["CGX_POISSON_XDEFER"] = xdefer
    for k, v in (extra or {}).items():
        os.environ[k] = v
    with cg.Solver(None, poisson_m=m) as s:
        s.fill(1.0, 0.0)
        s.begin()
        s.iterate(count, eps=-1.0)
        x = s.get_x()
        st = s.stats()
    for k in (extra or {}):
        del os.environ[k]
    return x, st.rr


for m in [int(a) for a in sys.argv[1:]] or [1040, 2048]:
    for count in (1, 2, 3, 4, 6):
        xa, ra = run(m, count, "1")
        xb, rb = run(m, count, "0")
        print(f"m={m} count={count} x_equal={np.array_equal(xa, xb)} rr_equal={ra == rb} "
              f"maxdiff={np.max(np.abs(xa - xb)):.3e} rr {ra!r} {rb!r}", flush=True)
