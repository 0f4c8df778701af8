#!/usr/bin/env python3
"""A/B of the CGX_F32_REF kernels (the bit-exact serialConjugate.c mode):
matVec  CGX_REF_MV=1 (64 rows x 128-column tiles per wave) vs 2 (16 rows x
512-column tiles) vs 4 (32 rows per block, two tiles in flight, wave 0 adds
and loads) vs 3 (the same with a wave that only adds: the default), vecVec CGX_REF_DOT=1 (one wave) vs 2
(4 waves, loads off the chain).  Whole solves of generateSPDmatrix(n) from x0 = 0 at
EPSILON = 1e-6, interleaved in one process; every variant's x must be the
oracle's (== serialConjugate.c) bit for bit.  Per-kernel times come from
running this under rocprofv3 --kernel-trace --stats.

  python tools/ref_f32_ab.py [n ...]        (default 4096 8192)
"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402

VARIANTS = {"mv1_dot1": ("1", "1"), "mv2_dot1": ("2", "1"), "mv2_dot2": ("2", "2"), "mv4_dot2": ("4", "2"),
            "mv3_dot2": ("3", "2")}


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [2048, 4096, 8192]
    for n in sizes:
        A, b = oracle.spd_matlab(n, np.float32)
        xr, sr = oracle.cg_f32ref(A, b, np.zeros(n, np.float32), eps=1e-6)
        s = cg.Solver(n, flags=cg.CGX_F32_REF)
        s.set_system(A, b, np.zeros(n, np.float32))
        times = {k: [] for k in VARIANTS}
        for rnd in range(6):
            for name, (mv, dot) in VARIANTS.items():
                os.environ["CGX_REF_MV"], os.environ["CGX_REF_DOT"] = mv, dot
                x, st = s.solve(np.zeros(n, np.float32), eps=1e-6)
                assert st.iterations == sr.iterations, (name, st.iterations, sr.iterations)
                assert np.array_equal(x.view(np.uint32), xr.view(np.uint32)), name
                if rnd:
                    times[name].append(st.solve_ms)
        s.close()
        row = {"n": n, "iterations": sr.iterations, "bit_identical_to_reference": True}
        for name in VARIANTS:
            row[name + "_solve_ms_med"] = statistics.median(times[name])
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
