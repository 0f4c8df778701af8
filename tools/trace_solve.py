#!/usr/bin/env python3
"""Three convergence-tested solves of the N=16384 system (x0 = 0, eps 1e-10)
for a timeline: run under
  rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace -o t --output-format csv -- \\
      python3 tools/trace_solve.py
libcgx's roctx ranges (cgx_generate_spd, cgx_solve, cgx_solve_begin,
cgx_iterate, cgx_get_x, ...) bracket the kernels of each phase."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import conjugate_gradient_amd as cg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
with cg.Solver(n) as s:
    s.generate_spd(42)
    for _ in range(3):
        x, st = s.solve(np.zeros(n), eps=1e-10)
        print(f"n={n} iterations={st.iterations} solve_ms={st.solve_ms:.3f}")
