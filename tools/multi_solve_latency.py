#!/usr/bin/env python3
"""The first and the next solves of a fresh process, several row blocks on
one GPU (cgx_create_multi, devices=[0]*P), CGX_F32_REF (parallel_cg.c's
arithmetic) with the collective or the p2p exchange: cgx_solve's own wall
time (solve_ms) for 5 solves from x0 = 0 in one context.  A fresh process
per configuration, as `cg_hip --gpus P` runs, so the first solve carries
whatever a process pays on first use.

  python tools/multi_solve_latency.py [n,...] [P,...] > profiles/rNN_multi_solve_latency.jsonl
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n, P, program):
    sys.path.insert(0, ROOT)
    import numpy as np

    import conjugate_gradient_amd as cg
    import oracle
    A, b = oracle.spd_matlab(n, np.float32)
    flags = cg.CGX_F32_REF | (cg.CGX_COMM_P2P if program == "p2p" else 0)
    ms = []
    with cg.Solver(n, flags=flags, devices=[0] * P) as s:
        s.set_system(A, b)
        for _ in range(5):
            s.set_x(np.zeros(n, np.float32))
            _, st = s.solve(None, eps=1e-6)
            ms.append(round(st.solve_ms, 3))
            its = st.iterations
    print(json.dumps({"n": n, "P": P, "program": program, "iterations": its, "solve_ms": ms}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
    sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4096, 8192]
    ps = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
    for n in sizes:
        for P in ps:
            for program in ("parallel", "p2p") if P > 1 else ("parallel",):
                r = subprocess.run([sys.executable, __file__, "--child", str(n), str(P), program],
                                   capture_output=True, text=True, timeout=300)
                sys.stdout.write(r.stdout if r.returncode == 0 else json.dumps(
                    {"n": n, "P": P, "program": program, "error": r.stderr[-500:]}) + "\n")
                sys.stdout.flush()


if __name__ == "__main__":
    main()
