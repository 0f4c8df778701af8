#!/usr/bin/env python3
"""Wall time of convergence-tested solves (cgx_solve, eps=1e-10) with the
device-side stopping decision (default) vs the host-checked loop
(CGX_GATED=0), on small and mid-size systems where per-iteration host
round trips matter.  Interleaved rounds in one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def main():
    out = []
    sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192, 16384]
    for n in sizes:
        s = cg.Solver(n)
        s.generate_spd(42)
        t = {"1": [], "0": []}
        its = {}
        for _ in range(7):
            for g in ("1", "0"):
                os.environ["CGX_GATED"] = g
                s.set_x(__import__("numpy").zeros(n))
                _, st = s.solve(None, eps=1e-10)
                t[g].append(st.solve_ms)
                its[g] = st.iterations
        s.close()
        row = {"n": n, "iterations": its, "gated_ms_med": statistics.median(t["1"]),
               "host_checked_ms_med": statistics.median(t["0"])}
        row["speedup"] = row["host_checked_ms_med"] / row["gated_ms_med"]
        print(json.dumps(row))
        out.append(row)


if __name__ == "__main__":
    main()
