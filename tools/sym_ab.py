#!/usr/bin/env python3
"""In-process A/B of the CGX_SYMMETRIC matVec (load policy CGX_SYM_PLAN nt=, read
per launch) against the row-major kernel on the same
system: interleaved rounds of fixed-count iterations, matVec time from HIP
events (CGX_TIMING), medians per variant.

  python tools/sym_ab.py [n ...]     (default 16384 65536)
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

VARIANTS = {"sym_nt": {"CGX_SYM_PLAN": "nt=1"}, "sym_default_policy": {"CGX_SYM_PLAN": "nt=0"}}


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [16384, 65536]
    for n in sizes:
        iters = 10 if n >= 65536 else 40
        s = cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_TIMING | cg.CGX_SYMMETRIC)
        s.generate_spd(42)
        d = cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_TIMING)
        d.generate_spd(42)
        res = {k: [] for k in VARIANTS}
        res["dense"] = []
        for rnd in range(5):
            for name, env in list(VARIANTS.items()) + [("dense", {})]:
                os.environ.update(env)
                solver = d if name == "dense" else s
                solver.begin()
                solver.iterate(2)
                solver.synchronize()
                solver.reset_timing()
                solver.iterate(iters)
                st = solver.stats()
                if rnd:
                    res[name].append(st.matvec_ms / st.matvec_count)
        s.close()
        d.close()
        nt = (n + 127) // 128
        sym_bytes = 8 * nt * (nt + 1) // 2 * 128 * 128 + 16 * n
        row = {"n": n}
        for k, v in res.items():
            ms = statistics.median(v)
            b = (8 * n * n + 16 * n) if k == "dense" else sym_bytes
            row[k] = {"matvec_ms": ms, "gbps": b / ms / 1e6}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
