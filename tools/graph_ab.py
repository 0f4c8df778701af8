#!/usr/bin/env python3
"""Fixed-count iterations from a hipGraph (CGX_GRAPH=1, opt-in, one GPU,
no per-launch timing) vs stream launches (CGX_GRAPH=0): wall time
per iteration over `iters` iterations, interleaved rounds in one process, and
x compared bit for bit between the two.

  python tools/graph_ab.py [--iters 400]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import conjugate_gradient_amd as cg  # noqa: E402


def run(s, iters, graph, reset):
    os.environ["CGX_GRAPH"] = "1" if graph else "0"
    reset()  # x0 again: begin() starts from the current x
    s.begin()
    s.iterate(4)  # the graph replays from k = 4
    s.synchronize()
    t0 = time.perf_counter()
    s.iterate(iters)
    s.synchronize()
    dt = time.perf_counter() - t0
    return dt / iters * 1e6, s.get_x()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    a = ap.parse_args()
    cases = [("dense", n) for n in (512, 1024, 4096, 16384)] + [("f32ref", 1024), ("poisson", 256), ("poisson", 1024)]
    for kind, n in cases:
        if kind == "poisson":
            s = cg.Solver(None, poisson_m=n)
            reset = lambda: s.fill(1.0, 0.0)  # noqa: E731
        else:
            s = cg.Solver(n, flags=cg.CGX_F32_REF if kind == "f32ref" else cg.CGX_F64)
            s.generate_spd(42)
            reset = lambda: s.set_x(np.zeros(s.n, s.dtype))  # noqa: E731
        t = {True: [], False: []}
        xs = {}
        for _ in range(4):
            for g in (False, True):
                us, x = run(s, a.iters, g, reset)
                t[g].append(us)
                xs[g] = x
        s.close()
        row = {"kind": kind, "n": n, "iters": a.iters,
               "stream_us_per_iter": statistics.median(t[False]), "graph_us_per_iter": statistics.median(t[True]),
               "x_bitwise_equal": bool((xs[True].view("u1") == xs[False].view("u1")).all())}
        row["speedup"] = row["stream_us_per_iter"] / row["graph_us_per_iter"]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
