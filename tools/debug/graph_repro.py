"""Repro for a host SIGSEGV in the LOCAL graph replay at 8 row blocks:
one solver per (S, G), fixed-count pieces, progress printed before each
step.  Loads /tmp/segv_bt.so (tools/debug/segv_bt.c) for a native backtrace.
Usage: python tools/debug/graph_repro.py S G [overlap 1|0]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402,F401
import conjugate_gradient_amd as cg  # noqa: E402


def say(*a):
    print(*a, flush=True)


S, G = int(sys.argv[1]), int(sys.argv[2])
overlap = len(sys.argv) < 4 or sys.argv[3] == "1"
os.environ["CGX_LOCAL_THREADS"] = "0"
os.environ["CGX_LOCAL_GRAPH"] = "2"
os.environ["CGX_LOCAL_GRAPH_ITERS"] = str(G)
n = 2048
flags = cg.CGX_F64 | (0 if overlap else cg.CGX_NO_OVERLAP)
say("create", S, G, overlap)
with cg.Solver(n, flags=flags, devices=[0] * S) as s:
    if os.path.exists("/tmp/segv_bt.so"):
        ctypes.CDLL("/tmp/segv_bt.so").segv_bt_install()
    s.generate_spd(42)
    say("begin")
    s.begin()
    for cnt in (G, 1, 2 * G):
        say("iterate", cnt)
        s.iterate(cnt, eps=-1.0)
        say("sync")
        s.synchronize()
    rn, bn = s.residual_norm()
    say("ok", rn / bn)
