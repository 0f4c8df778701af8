#!/usr/bin/env python3
"""Run a script against another build of libcgx (A/B of a kernel change in
one GPU session): python tools/ab_lib.py ab/libcgx_head.so bench.py --workload symmetric ...
The other build must export the same C ABI (include/cgx.h)."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

cg.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
