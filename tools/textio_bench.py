#!/usr/bin/env python3
"""Text I/O: cgx_text_read vs the reference's own
initialize() (serialConjugate.c:85-105, fscanf "%f%*c"), on a
generateSPDmatrix(n)-format matrixA file (one "%.4f" value per line).

The reference function is called from the unmodified serialConjugate.c object
through oracle/_ref/serial_ref --initialize (this container only: the
reference does not travel).  Values must agree bit for bit (float).

  python tools/textio_bench.py [--n 8192] [--threads 1,4,8] [--reps 3] [--out profiles/r01_textio_n8192.json]

Each thread count is timed --reps times after one warm-up read (median reported).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--threads", default="1,4,8")
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3, help="runs per thread count (the median is reported)")
    args = ap.parse_args()
    n = args.n
    exe = oracle.ref_binary()
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "matrixA.txt")
        A, _ = oracle.spd_matlab(n, np.float64)  # the values generateSPDmatrix.m writes
        t0 = time.perf_counter()
        A.ravel().tofile(path, sep="\n", format="%.4f")
        with open(path, "a") as f:
            f.write("\n")
        t_write = time.perf_counter() - t0
        del A
        size = os.path.getsize(path)
        res = {"n": n, "file_bytes": size, "values": n * n, "write_s": t_write, "host_cpus": os.cpu_count()}
        ours = {}
        cg.read_text(path, n * n, np.float32, threads=1)  # warm the page cache and the mapping path
        for t in map(int, args.threads.split(",")):
            times = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                v = cg.read_text(path, n * n, np.float32, threads=t)
                times.append(time.perf_counter() - t0)
            dt = sorted(times)[len(times) // 2]
            ours[t] = v
            res[f"cgx_text_read_t{t}_s"] = dt
            res[f"cgx_text_read_t{t}_s_all"] = times
            res[f"cgx_text_read_t{t}_MBps"] = size / dt / 1e6
        for t in ours:
            assert np.array_equal(ours[t], next(iter(ours.values())))
        if exe and n <= 8192:
            refout = os.path.join(td, "ref.f32")
            # the reference reads ROWS*col_num values with ROWS fixed at 8192
            if n == 8192:
                out = subprocess.run([exe, "--initialize", path, str(n), refout], check=True,
                                     capture_output=True, text=True).stdout
                t_ref = float(out.split()[-1])
                refv = np.fromfile(refout, dtype=np.float32)
                res["reference_initialize_s"] = t_ref
                res["reference_initialize_MBps"] = size / t_ref / 1e6
                res["bit_identical_to_reference"] = bool(np.array_equal(refv.view(np.uint32),
                                                                        next(iter(ours.values())).view(np.uint32)))
                for t in ours:
                    res[f"speedup_t{t}"] = t_ref / res[f"cgx_text_read_t{t}_s"]
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
