#!/usr/bin/env python3
"""The reference's only published numbers are CG-method seconds at
N = 512 ... 8192 (fp32, the mean of 3 runs; results.xlsx Sheet2!C5:C9,
BASELINE.md §1).  This runs the same measurement with cg_hip: for each N,
generateSPDmatrix(N) written as the MATLAB script writes it, then
`cg_hip --fp32-ref --stats` three times, reading the program's own
"average clock execution time in seconds" line (the CG loop, as
serialConjugate.c:208,249-251 times it), next to the published serial
figure.  The x is the reference's bit for bit in this mode (checked against
the oracle here).  One GPU; the MPI rows of the table need the 8-GPU node.

  python tools/published_sizes.py [--out profiles/r02_published_sizes.json]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402

PUBLISHED_SERIAL_S = {512: 0.005, 1024: 0.016, 2048: 0.039, 4096: 0.186, 8192: 0.562}  # Sheet2!C5:C9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    rows = []
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for n, pub in PUBLISHED_SERIAL_S.items():
            A, b = oracle.spd_matlab(n, np.float64)
            paths = [os.path.join(td, f) for f in ("A.txt", "b.txt", "x0.txt")]
            for p, arr, dec in zip(paths, (A, b, np.zeros(n)), (4, 4, 1)):
                oracle.write_text(p, arr, dec)
            A32, b32 = oracle.spd_matlab(n, np.float32)
            xr, sr = oracle.cg_f32ref(A32, b32, np.zeros(n, np.float32), eps=1e-6)
            times = []
            for _ in range(a.runs):
                out = subprocess.run([cg.CLI_PATH, "--fp32-ref", "--stats", "--print-x", *paths], check=True,
                                     capture_output=True, text=True).stdout
                times.append(float(out.split("average clock execution time in seconds:")[1].split()[0]))
                x = np.array([float(v) for v in out.strip().splitlines()[-n:]], dtype=np.float32)
                assert np.array_equal(x.view(np.uint32), xr.view(np.uint32)), n
                assert f"iterations: {sr.iterations} converged: 1" in out
            mean = statistics.mean(times)
            rows.append({"n": n, "iterations": int(sr.iterations), "cg_hip_cg_time_s_runs": times,
                         "cg_hip_cg_time_s_mean": mean, "published_serial_cg_time_s": pub,
                         "ratio_published_over_cg_hip": pub / mean, "x_bit_identical_to_reference": True})
            print(json.dumps(rows[-1]), flush=True)
    res = {"what": "CG-method seconds at the reference's published sizes: cg_hip --fp32-ref (one MI355X, "
                   "the program's own timer, mean of 3 runs as the reference averages) vs the published serial "
                   "fp32 figure (Intel Xeon, results.xlsx Sheet2!C5:C9)", "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
