#!/usr/bin/env python3
"""The reference's only published numbers are CG-method seconds at
N = 512 ... 8192 (fp32, the mean of 3 runs; results.xlsx Sheet2!C5:C9,
BASELINE.md §1).  This runs the same measurement with cg_hip: for each N,
generateSPDmatrix(N) written as the MATLAB script writes it, then
`cg_hip --fp32-ref --stats` three times, reading the program's own
"average clock execution time in seconds" line (the CG loop, as
serialConjugate.c:208,249-251 times it), next to the published serial
figure.  The x is the reference's bit for bit in this mode (checked against
the oracle here).

--mpi: the table's MPI rows (N = 4096 / 8192, P = 2 / 4 / 8, collective
parallel_cg.c and point-to-point_cg.c) with the one-process
drop-in `cg_hip --gpus P [--p2p] --fp32-ref`: P row blocks, here all on ONE
GPU, against the reference's P MPI ranks on CPU cores.  The program's own
"cg method execution time" line (parallel_cg.c times conjugrad the same way),
mean of 3 runs; x bit for bit the unmodified MPI program's under mpiexec -np
P (tests/golden/mpi/).  P GPUs would split the per-block work P ways; here
the blocks share one, so this is the study's structure on one device, not its
scaling.

  python tools/published_sizes.py [--mpi] [--out profiles/rNN_published_sizes.json]
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
# collective Sheet2!E25/I25/M25 (N=4096), E26/I26/M26 (8192);
# point-to-point Sheet2!E8/I8/M8, E9/I9/M9
PUBLISHED_MPI_S = {("parallel", 4096): {2: 0.176, 4: 0.117, 8: 0.062},
                   ("parallel", 8192): {2: 0.685, 4: 0.457, 8: 0.234},
                   ("p2p", 4096): {2: 0.182, 4: 0.121, 8: 0.065},
                   ("p2p", 8192): {2: 0.707, 4: 0.36, 8: 0.244}}
GOLDEN_MPI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "mpi")


def mpi_rows(runs):
    """The MPI rows: cg_hip --gpus P [--p2p] --fp32-ref on the same files."""
    with open(os.path.join(GOLDEN_MPI, "golden_mpi.json")) as f:
        gold = json.load(f)["runs"]
    rows = []
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for n in (4096, 8192):
            A, b = oracle.spd_matlab(n, np.float64)
            paths = [os.path.join(td, f) for f in ("A.txt", "b.txt", "x0.txt")]
            for p, arr, dec in zip(paths, (A, b, np.zeros(n)), (4, 4, 1)):
                oracle.write_text(p, arr, dec)
            for program in ("parallel", "p2p"):
                for P, pub in PUBLISHED_MPI_S[(program, n)].items():
                    key = f"{program}_spd{n}_np{P}"
                    xg = np.load(os.path.join(os.path.dirname(GOLDEN_MPI), gold[key]["x_file"]), allow_pickle=False)
                    times = []
                    for _ in range(runs):
                        cmd = [cg.CLI_PATH, "--gpus", str(P), "--fp32-ref", "--stats", "--print-x", *paths]
                        if program == "p2p":
                            cmd.insert(3, "--p2p")
                        out = subprocess.run(cmd, check=True, capture_output=True, text=True,
                                             env=dict(os.environ, HIP_VISIBLE_DEVICES="0")).stdout
                        times.append(float(out.split("cg method execution time in seconds:")[1].split()[0]))
                        x = np.array([float(v) for v in out.strip().splitlines()[-n:]], dtype=np.float32)
                        assert np.array_equal(x.view(np.uint32), xg.view(np.uint32)), key
                        assert f"iterations: {gold[key]['ref_iterations']} converged: 1" in out, key
                    mean = statistics.mean(times)
                    rows.append({"n": n, "program": program, "P": P, "iterations": gold[key]["ref_iterations"],
                                 "cg_hip_cg_time_s_runs": times, "cg_hip_cg_time_s_mean": mean,
                                 "published_mpi_cg_time_s": pub, "ratio_published_over_cg_hip": pub / mean,
                                 "x_bit_identical_to_reference": True})
                    print(json.dumps(rows[-1]), flush=True)
    return {"what": "the reference's MPI rows (results.xlsx Sheet2, BASELINE.md s1): cg_hip --gpus P [--p2p] "
                    "--fp32-ref, P row blocks in one process ALL ON ONE MI355X (the program's own cg-method timer, "
                    "mean of 3 runs), against the published P MPI ranks on Intel Xeon cores; x bit for bit "
                    "mpiexec -np P of the unmodified program", "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--mpi", action="store_true", help="the MPI rows (P row blocks on one GPU)")
    a = ap.parse_args()
    if a.mpi:
        res = mpi_rows(a.runs)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
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
                                     capture_output=True, text=True, env=dict(os.environ, HIP_VISIBLE_DEVICES="0")).stdout
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
