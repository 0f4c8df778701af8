#!/usr/bin/env python3
"""Generate tests/golden/mpi/ fixtures by running the UNMODIFIED reference MPI solvers.

Runs ``oracle/_ref/parallel_ref`` (/root/reference/parallel_cg.c: MPI_Allgather
of p, MPI_Allreduce of the two scalars) and ``oracle/_ref/p2p_ref``
(/root/reference/point-to-point_cg.c: allGather / allSum / BcastVector over
MPI_Send/Recv), both compiled from where they lie by ``oracle/Makefile``
(MPICH 3.3.2 ``mpicc``, only ``-Dmain=...`` and ``-fno-builtin-sqrt``; see
``oracle/ref/mpi_harness.c`` for how an n-row system is embedded in the
compiled-in ROWS=8192 with n/P real rows on every rank), under
``mpiexec -np P`` for P in 1, 2, 4, 8, on:

* the reference's 2x2 and 4x4 text fixtures (P dividing n);
* generateSPDmatrix(n) (MATLAB ``rng default``, "%.4f" text) at n = 512 ... 8192.

Writes ``mpi/golden_mpi.json`` (loop counts, input hashes) and
``mpi/x_<prog>_<case>_np<P>.npy`` (rank 0's float32 solution vector).

Usage:  python tests/golden/make_golden_mpi.py   (needs /root/reference and MPICH; ~2 min)
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import oracle  # noqa: E402
from make_golden import read_numbers  # noqa: E402

MPIEXEC = os.environ.get("MPIEXEC", "/opt/conda/bin/mpiexec")
OUT = os.path.join(HERE, "mpi")
PROGS = {
    "parallel": ("parallel_ref", "parallel_cg.c (MPI_Allgather + MPI_Allreduce, MPICH 3.3.2)"),
    "p2p": ("p2p_ref", "point-to-point_cg.c (MPI_Send/Recv allGather, allSum, BcastVector)"),
}


def run(prog: str, P: int, A, b, x0):
    exe = os.path.join(ROOT, "oracle", "_ref", PROGS[prog][0])
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} not built (make -C oracle, needs MPICH)")
    with tempfile.TemporaryDirectory() as td:
        paths = {k: os.path.join(td, k) for k in ("A", "b", "x0", "x")}
        np.ascontiguousarray(A, np.float32).tofile(paths["A"])
        np.ascontiguousarray(b, np.float32).tofile(paths["b"])
        np.ascontiguousarray(x0, np.float32).tofile(paths["x0"])
        out = subprocess.run([MPIEXEC, "-np", str(P), exe, str(b.size), paths["A"], paths["b"], paths["x0"],
                              paths["x"]], check=True, capture_output=True, text=True, timeout=600).stdout
        x = np.fromfile(paths["x"], dtype=np.float32)
    return x, int(re.search(r"iterations (\d+)", out).group(1))


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    fx = os.path.join(HERE, "ref_fixtures")
    A2 = read_numbers(os.path.join(fx, "matrixA.txt"), 4).reshape(2, 2)
    b2 = read_numbers(os.path.join(fx, "vectorb.txt"), 2)
    A4 = read_numbers(os.path.join(fx, "matrixA1.txt"), 16).reshape(4, 4)
    inputs = [
        ("kat2", lambda: (A2, b2, read_numbers(os.path.join(fx, "initialguess.txt"), 2))),
        ("kat2_x0", lambda: (A2, b2, read_numbers(os.path.join(fx, "initialguess1.txt"), 2))),
        ("kat4", lambda: (A4, read_numbers(os.path.join(fx, "vectorb1.txt"), 4),
                          read_numbers(os.path.join(fx, "X0.txt"), 4))),
    ]
    for n in (512, 1024, 2048, 4096, 8192):
        inputs.append((f"spd{n}", lambda n=n: (*oracle.spd_matlab(n, np.float32), np.zeros(n, np.float32))))

    runs = {}
    for name, make in inputs:
        A, b, x0 = make()
        n = b.size
        for P in (1, 2, 4, 8):
            if n % P:
                continue
            for prog in PROGS:
                x, iters = run(prog, P, A, b, x0)
                key = f"{prog}_{name}_np{P}"
                np.save(os.path.join(OUT, f"x_{key}.npy"), x, allow_pickle=False)
                runs[key] = {
                    "program": prog, "case": name, "np": P, "n": int(n),
                    "ref_iterations": iters,
                    "A_sha256": hashlib.sha256(np.ascontiguousarray(A, np.float32).tobytes()).hexdigest(),
                    "x_file": f"mpi/x_{key}.npy",
                }
                print(f"{key:28s} iters={iters} x[:3]={x[:3]}", flush=True)
        del A
    meta = {
        "generator": "tests/golden/make_golden_mpi.py",
        "programs": {k: v[1] for k, v in PROGS.items()},
        "harness": "oracle/ref/mpi_harness.c (n/P real rows per rank inside ROWS=8192)",
        "mpi": "MPICH 3.3.2 ch3:nemesis, mpiexec on one host",
        "EPSILON": 1e-6,
        "runs": runs,
    }
    with open(os.path.join(OUT, "golden_mpi.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
