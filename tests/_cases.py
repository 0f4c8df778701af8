"""Inputs of the golden cases (tests/golden/golden.json).

kat* come from the reference's own text fixtures (copied data under
tests/golden/ref_fixtures/); spd<n> are generateSPDmatrix(n) inputs regenerated
by the oracle's MATLAB-compatible generator.  Reading the fixtures with a
plain tokenizer here keeps the expected inputs independent of the product's
text reader (which is tested against these same files)."""
from __future__ import annotations

import functools
import os
import re

import numpy as np

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
FIX = os.path.join(GOLDEN, "ref_fixtures")
_NUM = re.compile(rb"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?")


def numbers(name: str, count: int, dtype=np.float32) -> np.ndarray:
    with open(os.path.join(FIX, name), "rb") as f:
        toks = _NUM.findall(f.read())[:count]
    assert len(toks) == count, name
    return np.array([float(t) for t in toks], dtype=dtype)


@functools.lru_cache(maxsize=8)
def _spd(n: int, dt: str):
    return oracle.spd_matlab(n, np.dtype(dt))


def case(name: str, dtype=np.float32):
    """(A, b, x0) of a golden case in `dtype` (values as the reference reads them)."""
    dt = np.dtype(dtype)
    if name == "kat2":
        return numbers("matrixA.txt", 4, dt).reshape(2, 2), numbers("vectorb.txt", 2, dt), numbers("initialguess.txt", 2, dt)
    if name == "kat2_x0":
        return numbers("matrixA.txt", 4, dt).reshape(2, 2), numbers("vectorb.txt", 2, dt), numbers("initialguess1.txt", 2, dt)
    if name == "kat4":
        return numbers("matrixA1.txt", 16, dt).reshape(4, 4), numbers("vectorb1.txt", 4, dt), numbers("X0.txt", 4, dt)
    if name.startswith("spd"):
        n = int(name[3:])
        A, b = _spd(n, dt.str)
        return A, b, np.zeros(n, dt)
    raise KeyError(name)


_HASH_ORACLE = {}


def hash_oracle(n: int, seed: int = 42):
    """conjgrad.m in fp64 on the bench's counter-hash system (seed 42), A
    regenerated row by row on 16 host threads (oracle_cg_f64_hash: no n*n
    memory, bit-identical to the stored form); computed once per session
    (shared by every test module that checks configs[2] / [3] at full size)."""
    if (n, seed) not in _HASH_ORACLE:
        oracle.set_threads(16)
        _HASH_ORACLE[(n, seed)] = oracle.cg_f64_hash(n, seed, eps=1e-10)
    return _HASH_ORACLE[(n, seed)]


def golden_x(golden: dict, name: str) -> np.ndarray:
    return np.load(os.path.join(GOLDEN, golden["cases"][name]["x_file"]), allow_pickle=False)


KATS = ["kat2", "kat2_x0", "kat4"]
SPD_SMALL = ["spd512", "spd1024", "spd2048"]
SPD_ALL = ["spd512", "spd1024", "spd2048", "spd4096", "spd8192"]


# ---- MPI goldens (tests/golden/mpi/, make_golden_mpi.py) -----------------------
# parallel_cg.c (MPI_Allreduce, MPICH order) and point-to-point_cg.c (allSum,
# rank order) run unmodified under mpiexec -np P on the cases above.
COMBINE_OF = {"parallel": "mpich", "p2p": "rank"}


@functools.lru_cache(maxsize=1)
def golden_mpi() -> dict:
    import json
    with open(os.path.join(GOLDEN, "mpi", "golden_mpi.json")) as f:
        return json.load(f)


def mpi_runs(min_np: int = 1, cases=None) -> list:
    """Keys of the MPI golden runs with np >= min_np (optionally of `cases`)."""
    return sorted(k for k, r in golden_mpi()["runs"].items()
                  if r["np"] >= min_np and (cases is None or r["case"] in cases))


def mpi_golden_x(key: str) -> np.ndarray:
    return np.load(os.path.join(GOLDEN, golden_mpi()["runs"][key]["x_file"]), allow_pickle=False)
