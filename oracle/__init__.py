"""CPU oracle for the CG hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package, and only as the checker (or as the timed CPU
baseline).  The product (``conjugate_gradient_amd`` / ``libcgx.so`` /
``cg_hip``) never imports it.

ctypes bindings over ``oracle/liboracle.so`` (built from ``cg_oracle.c`` by
``oracle/Makefile``), plus a pure-numpy restatement of ``conjgrad.m`` for small
cases.  What each function restates, with reference file:line citations, is in
``cg_oracle.h``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

# liboracle's OpenMP loops (generator, fp64 matVec): with the default active
# wait policy, idle team threads spin and the matVec ran SLOWER on 8 threads
# than on 1 in this container (2.3 vs 5.3 GB/s); passive waiting scales
# (43.7 GB/s on 8).  Read by libgomp when it is first loaded.
os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OracleStats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int64),
        ("converged", ctypes.c_int),
        ("rr", ctypes.c_double),
        ("t_init_s", ctypes.c_double),
        ("t_loop_s", ctypes.c_double),
    ]


def build() -> None:
    """Compile liboracle.so (and _ref/ when the reference is present)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        i64, f64, vp = ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
        L.oracle_mt_res53.argtypes = [ctypes.c_uint32, i64, vp]
        L.oracle_spd_matlab.argtypes = [i64, ctypes.c_int, vp, vp]
        L.oracle_spd_matlab.restype = ctypes.c_int
        L.oracle_spd_hash.argtypes = [i64, i64, i64, ctypes.c_uint64, ctypes.c_int, vp, vp]
        L.oracle_hash_u01.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_hash_u01.restype = f64
        L.oracle_matvec_f32ref.argtypes = [i64, i64, vp, vp, vp]
        L.oracle_dot_f32ref.argtypes = [i64, vp, vp]
        L.oracle_dot_f32ref.restype = ctypes.c_float
        L.oracle_matvec_f64.argtypes = [i64, i64, vp, vp, vp]
        L.oracle_dot_f64.argtypes = [i64, vp, vp]
        L.oracle_dot_f64.restype = f64
        L.oracle_cg_f32ref.argtypes = [i64, vp, vp, vp, i64, f64, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(OracleStats)]
        L.oracle_combine_f32.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.oracle_combine_f32.restype = ctypes.c_float
        L.oracle_cg_f32ref.restype = ctypes.c_int
        L.oracle_cg_f64.argtypes = [i64, vp, vp, vp, i64, f64, ctypes.POINTER(OracleStats)]
        L.oracle_cg_f64.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_hash_matvec_f64.argtypes = [i64, ctypes.c_uint64, i64, i64, vp, vp]
        L.oracle_write_text.argtypes = [ctypes.c_char_p, i64, vp, ctypes.c_int]
        L.oracle_write_text.restype = ctypes.c_int
        L.oracle_cg_f64_hash.argtypes = [i64, ctypes.c_uint64, vp, i64, f64, ctypes.POINTER(OracleStats)]
        L.oracle_cg_f64_hash.restype = ctypes.c_int
        L.oracle_poisson_apply.argtypes = [i64, vp, vp]
        L.oracle_cg_poisson_f64.argtypes = [i64, vp, vp, i64, f64, ctypes.POINTER(OracleStats)]
        L.oracle_cg_poisson_f64.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def set_threads(n: int) -> None:
    lib().oracle_set_threads(int(n))


def mt_res53(count: int, seed: int = 5489) -> np.ndarray:
    out = np.empty(count, dtype=np.float64)
    lib().oracle_mt_res53(seed, count, _p(out))
    return out


def spd_matlab(n: int, dtype=np.float32):
    """generateSPDmatrix(n) under `rng default`, through its %.4f text format."""
    dt = np.dtype(dtype)
    A = np.empty((n, n), dtype=dt)
    b = np.empty(n, dtype=dt)
    rc = lib().oracle_spd_matlab(n, 1 if dt == np.float32 else 0, _p(A), _p(b))
    if rc != 0:
        raise MemoryError("oracle_spd_matlab")
    return A, b


def spd_hash(n: int, seed: int = 42, dtype=np.float64, row0: int = 0, nrows: int | None = None):
    """Counter-hash SPD system rows [row0, row0+nrows)."""
    nrows = n - row0 if nrows is None else nrows
    dt = np.dtype(dtype)
    A = np.empty((nrows, n), dtype=dt)
    b = np.empty(nrows, dtype=dt)
    lib().oracle_spd_hash(n, row0, nrows, seed, 1 if dt == np.float32 else 0, _p(A), _p(b))
    return A, b


def hash_u01(seed: int, i: int, j: int) -> float:
    return lib().oracle_hash_u01(seed, i, j)


def matvec_f32ref(A: np.ndarray, v: np.ndarray) -> np.ndarray:
    A = np.ascontiguousarray(A, np.float32)
    v = np.ascontiguousarray(v, np.float32)
    out = np.empty(A.shape[0], np.float32)
    lib().oracle_matvec_f32ref(A.shape[0], A.shape[1], _p(A), _p(v), _p(out))
    return out


def dot_f32ref(a: np.ndarray, b: np.ndarray) -> np.float32:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return np.float32(lib().oracle_dot_f32ref(a.size, _p(a), _p(b)))


def matvec_f64(A: np.ndarray, v: np.ndarray) -> np.ndarray:
    A = np.ascontiguousarray(A, np.float64)
    v = np.ascontiguousarray(v, np.float64)
    out = np.empty(A.shape[0], np.float64)
    lib().oracle_matvec_f64(A.shape[0], A.shape[1], _p(A), _p(v), _p(out))
    return out


# How P row-block partials of a dot product are combined (cg_oracle.h):
#   "rank"  -- point-to-point_cg.c allSum (:339-359), sequential in rank order;
#   "mpich" -- parallel_cg.c's MPI_Allreduce (:287,294,313) as MPICH 3.3 does it
#              for one float: recursive doubling, a balanced pairwise tree.
COMBINE = {"rank": 0, "mpich": 1}


def combine_f32(parts, combine: str = "rank") -> np.float32:
    a = np.ascontiguousarray(parts, np.float32)
    return np.float32(lib().oracle_combine_f32(_p(a), a.size, COMBINE[combine]))


def cg_f32ref(A, b, x0, max_iter: int = -1, eps: float = 1e-6, nparts: int = 1, combine: str = "rank"):
    """serialConjugate.c conjugrad restated (nparts > 1: parallel_cg.c /
    point-to-point_cg.c on nparts ranks, partials combined in `combine`
    order); returns (x, OracleStats)."""
    A = np.ascontiguousarray(A, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    x = np.array(x0, dtype=np.float32, copy=True)
    st = OracleStats()
    rc = lib().oracle_cg_f32ref(b.size, _p(A), _p(b), _p(x), max_iter, eps, nparts, COMBINE[combine],
                                ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_cg_f32ref rc={rc}")
    return x, st


def cg_f64(A, b, x0, max_iter: int = -1, eps: float = 1e-10):
    """conjgrad.m restated in double; returns (x, OracleStats)."""
    A = np.ascontiguousarray(A, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    x = np.array(x0, dtype=np.float64, copy=True)
    st = OracleStats()
    rc = lib().oracle_cg_f64(b.size, _p(A), _p(b), _p(x), max_iter, eps, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_cg_f64 rc={rc}")
    return x, st


def hash_matvec_f64(n: int, v: np.ndarray, seed: int = 42, row0: int = 0, nrows: int | None = None) -> np.ndarray:
    """Rows [row0, row0+nrows) of spd_hash(n, seed)'s A times v, A regenerated on the fly."""
    nrows = n - row0 if nrows is None else nrows
    v = np.ascontiguousarray(v, np.float64)
    out = np.empty(nrows, np.float64)
    lib().oracle_hash_matvec_f64(n, seed, row0, nrows, _p(v), _p(out))
    return out


def cg_f64_hash(n: int, seed: int = 42, x0=None, max_iter: int = -1, eps: float = 1e-10):
    """conjgrad.m on spd_hash(n, seed) (A regenerated per matVec, no n*n memory);
    returns (x, OracleStats).  Same results as cg_f64(*spd_hash(n, seed))."""
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64, copy=True)
    st = OracleStats()
    rc = lib().oracle_cg_f64_hash(n, seed, _p(x), max_iter, eps, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_cg_f64_hash rc={rc}")
    return x, st


def write_text(path: str, values, decimals: int = 4) -> None:
    """One "%.<decimals>f" value per line (generateSPDmatrix.m's file format)."""
    v = np.ascontiguousarray(values, np.float64).ravel()
    if lib().oracle_write_text(path.encode(), v.size, _p(v), decimals) != 0:
        raise OSError(f"cannot write {path}")


def poisson_apply(m: int, p: np.ndarray) -> np.ndarray:
    p = np.ascontiguousarray(p, np.float64)
    out = np.empty(m * m, np.float64)
    lib().oracle_poisson_apply(m, _p(p), _p(out))
    return out


def cg_poisson_f64(m: int, b, x0, max_iter: int = -1, eps: float = 1e-10):
    """Matrix-free 5-point Poisson CG in double; returns (x, OracleStats)."""
    b = np.ascontiguousarray(b, np.float64)
    x = np.array(x0, dtype=np.float64, copy=True)
    st = OracleStats()
    rc = lib().oracle_cg_poisson_f64(m, _p(b), _p(x), max_iter, eps, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_cg_poisson_f64 rc={rc}")
    return x, st


def poisson_dense(m: int) -> np.ndarray:
    """The same operator as an explicit (m*m) x (m*m) matrix (small m only)."""
    n = m * m
    A = np.zeros((n, n))
    for i in range(m):
        for j in range(m):
            k = i * m + j
            A[k, k] = 4.0
            if i > 0:
                A[k, k - m] = -1.0
            if i < m - 1:
                A[k, k + m] = -1.0
            if j > 0:
                A[k, k - 1] = -1.0
            if j < m - 1:
                A[k, k + 1] = -1.0
    return A


def conjgrad_numpy(A, b, x, tol: float = 1e-10, max_iter: int | None = None):
    """conjgrad.m:1-18 line by line in numpy float64 (small cases only).
    Returns (x, iterations)."""
    A = np.asarray(A, np.float64)
    b = np.asarray(b, np.float64)
    x = np.array(x, np.float64, copy=True)
    r = b - A @ x                       # conjgrad.m:2
    p = r.copy()                        # :3
    rsold = r @ r                       # :4
    n = b.size if max_iter is None else max_iter
    it = 0
    for _ in range(n):                  # :6
        Ap = A @ p                      # :7
        alpha = rsold / (p @ Ap)        # :8
        x = x + alpha * p               # :9
        r = r - alpha * Ap              # :10
        rsnew = r @ r                   # :11
        it += 1
        if np.sqrt(rsnew) < tol:        # :12-14
            break
        p = r + (rsnew / rsold) * p     # :15
        rsold = rsnew                   # :16
    return x, it


def ref_binary() -> str | None:
    """Path of the reference build oracle/_ref/serial_ref, if built."""
    path = os.path.join(_HERE, "_ref", "serial_ref")
    return path if os.path.exists(path) else None
