"""conjugate_gradient_amd -- MI355X-native conjugate-gradient hot path.

Python mirror of the reference's solver interface over the C ABI of
``lib/libcgx.so`` (declared in ``include/cgx.h``).  The reference
(mawunyega/conjugate_gradient) is a set of C programs; the functions a user
of that code calls are reproduced here with the same names and argument
meaning so the parity tests read like the reference's own call sites:

=====================  ==============================================  =========================
reference               where                                           here
=====================  ==============================================  =========================
``conjugrad(A,b,x)``    serialConjugate.c:180-259                       :func:`conjugrad`
``conjugrad(..., P)``   parallel_cg.c:248-345 (row blocks, P ranks)     :func:`conjugrad` (shards)
``matVec``              serialConjugate.c:109-120                       :func:`matVec`
``vecVec``              serialConjugate.c:145-155                       :func:`vecVec`
``residual``            serialConjugate.c:124-131                       :func:`residual`
``scalarVec+vecAdd``    serialConjugate.c:221-243                       :func:`update_xr`,
                                                                        :func:`update_p`
``initialize``          serialConjugate.c:85-105                        :func:`read_text`
=====================  ==============================================  =========================

Everything runs on the GPU through libcgx.so; there is no CPU fallback.  If
the library is missing or no GPU is visible the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

__all__ = [
    "CGX_F64", "CGX_F32_REF", "CGX_TIMING", "CGX_HOST_STREAM", "CGX_NO_OVERLAP", "CGX_COMM_P2P", "CGX_SYMMETRIC",
    "CGX_PHASES", "CGX_PEER_ACTIVE", "CGX_SMALL_ACTIVE", "CGX_FOLD_ACTIVE", "CGX_XDEFER_ACTIVE", "CGX_XDEFER3_ACTIVE",
    "CGX_PULL_ACTIVE", "CGX_FOLDED_ACTIVE", "CGX_HALO_PULL_ACTIVE", "CGX_THREADS_ACTIVE", "CGX_HALO_OVERLAP_ACTIVE",
    "PHASE_NAMES", "overlap_rule", "CgxError", "Stats",
    "Solver", "lib", "build",
    "device_pci_bus_id", "device_link",
    "conjugrad", "matVec", "vecVec", "residual", "update_xr", "update_p", "read_text",
    "count_text", "read_dims", "device_count", "get_unique_id", "DeviceArray",
]

CGX_F64 = 0x0
CGX_F32_REF = 0x1
CGX_TIMING = 0x100
CGX_HOST_STREAM = 0x200
CGX_NO_OVERLAP = 0x400
CGX_OVERLAP_ACTIVE = 0x800
CGX_FUSED_ACTIVE = 0x2000
CGX_DETERMINISTIC = 0x4000
CGX_COMM_P2P = 0x1000
CGX_SYMMETRIC = 0x8000
CGX_PHASES = 0x10000
CGX_PEER_ACTIVE = 0x20000
CGX_SMALL_ACTIVE = 0x40000
CGX_FOLD_ACTIVE = 0x80000
CGX_XDEFER_ACTIVE = 0x100000
CGX_XDEFER3_ACTIVE = 0x200000
CGX_PULL_ACTIVE = 0x400000
CGX_FOLDED_ACTIVE = 0x800000
CGX_HALO_PULL_ACTIVE = 0x1000000
CGX_THREADS_ACTIVE = 0x2000000
CGX_HALO_OVERLAP_ACTIVE = 0x4000000

# cgx_phase_times indices (include/cgx.h), in the order the phases tile an iteration
PHASE_NAMES = ("matvec_own", "gather_exposed", "matvec", "combine_pap", "update_r", "combine_rr", "update_xp",
               "gap", "iteration", "matvec_busy")

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libcgx.so")
CLI_PATH = os.path.join(_HERE, "bin", "cg_hip")
_LIB = None


class CgxError(RuntimeError):
    def __init__(self, code: int, what: str):
        L = lib()
        msg = L.cgx_strerror(code).decode()
        detail = L.cgx_last_error().decode()
        super().__init__(f"{what}: {msg} ({detail})" if detail else f"{what}: {msg}")
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int64),
        ("converged", ctypes.c_int),
        ("rr", ctypes.c_double),
        ("solve_ms", ctypes.c_double),
        ("matvec_ms", ctypes.c_double),
        ("matvec_count", ctypes.c_int64),
        ("total_iterations", ctypes.c_int64),
    ]


class Info(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64), ("lda", ctypes.c_int64), ("nranks", ctypes.c_int),
        ("nshards", ctypes.c_int), ("rank0", ctypes.c_int), ("row0", ctypes.c_int64),
        ("nrows", ctypes.c_int64), ("flags", ctypes.c_int), ("elem_bytes", ctypes.c_int),
    ]


class PhaseTimes(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_int64 * 10), ("median_us", ctypes.c_double * 10),
                ("mean_us", ctypes.c_double * 10)]


class CommInfo(ctypes.Structure):
    _fields_ = [("rccl_nranks", ctypes.c_int), ("rccl_device", ctypes.c_int), ("rccl_rank", ctypes.c_int),
                ("device", ctypes.c_int), ("pci_bus_id", ctypes.c_char * 32)]


class OverlapInfo(ctypes.Structure):
    _fields_ = [("active", ctypes.c_int), ("decided_by", ctypes.c_int), ("allgather_us", ctypes.c_double),
                ("split_us", ctypes.c_double), ("one_launch_us", ctypes.c_double), ("split_cost_us", ctypes.c_double),
                ("overlap_form_us", ctypes.c_double), ("plain_form_us", ctypes.c_double), ("margin", ctypes.c_double),
                ("forms_ms", ctypes.c_double)]


# cgx_overlap_info.decided_by
OVERLAP_DECIDED_BY = {0: "measured", 1: "forced_on", 2: "off", 3: "n/a"}


def overlap_rule(info: dict) -> bool:
    """The library's decision rule on an overlap_info() dict (measured case):
    the overlapped form when it beat the plain form by more than the margin."""
    return info["overlap_form_us"] < (1.0 - info["margin"]) * info["plain_form_us"]


class UniqueId(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_char * 128)]


def build() -> None:
    """Compile libcgx.so and cg_hip for gfx950 (hipcc; works without a GPU)."""
    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)


def lib() -> ctypes.CDLL:
    """Load libcgx.so; raises if it has not been built (no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `make -C conjugate_gradient_amd/csrc` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    i64, i32, f64, vp, sz = ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t
    pctx = ctypes.POINTER(ctypes.c_void_p)
    sigs = {
        "cgx_strerror": ([i32], ctypes.c_char_p),
        "cgx_last_error": ([], ctypes.c_char_p),
        "cgx_version": ([], i32),
        "cgx_device_count": ([ctypes.POINTER(i32)], i32),
        "cgx_hip_last_error": ([], i32),
        "cgx_device_pci_bus_id": ([i32, ctypes.c_char_p, i32], i32),
        "cgx_device_link": ([i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "cgx_get_comm_info": ([vp, ctypes.POINTER(CommInfo)], i32),
        "cgx_get_overlap_info": ([vp, ctypes.POINTER(OverlapInfo)], i32),
        "cgx_get_phase_times": ([vp, ctypes.POINTER(PhaseTimes)], i32),
        "cgx_create": ([pctx, i64, i32, i32], i32),
        "cgx_create_multi": ([pctx, i64, i32, ctypes.POINTER(i32), i32], i32),
        "cgx_get_unique_id": ([ctypes.POINTER(UniqueId)], i32),
        "cgx_rccl_available": ([], i32),
        "cgx_create_rank": ([pctx, i64, i32, i32, ctypes.POINTER(UniqueId), i32, i32], i32),
        "cgx_create_poisson": ([pctx, i64, i32, i32], i32),
        "cgx_create_poisson_multi": ([pctx, i64, i32, ctypes.POINTER(i32), i32], i32),
        "cgx_create_poisson_rank": ([pctx, i64, i32, i32, ctypes.POINTER(UniqueId), i32, i32], i32),
        "cgx_fill": ([vp, f64, f64], i32),
        "cgx_destroy": ([vp], i32),
        "cgx_get_info": ([vp, ctypes.POINTER(Info)], i32),
        "cgx_set_rows": ([vp, i64, i64, vp, i64, vp, vp], i32),
        "cgx_set_system": ([vp, vp, vp, vp], i32),
        "cgx_generate_spd": ([vp, ctypes.c_uint64], i32),
        "cgx_get_x": ([vp, vp], i32),
        "cgx_set_x": ([vp, vp], i32),
        "cgx_solve": ([vp, vp, f64, i64, ctypes.POINTER(Stats)], i32),
        "cgx_solve_begin": ([vp], i32),
        "cgx_conjugrad": ([vp, vp, vp, i64, i32, f64, i64, ctypes.POINTER(Stats)], i32),
        "cgx_iterate": ([vp, i64, f64, ctypes.POINTER(i64), ctypes.POINTER(i32)], i32),
        "cgx_get_stats": ([vp, ctypes.POINTER(Stats)], i32),
        "cgx_reset_timing": ([vp], i32),
        "cgx_synchronize": ([vp], i32),
        "cgx_stream": ([vp], vp),
        "cgx_residual_norm": ([vp, ctypes.POINTER(f64), ctypes.POINTER(f64)], i32),
        "cgx_set_matvec_plan": ([vp, i32, i32, i32, i32], i32),
        "cgx_get_matvec_plan": ([vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32),
                                 ctypes.POINTER(i32)], i32),
        "cgx_dev_malloc": ([ctypes.POINTER(vp), sz], i32),
        "cgx_dev_free": ([vp], i32),
        "cgx_memcpy_h2d": ([vp, vp, sz], i32),
        "cgx_memcpy_d2h": ([vp, vp, sz], i32),
        "cgx_dev_synchronize": ([], i32),
        "cgx_matvec": ([i32, vp, i64, i64, i64, vp, vp, vp], i32),
        "cgx_dot": ([i32, i64, vp, vp, vp, vp], i32),
        "cgx_residual": ([i32, i64, vp, vp, vp, vp, vp, vp], i32),
        "cgx_update_xr": ([i32, i64, vp, vp, vp, vp, vp, vp, vp, vp], i32),
        "cgx_update_p": ([i32, i64, vp, vp, vp, vp, vp], i32),
        "cgx_text_count": ([ctypes.c_char_p], i64),
        "cgx_text_read": ([ctypes.c_char_p, i64, i32, vp, i32], i32),
        "cgx_text_dims": ([ctypes.c_char_p, ctypes.POINTER(i64)], i32),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _LIB = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise CgxError(rc, what)


def _ptr(a: np.ndarray) -> int:
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data


def _dtype(flags: int) -> np.dtype:
    return np.dtype(np.float32) if flags & CGX_F32_REF else np.dtype(np.float64)


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().cgx_device_count(ctypes.byref(n)), "cgx_device_count")
    return n.value


def device_pci_bus_id(device: int) -> str:
    buf = ctypes.create_string_buffer(32)
    _check(lib().cgx_device_pci_bus_id(device, buf, 32), "cgx_device_pci_bus_id")
    return buf.value.decode()


def device_link(a: int, b: int) -> dict:
    """The link between two visible devices: HSA link type (4 = xGMI, 2 = PCIe,
    -1 unknown), hop count, and whether a can access b's memory directly."""
    lt, hops, peer = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().cgx_device_link(a, b, ctypes.byref(lt), ctypes.byref(hops), ctypes.byref(peer)), "cgx_device_link")
    names = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
    return {"link": names.get(lt.value, "unknown" if lt.value < 0 else str(lt.value)), "hops": hops.value,
            "peer_access": bool(peer.value)}


def get_unique_id() -> bytes:
    """RCCL bootstrap id for cgx_create_rank (call on rank 0, broadcast)."""
    u = UniqueId()
    _check(lib().cgx_get_unique_id(ctypes.byref(u)), "cgx_get_unique_id")
    return ctypes.string_at(ctypes.addressof(u), 128)  # may contain NULs


# ----------------------------------------------------------------------------
# text I/O (initialize(), serialConjugate.c:85-105)
# ----------------------------------------------------------------------------
def count_text(path: str) -> int:
    c = lib().cgx_text_count(path.encode())
    if c < 0:
        raise FileNotFoundError(path)
    return int(c)


def read_text(path: str, count: int, dtype=np.float64, threads: int = 4) -> np.ndarray:
    dt = np.dtype(dtype)
    out = np.empty(count, dtype=dt)
    rc = lib().cgx_text_read(path.encode(), count, 1 if dt == np.float32 else 0, _ptr(out), threads)
    if rc == -1:
        raise FileNotFoundError(path)
    if rc == -2:
        raise ValueError(f"{path}: fewer than {count} numbers")
    if rc != 0:
        raise ValueError(f"{path}: malformed number")
    return out


def read_dims(path: str) -> tuple[int, int, int, int]:
    d = (ctypes.c_int64 * 4)()
    rc = lib().cgx_text_dims(path.encode(), d)
    if rc != 0:
        raise ValueError(f"{path}: cannot read dimensions (rc={rc})")
    return tuple(int(v) for v in d)


# ----------------------------------------------------------------------------
# device arrays (for the kernel-level entry points)
# ----------------------------------------------------------------------------
class DeviceArray:
    """A device buffer owned by libcgx (hipMalloc), with host copy helpers."""

    def __init__(self, count: int, dtype=np.float64):
        self.dtype = np.dtype(dtype)
        self.count = int(count)
        p = ctypes.c_void_p()
        _check(lib().cgx_dev_malloc(ctypes.byref(p), max(1, self.count) * self.dtype.itemsize), "cgx_dev_malloc")
        self.ptr = p.value

    @classmethod
    def from_host(cls, a: np.ndarray, dtype=None) -> "DeviceArray":
        a = np.ascontiguousarray(a, dtype=dtype or a.dtype)
        d = cls(a.size, a.dtype)
        if a.size:
            _check(lib().cgx_memcpy_h2d(d.ptr, _ptr(a), a.nbytes), "cgx_memcpy_h2d")
        return d

    def to_host(self) -> np.ndarray:
        out = np.empty(self.count, self.dtype)
        if self.count:
            _check(lib().cgx_dev_synchronize(), "cgx_dev_synchronize")
            _check(lib().cgx_memcpy_d2h(_ptr(out), self.ptr, out.nbytes), "cgx_memcpy_d2h")
        return out

    def free(self) -> None:
        if self.ptr:
            lib().cgx_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _dt_flag(dtype) -> int:
    return CGX_F32_REF if np.dtype(dtype) == np.float32 else CGX_F64


def _need(cond: bool, msg: str) -> None:
    """Explicit size check before a C call (not `assert`: python -O strips it;
    a short buffer passed on would be read or written past its end)."""
    if not cond:
        raise ValueError(msg)


def _fits(arrs, n: int, what: str) -> None:
    for a in arrs:
        if a is not None:
            _need(a.count >= n, f"{what}: device array of {a.count} elements, {n} needed")


def matVec(A: DeviceArray, v: DeviceArray, out: DeviceArray, rows: int, cols: int, lda: int | None = None) -> None:
    """serialConjugate.c:109-120 / parallel_cg.c:172-184 (rows = local_row)."""
    lda = lda or cols
    _need(rows >= 0 and cols >= 0 and lda >= cols, "matVec: need rows, cols >= 0 and lda >= cols")
    if rows and cols:
        _fits([A], (rows - 1) * lda + cols, "matVec A")
        _fits([v], cols, "matVec v")
        _fits([out], rows, "matVec out")
    _check(lib().cgx_matvec(_dt_flag(A.dtype), A.ptr, lda or cols, rows, cols, v.ptr, out.ptr, None), "cgx_matvec")


def vecVec(a: DeviceArray, b: DeviceArray, out: DeviceArray, n: int | None = None) -> None:
    """serialConjugate.c:145-155: out[0] = a . b (device scalar)."""
    n = n if n is not None else a.count
    _fits([a, b], n, "vecVec")
    _fits([out], 1, "vecVec out")
    _check(lib().cgx_dot(_dt_flag(a.dtype), n, a.ptr, b.ptr, out.ptr, None), "cgx_dot")


def residual(b, Ax, r, p, rr=None, n=None) -> None:
    """serialConjugate.c:210-212: r = p = b - Ax; rr[0] = r . r."""
    n = n if n is not None else b.count
    _fits([b, Ax, r, p], n, "residual")
    _fits([rr], 1, "residual rr")
    _check(lib().cgx_residual(_dt_flag(b.dtype), n, b.ptr, Ax.ptr, r.ptr, p.ptr,
                              rr.ptr if rr is not None else None, None), "cgx_residual")


def update_xr(x, r, p, Ap, rsold, pAp, rr, n=None) -> None:
    """serialConjugate.c:219-234: alpha = rsold/pAp; x += alpha p; r -= alpha Ap; rr = r.r."""
    n = n if n is not None else x.count
    _fits([x, r, p, Ap], n, "update_xr")
    _fits([rsold, pAp, rr], 1, "update_xr scalars")
    _check(lib().cgx_update_xr(_dt_flag(x.dtype), n, x.ptr, r.ptr, p.ptr, Ap.ptr,
                               rsold.ptr, pAp.ptr, rr.ptr, None), "cgx_update_xr")


def update_p(p, r, rr, rsold, n=None) -> None:
    """serialConjugate.c:239-243: p = r + (rr/rsold) p."""
    n = n if n is not None else p.count
    _fits([p, r], n, "update_p")
    _fits([rr, rsold], 1, "update_p scalars")
    _check(lib().cgx_update_p(_dt_flag(p.dtype), n, p.ptr, r.ptr, rr.ptr, rsold.ptr,
                              None), "cgx_update_p")


# ----------------------------------------------------------------------------
# the solver
# ----------------------------------------------------------------------------
class Solver:
    """A CG context: one GPU, several row-block shards in this process, or one
    rank of a one-process-per-GPU job (RCCL)."""

    def __init__(self, n: int, *, flags: int = CGX_F64, device: int = 0, devices=None,
                 rank: int | None = None, nranks: int | None = None, unique_id: bytes | None = None,
                 poisson_m: int | None = None):
        """Dense n x n system, or (poisson_m=m) the matrix-free 5-point Poisson
        operator on an m x m grid (n must then be m*m or None)."""
        L = lib()
        self.poisson_m = poisson_m
        if poisson_m is not None:
            n = poisson_m * poisson_m
        self.n = int(n)
        self.flags = flags
        self.dtype = _dtype(flags)
        h = ctypes.c_void_p()
        if poisson_m is not None:
            if rank is not None:
                u = UniqueId()
                ctypes.memmove(ctypes.addressof(u), unique_id, 128)
                rc = L.cgx_create_poisson_rank(ctypes.byref(h), poisson_m, rank, nranks, ctypes.byref(u), device, flags)
            elif devices is not None:
                arr = (ctypes.c_int * len(devices))(*devices)
                rc = L.cgx_create_poisson_multi(ctypes.byref(h), poisson_m, len(devices), arr, flags)
            else:
                rc = L.cgx_create_poisson(ctypes.byref(h), poisson_m, device, flags)
        elif rank is not None:
            u = UniqueId()
            if unique_id is None or len(unique_id) != 128:
                raise ValueError("unique_id must be the 128 bytes from get_unique_id()")
            ctypes.memmove(ctypes.addressof(u), unique_id, 128)
            rc = L.cgx_create_rank(ctypes.byref(h), self.n, rank, nranks, ctypes.byref(u), device, flags)
        elif devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = L.cgx_create_multi(ctypes.byref(h), self.n, len(devices), arr, flags)
        else:
            rc = L.cgx_create(ctypes.byref(h), self.n, device, flags)
        _check(rc, "cgx_create")
        self._h = h.value

    # lifetime
    def close(self) -> None:
        """cgx_destroy.  In rank mode it first drains the streams with the RCCL
        deadline; an error there (a peer died) is raised after the free."""
        if getattr(self, "_h", None):
            rc = lib().cgx_destroy(self._h)
            self._h = None
            _check(rc, "cgx_destroy")

    def __enter__(self):
        return self

    def __exit__(self, exc_type, *exc):
        if exc_type is None:
            self.close()
        else:  # keep the original error; the free still happens
            try:
                self.close()
            except CgxError:
                pass

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def info(self) -> Info:
        i = Info()
        _check(lib().cgx_get_info(self._h, ctypes.byref(i)), "cgx_get_info")
        return i

    # data
    def set_system(self, A: np.ndarray, b: np.ndarray, x0: np.ndarray | None = None) -> None:
        A = np.ascontiguousarray(A, self.dtype)
        b = np.ascontiguousarray(b, self.dtype)
        x0 = np.zeros(self.n, self.dtype) if x0 is None else np.ascontiguousarray(x0, self.dtype)
        _need(A.shape == (self.n, self.n), f"set_system: A has shape {A.shape}, ({self.n}, {self.n}) needed")
        _need(b.shape == (self.n,), f"set_system: b has shape {b.shape}, ({self.n},) needed")
        _need(x0.shape == (self.n,), f"set_system: x0 has shape {x0.shape}, ({self.n},) needed")
        _check(lib().cgx_set_system(self._h, _ptr(A), _ptr(b), _ptr(x0)), "cgx_set_system")

    def set_rows(self, row0: int, A_rows=None, b_rows=None, x_rows=None) -> None:
        arrs = [None if a is None else np.ascontiguousarray(a, self.dtype) for a in (A_rows, b_rows, x_rows)]
        _need(any(a is not None for a in arrs), "set_rows: nothing to set")
        nrows = next(a.shape[0] for a in arrs if a is not None)
        if arrs[0] is not None:
            _need(arrs[0].ndim == 2 and arrs[0].shape[1] >= self.n,
                  f"set_rows: A_rows has shape {arrs[0].shape}, (nrows, >= {self.n}) needed")
        for a, name in zip(arrs, ("A_rows", "b_rows", "x_rows")):
            if a is not None:
                _need(a.shape[0] == nrows and (a.ndim == 2 if name == "A_rows" else a.ndim == 1),
                      f"set_rows: {name} has shape {a.shape}; every argument needs the same {nrows} rows")
        _need(0 <= row0 and row0 + nrows <= self.n, f"set_rows: rows [{row0}, {row0 + nrows}) outside [0, {self.n})")
        lda = arrs[0].shape[1] if arrs[0] is not None else self.n
        _check(lib().cgx_set_rows(self._h, row0, nrows, *(None if a is None else _ptr(a) for a in arrs[:1]), lda,
                                  *(None if a is None else _ptr(a) for a in arrs[1:])), "cgx_set_rows")

    def fill(self, b_value: float, x_value: float = 0.0) -> None:
        _check(lib().cgx_fill(self._h, b_value, x_value), "cgx_fill")

    def generate_spd(self, seed: int = 42) -> None:
        _check(lib().cgx_generate_spd(self._h, seed), "cgx_generate_spd")

    def get_x(self) -> np.ndarray:
        x = np.empty(self.n, self.dtype)
        _check(lib().cgx_get_x(self._h, _ptr(x)), "cgx_get_x")
        return x

    def set_x(self, x: np.ndarray) -> None:
        x = np.ascontiguousarray(x, self.dtype)
        _need(x.shape == (self.n,), f"set_x: x has shape {x.shape}, ({self.n},) needed")
        _check(lib().cgx_set_x(self._h, _ptr(x)), "cgx_set_x")

    # solve
    def solve(self, x0: np.ndarray | None = None, eps: float = 1e-6, max_iter: int = -1) -> tuple[np.ndarray, Stats]:
        st = Stats()
        if x0 is not None:
            x = np.array(x0, dtype=self.dtype, copy=True)
            _need(x.shape == (self.n,), f"solve: x0 has shape {x.shape}, ({self.n},) needed")
            _check(lib().cgx_solve(self._h, _ptr(x), eps, max_iter, ctypes.byref(st)), "cgx_solve")
        else:
            _check(lib().cgx_solve(self._h, None, eps, max_iter, ctypes.byref(st)), "cgx_solve")
            x = self.get_x()
        return x, st

    def begin(self) -> None:
        _check(lib().cgx_solve_begin(self._h), "cgx_solve_begin")

    def iterate(self, count: int, eps: float = -1.0) -> tuple[int, bool]:
        done = ctypes.c_int64(0)
        conv = ctypes.c_int(0)
        _check(lib().cgx_iterate(self._h, count, eps, ctypes.byref(done), ctypes.byref(conv)), "cgx_iterate")
        return done.value, bool(conv.value)

    def stats(self) -> Stats:
        st = Stats()
        _check(lib().cgx_get_stats(self._h, ctypes.byref(st)), "cgx_get_stats")
        return st

    def residual_norm(self) -> tuple[float, float]:
        """(||b - A x||, ||b||) for the current x (ends a solve in progress)."""
        rn, bn = ctypes.c_double(), ctypes.c_double()
        _check(lib().cgx_residual_norm(self._h, ctypes.byref(rn), ctypes.byref(bn)), "cgx_residual_norm")
        return rn.value, bn.value

    def set_matvec_plan(self, rows_per_wave: int, chunks_in_flight: int, nontemporal: int = 1,
                        blocks_per_cu: int = 0) -> None:
        _check(lib().cgx_set_matvec_plan(self._h, rows_per_wave, chunks_in_flight, nontemporal, blocks_per_cu),
               "cgx_set_matvec_plan")

    def matvec_plan(self) -> dict:
        v = [ctypes.c_int() for _ in range(4)]
        _check(lib().cgx_get_matvec_plan(self._h, *(ctypes.byref(x) for x in v)), "cgx_get_matvec_plan")
        return dict(zip(("R", "U", "nt", "blocks"), (x.value for x in v)))

    def phase_times(self) -> dict:
        """CGX_PHASES: {phase: {"median_us", "mean_us", "samples"}} since the last reset_timing()."""
        t = PhaseTimes()
        _check(lib().cgx_get_phase_times(self._h, ctypes.byref(t)), "cgx_get_phase_times")
        return {name: {"median_us": t.median_us[i], "mean_us": t.mean_us[i], "samples": int(t.samples[i])}
                for i, name in enumerate(PHASE_NAMES)}

    def comm_info(self) -> dict:
        """What the exchange runs on: RCCL's rank count / device / rank (rank mode) and the PCI bus id."""
        ci = CommInfo()
        _check(lib().cgx_get_comm_info(self._h, ctypes.byref(ci)), "cgx_get_comm_info")
        return {"rccl_nranks": ci.rccl_nranks, "rccl_device": ci.rccl_device, "rccl_rank": ci.rccl_rank,
                "device": ci.device, "pci_bus_id": ci.pci_bus_id.decode()}

    def overlap_info(self) -> dict:
        """How the p exchange was chosen at creation (aligned row blocks,
        cgx_get_overlap_info): both whole forms, exchange + matVec, timed end
        to end; the overlapped one runs when overlap_form_us < (1 - margin) *
        plain_form_us.  The parts (allgather alone, the split, the one
        launch) are reported too.  Values as the library decided on them (not
        rounded); None where not measured."""
        o = OverlapInfo()
        _check(lib().cgx_get_overlap_info(self._h, ctypes.byref(o)), "cgx_get_overlap_info")
        r = lambda v: None if v < 0 else float(v)  # noqa: E731
        return {"on": bool(o.active), "decided_by": OVERLAP_DECIDED_BY.get(o.decided_by, str(o.decided_by)),
                "overlap_form_us": r(o.overlap_form_us), "plain_form_us": r(o.plain_form_us), "margin": o.margin,
                "forms_ms": r(o.forms_ms),
                "allgather_us": r(o.allgather_us), "split_cost_us": r(o.split_cost_us), "split_us": r(o.split_us),
                "one_launch_us": r(o.one_launch_us)}

    def reset_timing(self) -> None:
        _check(lib().cgx_reset_timing(self._h), "cgx_reset_timing")

    def synchronize(self) -> None:
        _check(lib().cgx_synchronize(self._h), "cgx_synchronize")


def conjugrad(A: np.ndarray, b: np.ndarray, x: np.ndarray, *, eps: float = 1e-6, max_iter: int = -1,
              flags: int | None = None, shards=None) -> Stats:
    """serialConjugate.c:180-259 ``conjugrad(A, b, x)``: solves in place (x is
    x0 on entry, the solution on exit).  ``shards`` = list of device ids gives
    parallel_cg.c's row-block split with P = len(shards) (parallel_cg.c:248).
    The dtype of ``x`` picks the arithmetic unless ``flags`` is given:
    float32 -> CGX_F32_REF (the reference's float results bit for bit),
    float64 -> CGX_F64."""
    if flags is None:
        flags = CGX_F32_REF if x.dtype == np.float32 else CGX_F64
    n = b.shape[0]
    with Solver(n, flags=flags, devices=shards) as s:
        s.set_system(A, b, x)
        xs, st = s.solve(None, eps=eps, max_iter=max_iter)
    x[...] = xs
    return st
