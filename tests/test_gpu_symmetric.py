"""CGX_SYMMETRIC: A kept as its upper triangle of 128 x 128 tiles, A.p from it.

Parity bar (the fp64 one of tests/test_gpu_solver.py): loop count equal to
the fp64 oracle's (conjgrad.m order) and x within 1e-10; the matVec itself
within the reordered-sum bound of the row-major kernel.  The sums run in a
different order than the row-major kernel, so x agrees to fp64 rounding, not
bit for bit; the result is deterministic run to run.
"""
import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle
from _cases import case

pytestmark = pytest.mark.gpu
TOL = 1e-10
SYM = cg.CGX_F64 | cg.CGX_SYMMETRIC


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1, "no GPU visible: the HIP path must run"


@pytest.mark.parametrize("n", [1, 5, 127, 128, 129, 300, 1000, 2304])
def test_symmetric_matvec(n):
    """b - A x through the tiled upper triangle == numpy, to the bound of a reordered fp64 sum."""
    rng = np.random.default_rng(n)
    R = rng.random((n, n))
    A = 0.5 * (R + R.T) + n * np.eye(n)
    b = rng.random(n)
    x = rng.random(n) - 0.5
    with cg.Solver(n, flags=SYM) as s:
        s.set_system(A, b, x)
        rn, bn = s.residual_norm()
    r = b - A @ x
    bound = 1e-13 * float(np.abs(A) @ np.abs(x) @ np.ones(n))
    assert abs(rn - np.linalg.norm(r)) <= bound + 1e-13 * np.linalg.norm(r)
    assert abs(bn - np.linalg.norm(b)) <= 1e-14 * np.linalg.norm(b)


@pytest.mark.parametrize("name", ["kat4", "spd512", "spd1024", "spd2048", "spd4096", "spd8192"])
def test_symmetric_solve_vs_oracle(golden, name):
    A, b, x0 = case(name, np.float64)
    with cg.Solver(b.size, flags=SYM) as s:
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert st.iterations == so.iterations == golden["cases"][name]["conjgrad_m_f64_iterations"]
    assert rel(x, xo) <= TOL and rn <= TOL * bn


def test_symmetric_reads_only_the_upper_tiles():
    """Entries below the diagonal tiles are never read (CG's A is symmetric by contract)."""
    A, b, x0 = case("spd1024", np.float64)
    G = A.copy()
    for I in range(1024 // 128):
        G[(I + 1) * 128:, I * 128:(I + 1) * 128] = np.nan  # strict lower tiles
    with cg.Solver(1024, flags=SYM) as s:
        s.set_system(G, b, x0)
        xg, sg = s.solve(None, eps=1e-10)
        s.set_system(A, b, x0)
        xa, sa = s.solve(None, eps=1e-10)
    assert sg.iterations == sa.iterations and np.array_equal(xg, xa)


@pytest.mark.parametrize("n", [1000, 5000, 16384])
def test_symmetric_generator_matches_dense(n):
    """cgx_generate_spd writes the same system into the tiles: the solves agree."""
    with cg.Solver(n, flags=SYM) as s:
        s.generate_spd(42)
        xs, ss = s.solve(None, eps=1e-10)
        xs2, _ = s.solve(np.zeros(n), eps=1e-10)
    with cg.Solver(n) as d:
        d.generate_spd(42)
        xd, sd = d.solve(None, eps=1e-10)
    assert ss.iterations == sd.iterations
    assert rel(xs, xd) <= 1e-12
    assert np.array_equal(xs, xs2)  # deterministic


def test_symmetric_rows_in_pieces_and_fixed_count():
    A, b, x0 = case("spd2048", np.float64)
    with cg.Solver(2048, flags=SYM | cg.CGX_TIMING) as s:
        for r0 in (0, 700, 1500):  # ragged row ranges, not tile aligned
            r1 = {0: 700, 700: 1500, 1500: 2048}[r0]
            s.set_rows(r0, A[r0:r1], b[r0:r1], x0[r0:r1])
        x, st = s.solve(None, eps=-1.0, max_iter=4)
        assert st.iterations == 4 and st.matvec_count >= 4
    xo, so = oracle.cg_f64(A, b, x0, eps=-1.0, max_iter=4)
    assert rel(x, xo) <= 1e-12


def test_symmetric_rejects_unsupported():
    for kw in ({"flags": SYM, "devices": [0, 0]}, {"flags": cg.CGX_F32_REF | cg.CGX_SYMMETRIC}):
        with pytest.raises(cg.CgxError):
            cg.Solver(1024, **kw)
    with cg.Solver(1024, flags=SYM) as s:
        with pytest.raises(cg.CgxError):
            s.set_matvec_plan(2, 8)


@pytest.mark.parametrize("name", ["kat4", "spd1024", "spd2048"])
def test_symmetric_host_streamed_solve(monkeypatch, golden, name):
    """CGX_SYMMETRIC | CGX_HOST_STREAM: the tiles stream from pinned host
    memory in 1 MiB chunks (8 tiles, so many chunks per matVec, ragged last)."""
    monkeypatch.setenv("CGX_STREAM_TILE_MB", "1")
    A, b, x0 = case(name, np.float64)
    with cg.Solver(b.size, flags=SYM | cg.CGX_HOST_STREAM) as s:
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert st.iterations == so.iterations == golden["cases"][name]["conjgrad_m_f64_iterations"]
    assert rel(x, xo) <= TOL


def test_symmetric_host_streamed_generator_matches_resident(monkeypatch):
    monkeypatch.setenv("CGX_STREAM_TILE_MB", "3")
    n = 5000
    with cg.Solver(n, flags=SYM | cg.CGX_HOST_STREAM) as s:
        s.generate_spd(42)
        xs, ss = s.solve(None, eps=1e-10)
    with cg.Solver(n, flags=SYM) as d:
        d.generate_spd(42)
        xd, sd = d.solve(None, eps=1e-10)
    assert ss.iterations == sd.iterations
    assert rel(xs, xd) <= 1e-12


@pytest.mark.parametrize("resident_mb", ["3", "1000"])
def test_symmetric_host_streamed_with_resident_tiles(monkeypatch, resident_mb):
    """CGX_STREAM_RESIDENT_MB with the tile stream: the first tiles stay in
    HBM (3 MB = 24 tiles: a resident part that ends inside a tile row; 1000
    MB: all of them) and only the rest streams.  Every chunking writes the
    same per-tile partials, so x is bit for bit the fully streamed solve's --
    rows set on the host, generated on the device, A replaced between solves."""
    monkeypatch.setenv("CGX_STREAM_TILE_MB", "1")
    n = 2000
    A, b = oracle.spd_hash(n, seed=3)
    A2, b2 = oracle.spd_hash(n, seed=4)
    out = {}
    for res in ("0", resident_mb):
        monkeypatch.setenv("CGX_STREAM_RESIDENT_MB", res)
        with cg.Solver(n, flags=SYM | cg.CGX_HOST_STREAM) as s:
            s.set_system(A, b)
            r1 = s.solve(None, eps=1e-10)
            s.set_system(A2, b2)
            r2 = s.solve(None, eps=1e-10)
            s.generate_spd(42)
            r3 = s.solve(None, eps=1e-10)
        out[res] = [(x, st.iterations) for x, st in (r1, r2, r3)]
    for (xa, ia), (xb, ib) in zip(out["0"], out[resident_mb]):
        assert ia == ib and np.array_equal(xa.view(np.uint8), xb.view(np.uint8))
    xo, so = oracle.cg_f64(A2, b2, np.zeros(n), eps=1e-10)
    assert out[resident_mb][1][1] == so.iterations and rel(out[resident_mb][1][0], xo) <= TOL
