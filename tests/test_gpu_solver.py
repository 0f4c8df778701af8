"""Solver-level parity on the GPU (conjugrad through the C ABI).

Pins:
  1. CGX_F32_REF x == serialConjugate.c x bit for bit, same loop count
     (golden vectors from the unmodified reference, tests/golden/);
  2. CGX_F64 x vs the fp64 oracle: ||dx||/||x|| <= 1e-10, ||b-Ax||/||b|| <= 1e-10,
     loop count == conjgrad.m's (tol 1e-10);
  3. CGX_F64 x vs the reference's fp32 x: ||dx||/||x|| <= 1e-5;
  4. KATs: 2x2 -> [2/3, 1/3], 4x4 -> [-1, 1, -1, 1] to 1e-12.
Multi-shard runs (several row blocks on this GPU, the parallel_cg.c split)
must give the reference MPI programs' results: F32_REF bit-exact to the
unmodified parallel_cg.c (collective exchange, MPICH's MPI_Allreduce order)
and point-to-point_cg.c (CGX_COMM_P2P, allSum order) run under mpiexec -np P
(tests/golden/mpi/), and to the oracle's P-part restatement of both beyond
the fixtures; 1e-10 in F64."""
import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle
from _cases import (COMBINE_OF, KATS, SPD_ALL, SPD_SMALL, case, golden_mpi, golden_x, hash_oracle, mpi_golden_x,
                    mpi_runs)

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1, "no GPU visible: the HIP path must run"


def rel(a, b):
    return np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b)


@pytest.mark.parametrize("name", KATS + SPD_ALL)
def test_f32ref_bit_exact_vs_reference(golden, name):
    A, b, x0 = case(name)
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=1e-6)
    ref = golden_x(golden, name)
    assert st.iterations == golden["cases"][name]["ref_iterations"]
    assert st.converged == 1
    assert np.array_equal(x.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name", KATS + SPD_ALL)
def test_f64_parity(golden, name):
    A, b, x0 = case(name, np.float64)
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert st.iterations == so.iterations == golden["cases"][name]["conjgrad_m_f64_iterations"]
    assert rel(x, xo) <= TOL
    assert np.linalg.norm(b - A @ x) <= TOL * np.linalg.norm(b)
    assert rel(golden_x(golden, name), x) <= 1e-5


@pytest.mark.parametrize("name", ["kat4", "spd512"])
def test_cgx_conjugrad_one_call_f64(golden, name):
    """cgx_conjugrad (the one-call drop-in, include/cgx.h) with CGX_F64 double
    arrays: x in place, bitwise equal to the context path's x, its stats filled;
    a size that does not fit a context fails with the create's error and leaves x."""
    import ctypes
    A, b, x0 = case(name, np.float64)
    x_ctx = x0.copy()
    st_ctx = cg.conjugrad(A, b, x_ctx, eps=1e-10)
    x = x0.copy()
    st = cg.Stats()
    L = cg.lib()
    A_c, b_c = np.ascontiguousarray(A), np.ascontiguousarray(b)
    rc = L.cgx_conjugrad(A_c.ctypes.data, b_c.ctypes.data, x.ctypes.data, A.shape[0], cg.CGX_F64, 1e-10, -1,
                         ctypes.byref(st))
    assert rc == 0, L.cgx_last_error().decode()
    assert np.array_equal(x.view(np.uint64), x_ctx.view(np.uint64))
    assert st.iterations == st_ctx.iterations == golden["cases"][name]["conjgrad_m_f64_iterations"]
    assert st.converged == 1
    x_bad = x0.copy()
    assert L.cgx_conjugrad(A_c.ctypes.data, b_c.ctypes.data, x_bad.ctypes.data, 0, cg.CGX_F64, 1e-10, -1,
                           None) != 0
    assert np.array_equal(x_bad, x0)


def test_known_answers():
    A, b, x0 = case("kat2", np.float64)
    x = x0.copy()
    cg.conjugrad(A, b, x, eps=1e-10)
    assert np.allclose(x, [2 / 3, 1 / 3], rtol=0, atol=1e-12)
    A, b, x0 = case("kat4", np.float64)
    x = x0.copy()
    cg.conjugrad(A, b, x, eps=1e-10)
    assert np.allclose(x, [-1, 1, -1, 1], rtol=0, atol=1e-12)


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("name", ["kat4", "spd512", "spd2048"])
def test_row_block_shards_f32ref(name, P):
    """P row blocks on this GPU == oracle with P-part dots (parallel_cg.c, MPICH order)."""
    A, b, x0 = case(name)
    if b.size % P:
        pytest.skip("n not divisible")
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=1e-6, shards=[0] * P)
    xo, so = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=P, combine="mpich")
    assert st.iterations == so.iterations
    assert np.array_equal(x.view(np.uint32), xo.view(np.uint32))


@pytest.mark.parametrize("key", mpi_runs(min_np=2))
def test_f32ref_shards_bit_exact_vs_mpi_reference(key):
    """P row blocks on this GPU == the unmodified MPI program under
    mpiexec -np P, bit for bit, same loop count: parallel_cg.c through the
    collective exchange (MPICH's MPI_Allreduce order), point-to-point_cg.c
    through CGX_COMM_P2P (allSum, rank order)."""
    r = golden_mpi()["runs"][key]
    A, b, x0 = case(r["case"])
    flags = cg.CGX_F32_REF | (cg.CGX_COMM_P2P if r["program"] == "p2p" else 0)
    with cg.Solver(b.size, flags=flags, devices=[0] * r["np"]) as s:
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-6)
    assert st.iterations == r["ref_iterations"] and st.converged == 1
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("kind", ["f64", "f64_nooverlap", "f32ref", "p2p_f64", "p2p_f32ref"])
def test_local_exchange_kernels_bitwise_equal_peer_copies(monkeypatch, kind, P):
    """The multi-shard exchange in one process: the pull kernels (one gather
    kernel per consuming shard; the scalar combines folded into the update
    kernels, the default, or one combine kernel each, CGX_LOCAL_FUSE=0) move
    the same bytes and add the same partials in the same order as round 3's
    per-pair peer copies (CGX_LOCAL_XCHG=copy): x bit for bit, the same loop
    count -- gated and fixed-count, with the overlapped gather, the plain one
    (3 shards: 2049/3 rows; CGX_NO_OVERLAP), the x0 allgather of a nonzero x0,
    F32_REF's MPICH-order combine (folded since round 6), and the p2p
    pattern (CGX_COMM_P2P: through block 0, rank order) by pull kernels or
    by copies."""
    n = 2048 if P != 3 else 2049
    f32 = kind.endswith("f32ref")
    dt = np.float32 if f32 else np.float64
    A, b = oracle.spd_hash(n, seed=11, dtype=dt)
    x0 = np.full(n, 0.125, dt)
    flags = cg.CGX_F32_REF if f32 else cg.CGX_F64 | (cg.CGX_NO_OVERLAP if kind == "f64_nooverlap" else 0)
    flags |= cg.CGX_COMM_P2P if kind.startswith("p2p") else 0
    res = {}
    # nofuse: a combine kernel per scalar instead of the folded sums; onethread: every block's work
    # enqueued by the calling thread instead of one thread per block (cgx_local_mt.hip)
    if kind == "f64":  # the overlapped gather (f64_nooverlap: the one-launch form of the same bits)
        monkeypatch.setenv("CGX_OVERLAP", "1")
    for form in ("kernel", "onethread", "nofuse", "copy"):
        monkeypatch.setenv("CGX_LOCAL_XCHG", "copy" if form == "copy" else "kernel")
        monkeypatch.setenv("CGX_LOCAL_FUSE", "0" if form == "nofuse" else "1")
        monkeypatch.setenv("CGX_LOCAL_THREADS", "0" if form == "onethread" else "1")
        with cg.Solver(n, flags=flags, devices=[0] * P) as s:
            if kind == "f64" and P in (2, 8):
                assert s.info.flags & cg.CGX_OVERLAP_ACTIVE
            s.set_system(A, b, x0)
            x, st = s.solve(None, eps=1e-6 if f32 else 1e-10)
            xf, stf = s.solve(x0, eps=-1.0, max_iter=7)
            rn, bn = s.residual_norm()
            monkeypatch.setenv("CGX_GATED", "0")  # host-checked: r.r read before the p update
            xh, sth = s.solve(x0, eps=1e-6 if f32 else 1e-10)
            monkeypatch.delenv("CGX_GATED")
        res[form] = (x, st.iterations, xf, rn, xh, sth.iterations)
    c = res["copy"]
    for form in ("kernel", "onethread", "nofuse"):
        r = res[form]
        assert r[1] == c[1] and r[5] == c[5] == c[1], form
        assert np.array_equal(r[0], c[0]) and np.array_equal(r[2], c[2]) and r[3] == c[3], form
        assert np.array_equal(r[4], c[0]), form
    xk, itk = res["kernel"][0], res["kernel"][1]
    if f32:
        xo, so = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=P, combine="rank" if kind.startswith("p2p") else "mpich")
        assert itk == so.iterations and np.array_equal(xk.view(np.uint32), xo.view(np.uint32))
    else:
        xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
        assert itk == so.iterations and rel(xk, xo) <= TOL


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("name", ["kat4", "spd1024", "spd4096"])
def test_row_block_shards_f64(golden, name, P):
    A, b, x0 = case(name, np.float64)
    x = x0.copy()
    if b.size % P:  # parallel_cg.c:86-90: N must split into P equal row blocks
        with pytest.raises(cg.CgxError, match="not divisible"):
            cg.conjugrad(A, b, x, eps=1e-10, shards=[0] * P)
        return
    st = cg.conjugrad(A, b, x, eps=1e-10, shards=[0] * P)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert st.iterations == so.iterations
    assert rel(x, xo) <= TOL


@pytest.mark.parametrize("mode", ["collective", "overlap", "p2p", "deterministic"])
def test_rccl_rank_mode_world1(monkeypatch, mode):
    """The one-process-per-GPU path (RCCL allgather/allreduce) at world size 1:
    plain collectives; the overlapped exchange forced on (CGX_OVERLAP=force:
    in-place ncclAllGather on the comm stream, event hand-offs, own-block then
    remaining-columns matVec with a zero-width second piece); the
    point-to-point_cg.c pattern (CGX_COMM_P2P)."""
    A, b, x0 = case("spd1024", np.float64)
    if mode == "overlap":
        monkeypatch.setenv("CGX_OVERLAP", "force")
    flags = cg.CGX_F64 | {"p2p": cg.CGX_COMM_P2P, "deterministic": cg.CGX_DETERMINISTIC}.get(mode, 0)
    uid = cg.get_unique_id()
    with cg.Solver(b.size, rank=0, nranks=1, unique_id=uid, device=0, flags=flags) as s:
        assert bool(s.info.flags & cg.CGX_OVERLAP_ACTIVE) == (mode == "overlap")
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert st.iterations == so.iterations and rel(x, xo) <= TOL
    assert rn <= TOL * bn
    if mode == "deterministic":  # rank-order combine: the single-shard bits
        xs = x0.copy()
        cg.conjugrad(A, b, xs, eps=1e-10)
        assert np.array_equal(x, xs)
    if mode != "collective":
        return
    with cg.Solver(b.size, rank=0, nranks=1, unique_id=cg.get_unique_id(), flags=cg.CGX_F32_REF) as s:
        A32, b32, x032 = case("spd1024")
        s.set_system(A32, b32, x032)
        x32, st32 = s.solve(None, eps=1e-6)
    ref, _ = oracle.cg_f32ref(A32, b32, x032)
    assert np.array_equal(x32, ref)


def test_set_rows_partial_and_generator_rows():
    """cgx_set_rows with each shard's own block only (MPI_Scatter)."""
    A, b, x0 = case("spd2048", np.float64)
    P = 4
    with cg.Solver(b.size, devices=[0] * P) as s:
        loc = b.size // P
        for q in range(P):
            sl = slice(q * loc, (q + 1) * loc)
            s.set_rows(q * loc, A[sl], b[sl], x0[sl])
        x, st = s.solve(None, eps=1e-10)
    xo, _ = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert rel(x, xo) <= TOL


@pytest.mark.parametrize("n,shards", [(1000, None), (2048, [0, 0]), (4096, [0] * 4)])
def test_device_generator_matches_oracle(n, shards):
    """cgx_generate_spd == oracle_spd_hash: identical A, b give identical solves."""
    with cg.Solver(n, devices=shards) as s:
        s.generate_spd(seed=42)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    A, b = oracle.spd_hash(n, seed=42)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert st.iterations == so.iterations
    assert rel(x, xo) <= 1e-12
    assert abs(bn - np.linalg.norm(b)) <= 1e-14 * np.linalg.norm(b)
    assert rn <= TOL * bn
    with cg.Solver(n, flags=cg.CGX_F32_REF, devices=shards) as s:
        s.generate_spd(seed=42)
        x32, st32 = s.solve(None, eps=1e-6)
    A32, b32 = oracle.spd_hash(n, seed=42, dtype=np.float32)
    xo32, _ = oracle.cg_f32ref(A32, b32, np.zeros(n, np.float32), nparts=len(shards) if shards else 1,
                               combine="mpich")
    assert np.array_equal(x32, xo32)


def test_n16384_against_cpu_oracle():
    """configs[1]: N=16384 dense SPD fp64 on one GPU vs the CPU fp64 oracle."""
    n = 16384
    with cg.Solver(n) as s:
        s.generate_spd(seed=42)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    oracle.set_threads(16)
    A, b = oracle.spd_hash(n, seed=42)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    del A
    assert st.iterations == so.iterations
    assert rel(x, xo) <= TOL
    assert rn <= TOL * bn


@pytest.mark.parametrize("P", [1, 8])
def test_n65536_full_size_against_cpu_oracle(P):
    """BASELINE.json's headline size, N=65536 (34.4 GB of A): one row block,
    and the 8-GPU partition (8 blocks of 8192 rows) as 8 shards on this GPU.
    Same loop count as conjgrad.m at tol 1e-10, x within 1e-10 of the fp64
    oracle (16 host threads), true residual ||b-Ax|| <= 1e-10 ||b||."""
    n = 65536
    with cg.Solver(n, devices=[0] * P if P > 1 else None) as s:
        s.generate_spd(seed=42)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    xo, so = _oracle_n65536()
    assert st.converged and st.iterations == so.iterations
    assert rel(x, xo) <= TOL
    assert rn <= TOL * bn


def _oracle_n65536():
    return hash_oracle(65536)


def _oracle_hash(n, seed=42):
    return hash_oracle(n, seed)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("layout", ["rows", "symmetric"])
def test_configs3_streamed_n131072_full_size(layout):
    """BASELINE configs[3] at its stated size: N=131072 fp64 (137 GB of A, or
    68.7 GB of upper-triangle tiles) kept in pinned host memory and streamed
    through the GPU every matVec (CGX_HOST_STREAM).  Solved to eps 1e-10 from
    x0 = 0: loop count == conjgrad.m's, x within 1e-10 of the fp64 oracle
    (A regenerated on 16 host threads), true residual <= 1e-10 ||b||."""
    n = 131072
    flags = cg.CGX_F64 | cg.CGX_HOST_STREAM | (cg.CGX_SYMMETRIC if layout == "symmetric" else 0)
    with cg.Solver(n, flags=flags) as s:
        s.generate_spd(seed=42)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    xo, so = _oracle_hash(n)
    assert st.converged and st.iterations == so.iterations
    assert rel(x, xo) <= TOL
    assert rn <= TOL * bn


@pytest.mark.timeout(600)
def test_configs4_poisson_m8192_full_size():
    """BASELINE configs[4] at its stated size: the matrix-free 5-point Poisson
    operator on an 8192 x 8192 grid (N = 67.1 M), b = 1, x0 = 0, 25 fixed
    iterations (the fused two-kernel iteration) against the fp64 oracle: x to
    1e-9 (a fixed-count solve far from convergence; the sums are reordered),
    and the true residual equal to the oracle's to 1e-9."""
    m, iters = 8192, 25
    n = m * m
    with cg.Solver(None, poisson_m=m) as s:
        assert s.info.flags & cg.CGX_FUSED_ACTIVE
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=-1.0, max_iter=iters)
        rn, bn = s.residual_norm()
    assert st.iterations == iters
    oracle.set_threads(16)
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=-1.0, max_iter=iters)
    assert so.iterations == iters
    assert rel(x, xo) <= 1e-9
    ro = np.linalg.norm(1.0 - oracle.poisson_apply(m, xo))
    assert abs(rn - ro) <= 1e-9 * ro and abs(bn - m) <= 1e-12 * m


@pytest.mark.timeout(600)
def test_poisson_slab_over_4gib_byte_offsets():
    """k_poisson_p addresses a slab's rows by 32-bit byte offsets while every
    offset fits (halo rows included: (m + 2) m 8 B <= 2^32 - 1), else by 64-bit
    ones.  m = 23172 is the first even grid past that bound on one slab: 5
    fixed iterations against the fp64 oracle (x and the true residual to 1e-9)."""
    m, iters = 23172, 5
    assert (m + 2) * m * 8 > 2**32 - 1 >= (m // 2 + 2) * m * 8
    n = m * m
    with cg.Solver(None, poisson_m=m) as s:
        assert s.info.flags & cg.CGX_FUSED_ACTIVE
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=-1.0, max_iter=iters)
        rn, bn = s.residual_norm()
    assert st.iterations == iters
    oracle.set_threads(16)
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=-1.0, max_iter=iters)
    assert so.iterations == iters
    assert rel(x, xo) <= 1e-9
    del x
    ro = np.linalg.norm(1.0 - oracle.poisson_apply(m, xo))
    assert abs(rn - ro) <= 1e-9 * ro and abs(bn - m) <= 1e-12 * m


def test_solve_in_pieces_and_fixed_count():
    """cgx_solve_begin + cgx_iterate == cgx_solve; eps < 0 runs exactly max_iter."""
    A, b, x0 = case("spd1024", np.float64)
    with cg.Solver(b.size) as s:
        s.set_system(A, b, x0)
        x_full, st = s.solve(None, eps=1e-10)
        s.set_x(x0)
        s.begin()
        total = 0
        while True:
            done, conv = s.iterate(2, eps=1e-10)
            total += done
            if conv or done == 0:
                break
        assert total == st.iterations
        assert np.array_equal(s.get_x(), x_full)
        s.set_x(x0)
        _, st2 = s.solve(None, eps=-1.0, max_iter=9)
        assert st2.iterations == 9 and st2.converged == 0


@pytest.mark.parametrize("kind,fuse_p", [("dense", None), ("dense", "0"), ("shards", None), ("symmetric", None),
                                         ("poisson", None)])
def test_fixed_count_past_convergence_stays_finite(monkeypatch, kind, fuse_p):
    """bench.py's fixed-count mode runs on long after CG has converged: r.r
    shrinks until it underflows to 0, and alpha / beta would then be 0/0.
    The fp64 kernels treat a zero denominator as the exact convergence it is
    (alpha = beta = 0, cg_ratio in cgx_device.h): x stays at the solution, no
    NaN (bench.py at N=16384, 300 steps, reported relres NaN before)."""
    if fuse_p is not None:
        monkeypatch.setenv("CGX_FUSE_P", fuse_p)
    if kind == "poisson":
        kw, n, steps = {"poisson_m": 8}, None, 3000
    else:
        kw = {"flags": cg.CGX_F64 | (cg.CGX_SYMMETRIC if kind == "symmetric" else 0)}
        if kind == "shards":
            kw["devices"] = [0, 0]
        n, steps = 1024, 600
    with cg.Solver(n, **kw) as s:
        if kind == "poisson":
            s.fill(1.0, 0.0)
        else:
            s.generate_spd(3)
        x_conv, st = s.solve(None, eps=1e-12)
        assert st.converged
        rn_conv, bn = s.residual_norm()
        s.set_x(np.zeros(s.n))
        _, st2 = s.solve(None, eps=-1.0, max_iter=steps)
        assert st2.iterations == steps
        x = s.get_x()
        rn, bn2 = s.residual_norm()
    assert np.all(np.isfinite(x)), kind
    assert rn / bn2 <= max(1e-12, 10 * rn_conv / bn), (rn / bn2, rn_conv / bn)
    assert rel(x, x_conv) <= 1e-10


@pytest.mark.parametrize("shards", [None, [0, 0]])
def test_indefinite_breakdown_is_not_hidden(shards):
    """An A that is not positive definite can give p.Ap = 0 with r.r != 0: a
    real breakdown.  alpha = r.r / p.Ap is then Inf, as in the reference's
    division (serialConjugate.c:220), and x stops being finite -- not a quiet
    alpha = 0 that would stall the solve at x0 until max_iter (cg_ratio keeps
    0 only for an underflowed numerator, the exact-convergence case)."""
    A = np.diag([1.0, -1.0])
    b = np.ones(2)
    with cg.Solver(2, devices=shards) as s:
        s.set_system(A, b, np.zeros(2))
        x, st = s.solve(None, eps=1e-10)
    assert not st.converged and st.iterations == 2  # the reference's k < ROWS cap
    assert not np.all(np.isfinite(x)), x


def test_create_multi_leaves_no_hip_error():
    """cgx_create_multi enables peer access only between distinct devices,
    after hipDeviceCanAccessPeer, and consumes every HIP error it meets: the
    thread's pending HIP error is clean afterwards (a stale one would surface
    as a spurious CGX_ERR_HIP at the first kernel launch).  CGX_PEER_ACTIVE
    reports whether the blocks span several devices with peer access on."""
    L = cg.lib()
    with cg.Solver(1024, devices=[0, 0]) as s:
        assert L.cgx_hip_last_error() == 0
        assert not s.info.flags & cg.CGX_PEER_ACTIVE  # one device: nothing to enable
        s.generate_spd(1)
        _, st = s.solve(None, eps=1e-10)
        assert st.converged
    # (distinct devices: tests/test_gpu_multidevice.py::test_create_multi_distinct_devices_peer_access)
    assert cg.device_link(0, 0)["link"] == "unknown" and len(cg.device_pci_bus_id(0)) >= 12


@pytest.mark.parametrize("kind", ["single", "small_fused", "shards_overlap", "shards_one", "shards_plain", "gated"])
def test_phase_times_tile_the_iteration(monkeypatch, kind):
    """CGX_PHASES: the iteration's kernels stamp their start and end on the
    device clock; the phases are resolved after the fact.  Every kernel phase
    gets one sample per iteration (the gap and the iteration one fewer), more
    iterations than one stamp ring holds (1024) are carried across resolves,
    and the consecutive phases tile the iteration: their means add up to the
    mean iteration.  A converged, device-gated solve stops sampling where the
    kernels stop running."""
    n, steps = {"small_fused": 2048, "single": 16384}.get(kind, 4096), 1100  # > the 1024-iteration stamp ring
    devices = {"shards_overlap": [0, 0], "shards_one": [0, 0], "shards_plain": [0, 0, 0]}.get(kind)
    if kind == "shards_plain":  # 4095/3 rows: not 128-aligned, one launch in column order
        n = 4095
    if kind in ("shards_overlap", "shards_one"):  # aligned: the overlapped form, or the one-launch form
        monkeypatch.setenv("CGX_OVERLAP", "1" if kind == "shards_overlap" else "0")
    with cg.Solver(n, flags=cg.CGX_PHASES | cg.CGX_TIMING, devices=devices) as s:
        s.generate_spd(5)
        if kind == "gated":
            _, st = s.solve(None, eps=1e-10)
            ph = s.phase_times()
            assert ph["matvec"]["samples"] == st.iterations and ph["iteration"]["samples"] == st.iterations - 1
            return
        s.begin()
        s.iterate(3, eps=-1.0)
        s.reset_timing()
        s.iterate(steps, eps=-1.0)
        ph = s.phase_times()
    assert ph["iteration"]["samples"] == steps - 1, ph["iteration"]
    # samples per phase: one per iteration for a kernel and for the span between
    # two kernels of an iteration; one fewer for the span before an
    # iteration's first kernel (the gap; p's allgather when not overlapped)
    S, F = steps, steps - 1
    want = {"single": {"matvec": S, "combine_pap": S, "update_r": S, "combine_rr": S, "update_xp": S, "gap": F},
            "small_fused": {"matvec": S, "combine_pap": S, "update_xp": S, "gap": F},
            "shards_overlap": {"matvec_own": S, "gather_exposed": S, "matvec": S, "combine_pap": S, "update_r": S,
                               "combine_rr": S, "update_xp": S, "gap": F},
            "shards_plain": {"gather_exposed": F, "matvec": S, "combine_pap": S, "update_r": S, "combine_rr": S,
                             "update_xp": S}}
    want["shards_one"] = want["shards_plain"]
    want = want[kind]
    for name in cg.PHASE_NAMES[:8]:
        assert ph[name]["samples"] == want.get(name, 0), (name, ph[name])
    # matvec_busy (not a tile): the union of the matVec kernels' spans, one per iteration -- the matVec
    # itself without the overlap; with it at least the own block, and within own block + the wait for p
    # (gather_exposed) + the rest launch, all three on the compute stream
    busy = ph["matvec_busy"]
    assert busy["samples"] == S, busy
    if kind == "shards_overlap":
        assert ph["matvec_own"]["mean_us"] <= busy["mean_us"]
        assert busy["mean_us"] <= 1.01 * (ph["matvec_own"]["mean_us"] + ph["gather_exposed"]["mean_us"]
                                          + ph["matvec"]["mean_us"])
    else:
        assert abs(busy["mean_us"] - ph["matvec"]["mean_us"]) <= 0.01 * ph["matvec"]["mean_us"] + 0.05
        if name in want:
            assert ph[name]["mean_us"] > 0, (name, ph[name])
    tiles = sum(ph[k]["mean_us"] * ph[k]["samples"] for k in cg.PHASE_NAMES[:8]) / (steps - 1)
    assert abs(tiles / ph["iteration"]["mean_us"] - 1) <= 0.02, (tiles, ph["iteration"])


@pytest.mark.parametrize("flags,kw", [(cg.CGX_F32_REF, {}), (cg.CGX_HOST_STREAM, {}), (cg.CGX_SYMMETRIC, {}),
                                      (0, {"poisson_m": 8})])
def test_phase_times_refused_where_not_stamped(flags, kw):
    """CGX_PHASES covers the dense fp64 kernels with A resident; the other
    operators are refused at creation, and a context without the flag
    refuses cgx_get_phase_times."""
    with pytest.raises(cg.CgxError, match="CGX_PHASES"):
        cg.Solver(64, flags=flags | cg.CGX_PHASES, **kw)
    with cg.Solver(64) as s, pytest.raises(cg.CgxError):
        s.phase_times()


def test_timing_events_count():
    """CGX_TIMING times every matVec launch.  With x0 = 0 the initial A x0 is
    skipped (exactly zero); with any other x0 it runs."""
    n = 4096
    with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_TIMING) as s:
        s.generate_spd(1)
        s.solve(None, eps=-1.0, max_iter=5)
        st = s.stats()
        assert st.matvec_count == 5  # x0 = 0: 5 iterations, no initial matVec
        assert st.matvec_ms > 0
        s.reset_timing()
        s.solve(np.full(n, 0.5), eps=-1.0, max_iter=5)
        assert s.stats().matvec_count == 6  # initial residual + 5 iterations


@pytest.mark.parametrize("shards", [None, [0, 0]])
def test_zero_x0_skips_initial_matvec_same_result(monkeypatch, shards):
    """Skipping A x0 for x0 = 0 changes nothing: the same x, bit for bit, as a
    solve from x0 = [0, ..., 0, 0] with the last entry first set nonzero and
    then zeroed (partial set_rows), which keeps the initial matVec.  (The
    host-checked loop: with device-side gating a single process may stop
    enqueueing at a timing-dependent point, so the launch count varies.)"""
    monkeypatch.setenv("CGX_GATED", "0")
    A, b, x0 = case("spd1024", np.float64)
    n = b.size
    res = []
    for partial in (False, True):
        with cg.Solver(n, devices=shards, flags=cg.CGX_F64 | cg.CGX_TIMING) as s:
            s.set_system(A, b, np.full(n, 1.0) if partial else x0)
            if partial:  # zero x through partial writes: the library cannot know it is all zeros
                s.set_rows(0, None, None, np.zeros(300))
                s.set_rows(300, None, None, np.zeros(n - 300))
            x, st = s.solve(None, eps=1e-10)
            res.append((x, st.iterations, s.stats().matvec_count))
    (x1, it1, mv1), (x2, it2, mv2) = res
    assert it1 == it2 and np.array_equal(x1, x2)
    assert mv2 == mv1 + 1


def test_f32ref_nonfinite_A_follows_the_reference():
    """CGX_F32_REF keeps the initial matVec for x0 = 0: with an Inf in A the
    reference's r0 = b - A x0 has a NaN (Inf * 0, serialConjugate.c:209) and
    the loop never meets EPSILON; the GPU does the same (NaN where the oracle
    has NaN, the k < n cap, not converged).  fp64 mode documents finite A."""
    A, b, x0 = case("spd512")
    A = A.copy()
    A[7, 3] = np.inf
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=1e-6)
    xo, so = oracle.cg_f32ref(A, b, x0, eps=1e-6)
    assert st.iterations == so.iterations == 512 and st.converged == so.converged == 0
    assert np.array_equal(np.isnan(x), np.isnan(xo)) and np.isnan(x).any()


@pytest.mark.parametrize("n,seed", [(130, 5), (512, 1), (1000, 2), (2048, 6), (4096, 7), (8192, 3), (8193, 4)])
def test_two_launch_iteration_bitwise_equals_three(monkeypatch, n, seed):
    """Small dense fp64 systems on one GPU iterate in two launches instead of
    three (CGX_FUSE_P): matVec + k_update_xrp_f64, whose last block forms p;
    or, folded (CGX_FOLD_P=1), k_matvec_fold_f64 forming p_k as it multiplies
    it + the fully parallel k_update_xr_stop_f64.  Same expressions, same
    order: x bit for bit and the same loop count as the three-launch iteration
    -- device-gated, host-checked, fixed-count and in pieces; with several
    blocks (n = 8192: r handed to the last block write-through), odd n, rows
    not a whole number of 128-column chunks (the fold's tail columns) and both
    row plans (R = 2 at n = 2048, R = 1 at 4096-8192).  At n = 2048-8192 every
    form's matVec is k_matvec_small_f64 (p staged in LDS; the fold forms
    p_k into LDS).  All agree with the fp64 oracle."""
    A, b = oracle.spd_hash(n, seed=seed)
    res = {}
    for form, fuse, fold in (("three", "0", "0"), ("two", "1", "0"), ("fold", "1", "1")):
        monkeypatch.setenv("CGX_FUSE_P", fuse)
        monkeypatch.setenv("CGX_FOLD_P", fold)
        for gated in ("1", "0"):
            monkeypatch.setenv("CGX_GATED", gated)
            with cg.Solver(n) as s:
                assert bool(s.info.flags & cg.CGX_FUSED_ACTIVE) == (fuse == "1")
                assert bool(s.info.flags & cg.CGX_FOLD_ACTIVE) == (fold == "1")
                assert bool(s.info.flags & cg.CGX_SMALL_ACTIVE) == (2048 <= n <= 8192)
                s.set_system(A, b)
                x, st = s.solve(np.zeros(n), eps=1e-10)
                xf, stf = s.solve(np.zeros(n), eps=-1.0, max_iter=9)
                s.set_x(np.zeros(n))
                s.begin()
                d1, _ = s.iterate(3)
                d2, conv = s.iterate(100, eps=1e-10)
                xp = s.get_x()
            res[(form, gated)] = (x, st.iterations, xf, stf.iterations, xp, d1 + d2, conv)
    ref = res[("three", "0")]
    for key, (x, it, xf, itf, xp, dp, conv) in res.items():
        assert it == ref[1] and np.array_equal(x, ref[0]), key
        assert itf == 9 and np.array_equal(xf, ref[2]), key
        assert conv and dp == it and np.array_equal(xp, ref[0]), key
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert ref[1] == so.iterations and rel(ref[0], xo) <= TOL


@pytest.mark.parametrize("n", [1024, 2048])
def test_plan_change_inside_a_folded_solve_is_refused(n):
    """A matVec plan with more than 2 rows per wave turns the folded iteration
    off.  Inside a solve that would multiply a stale p (p_k lives in pfull or
    p_alt by the parity of k), so cgx_set_matvec_plan refuses it there
    (CGX_ERR_STATE) and the solve goes on bit for bit.  A plan that keeps the
    fold may change between cgx_iterate calls (x agrees with the oracle), and
    the R = 4 plan is taken between solves (the next solve runs unfolded)."""
    A, b = oracle.spd_hash(n, seed=6)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    with cg.Solver(n) as s:
        assert s.info.flags & cg.CGX_FOLD_ACTIVE
        s.set_system(A, b)
        x_ref, st = s.solve(np.zeros(n), eps=1e-10)
        s.set_x(np.zeros(n))
        s.begin()
        d1, _ = s.iterate(3)
        with pytest.raises(cg.CgxError) as e:
            s.set_matvec_plan(4, 8)
        assert e.value.code == -6  # CGX_ERR_STATE
        assert s.info.flags & cg.CGX_FOLD_ACTIVE
        d2, conv = s.iterate(100, eps=1e-10)
        assert conv and d1 + d2 == st.iterations and np.array_equal(s.get_x(), x_ref)
        s.set_x(np.zeros(n))
        s.begin()
        s.iterate(3)
        s.set_matvec_plan(2, 4)
        assert s.info.flags & cg.CGX_FOLD_ACTIVE
        _, conv = s.iterate(100, eps=1e-10)
        assert conv and rel(s.get_x(), xo) <= TOL
        s.set_matvec_plan(4, 8)
        assert not s.info.flags & cg.CGX_FOLD_ACTIVE
        x4, st4 = s.solve(np.zeros(n), eps=1e-10)
    assert st4.iterations == so.iterations and rel(x4, xo) <= TOL


@pytest.mark.parametrize("n,seed", [(2048, 6), (2100, 8), (4096, 7), (5000, 9), (8192, 3)])
def test_small_matvec_lds_agrees_with_l2_kernel(monkeypatch, n, seed):
    """k_matvec_small_f64 (one GPU, 2048 <= lda <= 8192: the vector staged in
    LDS once per CU, one block per CU) sums each row as k_matvec_f64 does;
    only the fused p.Ap adds in another order.  Default and folded forms
    converge in the oracle's loop count, agree with the oracle and, to fp64
    rounding, with round 2's kernel (CGX_MV_SMALL=0).  lda = 2176 (17 chunks,
    not a whole number of steps) keeps k_matvec_f64."""
    A, b = oracle.spd_hash(n, seed=seed)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    res = {}
    for small in ("1", "0"):
        for fold in ("1", "0"):
            monkeypatch.setenv("CGX_MV_SMALL", small)
            monkeypatch.setenv("CGX_FOLD_P", fold)
            with cg.Solver(n) as s:
                assert bool(s.info.flags & cg.CGX_SMALL_ACTIVE) == (small == "1" and n != 2100)
                s.set_system(A, b)
                x, st = s.solve(np.zeros(n), eps=1e-10)
            assert st.converged and st.iterations == so.iterations and rel(x, xo) <= TOL, (small, fold)
            res[(small, fold)] = x
    for key, x in res.items():
        assert rel(x, res[("0", "0")]) <= 1e-12, key
    assert np.array_equal(res[("1", "1")], res[("1", "0")])  # the fold: same kernel, same bits


def _f32_system(name):
    if name.startswith("hash"):  # ragged sizes: rows not a multiple of 32, columns not of 512, 2 dot chunks
        n = int(name[4:])
        A, b = oracle.spd_hash(n, seed=11)
        return A.astype(np.float32), b.astype(np.float32), np.zeros(n, np.float32)
    return case(name, np.float32)


@pytest.mark.parametrize("name", ["kat2_x0", "kat4", "spd512", "spd2048", "spd8192", "hash1000", "hash4100",
                                  "hash1", "hash3", "hash33", "hash513", "hash4097"])
def test_f32ref_two_launch_iteration_bitwise_equals_four(monkeypatch, name):
    """CGX_F32_REF on one GPU iterates in two launches (CGX_REF_FUSE): the
    matVec whose last block runs vecVec(p, Ap), then one block for x/r, r.r,
    the stopping test and p -- instead of four (matVec, vecVec, x/r + r.r,
    p).  The same float operations in the same order: x bit for bit and the
    same loop count as the four-launch iteration and as serialConjugate.c's
    restatement, device-gated, host-checked, fixed-count and in pieces."""
    A, b, x0 = _f32_system(name)
    n = A.shape[0]
    xr, sr = oracle.cg_f32ref(A, b, x0, eps=1e-6)
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("CGX_REF_FUSE", fuse)
        for gated in ("1", "0"):
            monkeypatch.setenv("CGX_GATED", gated)
            with cg.Solver(n, flags=cg.CGX_F32_REF) as s:
                assert bool(s.info.flags & cg.CGX_FUSED_ACTIVE) == (fuse == "1")
                s.set_system(A, b, x0)
                x, st = s.solve(x0.copy(), eps=1e-6)
                xf, _ = s.solve(x0.copy(), eps=-1.0, max_iter=3)
                s.set_x(x0)
                s.begin()
                d1, _ = s.iterate(1, eps=1e-6)
                d2, conv = s.iterate(100, eps=1e-6)
                xp = s.get_x()
            res[(fuse, gated)] = (x, st.iterations, xf, xp, d1 + d2, conv)
    bits = lambda v: v.view(np.uint32)
    for key, (x, it, xf, xp, dp, conv) in res.items():
        assert it == sr.iterations and np.array_equal(bits(x), bits(xr)), key
        assert np.array_equal(bits(xf), bits(res[("0", "0")][2])), key
        assert conv and dp == it and np.array_equal(bits(xp), bits(xr)), key


def test_errors_are_reported():
    with cg.Solver(8) as s:
        with pytest.raises(cg.CgxError) as ei:
            s.iterate(1)
        assert ei.value.code == -6
    with pytest.raises(cg.CgxError):
        cg.Solver(8, device=99)


@pytest.mark.parametrize("shards", [None, [0, 0]])
def test_host_streamed_matvec(monkeypatch, shards):
    """CGX_HOST_STREAM (configs[3] design): A in pinned host memory, row tiles
    streamed through 3 device buffers.  Row sums are the resident kernel's
    (same per-lane order), so the solve matches the resident one to rounding
    of the separate p.Ap reduction, and F32_REF stays bit-exact."""
    monkeypatch.setenv("CGX_STREAM_TILE_MB", "1")  # 1 MiB tiles: many tiles per matVec
    n = 2048
    A, b = oracle.spd_hash(n, seed=5)
    flags = cg.CGX_F64 | cg.CGX_HOST_STREAM | cg.CGX_TIMING
    with cg.Solver(n, flags=flags, devices=shards) as s:
        s.set_system(A, b)
        x, st = s.solve(None, eps=1e-10)
        assert s.stats().matvec_count == st.iterations  # x0 = 0: no initial A x0
    with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_HOST_STREAM, devices=shards) as s:
        s.generate_spd(seed=5)  # generated tile by tile on the device, kept on the host
        xg, stg = s.solve(None, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert st.iterations == stg.iterations == so.iterations
    assert rel(x, xo) <= TOL and rel(xg, xo) <= TOL
    A32, b32, x032 = case("spd1024")
    with cg.Solver(1024, flags=cg.CGX_F32_REF | cg.CGX_HOST_STREAM, devices=shards) as s:
        s.set_system(A32, b32, x032)
        x32, st32 = s.solve(None, eps=1e-6)
    ref, sr = oracle.cg_f32ref(A32, b32, x032, nparts=len(shards) if shards else 1, combine="mpich")
    assert st32.iterations == sr.iterations
    assert np.array_equal(x32, ref)


@pytest.mark.parametrize("resident_mb,shards", [("5", None), ("5", [0, 0]), ("1000", None)])
def test_host_streamed_with_resident_rows(monkeypatch, resident_mb, shards):
    """CGX_STREAM_RESIDENT_MB: the first rows of each shard's block stay in
    HBM and only the rest streams (an out-of-core matrix keeps what fits).
    The row sums are the same whichever plan adds them, so x is bit for bit
    the fully streamed solve's -- rows set on the host, generated on the
    device, an A replaced between solves (the resident copy follows), all
    rows resident (1000 MB) -- and F32_REF stays the reference's."""
    monkeypatch.setenv("CGX_STREAM_TILE_MB", "1")
    n = 2048  # 16 KiB rows: 5 MB keeps 320 of them
    A, b = oracle.spd_hash(n, seed=5)
    A2, b2 = oracle.spd_hash(n, seed=6)
    out = {}
    for res in ("0", resident_mb):
        monkeypatch.setenv("CGX_STREAM_RESIDENT_MB", res)
        with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_HOST_STREAM, devices=shards) as s:
            s.set_system(A, b)
            x1, st1 = s.solve(None, eps=1e-10)
            s.begin()
            s.iterate(4, eps=-1.0)  # left in flight: set_system must wait for its copies of A
            s.set_system(A2, b2)
            x2, st2 = s.solve(np.zeros(n), eps=1e-10)
            s.generate_spd(seed=5)
            x3, st3 = s.solve(None, eps=1e-10)
        A32, b32, x032 = case("spd1024")
        with cg.Solver(1024, flags=cg.CGX_F32_REF | cg.CGX_HOST_STREAM, devices=shards) as s:
            s.set_system(A32, b32, x032)
            x4, st4 = s.solve(None, eps=1e-6)
        out[res] = [(x1, st1.iterations), (x2, st2.iterations), (x3, st3.iterations), (x4, st4.iterations)]
    for (xa, ia), (xb, ib) in zip(out["0"], out[resident_mb]):
        assert ia == ib and np.array_equal(xa.view(np.uint8), xb.view(np.uint8))
    xo, so = oracle.cg_f64(A2, b2, np.zeros(n), eps=1e-10)
    assert out["0"][1][1] == so.iterations and rel(out["0"][1][0], xo) <= TOL
    ref, sr = oracle.cg_f32ref(A32, b32, x032, nparts=len(shards) if shards else 1, combine="mpich")
    assert np.array_equal(out[resident_mb][3][0], ref)


# ---------------------------------------------------------------------------
# matrix-free 5-point Poisson (configs[4]); oracle: oracle_cg_poisson_f64
# ---------------------------------------------------------------------------
# The stopping test is absolute (sqrt(r.r) < eps, serialConjugate.c:235).  With
# b = 1, ||b|| = m, and the attainable residual is about cond(A) * 2^-53 * ||b||
# (cond ~ 0.4 m^2): at m = 520, eps = 1e-10 sits at that floor, where the loop
# count depends on rounding (both the split and the fused GPU iteration stop
# 2 iterations before the sequential oracle).  The large case uses eps = 1e-7.
@pytest.mark.parametrize("m,shards,eps", [(1, None, 1e-10), (7, None, 1e-10), (64, None, 1e-10), (64, [0, 0], 1e-10),
                                          (64, [0] * 4, 1e-10), (96, [0] * 8, 1e-10), (130, [0, 0], 1e-10),
                                          (520, [0] * 4, 1e-7)])
def test_poisson_matches_oracle(m, shards, eps):
    n = m * m
    with cg.Solver(None, poisson_m=m, devices=shards) as s:
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=eps)
        rn, bn = s.residual_norm()
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=eps)
    assert st.iterations == so.iterations
    assert rel(x, xo) <= TOL
    assert rn <= 10 * eps
    assert np.linalg.norm(oracle.poisson_apply(m, x) - 1.0) <= 1e-9 * np.sqrt(n)


@pytest.mark.parametrize("shards", [None, [0] * 4])
@pytest.mark.parametrize("gated", ["1", "0"])
def test_poisson_fused_iteration_matches_split(monkeypatch, shards, gated):
    """The fused two-kernel iteration (k_poisson_p + k_poisson_xr, 64 B/point)
    against the stencil / r / x,p split (CGX_POISSON_FUSED=0): same loop count,
    x to 1e-12, with device-side gating on and off; odd m runs the split."""
    m = 96
    monkeypatch.setenv("CGX_GATED", gated)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("CGX_POISSON_FUSED", fused)
        with cg.Solver(None, poisson_m=m, devices=shards) as s:
            assert bool(s.info.flags & cg.CGX_FUSED_ACTIVE) == (fused == "1")
            s.fill(1.0, 0.0)
            res[fused] = s.solve(None, eps=1e-10)
    (xf, stf), (xs, sts) = res["1"], res["0"]
    assert stf.converged and sts.converged and stf.iterations == sts.iterations
    assert rel(xf, xs) <= 1e-12
    monkeypatch.setenv("CGX_POISSON_FUSED", "1")
    with cg.Solver(None, poisson_m=7) as s:
        assert not s.info.flags & cg.CGX_FUSED_ACTIVE


@pytest.mark.parametrize("m,P,eps", [(96, 4, 1e-10), (256, 2, 1e-8), (64, 8, 1e-10)])
def test_poisson_halo_overlap_matches(monkeypatch, m, P, eps):
    """Several slabs: r's halo exchange runs on the comm streams while
    k_poisson_p does the slab's interior runs; its two edge runs follow the
    exchange and add their p.Ap share.  Same loop count and x (to 1e-12) as the
    exchange-then-kernel order (CGX_HALO_OVERLAP=0), gated and host-checked.
    In one process the overlap exists with the peer-copy exchange
    (CGX_LOCAL_XCHG=copy; the default pull has nothing to overlap).
    (eps above the attainable-residual floor: see test_poisson_matches_oracle.)"""
    n = m * m
    monkeypatch.setenv("CGX_LOCAL_XCHG", "copy")
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=eps)
    for gated in ("1", "0"):
        monkeypatch.setenv("CGX_GATED", gated)
        res = []
        for ov in ("1", "0"):
            monkeypatch.setenv("CGX_HALO_OVERLAP", ov)
            with cg.Solver(None, poisson_m=m, devices=[0] * P) as s:
                s.fill(1.0, 0.0)
                res.append(s.solve(None, eps=eps))
        (x1, st1), (x0, st0) = res
        assert st1.iterations == st0.iterations == so.iterations
        assert rel(x1, x0) <= 1e-12 and rel(x1, xo) <= TOL


def _poisson_x_runs(m, shards, xdefer, monkeypatch):
    """x after each way of driving a fused Poisson solve (x updated every other
    iteration, or every iteration with CGX_POISSON_XDEFER=0)."""
    monkeypatch.setenv("CGX_POISSON_XDEFER", xdefer)
    out = {}
    with cg.Solver(None, poisson_m=m, devices=shards) as s:
        assert s.info.flags & cg.CGX_FUSED_ACTIVE
        assert bool(s.info.flags & cg.CGX_XDEFER_ACTIVE) == (xdefer != "0")
        assert bool(s.info.flags & cg.CGX_XDEFER3_ACTIVE) == (xdefer == "3")
        for gated in ("1", "0"):
            monkeypatch.setenv("CGX_GATED", gated)
            s.fill(1.0, 0.0)
            x, st = s.solve(None, eps=1e-10)
            out["solve" + gated] = (x, st.iterations)
        for count in (1, 2, 3, 7, 8, 9):  # fixed count, every residue of 2 and 3
            s.fill(1.0, 0.0)
            s.begin()
            d, _ = s.iterate(count, eps=-1.0)
            out[f"fixed{count}"] = (s.get_x(), d)
        s.fill(1.0, 0.0)  # pieces of odd length, then convergence-tested
        s.begin()
        s.iterate(3, eps=-1.0)
        s.iterate(5, eps=-1.0)
        d, c = s.iterate(10 ** 6, eps=1e-10)
        out["pieces"] = (s.get_x(), d, c)
    return out


@pytest.mark.parametrize("period", ["2", "3"])
@pytest.mark.parametrize("m,shards", [(64, None), (96, [0] * 4), (130, [0, 0]), (1040, None)])
def test_poisson_x_every_other_iteration_is_bitwise(monkeypatch, m, shards, period):
    """k_poisson_xr_f64 updates x every other (every third: the default) iteration
    (the left-out iterations' alphas kept, p_{k-1} (and p_{k-2}) read from the
    other slabs; 60 (58.7) instead of 64 B per point) with the every-iteration
    update's FMAs in the same order: x is bit for bit CGX_POISSON_XDEFER=0's
    after every way a solve can end (gated and host-checked convergence at every
    residue, fixed counts 1/2/3/7/8/9, pieces of 3 and 5), with the same loop
    counts."""
    monkeypatch.setenv("CGX_POISSON_FUSED", "1")
    a = _poisson_x_runs(m, shards, period, monkeypatch)  # x every 2nd / 3rd iteration (3: a third p slab)
    b = _poisson_x_runs(m, shards, "0", monkeypatch)
    assert a.keys() == b.keys()
    for key in a:
        assert np.array_equal(a[key][0], b[key][0]), key
        assert a[key][1:] == b[key][1:], key
    if m >= 520:  # eps = 1e-10 is below the attainable residual there (test_poisson_matches_oracle)
        return
    n = m * m
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=1e-10)
    assert a["solve1"][1] == a["solve0"][1] == so.iterations
    assert rel(a["solve1"][0], xo) <= TOL


@pytest.mark.parametrize("period", ["2", "3"])
@pytest.mark.parametrize("m,shards", [(1024, None), (1024, [0, 0]), (512, [0] * 4)])
def test_poisson_xr_pipelined_kernel_is_bitwise(monkeypatch, m, shards, period):
    """The software-pipelined x catch-up (k_poisson_xr_pipe_f64, the default
    for full 512-column strips and 8-row items) does k_poisson_xr_f64's
    arithmetic row by row and item by item in the same order on the same
    grid: x and the loop counts are bit for bit the plain kernel's
    (CGX_POISSON_PLAN=pipe=0) after every way a solve can end, with x every
    other and every third iteration."""
    monkeypatch.setenv("CGX_POISSON_FUSED", "1")
    monkeypatch.delenv("CGX_POISSON_PLAN", raising=False)
    a = _poisson_x_runs(m, shards, period, monkeypatch)
    monkeypatch.setenv("CGX_POISSON_PLAN", "pipe=0")
    b = _poisson_x_runs(m, shards, period, monkeypatch)
    assert a.keys() == b.keys()
    for key in a:
        assert np.array_equal(a[key][0], b[key][0]), key
        assert a[key][1:] == b[key][1:], key


@pytest.mark.parametrize("m,shards", [(96, [0] * 4), (130, [0, 0]), (1024, [0] * 8), (512, [0] * 2)])
def test_poisson_local_pull_bitwise_equal_copies(monkeypatch, m, shards):
    """One process, several slabs: k_poisson_p reads r's halo rows in place
    from the neighbouring slabs (system-scope loads after the r.r combine's
    events), and the two scalar combines are summed by the kernels that use
    them (p.Ap by k_poisson_xr, r.r by the next k_poisson_p; a combine kernel
    only when the host reads r.r).  Against round 3's per-neighbour peer
    copies with combine kernels (CGX_LOCAL_XCHG=copy) and the pull with
    combine kernels (CGX_LOCAL_FUSE=0): x and the loop counts bit for bit,
    gated, host-checked, fixed counts and pieces, x every third iteration.
    (The copies run before k_poisson_p, CGX_HALO_OVERLAP=0: behind its interior
    runs p.Ap would add the edge runs' share separately, other bits.)"""
    monkeypatch.setenv("CGX_POISSON_FUSED", "1")
    monkeypatch.setenv("CGX_HALO_OVERLAP", "0")
    res = {}
    for form in ("pull", "nofuse", "copy"):
        monkeypatch.setenv("CGX_LOCAL_XCHG", "copy" if form == "copy" else "kernel")
        monkeypatch.setenv("CGX_LOCAL_FUSE", "0" if form == "nofuse" else "1")
        res[form] = _poisson_x_runs(m, shards, "3", monkeypatch)
    for form in ("pull", "nofuse"):
        assert res[form].keys() == res["copy"].keys()
        for key in res["copy"]:
            assert np.array_equal(res[form][key][0], res["copy"][key][0]), (form, key)
            assert res[form][key][1:] == res["copy"][key][1:], (form, key)
    if m <= 130:  # eps 1e-10 is above the attainable-residual floor only on small grids (test_poisson_matches_oracle)
        n = m * m
        xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=1e-10)
        assert res["pull"]["solve1"][1] == so.iterations and rel(res["pull"]["solve1"][0], xo) <= 1e-9


def test_poisson_fused_in_pieces_and_iteration_cap():
    """Iterations issued in several cgx_iterate calls (fixed count, then
    convergence-tested) give the one-call solve; a cap that stops exactly at
    the converging iteration still reports convergence."""
    m = 64
    n = m * m
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=1e-10)
    with cg.Solver(None, poisson_m=m) as s:
        s.fill(1.0, 0.0)
        s.begin()
        d1, c1 = s.iterate(5, eps=-1.0)
        d2, c2 = s.iterate(10 ** 6, eps=1e-10)
        assert d1 == 5 and not c1 and c2 and 5 + d2 == so.iterations
        assert rel(s.get_x(), xo) <= TOL
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=1e-10, max_iter=so.iterations)
        assert st.converged and st.iterations == so.iterations
        assert rel(x, xo) <= TOL


def test_poisson_equals_dense_operator():
    """The stencil is the explicit matrix: same solve through the dense path."""
    m = 16
    A = oracle.poisson_dense(m)
    b = np.random.default_rng(0).random(m * m)
    with cg.Solver(None, poisson_m=m) as s:
        s.set_rows(0, None, b, np.zeros(m * m))
        xs, sts = s.solve(None, eps=1e-12)
    xd = np.zeros(m * m)
    std = cg.conjugrad(A, b, xd, eps=1e-12)
    assert sts.iterations == std.iterations
    assert rel(xs, xd) <= 1e-12


@pytest.mark.parametrize("halo", ["default", "force"])
def test_poisson_rank_mode_world1_and_fixed_count(monkeypatch, halo):
    """Rank mode at world size 1; `force` also runs the overlapped r halo
    exchange (empty ncclSend/Recv group on the comm stream, split k_poisson_p)."""
    if halo == "force":
        monkeypatch.setenv("CGX_HALO_OVERLAP", "force")
    m = 128
    with cg.Solver(None, poisson_m=m, rank=0, nranks=1, unique_id=cg.get_unique_id()) as s:
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=-1.0, max_iter=150)
    xo, so = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), eps=-1.0, max_iter=150)
    assert st.iterations == so.iterations == 150
    assert rel(x, xo) <= 1e-9
    with cg.Solver(None, poisson_m=m, rank=0, nranks=1, unique_id=cg.get_unique_id()) as s:
        s.fill(1.0, 0.0)
        x, st = s.solve(None, eps=1e-8)  # convergence-tested (device-gated)
    xo, so = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), eps=1e-8)
    assert st.converged and st.iterations == so.iterations and rel(x, xo) <= TOL


def test_poisson_rejects_bad_use():
    with pytest.raises(cg.CgxError):
        cg.Solver(None, poisson_m=10, devices=[0, 0, 0])   # 10 % 3
    with pytest.raises(cg.CgxError):
        cg.Solver(None, poisson_m=8, flags=cg.CGX_F32_REF)
    with cg.Solver(None, poisson_m=8) as s:
        with pytest.raises(cg.CgxError):
            s.generate_spd(1)
        with pytest.raises(cg.CgxError):
            s.set_rows(0, np.zeros((64, 64)), np.ones(64))


@pytest.mark.parametrize("P", [2, 4, 8])
def test_overlap_choice_is_bitwise_neutral(monkeypatch, P):
    """Aligned row blocks: the context times both whole forms at creation and
    picks the overlapped form (own column block beside the exchange, then the
    rest) or the plain one (the exchange, then one launch).  The one launch sums the own block and the
    rest apart and adds them, as the two launches do: x is the same bits in
    every form (forced on, forced off by env or flag, measured), gated and
    fixed-count, from x0 = 0 and from a nonzero x0; all == oracle."""
    n = 2048
    A, b = oracle.spd_hash(n, seed=11)
    x0 = np.full(n, 0.125)
    res = {}
    for form, env, flags in (("on", "1", 0), ("off", "0", 0), ("flag", None, cg.CGX_NO_OVERLAP),
                             ("measured", None, 0)):
        if env is None:
            monkeypatch.delenv("CGX_OVERLAP", raising=False)
        else:
            monkeypatch.setenv("CGX_OVERLAP", env)
        with cg.Solver(n, flags=cg.CGX_F64 | flags, devices=[0] * P) as s:
            info = s.overlap_info()
            on = bool(s.info.flags & cg.CGX_OVERLAP_ACTIVE)
            assert info["on"] == on and info["one_launch_us"] > 0 and info["allgather_us"] > 0
            assert info["overlap_form_us"] > 0 and info["plain_form_us"] > 0 and info["margin"] == 0.01
            assert 0 < info["forms_ms"] < 60_000
            assert info["decided_by"] == {"on": "forced_on", "off": "off", "flag": "off"}.get(form, "measured")
            assert on == {"on": True, "off": False, "flag": False}.get(form, cg.overlap_rule(info))
            s.set_system(A, b)
            xg, st = s.solve(None, eps=1e-10)
            xf, _ = s.solve(x0, eps=-1.0, max_iter=9)
        res[form] = (xg, st.iterations, xf)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    ref = res["on"]
    assert ref[1] == so.iterations and rel(ref[0], xo) <= TOL
    for form, r in res.items():
        assert r[1] == ref[1] and np.array_equal(r[0], ref[0]) and np.array_equal(r[2], ref[2]), form


@pytest.mark.parametrize("P", [2, 4])
def test_p2p_exchange_mode(P):
    """CGX_COMM_P2P (point-to-point_cg.c's gather-to-root + send-to-all) gives
    the collective mode's results bit for bit (fp64: both sum scalars in rank
    order); F32_REF == oracle with P-part dots (point-to-point_cg.c allSum)."""
    A, b, x0 = case("spd1024", np.float64)
    out = {}
    for flags in (cg.CGX_F64 | cg.CGX_NO_OVERLAP, cg.CGX_F64 | cg.CGX_COMM_P2P):
        with cg.Solver(b.size, flags=flags, devices=[0] * P) as s:
            s.set_system(A, b, x0)
            out[flags] = s.solve(None, eps=1e-10)
    (xa, sa), (xb, sb) = out.values()
    assert sa.iterations == sb.iterations and np.array_equal(xa, xb)
    A32, b32, x032 = case("spd1024")
    with cg.Solver(b.size, flags=cg.CGX_F32_REF | cg.CGX_COMM_P2P, devices=[0] * P) as s:
        s.set_system(A32, b32, x032)
        x32, st32 = s.solve(None, eps=1e-6)
    ref, sr = oracle.cg_f32ref(A32, b32, x032, nparts=P, combine="rank")
    assert st32.iterations == sr.iterations and np.array_equal(x32, ref)
    uid = cg.get_unique_id()
    with cg.Solver(b.size, flags=cg.CGX_F64 | cg.CGX_COMM_P2P, rank=0, nranks=1, unique_id=uid) as s:
        s.set_system(A, b, x0)
        x1, s1 = s.solve(None, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert s1.iterations == so.iterations and rel(x1, xo) <= TOL


def test_p2p_local_exchange_is_ordered():
    """Multi-shard CGX_COMM_P2P: shard 0 gathers, then every shard copies from
    it.  Shard 0's next kernels must wait for those copies (with x0 gathered
    for A x0 the residual rewrote shard 0's p while the others were still
    copying it: wrong x in about 1 solve in 5).  Repeated short fixed-count
    solves, each bit-exact to the P-part oracle (allSum order)."""
    A, b, x0 = case("kat4")
    for _ in range(10):
        for it in (1, 2, 3, 4):
            with cg.Solver(4, flags=cg.CGX_F32_REF | cg.CGX_COMM_P2P, devices=[0, 0]) as s:
                s.set_system(A, b, x0)
                x, _ = s.solve(None, eps=-1.0, max_iter=it)
            xo, _ = oracle.cg_f32ref(A, b, x0, eps=-1.0, max_iter=it, nparts=2, combine="rank")
            assert np.array_equal(x.view(np.uint32), xo.view(np.uint32)), it


@pytest.mark.parametrize("n,P", [(1, 1), (3, 3), (1001, 7), (1000, 8), (640, 5)])
def test_ragged_sizes_and_blocks(n, P):
    """Odd n, row blocks of odd length (unaligned vector slices -> scalar
    kernels), blocks not 128-aligned (no overlap): fp64 within 1e-10 of the
    oracle, F32_REF bit-exact to the P-part oracle (MPICH order, also for P
    that is not a power of two: pairs first, then the tree)."""
    A, b = oracle.spd_hash(n, seed=n)
    with cg.Solver(n, devices=[0] * P) as s:
        s.set_system(A, b)
        x, st = s.solve(None, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert st.iterations == so.iterations and rel(x, xo) <= TOL
    A32, b32 = A.astype(np.float32), b.astype(np.float32)
    with cg.Solver(n, flags=cg.CGX_F32_REF, devices=[0] * P) as s:
        s.set_system(A32, b32)
        x32, st32 = s.solve(None, eps=1e-6)
    ref, sr = oracle.cg_f32ref(A32, b32, np.zeros(n, np.float32), nparts=P, combine="mpich")
    assert st32.iterations == sr.iterations and np.array_equal(x32, ref)


@pytest.mark.parametrize("n,P", [(129, 1), (4095, 1), (4097, 1), (5000, 1), (8191, 1), (9000, 2)])
def test_f32ref_partial_dot_chunks(n, P):
    """The sequential dots walk 4096-element chunks; a short chunk (n below
    4096, or the last one) runs the pipelined chain over +0 padding.  Sizes
    around and past one chunk, on one GPU and as two row blocks of 4500:
    x and the loop count bit for bit the P-part oracle's."""
    A, b = oracle.spd_hash(n, seed=n)
    A32, b32 = A.astype(np.float32), b.astype(np.float32)
    del A
    x0 = np.zeros(n, np.float32)
    with cg.Solver(n, flags=cg.CGX_F32_REF, devices=[0] * P if P > 1 else None) as s:
        s.set_system(A32, b32, x0)
        x, st = s.solve(None, eps=1e-6)
    ref, sr = oracle.cg_f32ref(A32, b32, x0, nparts=P, combine="mpich")
    assert st.iterations == sr.iterations and st.converged == 1
    assert np.array_equal(x.view(np.uint32), ref.view(np.uint32))
    assert np.float32(st.rr) == np.float32(sr.rr)


@pytest.mark.parametrize("n,P,seed", [(777, 3, 1), (1000, 4, 2), (2304, 2, 3)])
def test_f32ref_bit_exact_many_iterations(n, P, seed):
    """A harder system than generateSPDmatrix (eigenvalues spread over two
    decades, so 30-80 iterations instead of 4-5) from a nonzero x0: the
    F32_REF path must still reproduce the reference's loop bit for bit,
    iteration after iteration, with the P-part dot order."""
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    lam = np.logspace(0, 2, n)
    A = ((Q * lam) @ Q.T).astype(np.float32)
    A = (A + A.T) / np.float32(2)
    b = rng.random(n, dtype=np.float32)
    x0 = (rng.random(n, dtype=np.float32) - np.float32(0.5))
    with cg.Solver(n, flags=cg.CGX_F32_REF, devices=[0] * P) as s:
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-4)
    ref, sr = oracle.cg_f32ref(A, b, x0, eps=1e-4, nparts=P, combine="mpich")
    assert st.iterations == sr.iterations and st.iterations >= 20
    assert np.array_equal(x.view(np.uint32), ref.view(np.uint32))


def test_max_iter_cap_and_nonconvergence():
    """Loop bound k < n (serialConjugate.c:213): a system that cannot meet eps
    stops after exactly n iterations, unconverged."""
    A, b, x0 = case("kat4", np.float64)
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=0.0)           # sqrt(rr) < 0 never holds
    assert st.iterations == 4 and st.converged == 0
    assert np.allclose(x, [-1, 1, -1, 1], atol=1e-10)
    x = x0.copy()
    st = cg.conjugrad(A, b, x, eps=1e-12, max_iter=2)
    assert st.iterations == 2 and st.converged == 0


@pytest.mark.parametrize("shards", [None, [0, 0, 0, 0]])
def test_device_gated_convergence_matches_host_checked(monkeypatch, shards):
    """Device-side stopping decision (default for fp64) == the host-checked
    loop (CGX_GATED=0): same loop count, same x bits, no extra iteration
    leaks into x; stats report the converged count and r.r."""
    A, b = oracle.spd_hash(2048, seed=3)
    res = {}
    for gated in ("1", "0"):
        monkeypatch.setenv("CGX_GATED", gated)
        for look in ("1", "2", "5"):
            monkeypatch.setenv("CGX_LOOKAHEAD", look)
            with cg.Solver(2048, devices=shards) as s:
                s.set_system(A, b)
                x, st = s.solve(None, eps=1e-10)
                res[(gated, look)] = (x, st.iterations, st.converged, st.rr, s.stats().total_iterations)
    ref = res[("0", "1")]
    for key, (x, it, conv, rr, tot) in res.items():
        assert it == ref[1] and conv == 1 and tot == it, key
        assert np.array_equal(x, ref[0]), key
        assert rr == ref[3] and np.sqrt(rr) < 1e-10
    xo, so = oracle.cg_f64(A, b, np.zeros(2048), eps=1e-10)
    assert ref[1] == so.iterations and rel(ref[0], xo) <= TOL


@pytest.mark.parametrize("case_name,shards", [("spd512", None), ("spd1024", [0, 0]), ("spd2048", [0, 0, 0, 0]),
                                             ("kat4", None), ("kat2_x0", None)])
def test_f32ref_device_gated_equals_host_checked_and_reference(monkeypatch, case_name, shards):
    """CGX_F32_REF with the stopping decision on the device (default) and
    host-checked (CGX_GATED=0), at every lookahead: the same loop count and
    x bits as the reference (serial, or the P-part oracle in MPICH order),
    no extra iteration leaking into x, the converged r.r reported."""
    A, b, x0 = case(case_name, np.float32)
    n = A.shape[0]
    P = len(shards) if shards else 1
    xr, sr = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=P, combine="mpich")
    for gated in ("1", "0"):
        monkeypatch.setenv("CGX_GATED", gated)
        for look in ("1", "2", "5"):
            monkeypatch.setenv("CGX_LOOKAHEAD", look)
            with cg.Solver(n, flags=cg.CGX_F32_REF, devices=shards) as s:
                s.set_system(A, b, x0)
                x, st = s.solve(x0.copy(), eps=1e-6)
                assert st.iterations == sr.iterations and st.converged == 1, (gated, look)
                assert s.stats().total_iterations == st.iterations, (gated, look)
                assert np.array_equal(x.view(np.uint32), xr.view(np.uint32)), (gated, look)
                assert np.float32(st.rr) == np.float32(sr.rr) and np.sqrt(st.rr) < 1e-6


def test_poisson_fixed_count_is_deterministic():
    """The same fixed-count Poisson solve twice on one context: x bit for bit
    (fixed-order reductions; x0 reset, since begin() starts from the current x)."""
    xs = []
    with cg.Solver(None, poisson_m=520) as s:
        for _ in range(2):
            s.fill(1.0, 0.0)
            x, _ = s.solve(None, eps=-1.0, max_iter=25)
            xs.append(x)
    assert np.array_equal(xs[0].view(np.uint8), xs[1].view(np.uint8))
