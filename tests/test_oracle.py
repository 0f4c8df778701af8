"""The oracle (CPU restatement, oracle/cg_oracle.c) pinned against the
reference: bit-exact to the unmodified serialConjugate.c outputs in
tests/golden/, its generators against independent implementations."""
import hashlib

import numpy as np
import pytest

import oracle
from _cases import COMBINE_OF, KATS, SPD_ALL, SPD_SMALL, case, golden_mpi, golden_x, mpi_golden_x, mpi_runs


def test_mt19937_matches_numpy():
    # MATLAB `rng default` == MT19937(5489) + genrand_res53 == numpy RandomState(5489)
    ours = oracle.mt_res53(5000)
    ref = np.random.RandomState(5489).random_sample(5000)
    assert np.array_equal(ours, ref)
    assert np.allclose(ours[:5], [0.8147, 0.9058, 0.1270, 0.9134, 0.6324], atol=5e-5)


def test_spd_matlab_matches_numpy_restatement():
    # generateSPDmatrix.m:4-17 via numpy: column-major rand fill, 0.5(R+R') + nI, "%.4f"
    n = 48
    draws = np.random.RandomState(5489).random_sample(n * n + n)
    R = draws[: n * n].reshape(n, n).T
    A = 0.5 * (R + R.T) + n * np.eye(n)
    b = draws[n * n:]
    A32 = np.array([np.float32(f"{v:.4f}") for v in A.ravel()], np.float32).reshape(n, n)
    b32 = np.array([np.float32(f"{v:.4f}") for v in b], np.float32)
    oA, ob = oracle.spd_matlab(n, np.float32)
    assert np.array_equal(oA, A32) and np.array_equal(ob, b32)
    oA64, _ = oracle.spd_matlab(n, np.float64)
    assert np.array_equal(oA64, np.array([float(f"{v:.4f}") for v in A.ravel()]).reshape(n, n))
    assert np.array_equal(oA, oA.T)


@pytest.mark.parametrize("name", ["spd512", "spd1024", "spd2048"])
def test_golden_inputs_unchanged(golden, name):
    A, b, _ = case(name)
    g = golden["cases"][name]
    assert hashlib.sha256(A.tobytes()).hexdigest() == g["A_sha256"]
    assert hashlib.sha256(b.tobytes()).hexdigest() == g["b_sha256"]


@pytest.mark.parametrize("name", KATS + SPD_ALL)
def test_f32ref_bit_exact_vs_reference(golden, name):
    """oracle_cg_f32ref == unmodified serialConjugate.c, bit for bit, same loop count."""
    A, b, x0 = case(name)
    x, st = oracle.cg_f32ref(A, b, x0, eps=1e-6)
    ref = golden_x(golden, name)
    assert st.iterations == golden["cases"][name]["ref_iterations"]
    assert st.converged == 1
    assert np.array_equal(x.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name", KATS + SPD_SMALL)
def test_f64_oracle_matches_conjgrad_m(golden, name):
    A, b, x0 = case(name, np.float64)
    x, st = oracle.cg_f64(A, b, x0, eps=1e-10)
    xn, itn = oracle.conjgrad_numpy(A, b, x0, tol=1e-10)
    assert st.iterations == itn == golden["cases"][name]["conjgrad_m_f64_iterations"]
    assert np.linalg.norm(x - xn) <= 1e-12 * np.linalg.norm(xn)
    assert np.linalg.norm(b - A @ x) <= 1e-10 * np.linalg.norm(b)


def test_known_answers_f64():
    A, b, x0 = case("kat2", np.float64)
    x, _ = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert np.allclose(x, [2 / 3, 1 / 3], rtol=0, atol=1e-12)
    A, b, x0 = case("kat4", np.float64)
    x, _ = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert np.allclose(x, [-1, 1, -1, 1], rtol=0, atol=1e-12)


def test_reference_x_close_to_f64(golden):
    # fp32 reference vs fp64 solution: the 1e-5 parity pin (SURVEY.md s8(c) pin 3)
    for name in SPD_SMALL:
        A, b, x0 = case(name, np.float64)
        x64, _ = oracle.cg_f64(A, b, x0, eps=1e-10)
        ref = golden_x(golden, name).astype(np.float64)
        assert np.linalg.norm(ref - x64) <= 1e-5 * np.linalg.norm(x64)


def test_hash_generator_properties():
    n = 300
    A, b = oracle.spd_hash(n, seed=7)
    assert np.array_equal(A, A.T)
    off = A - np.diag(np.diag(A))
    assert off.min() >= 0 and off.max() < 1
    assert np.all(np.diag(A) >= n) and np.all(np.diag(A) < n + 1)
    assert b.min() >= 0 and b.max() < 1
    # rows are independent of the block they are generated in
    A2, b2 = oracle.spd_hash(n, seed=7, row0=100, nrows=50)
    assert np.array_equal(A2, A[100:150]) and np.array_equal(b2, b[100:150])
    # u(i, j) is the documented counter hash
    assert A[3, 5] == 0.5 * (oracle.hash_u01(7, 3, 5) + oracle.hash_u01(7, 5, 3))
    A32, b32 = oracle.spd_hash(n, seed=7, dtype=np.float32)
    assert np.array_equal(A32, A.astype(np.float32)) and np.array_equal(b32, b.astype(np.float32))


@pytest.mark.parametrize("key", mpi_runs())
def test_f32ref_nparts_bit_exact_vs_mpi_reference(key):
    """oracle_cg_f32ref(nparts=P) == the unmodified parallel_cg.c (combine
    "mpich") / point-to-point_cg.c (combine "rank") under mpiexec -np P, bit
    for bit, same loop count (tests/golden/mpi/)."""
    r = golden_mpi()["runs"][key]
    A, b, x0 = case(r["case"])
    assert hashlib.sha256(A.tobytes()).hexdigest() == r["A_sha256"]
    x, st = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=r["np"], combine=COMBINE_OF[r["program"]])
    assert st.iterations == r["ref_iterations"] and st.converged == 1
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


def test_mpi_goldens_discriminate_the_combine_order():
    """The fixtures pin the order: at np >= 4 the two MPI programs differ, and
    the wrong order misses the golden on most cases (np <= 2 the orders agree)."""
    runs = golden_mpi()["runs"]
    wrong = 0
    for key in mpi_runs(min_np=4, cases=KATS + SPD_SMALL):
        r = runs[key]
        A, b, x0 = case(r["case"])
        other = "rank" if COMBINE_OF[r["program"]] == "mpich" else "mpich"
        x, st = oracle.cg_f32ref(A, b, x0, eps=1e-6, nparts=r["np"], combine=other)
        wrong += not (st.iterations == r["ref_iterations"]
                      and np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32)))
    assert wrong >= 6
    # np=1: both programs reduce to serialConjugate.c
    g = {k: r for k, r in runs.items() if r["np"] == 1}
    assert len(g) == 16
    assert all(np.array_equal(mpi_golden_x(k), mpi_golden_x(k.replace("parallel_", "p2p_"))) for k in g
               if k.startswith("parallel_"))


def test_combine_orders():
    parts = np.array([1e8, 1.0, -1e8, 1.0, 3.0, 0.5, 0.25, 7.0], np.float32)
    seq = np.float32(0)
    for q, v in enumerate(parts):
        seq = v if q == 0 else np.float32(seq + v)
    assert oracle.combine_f32(parts, "rank") == seq
    t = lambda a, b: np.float32(a + b)  # noqa: E731
    tree = t(t(t(parts[0], parts[1]), t(parts[2], parts[3])), t(t(parts[4], parts[5]), t(parts[6], parts[7])))
    assert oracle.combine_f32(parts, "mpich") == tree
    # non-power-of-two: first 2*rem pairs, then the tree (MPICH recursive doubling)
    p6 = parts[:6]
    assert oracle.combine_f32(p6, "mpich") == t(t(t(p6[0], p6[1]), t(p6[2], p6[3])), t(p6[4], p6[5]))
    p3 = parts[:3]
    assert oracle.combine_f32(p3, "mpich") == t(t(p3[0], p3[1]), p3[2])


def test_nparts_dot_order():
    """nparts=P reorders only the dot products (point-to-point_cg.c allSum):
    P=1 is the serial result; P>1 stays within fp32 noise of it."""
    A, b, x0 = case("spd512")
    x1, s1 = oracle.cg_f32ref(A, b, x0, nparts=1)
    x1b, _ = oracle.cg_f32ref(A, b, x0)
    assert np.array_equal(x1, x1b)
    for P in (2, 4, 8):
        xp, sp = oracle.cg_f32ref(A, b, x0, nparts=P)
        assert np.linalg.norm(xp - x1) <= 1e-5 * np.linalg.norm(x1)
        assert abs(sp.iterations - s1.iterations) <= 1


def test_hash_oracle_without_storage_equals_stored():
    """cg_f64_hash (A regenerated per matVec, for N = 65536 / 131072) == cg_f64
    on the stored spd_hash system, bit for bit; its matVec rows likewise."""
    n = 700
    A, b = oracle.spd_hash(n, seed=9)
    v = np.random.default_rng(1).random(n)
    assert np.array_equal(oracle.hash_matvec_f64(n, v, seed=9), oracle.matvec_f64(A, v))
    assert np.array_equal(oracle.hash_matvec_f64(n, v, seed=9, row0=100, nrows=37), oracle.matvec_f64(A[100:137], v))
    oracle.set_threads(4)
    try:
        x1, s1 = oracle.cg_f64_hash(n, seed=9, eps=1e-10)
    finally:
        oracle.set_threads(1)
    x2, s2 = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert s1.iterations == s2.iterations and np.array_equal(x1, x2)


def test_fixed_count_mode():
    A, b, x0 = case("spd512", np.float64)
    _, st = oracle.cg_f64(A, b, x0, eps=-1.0, max_iter=12)
    assert st.iterations == 12 and st.converged == 0


def test_poisson_oracle_is_the_laplacian():
    m = 12
    A = oracle.poisson_dense(m)
    assert np.array_equal(A, A.T)
    assert np.all(np.linalg.eigvalsh(A) > 0)
    p = np.random.default_rng(2).random(m * m)
    assert np.abs(A @ p - oracle.poisson_apply(m, p)).max() <= 1e-14
    b = np.ones(m * m)
    x, st = oracle.cg_poisson_f64(m, b, np.zeros(m * m), eps=1e-10)
    xn, itn = oracle.conjgrad_numpy(A, b, np.zeros(m * m), tol=1e-10)
    assert st.iterations == itn
    assert np.linalg.norm(x - xn) <= 1e-12 * np.linalg.norm(xn)


def test_bench_reference_baseline_leg():
    """bench.py's cpu_baseline_reference: serialConjugate.c itself (oracle/_ref)
    at its compiled N=8192 on the bench generator's fp32 system; the same
    loop count as the bit-exact restatement on that system."""
    if not oracle.ref_binary():
        pytest.skip("oracle/_ref/serial_ref not built (no /root/reference here)")
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    r = bench.cpu_baseline_reference()
    assert r["kind"] == "reference" and r["cores"] == 1 and r["n"] == 8192 and r["value"] > 0
    A, b = oracle.spd_hash(8192, seed=bench.SEED, dtype=np.float32)
    _, st = oracle.cg_f32ref(A, b, np.zeros(8192, np.float32), eps=1e-6)
    assert f"{st.iterations} loop iterations" in r["sample"]
