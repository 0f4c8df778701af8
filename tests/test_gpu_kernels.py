"""Kernel-level parity (device pointers through the C ABI) on the GPU.

fp32-ref kernels must equal the oracle / numpy float32 bit for bit (the
reference's operation order).  fp64 kernels are checked against the oracle's
sequential fp64 loops with a stated tolerance: a reordered fp64 sum of n
terms differs by at most ~n * 2^-53 * sum|a_i b_i|; we use 1e-13 relative to
sum|a_i b_i| for n <= 8192 (bound 9e-13 worst case, ~1e-15 typical)."""
import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle

pytestmark = pytest.mark.gpu

F64_TOL = 1e-13


def dev(a, dtype=None):
    return cg.DeviceArray.from_host(np.ascontiguousarray(a, dtype=dtype))


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1, "no GPU visible: the HIP path must run"


@pytest.mark.parametrize("rows,cols", [(64, 1024), (40, 1000)])
def test_matvec_ref_f32_nonfinite_bitwise(rows, cols):
    """Inf, -Inf and NaN entries flow through the chains as in the reference
    (the zero products the default kernel gives padded columns stay exact)."""
    rng = np.random.default_rng(11)
    A = rng.random((rows, cols), dtype=np.float32) - 0.5
    A[3, 7], A[5, cols - 1], A[rows - 1, 0], A[9, 100] = np.inf, -np.inf, np.nan, 3e38
    v = rng.random(cols, dtype=np.float32) * 4
    out = cg.DeviceArray(rows, np.float32)
    cg.matVec(dev(A), dev(v), out, rows, cols)
    ref = oracle.matvec_f32ref(A, v)
    assert np.array_equal(out.to_host().view(np.uint32), ref.view(np.uint32))


# The 32-row blocks with two 512-column tiles in flight and a dedicated adding wave: their FULL form when
# rows % 32 == 0 and cols % 512 == 0, a bounds-checked form for other multiples of 4; the 16-row kernel
# when cols % 4 != 0 (rows not 16-B aligned).
@pytest.mark.parametrize("rows,cols", [(1, 1), (2, 2), (5, 3), (64, 64), (300, 257), (1000, 1000), (8192, 96),
                                       (16, 512), (17, 513), (33, 1536), (48, 1025), (100, 4100), (32, 512),
                                       (64, 1024), (96, 2560), (31, 4), (33, 516), (1024, 8192), (8192, 8192)])
def test_matvec_ref_f32_bitwise(rows, cols):
    rng = np.random.default_rng(rows * 7 + cols)
    A = rng.random((rows, cols), dtype=np.float32) - 0.5
    v = rng.random(cols, dtype=np.float32)
    out = cg.DeviceArray(rows, np.float32)
    cg.matVec(dev(A), dev(v), out, rows, cols)
    ref = oracle.matvec_f32ref(A, v)
    assert np.array_equal(out.to_host().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4096, 4097, 8192, 8193, 20000])
def test_dot_ref_f32_bitwise(n):
    rng = np.random.default_rng(n)
    a = rng.random(n, dtype=np.float32) - 0.5
    b = rng.random(n, dtype=np.float32)
    out = cg.DeviceArray(1, np.float32)
    cg.vecVec(dev(a), dev(b), out)
    assert out.to_host()[0].view(np.uint32) == oracle.dot_f32ref(a, b).view(np.uint32)


def test_vector_updates_ref_f32_bitwise():
    rng = np.random.default_rng(3)
    n = 5000
    f = np.float32
    b, Ax, x, p, Ap = (rng.random(n, dtype=f) for _ in range(5))
    r_d, p_d, rr_d = cg.DeviceArray(n, f), cg.DeviceArray(n, f), cg.DeviceArray(1, f)
    cg.residual(dev(b), dev(Ax), r_d, p_d, rr_d)
    r = b - Ax  # numpy float32: one rounding per op, like serialConjugate.c:129
    assert np.array_equal(r_d.to_host(), r) and np.array_equal(p_d.to_host(), r)
    assert rr_d.to_host()[0] == oracle.dot_f32ref(r, r)

    rsold, pAp = np.array([f(2.5)]), np.array([f(7.25)])
    x_d, r2_d, rr2_d = dev(x), dev(r), cg.DeviceArray(1, f)
    cg.update_xr(x_d, r2_d, dev(p), dev(Ap), dev(rsold), dev(pAp), rr2_d)
    alpha = f(rsold[0] / pAp[0])
    x_ref = x + p * alpha
    r_ref = r - Ap * alpha
    assert np.array_equal(x_d.to_host(), x_ref) and np.array_equal(r2_d.to_host(), r_ref)
    assert rr2_d.to_host()[0] == oracle.dot_f32ref(r_ref, r_ref)

    p_d2 = dev(p)
    cg.update_p(p_d2, dev(r_ref), dev(np.array([f(1.5)])), dev(rsold))
    ratio = f(f(1.5) / rsold[0])
    assert np.array_equal(p_d2.to_host(), r_ref + p * ratio)


@pytest.mark.parametrize("rows,cols,lda", [(1, 1, 1), (3, 5, 5), (7, 129, 131), (128, 128, 128),
                                           (1000, 1000, 1000), (4096, 4096, 4096), (33, 8192, 8200),
                                           (20000, 256, 256)])
def test_matvec_f64(rows, cols, lda):
    rng = np.random.default_rng(rows + cols)
    A = rng.random((rows, lda)) - 0.5
    v = rng.random(cols)
    out = cg.DeviceArray(rows, np.float64)
    cg.matVec(dev(A), dev(v), out, rows, cols, lda)
    ref = oracle.matvec_f64(np.ascontiguousarray(A[:, :cols]), v)
    scale = np.abs(A[:, :cols]) @ np.abs(v)
    assert np.all(np.abs(out.to_host() - ref) <= F64_TOL * scale + 1e-300)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 100000, 1 << 20])
def test_dot_and_updates_f64(n):
    rng = np.random.default_rng(n)
    a, b = rng.random(n) - 0.5, rng.random(n)
    out = cg.DeviceArray(1, np.float64)
    cg.vecVec(dev(a), dev(b), out)
    assert abs(out.to_host()[0] - a @ b) <= F64_TOL * (np.abs(a) @ np.abs(b))
    # deterministic: the same launch twice gives the same bits
    cg.vecVec(dev(a), dev(b), out)
    first = out.to_host()[0]
    cg.vecVec(dev(a), dev(b), out)
    assert out.to_host()[0] == first

    x, r, p, Ap = (rng.random(n) for _ in range(4))
    x_d, r_d, rr_d = dev(x), dev(r), cg.DeviceArray(1, np.float64)
    cg.update_xr(x_d, r_d, dev(p), dev(Ap), dev(np.array([3.0])), dev(np.array([4.0])), rr_d)
    alpha = 0.75
    np.testing.assert_allclose(x_d.to_host(), x + alpha * p, rtol=1e-15, atol=0)
    r_ref = r - alpha * Ap
    np.testing.assert_allclose(r_d.to_host(), r_ref, rtol=1e-13, atol=1e-15)
    assert abs(rr_d.to_host()[0] - r_ref @ r_ref) <= F64_TOL * (r_ref @ r_ref)


# every plan libcgx ships: R rows per wave x U chunks in flight x load policy
# (0 plain, 1 non-temporal, 2 / 8 pipelined plain / non-temporal = default); R=8 U=8
# pipelined spills and is never planned
MV_PLANS = [(R, U, nt) for R in (1, 2, 4, 8) for U in (2, 4, 8) for nt in (0, 1, 2, 8)
            if not (R == 8 and U == 8 and nt in (2, 8))]


@pytest.mark.parametrize("rows,cols", [(300, 2048), (2048, 4096), (5000, 5120), (8192, 8192), (77, 2560)])
def test_matvec_small_lds_bitwise_equals_l2_kernel(monkeypatch, rows, cols):
    """k_matvec_small_f64 (the vector staged in LDS, one block per CU; the
    solver's matVec on one GPU at 2048 <= lda <= 8192) sums every row as
    k_matvec_f64 does -- per lane, chunks in ascending order, then the wave
    sum -- so Ap is bit for bit the L2 kernel's: rows fewer than the grid's
    waves (77, 300), several rows per wave (5000, 8192), 4 chunks per step
    (2560 = 20 chunks).  CGX_MV_SMALL=2 routes the kernel-level cgx_matvec
    through it."""
    rng = np.random.default_rng(rows * 7 + cols)
    A = rng.random((rows, cols)) - 0.5
    v = rng.random(cols)
    A_d, v_d = dev(A), dev(v)
    out = cg.DeviceArray(rows)
    cg.matVec(A_d, v_d, out, rows, cols)
    base = out.to_host()
    assert np.all(np.abs(base - oracle.matvec_f64(A, v)) <= F64_TOL * (np.abs(A) @ np.abs(v)))
    monkeypatch.setenv("CGX_MV_SMALL", "2")
    for nt, u in (("512", "8"), ("512", "4"), ("1024", "4"), ("1024", "8")):
        monkeypatch.setenv("CGX_SMALL_PLAN", f"threads={nt},U={u}")
        out = cg.DeviceArray(rows)
        cg.matVec(A_d, v_d, out, rows, cols)
        assert np.array_equal(out.to_host(), base), (nt, u)


@pytest.mark.parametrize("rows,cols", [(300, 1000), (1000, 1024), (517, 2176), (2048, 4096), (8192, 3200)])
def test_matvec_f64_every_plan_bitwise_equal(monkeypatch, rows, cols):
    """Every (rows per wave, chunks in flight, load policy) plan, including the
    software-pipelined kernel (8) with chunk counts that are not a multiple of
    U, gives the same row sums bit for bit: each lane accumulates its columns
    in ascending order whatever the plan.  The default plan is checked against
    the fp64 oracle.  (The rejected variants are checked the same way by
    tools/microbench/matvec_variants.hip.)"""
    rng = np.random.default_rng(rows + cols)
    A = rng.random((rows, cols)) - 0.5
    v = rng.random(cols)
    A_d, v_d = dev(A), dev(v)
    ref = oracle.matvec_f64(A, v)
    out = cg.DeviceArray(rows)
    cg.matVec(A_d, v_d, out, rows, cols)
    base = out.to_host()
    bound = F64_TOL * (np.abs(A) @ np.abs(v))
    assert np.all(np.abs(base - ref) <= bound)
    for R, U, nt in MV_PLANS:
        monkeypatch.setenv("CGX_MV_PLAN", f"R={R},U={U},nt={nt}")
        out = cg.DeviceArray(rows)
        cg.matVec(A_d, v_d, out, rows, cols)
        assert np.array_equal(out.to_host(), base), (R, U, nt)
