// cgx_vector.hip -- the fp64 BLAS-1 kernels of the CG iteration (residual,
// the x/r/p updates with the device-side stopping decision, dot), the
// counter-hash SPD generator, fill and the rank-ordered scalar sum.
// serialConjugate.c:122-177 (vecVec, scalarVec, vecAdd, vecSub) and :209-243.
#include "cgx_device.h"

namespace cgx {
namespace {

// residual x2 + vecVec (serialConjugate.c:210-212).  Ax == nullptr: A x0 is
// exactly zero (x0 = 0), so r = b - 0.0 without reading an Ap buffer (the same
// operation, the same bits).  clear2 != nullptr: the solve's device-side
// convergence record {kdone, r.r} is reset here, by block 0, instead of by a
// separate memset launch (every gated kernel of the solve follows in stream
// order).
template <bool VEC>
__global__ __launch_bounds__(kNT) void k_residual_f64(int64_t n, const double *__restrict__ b,
                                                      const double *__restrict__ Ax,
                                                      double *__restrict__ r, double *__restrict__ p,
                                                      double *rr_out, double *partials,
                                                      unsigned *ticket, int64_t *clear2) {
    if (clear2 && blockIdx.x == 0 && threadIdx.x < 2) clear2[threadIdx.x] = 0;
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 bv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) { const int64_t i = 2 * (base + u * kNT); bv[u] = ld2(b + i); av[u] = Ax ? ld2(Ax + i) : (d2)(0.0); }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                const d2 ri = bv[u] - av[u];
                st2(r + i, ri);
                if (p) st2(p + i, ri);
                acc += ri.x * ri.x + ri.y * ri.y;
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const double ri = b[n - 1] - (Ax ? Ax[n - 1] : 0.0);
            r[n - 1] = ri;
            if (p) p[n - 1] = ri;
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            const double ri = b[i] - (Ax ? Ax[i] : 0.0);
            r[i] = ri;
            if (p) p[i] = ri;
            acc += ri * ri;
        }
    }
    if (rr_out) grid_sum_last_block(acc, partials, ticket, rr_out);
}

// x += alpha p; r -= alpha Ap; r.r  (serialConjugate.c:219-234, conjgrad.m:8-11)
template <bool VEC, int VP = 0>
__global__ __launch_bounds__(kNT) void k_update_xr_f64(int64_t n, double *__restrict__ x,
                                                       double *__restrict__ r,
                                                       const double *__restrict__ p,
                                                       const double *__restrict__ Ap,
                                                       const double *rsold, const double *pAp,
                                                       double *rr_out, double *partials,
                                                       unsigned *ticket) {
    const double alpha = cg_ratio(*rsold, *pAp);
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 xv[kVU], rv[kVU], pv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                xv[u] = ldv<VP>(x + i); rv[u] = ldv<VP>(r + i); pv[u] = ldv<VP>(p + i); av[u] = ldv<VP>(Ap + i);
            }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                stv<VP>(x + i, xv[u] + alpha * pv[u]);
                const d2 ri = rv[u] - alpha * av[u];
                stv<VP>(r + i, ri);
                acc += ri.x * ri.x + ri.y * ri.y;
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const int64_t i = n - 1;
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            r[i] = ri;
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            r[i] = ri;
            acc += ri * ri;
        }
    }
    grid_sum_last_block(acc, partials, ticket, rr_out);
}

// p = r + beta p  (serialConjugate.c:239-243, conjgrad.m:15)
template <bool VEC, int VP = 0>
__global__ __launch_bounds__(kNT) void k_update_p_f64(int64_t n, double *__restrict__ p,
                                                      const double *__restrict__ r,
                                                      const double *rr, const double *rsold) {
    const double beta = cg_ratio(*rr, *rsold);
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 pv[kVU], rv[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) { const int64_t i = 2 * (base + u * kNT); pv[u] = ldv<VP>(p + i); rv[u] = ldv<VP>(r + i); }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) stv<VP>(p + 2 * (base + u * kNT), rv[u] + beta * pv[u]);
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) p[n - 1] = r[n - 1] + beta * p[n - 1];
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
            p[i] = r[i] + beta * p[i];
    }
}

// The two-launch iteration (small systems, one GPU; cgx_iterate.hip): after
// the matVec (with its fused p.Ap) ONE kernel does
//   x += alpha p; r -= alpha Ap; r.r                 (every block, its rows)
// and the block that sums the r.r partials then decides the stop
// (serialConjugate.c:235) and, if the loop goes on, forms
//   p = r + (r.r / rsold) p                          (the whole vector)
// -- the update kernel of the three-launch iteration folded into this one's
// last block.  r crosses blocks inside the launch, so it is stored
// write-through (sc1) and that block reads it with sc1 loads (Guideline 16's
// one-counter row).  The expressions are the three-launch kernels' own, so
// x, r, p and r.r come out bit for bit the same.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t vec_rsrc(const double *p, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(n * 8), 0x00020000);
}
__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t rs, int64_t i, d2 v) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, (int)(i * 8), 0, 16);  // aux 16 = sc1
}
__device__ __forceinline__ d2 ld2_sc1(__amdgpu_buffer_rsrc_t rs, int64_t i) {
    return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 8), 0, 16));
}

template <bool VEC>
__global__ __launch_bounds__(kNT) void k_update_xrp_f64(int64_t n, double *__restrict__ x, double *__restrict__ r,
                                                        double *__restrict__ p, const double *__restrict__ Ap,
                                                        const double *rsold, const double *pAp, double *rr_out,
                                                        double *partials, unsigned *ticket, const int64_t *gate,
                                                        ConvArgs cv, int64_t *ts) {
    if (gate && *gate) return;
    ts_start(ts);
    const double rs = *rsold;
    const double alpha = cg_ratio(rs, *pAp);
    const __amdgpu_buffer_rsrc_t rrs = vec_rsrc(r, n);
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 xv[kVU], rv[kVU], pv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                xv[u] = ld2(x + i); rv[u] = ld2(r + i); pv[u] = ld2(p + i); av[u] = ld2(Ap + i);
            }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                st2(x + i, xv[u] + alpha * pv[u]);
                const d2 ri = rv[u] - alpha * av[u];
                st2_sc1(rrs, i, ri);
                acc += ri.x * ri.x + ri.y * ri.y;
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const int64_t i = n - 1;
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            __hip_atomic_store(r + i, ri, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            __hip_atomic_store(r + i, ri, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += ri * ri;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's r stores land before the ticket
    double rr;
    if (!grid_sum_keep_last(acc, partials, ticket, rr_out, rr)) {
        ts_end(ts);
        return;
    }
    // ---- the last block: the stopping test, then p = r + beta p for all of p
    if (cv.kdone && cv.eps >= 0.0 && sqrt(rr) < cv.eps) {
        if (threadIdx.x == 0) record_convergence(cv, cv.k + 1, rr);
        ts_end(ts);
        return;
    }
    const double beta = cg_ratio(rr, rs);
    if constexpr (VEC) {
        // One CU does all of p: every load of a thread's share (up to kPU
        // pairs, n <= 8192 in one step) is issued before the first store, so
        // the pass costs one round trip to memory instead of one per kVU pairs
        // (n = 8192: 4 dependent steps before).
        constexpr int kPU = 16;
        const int64_t npairs = n >> 1;
        for (int64_t b0 = threadIdx.x; b0 < npairs; b0 += (int64_t)kNT * kPU) {
            d2 rv[kPU], pv[kPU];
#pragma unroll
            for (int u = 0; u < kPU; ++u)
                if (b0 + u * kNT < npairs) {
                    const int64_t i = 2 * (b0 + u * kNT);
                    rv[u] = ld2_sc1(rrs, i);
                    pv[u] = ld2(p + i);
                }
#pragma unroll
            for (int u = 0; u < kPU; ++u)
                if (b0 + u * kNT < npairs) st2(p + 2 * (b0 + u * kNT), rv[u] + beta * pv[u]);
        }
        if ((n & 1) && threadIdx.x == 0)
            p[n - 1] = __hip_atomic_load(r + n - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + beta * p[n - 1];
    } else {
        for (int64_t i = threadIdx.x; i < n; i += kNT)
            p[i] = __hip_atomic_load(r + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + beta * p[i];
    }
    ts_end(ts);
}

// The update of the folded two-launch iteration (k_matvec_fold_f64 formed
// p_k): x += alpha p_k; r -= alpha Ap; r.r, and the block that sums the r.r
// partials decides the stop (serialConjugate.c:235).  Fully parallel: the
// p update is the next matVec's.  The expressions are k_update_xrp_f64's.
template <bool VEC>
__global__ __launch_bounds__(kNT) void k_update_xr_stop_f64(int64_t n, double *__restrict__ x, double *__restrict__ r,
                                                            const double *__restrict__ p, const double *__restrict__ Ap,
                                                            const double *rsold, const double *pAp, double *rr_out,
                                                            double *partials, unsigned *ticket, const int64_t *gate,
                                                            ConvArgs cv, int64_t *ts) {
    if (gate && *gate) return;
    ts_start(ts);
    const double alpha = cg_ratio(*rsold, *pAp);
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 xv[kVU], rv[kVU], pv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                xv[u] = ld2(x + i); rv[u] = ld2(r + i); pv[u] = ld2(p + i); av[u] = ld2(Ap + i);
            }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                st2(x + i, xv[u] + alpha * pv[u]);
                const d2 ri = rv[u] - alpha * av[u];
                st2(r + i, ri);
                acc += ri.x * ri.x + ri.y * ri.y;
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const int64_t i = n - 1;
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            r[i] = ri;
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            x[i] = x[i] + alpha * p[i];
            const double ri = r[i] - alpha * Ap[i];
            r[i] = ri;
            acc += ri * ri;
        }
    }
    double rr;
    if (grid_sum_keep_last(acc, partials, ticket, rr_out, rr) && cv.kdone && cv.eps >= 0.0 && sqrt(rr) < cv.eps &&
        threadIdx.x == 0)
        record_convergence(cv, cv.k + 1, rr);
    ts_end(ts);
}

// The solver's split of the x/r/p updates (fp64): x's update moves into the
// p update, which reads p anyway -- 24 + 40 B per element instead of 48 + 24.
// r -= alpha Ap; r.r   (alpha = rsold / pAp)
template <bool VEC, int VP = 2>
__global__ __launch_bounds__(kNT) void k_update_r_f64(int64_t n, double *__restrict__ r, const double *__restrict__ Ap,
                                                      const double *rsold, const double *pAp, double *rr_out,
                                                      double *partials, unsigned *ticket, const int64_t *gate,
                                                      int64_t *ts, PeerSum pap_sum) {
    if (gate && *gate) return;
    ts_start(ts);
    const double alpha = cg_ratio(*rsold, pap_sum.cnt ? peer_sum_wave(pap_sum) : *pAp);
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 rv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) { const int64_t i = 2 * (base + u * kNT); rv[u] = ldv<VP>(r + i); av[u] = ldv<VP>(Ap + i); }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const d2 ri = rv[u] - alpha * av[u];
                stv<VP>(r + 2 * (base + u * kNT), ri);
                acc += ri.x * ri.x + ri.y * ri.y;
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            const double ri = r[n - 1] - alpha * Ap[n - 1];
            r[n - 1] = ri;
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            const double ri = r[i] - alpha * Ap[i];
            r[i] = ri;
            acc += ri * ri;
        }
    }
    grid_sum_last_block(acc, partials, ticket, rr_out);
    ts_end(ts);
}

// x += alpha p (alpha = rsold / pAp); then, if rr != nullptr, p = r + (rr / rsold) p.
// With cv.kdone != nullptr (device-side gating) the kernel also makes the
// reference's stopping decision, `sqrt(r.r) < EPSILON` (serialConjugate.c:235):
// on convergence it does only the x update and records k+1 and r.r; in a
// later iteration (kdone in (0, k]) it does nothing.

template <bool VEC, int VP = 2>
__global__ __launch_bounds__(kNT) void k_update_xp_f64(int64_t n, double *__restrict__ x, double *__restrict__ p,
                                                       const double *__restrict__ r, const double *rsold,
                                                       const double *pAp, const double *rr, ConvArgs cv,
                                                       int64_t *ts, PeerSum rr_sum) {
    bool upd_p = rr != nullptr;
    if (cv.kdone && *cv.kdone != 0 && *cv.kdone <= cv.k) return;
    // the r.r combine folded in (multi-shard): every block sums the partials
    const double rrv = rr_sum.cnt ? peer_sum_wave(rr_sum) : rr ? *rr : 0.0;
    if (cv.kdone) {
        const double rrn = rrv;
        if (cv.eps >= 0.0 && sqrt(rrn) < cv.eps) {
            upd_p = false;
            if (blockIdx.x == 0 && threadIdx.x == 0) record_convergence(cv, cv.k + 1, rrn);
        }
    }
    ts_start(ts);
    const double alpha = cg_ratio(*rsold, *pAp);
    const double beta = upd_p ? cg_ratio(rrv, *rsold) : 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 xv[kVU], pv[kVU], rv[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                xv[u] = ldv<VP>(x + i);
                pv[u] = ldv<VP>(p + i);
                if (upd_p) rv[u] = ldv<VP>(r + i);
            }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) {
                const int64_t i = 2 * (base + u * kNT);
                stv<VP>(x + i, xv[u] + alpha * pv[u]);
                if (upd_p) stv<VP>(p + i, rv[u] + beta * pv[u]);
            }
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
            x[n - 1] = x[n - 1] + alpha * p[n - 1];
            if (upd_p) p[n - 1] = r[n - 1] + beta * p[n - 1];
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            x[i] = x[i] + alpha * p[i];
            if (upd_p) p[i] = r[i] + beta * p[i];
        }
    }
    ts_end(ts);
}

template <bool VEC>
__global__ __launch_bounds__(kNT) void k_dot_f64(int64_t n, const double *__restrict__ a,
                                                 const double *__restrict__ b, double *out,
                                                 double *partials, unsigned *ticket) {
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 av[kVU], bv[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) { const int64_t i = 2 * (base + u * kNT); av[u] = ld2(a + i); bv[u] = ld2(b + i); }
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) acc += av[u].x * bv[u].x + av[u].y * bv[u].y;
        CGX_VEC_LOOP_END
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) acc += a[n - 1] * b[n - 1];
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
            acc += a[i] * b[i];
    }
    grid_sum_last_block(acc, partials, ticket, out);
}

// counter-hash SPD generator (generateSPDmatrix.m:4-17 distribution)
// ---------------------------------------------------------------------------

template <typename T>
__global__ __launch_bounds__(kNT) void k_gen_spd(int64_t n, int64_t lda, int64_t row0, int64_t nrows,
                                                 uint64_t salt, uint64_t salt_b, T *A, T *b) {
#pragma clang fp contract(off)
    for (int64_t rr = blockIdx.x; rr < nrows; rr += gridDim.x) {
        const uint64_t i = (uint64_t)(row0 + rr);
        T *row = A + rr * lda;
        for (int64_t jj = threadIdx.x; jj < lda; jj += kNT) {
            double val = 0.0;
            if (jj < n) {
                const uint64_t j = (uint64_t)jj;
                val = 0.5 * (u01(salt, i, j) + u01(salt, j, i));
                if (i == j) val = val + (double)n;
            }
            row[jj] = (T)val;
        }
        if (threadIdx.x == 0) {
            const uint64_t h = mix64(i ^ salt_b);
            b[rr] = (T)((double)(h >> 11) * 0x1.0p-53);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_fill(T *p, int64_t n, T v) {
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) p[i] = v;
}

// Scalars combined in a fixed order.  Inputs sit in 8-byte slots (a float at
// the slot start for F32_REF): element q at in[q*stride].
//   rank order  ((in0 + in1) + in2) + ...   point-to-point_cg.c allSum :344-352
//   MPICH order (mpich != 0): MPI_Allreduce(MPI_SUM) of one value as MPICH 3.3
//     runs it (recursive doubling, parallel_cg.c:287,294,313): with pof2 the
//     largest power of two <= cnt and rem = cnt - pof2, pairs (2q, 2q+1), q < rem,
//     combine first, then a balanced pairwise tree over the pof2 values.
//     Pinned by tests/golden/mpi/ (mpiexec -np 2/4/8 of the unmodified program).
template <typename T>
__global__ void k_sum_ordered(const T *in, int cnt, int stride, int mpich, T *out) {
#pragma clang fp contract(off)
    if (!mpich) {
        T s = in[0];
        for (int q = 1; q < cnt; ++q) s = s + in[q * stride];
        *out = s;
        return;
    }
    int pof2 = 1;
    while (pof2 * 2 <= cnt) pof2 *= 2;
    const int rem = cnt - pof2;
    T v[kMaxCombine];
    for (int q = 0; q < pof2; ++q)
        v[q] = q < rem ? in[2 * q * stride] + in[(2 * q + 1) * stride] : in[(q + rem) * stride];
    for (int d = 1; d < pof2; d *= 2)
        for (int q = 0; q < pof2; q += 2 * d) v[q] = v[q] + v[q + d];
    *out = v[0];
}

// The pull kernels of the one-process multi-shard exchange read other
// shards' memory -- on distinct devices, peer memory over xGMI, which this
// device's L2 may hold from an earlier iteration's read of the same address.
// So every such read is a system-scope load (sc0 sc1: served coherently, not
// from a stale L2 line); the producers' event records carry the system-scope
// release that wrote their data back.  On one device these are plain loads'
// worth of traffic (512 KB of p per iteration at N = 65536).  (load_sys:
// cgx_device.h.)

// The same combines over a table of peer pointers (one partial per shard),
// by one wave: lane q loads partial q (one round trip for all of them), then
// the rank-order sum in lane order, or MPICH's recursive doubling with the
// values kept in lanes (pairs (2q, 2q+1) for q < rem, then a pairwise tree:
// the same adds in the same order as k_sum_ordered).
template <typename T>
__global__ __launch_bounds__(64) void k_combine_peers(PeerTable src, int cnt, int mpich, T *out) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x;
    const T x = peer_lane_load<T>(src, cnt);
    if (!mpich) {
        T s = __shfl(x, 0, 64);
        for (int q = 1; q < cnt; ++q) s = s + __shfl(x, q, 64);
        if (lane == 0) *out = s;
        return;
    }
    int pof2 = 1;
    while (pof2 * 2 <= cnt) pof2 *= 2;
    const int rem = cnt - pof2;
    const T a = __shfl(x, lane < rem ? 2 * lane : (lane + rem) & 63, 64);
    const T b = __shfl(x, (2 * lane + 1) & 63, 64);
    T v = lane < rem ? a + b : a;
    for (int d = 1; d < pof2; d *= 2) {
        const T w = __shfl(v, (lane + d) & 63, 64);
        if (lane % (2 * d) == 0 && lane + d < pof2) v = v + w;
    }
    if (lane == 0) *out = v;
}

// blockIdx.y = the source slice; each thread moves kGU words of W (8 or 4)
// bytes per pass with all its loads issued before the stores (remote reads
// over xGMI are latency-bound: keep many in flight).
constexpr int kGU = 8;
template <typename W>
__global__ __launch_bounds__(kNT) void k_gather_slices(PeerTable src, int skip, int64_t words, char *dst) {
    const int q = blockIdx.y;
    if (q == skip) return;
    const W *__restrict__ in = reinterpret_cast<const W *>(src.p[q]);
    W *__restrict__ out = reinterpret_cast<W *>(dst) + (int64_t)q * words;
    const int64_t stride = (int64_t)gridDim.x * kNT * kGU;
    for (int64_t base = (int64_t)blockIdx.x * kNT * kGU + threadIdx.x; base < words; base += stride) {
        W v[kGU];
#pragma unroll
        for (int u = 0; u < kGU; ++u)
            if (base + u * kNT < words) v[u] = load_sys(in + base + u * kNT);
#pragma unroll
        for (int u = 0; u < kGU; ++u)
            if (base + u * kNT < words) out[base + u * kNT] = v[u];
    }
}

}  // namespace

hipError_t gather_slices(const PeerTable &src, int cnt, int skip, int64_t slice_bytes, char *dst, hipStream_t s) {
    if (cnt < 1 || cnt > kMaxPeers || slice_bytes < 0 || (slice_bytes & 3)) return hipErrorInvalidValue;
    if (slice_bytes == 0) return hipSuccess;
    bool a8 = (slice_bytes % 8) == 0 && (reinterpret_cast<uintptr_t>(dst) % 8) == 0;
    for (int q = 0; q < cnt; ++q) a8 = a8 && (reinterpret_cast<uintptr_t>(src.p[q]) % 8) == 0;
    const int64_t wb = a8 ? 8 : 4, words = slice_bytes / wb;
    const int64_t per_block = (int64_t)kNT * kGU;
    const unsigned gx = (unsigned)std::min<int64_t>((words + per_block - 1) / per_block, 64);
    const dim3 grid(gx, (unsigned)cnt);
    if (a8) hipLaunchKernelGGL(k_gather_slices<uint64_t>, grid, dim3(kNT), 0, s, src, skip, words, dst);
    else hipLaunchKernelGGL(k_gather_slices<uint32_t>, grid, dim3(kNT), 0, s, src, skip, words, dst);
    return hipGetLastError();
}

hipError_t combine_peers_f64(const PeerTable &src, int cnt, double *out, hipStream_t s) {
    if (cnt < 1 || cnt > kMaxPeers) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_combine_peers<double>, dim3(1), dim3(64), 0, s, src, cnt, 0, out);
    return hipGetLastError();
}

hipError_t combine_peers_f32(const PeerTable &src, int cnt, float *out, hipStream_t s, bool mpich) {
    if (cnt < 1 || cnt > kMaxPeers) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_combine_peers<float>, dim3(1), dim3(64), 0, s, src, cnt, mpich ? 1 : 0, out);
    return hipGetLastError();
}

hipError_t residual_f64(int64_t n, const double *b, const double *Ax, double *r, double *p,
                        double *rr_out, const RedWs &ws, hipStream_t s, int64_t *clear2) {
    const bool vec = al16(b) && al16(Ax) && al16(r) && al16(p);
    hipLaunchKernelGGL(vec ? k_residual_f64<true> : k_residual_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, b,
                       Ax, r, p, rr_out, ws.partials, ws.tickets + T_RESID, clear2);
    return hipGetLastError();
}

hipError_t update_xr_f64(int64_t n, double *x, double *r, const double *p, const double *Ap,
                         const double *rsold, const double *pAp, double *rr_out, const RedWs &ws,
                         hipStream_t s) {
    const bool vec = al16(x) && al16(r) && al16(p) && al16(Ap);
    auto fn = !vec ? k_update_xr_f64<false> : k_update_xr_f64<true, 2>;  // the solver kernels' policy (ldv)
    hipLaunchKernelGGL(fn, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x, r, p, Ap, rsold, pAp, rr_out, ws.partials,
                       ws.tickets + T_XR);
    return hipGetLastError();
}

hipError_t update_p_f64(int64_t n, double *p, const double *r, const double *rr, const double *rsold,
                        hipStream_t s) {
    const bool vec = al16(p) && al16(r);
    auto fn = !vec ? k_update_p_f64<false> : k_update_p_f64<true, 2>;
    hipLaunchKernelGGL(fn, dim3(grid_vec(n)), dim3(kNT), 0, s, n, p, r, rr, rsold);
    return hipGetLastError();
}

hipError_t update_r_f64(int64_t n, double *r, const double *Ap, const double *rsold, const double *pAp,
                        double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate, int64_t *ts,
                        const PeerSum *pap_sum) {
    const bool vec = al16(r) && al16(Ap);
    PeerSum ps{};
    if (pap_sum) ps = *pap_sum;
    hipLaunchKernelGGL(vec ? k_update_r_f64<true> : k_update_r_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, r,
                       Ap, rsold, pAp, rr_out, ws.partials, ws.tickets + T_XR, gate, ts, ps);
    return hipGetLastError();
}

hipError_t update_xrp_f64(int64_t n, double *x, double *r, double *p, const double *Ap, const double *rsold,
                          const double *pAp, double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate,
                          double eps, int64_t k, int64_t *kdone, double *rrfinal, int64_t *hrec, int64_t *ts) {
    if (n * 8 > INT32_MAX) return hipErrorInvalidValue;  // buffer-resource offsets are 32-bit
    const bool vec = al16(x) && al16(r) && al16(p) && al16(Ap);
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(vec ? k_update_xrp_f64<true> : k_update_xrp_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s,
                       n, x, r, p, Ap, rsold, pAp, rr_out, ws.partials, ws.tickets + T_XR, gate, cv, ts);
    return hipGetLastError();
}

hipError_t update_xr_stop_f64(int64_t n, double *x, double *r, const double *p, const double *Ap,
                              const double *rsold, const double *pAp, double *rr_out, const RedWs &ws, hipStream_t s,
                              const int64_t *gate, double eps, int64_t k, int64_t *kdone, double *rrfinal,
                              int64_t *hrec, int64_t *ts) {
    const bool vec = al16(x) && al16(r) && al16(p) && al16(Ap);
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(vec ? k_update_xr_stop_f64<true> : k_update_xr_stop_f64<false>, dim3(grid_vec(n)), dim3(kNT),
                       0, s, n, x, r, p, Ap, rsold, pAp, rr_out, ws.partials, ws.tickets + T_XR, gate, cv, ts);
    return hipGetLastError();
}

hipError_t update_xp_f64(int64_t n, double *x, double *p, const double *r, const double *rsold, const double *pAp,
                         const double *rr, hipStream_t s, double eps, int64_t k, int64_t *kdone, double *rrfinal,
                         int64_t *hrec, int64_t *ts, const PeerSum *rr_sum) {
    const bool vec = al16(x) && al16(p) && al16(r);
    PeerSum ps{};
    if (rr_sum) ps = *rr_sum;
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(vec ? k_update_xp_f64<true> : k_update_xp_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x,
                       p, r, rsold, pAp, rr, cv, ts, ps);
    return hipGetLastError();
}

hipError_t dot_f64(int64_t n, const double *a, const double *b, double *out, const RedWs &ws,
                   hipStream_t s) {
    const bool vec = al16(a) && al16(b);
    hipLaunchKernelGGL(vec ? k_dot_f64<true> : k_dot_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, a, b, out,
                       ws.partials, ws.tickets + T_DOT);
    return hipGetLastError();
}

hipError_t gen_spd_f64(int64_t n, int64_t lda, int64_t row0, int64_t nrows, uint64_t seed, double *A,
                       double *b, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_spd<double>, dim3(grid_1d(nrows, 1, 65536)), dim3(kNT), 0, s, n, lda, row0,
                       nrows, mix64(seed), mix64(seed + 1), A, b);
    return hipGetLastError();
}

hipError_t gen_spd_f32(int64_t n, int64_t lda, int64_t row0, int64_t nrows, uint64_t seed, float *A,
                       float *b, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_spd<float>, dim3(grid_1d(nrows, 1, 65536)), dim3(kNT), 0, s, n, lda, row0,
                       nrows, mix64(seed), mix64(seed + 1), A, b);
    return hipGetLastError();
}

hipError_t fill_f64(double *p, int64_t n, double v, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill<double>, dim3(grid_vec(n)), dim3(kNT), 0, s, p, n, v);
    return hipGetLastError();
}

hipError_t fill_f32(float *p, int64_t n, float v, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill<float>, dim3(grid_vec(n)), dim3(kNT), 0, s, p, n, v);
    return hipGetLastError();
}

hipError_t sum_ordered_f64(const double *in, int cnt, double *out, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_ordered<double>, dim3(1), dim3(1), 0, s, in, cnt, 1, 0, out);
    return hipGetLastError();
}

hipError_t sum_ordered_f32(const float *in, int cnt, float *out, hipStream_t s, bool mpich) {
    if (cnt < 1 || cnt > kMaxCombine) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sum_ordered<float>, dim3(1), dim3(1), 0, s, in, cnt, 2, mpich ? 1 : 0, out);
    return hipGetLastError();
}

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_vector() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_fill<double>));
}

}  // namespace cgx
