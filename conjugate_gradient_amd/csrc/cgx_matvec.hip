// cgx_matvec.hip -- the dense fp64 matVec (the CG hot path's HBM-bound kernel).
//
// The reference's matVec (serialConjugate.c:109-120, parallel_cg.c:172-184)
// becomes k_matvec_f64 (+ the p.Ap vecVec fused into its epilogue).  The other kernels of
// the iteration live beside it: cgx_vector.hip (residual, x/r/p updates, dot),
// cgx_poisson.hip, cgx_ref_f32.hip (CGX_F32_REF) and cgx_symv.hip
// (CGX_SYMMETRIC); shared helpers in cgx_device.h.
//
// Design: the matVec is HBM-bound (0.25 flop/B in fp64), so it
// streams A once with 16-B-per-lane coalesced loads (a wave covers one
// 1-KiB, 128-column chunk of a row per instruction), R rows per wave share
// each p chunk held in registers (p re-reads hit L1/L2: p is <= 1 MiB), U
// chunks per row are in flight per lane, and the grid is sized to the
// resident-wave capacity and grid-strides over row groups; the next step's
// loads are issued before the current step's FMAs (software pipeline).  No
// MFMA: a GEMV has no reuse of A.  Reductions are deterministic: per-block
// partials in fixed slots, summed in index order by the last block to arrive
// (write-through sc1 partials and a relaxed ticket, the fence-free form of
// cdna_hip_programming.md Guideline 16).
#include "cgx_device.h"

#include <algorithm>

namespace cgx {
namespace {

// Load policy of the A stream (the only data a matVec reads once):
//   0 plain global_load, 1 global_load ... nt, 2 / 8 software-pipelined
//   global_load, default policy / nt (8 = the default plan).  The variants measured and not
//   adopted (buffer loads with other cache bits, a flattened pipeline,
//   LDS-staged p, SGPR row bases) live in tools/microbench/matvec_variants.hip.
//   All give the same row sums bit for bit.
template <int POL>
__device__ __forceinline__ d2 load_a(const d2 *p) {
    if constexpr (POL == 1) return __builtin_nontemporal_load(p);
    else return *p;
}

// ---------------------------------------------------------------------------
// matVec (serialConjugate.c:109-120 / parallel_cg.c:172-184), fp64.
// Wave w owns row groups g = w, w + waves, ...; a group is R consecutive rows.
// Per step a lane holds U 16-B chunks of p and R*U 16-B chunks of A.
// ---------------------------------------------------------------------------
// Accumulate 128-column chunks [c0, c1) of R rows into acc (U chunks per step).
template <int R, int U, int NT>
__device__ __forceinline__ void mv_chunks(const d2 *const (&arow)[R], int lane, const d2 *v2, int64_t c0, int64_t c1,
                                          d2 (&acc)[R]) {
    int64_t c = c0;
    for (; c + U <= c1; c += U) {
        d2 pv[U];
        d2 av[R][U];
#pragma unroll
        for (int u = 0; u < U; ++u) pv[u] = v2[(c + u) * 64];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                av[r][u] = load_a<NT>(arow[r] + (c + u) * 64);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc[r].x = __builtin_fma(av[r][u].x, pv[u].x, acc[r].x);
                acc[r].y = __builtin_fma(av[r][u].y, pv[u].y, acc[r].y);
            }
    }
    for (; c < c1; ++c) {
        const d2 pv = v2[c * 64];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const d2 a = load_a<NT>(arow[r] + c * 64);
            acc[r].x = __builtin_fma(a.x, pv.x, acc[r].x);
            acc[r].y = __builtin_fma(a.y, pv.y, acc[r].y);
        }
    }
}

// Software-pipelined variant: the loads of step c+U are issued before the
// FMAs of step c (two register sets, ping-pong), so a wave always has a
// step's loads in flight.
template <int R, int U, int NT>
__device__ __forceinline__ void mv_load_step(const d2 *const (&arow)[R], int lane, const d2 *v2, int64_t c, d2 (&pv)[U],
                                             d2 (&av)[R][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) pv[u] = v2[(c + u) * 64];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            av[r][u] = load_a<NT>(arow[r] + (c + u) * 64);
        }
}

template <int R, int U>
__device__ __forceinline__ void mv_fma_step(const d2 (&pv)[U], const d2 (&av)[R][U], d2 (&acc)[R]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc[r].x = __builtin_fma(av[r][u].x, pv[u].x, acc[r].x);
            acc[r].y = __builtin_fma(av[r][u].y, pv[u].y, acc[r].y);
        }
}

template <int R, int U, int NT>
__device__ __forceinline__ void mv_chunks_pipe(const d2 *const (&arow)[R], int lane, const d2 *v2, int64_t c0, int64_t c1,
                                               d2 (&acc)[R]) {
    d2 pa[U], aa[R][U], pb[U], ab[R][U];
    int64_t c = c0;
    if (c + U <= c1) mv_load_step<R, U, NT>(arow, lane, v2, c, pa, aa);
    while (c + U <= c1) {
        const bool more = c + 2 * U <= c1;
        if (more) mv_load_step<R, U, NT>(arow, lane, v2, c + U, pb, ab);
        mv_fma_step<R, U>(pa, aa, acc);
        c += U;
        if (!more) break;
        const bool more2 = c + 2 * U <= c1;
        if (more2) mv_load_step<R, U, NT>(arow, lane, v2, c + U, pa, aa);
        mv_fma_step<R, U>(pb, ab, acc);
        c += U;
        if (!more2) break;
    }
    // remaining single chunks
    for (; c < c1; ++c) {
        const d2 pv = v2[c * 64];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const d2 a = load_a<NT>(arow[r] + c * 64);
            acc[r].x = __builtin_fma(a.x, pv.x, acc[r].x);
            acc[r].y = __builtin_fma(a.y, pv.y, acc[r].y);
        }
    }
}

// Column range: the `ccount` 128-column chunks starting at chunk `cfirst`,
// wrapping modulo the vec_cols/128 aligned chunks; `tail` adds the scalar
// columns [vec_cols, cols).  `accumulate` adds the existing out[i] (the
// overlap path computes the shard's own column block first, then the rest).
template <int R, int U, int NT, bool PIPE = false>
__global__ __launch_bounds__(kNT) void k_matvec_f64(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
    const double *__restrict__ pown, double *dot_out, double *partials, unsigned *ticket, const int64_t *gate,
    int64_t *ts) {
    if (gate && *gate) return;  // the solve converged in an earlier iteration (device-side gating)
    ts_start(ts);
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int64_t ngroups = (rows + R - 1) / R;
    const int64_t wstride = (int64_t)gridDim.x * (kNT / 64);
    const int64_t nchunk = vec_cols >> 7;  // 16-B-aligned 128-column chunks
    const int64_t ctail = nchunk << 7;
    const int64_t ca = cfirst, cb = (cfirst + ccount < nchunk) ? cfirst + ccount : nchunk;  // first piece
    const int64_t wrap = cfirst + ccount - cb;                                              // wrapped piece
    const d2 *v2 = reinterpret_cast<const d2 *>(v) + lane;
    double dacc = 0.0;

    for (int64_t g = (int64_t)blockIdx.x * (kNT / 64) + wid; g < ngroups; g += wstride) {
        const int64_t r0 = g * R;
        int64_t ridx[R];
        const d2 *arow[R];
        d2 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            ridx[r] = (r0 + r < rows) ? (r0 + r) : (rows - 1);
            arow[r] = reinterpret_cast<const d2 *>(A + ridx[r] * lda) + lane;
            acc[r] = (d2)(0.0);
        }
        if constexpr (PIPE) {
            mv_chunks_pipe<R, U, NT>(arow, lane, v2, ca, cb, acc);
            if (wrap > 0) mv_chunks_pipe<R, U, NT>(arow, lane, v2, 0, wrap, acc);
        } else {
            mv_chunks<R, U, NT>(arow, lane, v2, ca, cb, acc);
            if (wrap > 0) mv_chunks<R, U, NT>(arow, lane, v2, 0, wrap, acc);
        }
        if (tail)
            for (int64_t j = ctail + lane; j < cols; j += 64) {
                const double vj = v[j];
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r].x = __builtin_fma(A[ridx[r] * lda + j], vj, acc[r].x);
            }
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double s = wave_sum(acc[r].x + acc[r].y);
            if (lane == r) mine = s;
        }
        if (lane < R && r0 + lane < rows) {
            if (accumulate) mine = out[r0 + lane] + mine;
            out[r0 + lane] = mine;
            if (pown) dacc += pown[r0 + lane] * mine;
        }
    }
    if (pown) grid_sum_last_block(dacc, partials, ticket, dot_out);
    ts_end(ts);
}

// ---------------------------------------------------------------------------
// The matVec of a small system's two-launch iteration with the previous
// iteration's p update folded in (one GPU, n <= kFusePMax): p_k is never
// formed by a pass of its own -- every wave forms the chunks it multiplies,
//   p_k[j] = r_k[j] + beta p_{k-1}[j],   beta = r.r_k / r.r_{k-1}
// (serialConjugate.c:239-243, the expression k_update_xp_f64 evaluates, so
// the same bits), multiplies them, and the wave that owns row i also stores
// p_k[i] into the other p buffer (p_{k-1} and p_k never share one: no
// write-after-read race) and adds p_k[i] * (A p_k)[i] to the fused p.Ap.
// The next kernel (k_update_xr_stop_f64) is then fully parallel: no
// single-block pass over p at the end of the iteration.
// Loads of r and p_{k-1} for step c + U go out before the FMAs of step c,
// like k_matvec_f64's pipeline; the combine waits until the FMA step.
template <int R, int U>
__device__ __forceinline__ void fold_load_step(const d2 *const (&arow)[R], const d2 *r2, const d2 *q2, int64_t c,
                                               d2 (&rv)[U], d2 (&qv)[U], d2 (&av)[R][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        rv[u] = r2[(c + u) * 64];
        qv[u] = q2[(c + u) * 64];
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) av[r][u] = load_a<1>(arow[r] + (c + u) * 64);
}

template <int R, int U>
__device__ __forceinline__ void fold_fma_step(const d2 (&rv)[U], const d2 (&qv)[U], const d2 (&av)[R][U], double beta,
                                              d2 (&acc)[R]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const d2 pv = rv[u] + beta * qv[u];  // p = r + beta p (k_update_xp_f64's expression)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc[r].x = __builtin_fma(av[r][u].x, pv.x, acc[r].x);
            acc[r].y = __builtin_fma(av[r][u].y, pv.y, acc[r].y);
        }
    }
}

template <int R, int U>
__global__ __launch_bounds__(kNT) void k_matvec_fold_f64(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols,
    const double *__restrict__ r, const double *__restrict__ pold, double *__restrict__ pnew, const double *rr_new,
    const double *rr_old, double *__restrict__ out, double *dot_out, double *partials, unsigned *ticket,
    const int64_t *gate, int64_t *ts) {
    if (gate && *gate) return;
    ts_start(ts);
    const double beta = cg_ratio(*rr_new, *rr_old);
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int64_t ngroups = (rows + R - 1) / R;
    const int64_t wstride = (int64_t)gridDim.x * (kNT / 64);
    const int64_t nchunk = vec_cols >> 7;
    const d2 *r2 = reinterpret_cast<const d2 *>(r) + lane;
    const d2 *q2 = reinterpret_cast<const d2 *>(pold) + lane;
    double dacc = 0.0;
    for (int64_t g = (int64_t)blockIdx.x * (kNT / 64) + wid; g < ngroups; g += wstride) {
        const int64_t r0 = g * R;
        int64_t ridx[R];
        const d2 *arow[R];
        d2 acc[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            ridx[q] = (r0 + q < rows) ? (r0 + q) : (rows - 1);
            arow[q] = reinterpret_cast<const d2 *>(A + ridx[q] * lda) + lane;
            acc[q] = (d2)(0.0);
        }
        {
            d2 ra[U], qa[U], aa[R][U], rb[U], qb[U], ab[R][U];
            int64_t c = 0;
            if (c + U <= nchunk) fold_load_step<R, U>(arow, r2, q2, c, ra, qa, aa);
            while (c + U <= nchunk) {
                const bool more = c + 2 * U <= nchunk;
                if (more) fold_load_step<R, U>(arow, r2, q2, c + U, rb, qb, ab);
                fold_fma_step<R, U>(ra, qa, aa, beta, acc);
                c += U;
                if (!more) break;
                const bool more2 = c + 2 * U <= nchunk;
                if (more2) fold_load_step<R, U>(arow, r2, q2, c + U, ra, qa, aa);
                fold_fma_step<R, U>(rb, qb, ab, beta, acc);
                c += U;
                if (!more2) break;
            }
            for (; c < nchunk; ++c) {
                const d2 pv = r2[c * 64] + beta * q2[c * 64];
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const d2 a = load_a<1>(arow[q] + c * 64);
                    acc[q].x = __builtin_fma(a.x, pv.x, acc[q].x);
                    acc[q].y = __builtin_fma(a.y, pv.y, acc[q].y);
                }
            }
        }
        for (int64_t j = (nchunk << 7) + lane; j < cols; j += 64) {  // columns past the last whole chunk
            const double pj = r[j] + beta * pold[j];
#pragma unroll
            for (int q = 0; q < R; ++q) acc[q].x = __builtin_fma(A[ridx[q] * lda + j], pj, acc[q].x);
        }
        double mine = 0.0;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const double sum = wave_sum(acc[q].x + acc[q].y);
            if (lane == q) mine = sum;
        }
        if (lane < R && r0 + lane < rows) {
            const int64_t i = r0 + lane;
            const double pi = r[i] + beta * pold[i];
            pnew[i] = pi;
            out[i] = mine;
            dacc += pi * mine;
        }
    }
    grid_sum_last_block(dacc, partials, ticket, dot_out);
    ts_end(ts);
}

using FoldFn = decltype(&k_matvec_fold_f64<1, 8>);
FoldFn pick_fold(int R, int U) {
    if (R == 1) return U == 2 ? k_matvec_fold_f64<1, 2> : U == 4 ? k_matvec_fold_f64<1, 4> : k_matvec_fold_f64<1, 8>;
    return U == 2 ? k_matvec_fold_f64<2, 2> : U == 4 ? k_matvec_fold_f64<2, 4> : k_matvec_fold_f64<2, 8>;
}

using MvFn = void (*)(const double *, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int,
                      const double *, double *, const double *, double *, double *, unsigned *, const int64_t *,
                      int64_t *);

template <int R, int U>
MvFn pick_nt(int nt) {
    switch (nt) {
        case 0: return k_matvec_f64<R, U, 0>;
        case 2: return k_matvec_f64<R, U, 0, true>;  // pipelined, default-policy loads
        case 8: return k_matvec_f64<R, U, 1, true>;  // pipelined, global nt (the default)
        default: return k_matvec_f64<R, U, 1>;
    }
}
template <int R>
MvFn pick_u(int U, int nt) {
    switch (U) {
        case 2: return pick_nt<R, 2>(nt);
        case 8: return pick_nt<R, 8>(nt);
        default: return pick_nt<R, 4>(nt);
    }
}
MvFn pick_mv(int R, int U, int nt) {
    switch (R) {
        case 1: return pick_u<1>(U, nt);
        case 2: return pick_u<2>(U, nt);
        case 8: return pick_u<8>(U, nt);
        default: return pick_u<4>(U, nt);
    }
}

}  // namespace

MatvecPlan plan_matvec_f64(int device, int64_t rows, int R, int U, int nt, int blocks_per_cu, int64_t cols) {
    MatvecPlan pl;
    const int cus = cu_count(device);
    // Software-pipelined (loads of step c+U issued before the FMAs of step c),
    // 2 rows per wave, U=8, global_load ... nt: 256 VGPRs, one wave per SIMD,
    // 32 KiB of A in flight per wave.  Measured on MI355X, interleaved against
    // every (R, U, policy) of the unpipelined kernel (profiles/r01_sweep_pipe*):
    // 7.24 TB/s at 65536^2 (unpipelined best R=8,U=8,buffer-nt: 7.09),
    // 7.21 TB/s on an 8192 x 65536 row block (7.05), 6.81 TB/s at 16384^2 (6.60).
    // R=1 when there are fewer than 2 rows per resident wave.
    // Rows of 4096-8192 columns keep R = 1, one row per wave and twice the
    // waves: 81.0-82.5 vs 82.6 us at 8192^2, 20.9 vs 21.7 at 4096^2, but
    // 5.3 vs 5.2 at 2048^2 (profiles/r02_sweep_square_n*.jsonl); per CG
    // iteration at N=8192 93.1-94.1 vs 94.2-95.7 us, at N=2048 16.5 vs 14.0
    // (profiles/r02_floor_plan_r1_vs_r2.jsonl).
    const int64_t want_waves = (int64_t)cus * 4;
    pl.R = (rows >= 2 * want_waves && !(cols >= 4096 && cols <= 8192)) ? 2 : 1;
    // a row of fewer than 8 chunks: with U = 8 its chunks would go through the
    // one-chunk remainder loop, one dependent memory round trip each (N = 512:
    // 4 chunks); U = 4 / 2 issues them together
    const int64_t chunks = cols >> 7;
    pl.U = (cols <= 0 || chunks >= 8) ? 8 : chunks >= 4 ? 4 : 2;
    pl.nt = 8;
    pl.R = env_int("CGX_MV_R", pl.R);
    pl.U = env_int("CGX_MV_U", pl.U);
    pl.nt = env_int("CGX_MV_NT", pl.nt);
    if (R > 0) pl.R = R;
    if (U > 0) pl.U = U;
    if (nt >= 0) pl.nt = nt;
    if (pl.R != 1 && pl.R != 2 && pl.R != 4 && pl.R != 8) pl.R = 4;
    if (pl.U != 2 && pl.U != 4 && pl.U != 8) pl.U = 4;
    if (pl.nt != 0 && pl.nt != 1 && pl.nt != 2 && pl.nt != 8) pl.nt = 8;
    int per_cu = 0;
    const void *fn = reinterpret_cast<const void *>(pick_mv(pl.R, pl.U, pl.nt));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, 0) != hipSuccess || per_cu <= 0)
        per_cu = 2;
    per_cu = env_int("CGX_MV_BLOCKS_PER_CU", per_cu);
    if (blocks_per_cu > 0) per_cu = blocks_per_cu;
    const int64_t groups = (rows + pl.R - 1) / pl.R;
    const int64_t need = (groups + (kNT / 64) - 1) / (kNT / 64);
    int64_t cap = (int64_t)per_cu * cus;
    if (cap > kMaxRedBlocks) cap = kMaxRedBlocks;
    pl.blocks = (int)std::max<int64_t>(1, std::min(need, cap));
    return pl;
}

hipError_t matvec_f64(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                      const double *v, double *out, const double *pown, double *dot_out,
                      const RedWs &ws, hipStream_t s, const int64_t *gate, int64_t *ts) {
    if (rows <= 0) return hipSuccess;
    // The vector path needs 16-B-aligned rows and p; otherwise every column
    // goes through the scalar tail loop.
    const bool aligned = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15) == 0 &&
                         (lda & 1) == 0;
    const int64_t vec_cols = aligned ? (cols & ~int64_t(127)) : 0;
    MvFn fn = pick_mv(pl.R, pl.U, pl.nt);
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, vec_cols, int64_t(0),
                       vec_cols >> 7, 1, 0, v, out, pown, dot_out, ws.partials, ws.tickets + T_MATVEC, gate, ts);
    return hipGetLastError();
}

hipError_t matvec_f64_cols(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t col_first, int64_t col_count, bool accumulate, const double *v, double *out,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate, int64_t *ts) {
    if (rows <= 0) return hipSuccess;
    if ((cols & 127) || (col_first & 127) || (col_count & 127) || (lda & 1) ||
        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15))
        return hipErrorInvalidValue;
    MvFn fn = pick_mv(pl.R, pl.U, pl.nt);
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, cols, col_first >> 7,
                       col_count >> 7, 0, accumulate ? 1 : 0, v, out, pown, dot_out, ws.partials,
                       ws.tickets + T_MATVEC, gate, ts);
    return hipGetLastError();
}

hipError_t matvec_fold_f64(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           const double *r, const double *pold, double *pnew, const double *rr_new,
                           const double *rr_old, double *out, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate, int64_t *ts) {
    if (rows <= 0) return hipSuccess;
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(r) | reinterpret_cast<uintptr_t>(pold)) & 15) ||
        (lda & 1))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(pick_fold(pl.R == 1 ? 1 : 2, pl.U), dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols,
                       cols & ~int64_t(127), r, pold, pnew, rr_new, rr_old, out, dot_out, ws.partials,
                       ws.tickets + T_MATVEC, gate, ts);
    return hipGetLastError();
}

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_matvec() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_f64<2, 8, 1, true>));
}

}  // namespace cgx
