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

// The virtual chunks [v0, v1) of the rotated order that starts at physical
// chunk cfirst (virtual v = physical (cfirst + v) mod nchunk), as at most two
// physical pieces in order.
template <int R, int U, int NT, bool PIPE>
__device__ __forceinline__ void mv_range(const d2 *const (&arow)[R], int lane, const d2 *v2, int64_t nchunk,
                                         int64_t cfirst, int64_t v0, int64_t v1, d2 (&acc)[R]) {
    if (v1 <= v0) return;
    const int64_t a = cfirst + v0 < nchunk ? cfirst + v0 : cfirst + v0 - nchunk;
    const int64_t b = a + (v1 - v0) < nchunk ? a + (v1 - v0) : nchunk;
    const int64_t wrap = (v1 - v0) - (b - a);
    if constexpr (PIPE) {
        mv_chunks_pipe<R, U, NT>(arow, lane, v2, a, b, acc);
        if (wrap > 0) mv_chunks_pipe<R, U, NT>(arow, lane, v2, 0, wrap, acc);
    } else {
        mv_chunks<R, U, NT>(arow, lane, v2, a, b, acc);
        if (wrap > 0) mv_chunks<R, U, NT>(arow, lane, v2, 0, wrap, acc);
    }
}

// The one-launch form of the overlapped matVec (rotated column order, two
// accumulators): one software pipeline runs through the whole rotated row --
// the own column block (virtual chunks [0, cseg)) into acc1, then the rest,
// across the wrap, into acc -- with the next step's loads issued before the
// current step's FMAs, the segment end and the wrap included.  Each
// accumulator sees the FMA chain the own / rest launches apply, in the same
// order, so the row sums are theirs bit for bit.  Needs U | cseg, U | ccount
// and U | (nchunk - cfirst) (no step straddles the segment end or the wrap).
template <int R, int U, int NT>
__device__ __forceinline__ void mv_rot_pipe(const d2 *const (&arow)[R], int lane, const d2 *v2, int64_t nchunk,
                                            int64_t cfirst, int64_t cseg, int64_t ccount, d2 (&acc1)[R],
                                            d2 (&acc)[R]) {
    d2 pa[U], aa[R][U], pb[U], ab[R][U];
    const int64_t wrapv = nchunk - cfirst;  // the first virtual chunk past the wrap
    auto phys = [&](int64_t vc) { return vc < wrapv ? cfirst + vc : vc - wrapv; };
    auto seg_end = [&](int64_t vc) {
        if (vc == cseg) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc1[r] = acc[r];
                acc[r] = (d2)(0.0);
            }
        }
    };
    int64_t vc = 0;
    mv_load_step<R, U, NT>(arow, lane, v2, phys(0), pa, aa);
    for (;;) {
        const bool more = vc + U < ccount;
        if (more) mv_load_step<R, U, NT>(arow, lane, v2, phys(vc + U), pb, ab);
        mv_fma_step<R, U>(pa, aa, acc);
        vc += U;
        seg_end(vc);
        if (!more) break;
        const bool more2 = vc + U < ccount;
        if (more2) mv_load_step<R, U, NT>(arow, lane, v2, phys(vc + U), pa, aa);
        mv_fma_step<R, U>(pb, ab, acc);
        vc += U;
        seg_end(vc);
        if (!more2) break;
    }
}

// Column range: the `ccount` 128-column chunks starting at chunk `cfirst`,
// wrapping modulo the vec_cols/128 aligned chunks; `tail` adds the scalar
// columns [vec_cols, cols).  `accumulate` adds the existing out[i] (the
// overlap path computes the shard's own column block first, then the rest).
// ROT (0 < cseg < ccount): the own block and the rest in one launch -- the
// first cseg chunks of the range and the others summed separately and added,
// out[i] = own + rest, which is what the own launch followed by the
// accumulating rest launch stores (the overlapped exchange's two launches and
// the one launch after the exchange give the same bits).
template <int R, int U, int NT, bool PIPE = false, bool ROT = false>
__global__ __launch_bounds__(kNT) void k_matvec_f64(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int64_t cseg, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
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
        double mine = 0.0;
        if constexpr (ROT) {
            d2 acc1[R];
#pragma unroll
            for (int r = 0; r < R; ++r) acc1[r] = (d2)(0.0);
            if (PIPE && cseg % U == 0 && ccount % U == 0 && (nchunk - cfirst) % U == 0)
                mv_rot_pipe<R, U, NT>(arow, lane, v2, nchunk, cfirst, cseg, ccount, acc1, acc);
            else {
                mv_range<R, U, NT, PIPE>(arow, lane, v2, nchunk, cfirst, 0, cseg, acc1);
                mv_range<R, U, NT, PIPE>(arow, lane, v2, nchunk, cfirst, cseg, ccount, acc);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double s1 = wave_sum(acc1[r].x + acc1[r].y);
                const double s2 = wave_sum(acc[r].x + acc[r].y);
                if (lane == r) mine = s1 + s2;  // the rest launch's out[i] (= s1) + its own sum
            }
        } else {
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
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double s = wave_sum(acc[r].x + acc[r].y);
                if (lane == r) mine = s;
            }
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
template <int R, int U, int NTA>
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
        for (int u = 0; u < U; ++u) av[r][u] = load_a<NTA>(arow[r] + (c + u) * 64);
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

template <int R, int U, int NTA = 1>
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
            if (c + U <= nchunk) fold_load_step<R, U, NTA>(arow, r2, q2, c, ra, qa, aa);
            while (c + U <= nchunk) {
                const bool more = c + 2 * U <= nchunk;
                if (more) fold_load_step<R, U, NTA>(arow, r2, q2, c + U, rb, qb, ab);
                fold_fma_step<R, U>(ra, qa, aa, beta, acc);
                c += U;
                if (!more) break;
                const bool more2 = c + 2 * U <= nchunk;
                if (more2) fold_load_step<R, U, NTA>(arow, r2, q2, c + U, ra, qa, aa);
                fold_fma_step<R, U>(rb, qb, ab, beta, acc);
                c += U;
                if (!more2) break;
            }
            for (; c < nchunk; ++c) {
                const d2 pv = r2[c * 64] + beta * q2[c * 64];
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const d2 a = load_a<NTA>(arow[q] + c * 64);
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

// ---------------------------------------------------------------------------
// Small systems on one GPU (2048 <= lda <= 8192, the reference's published
// sizes): the vector staged in LDS, one block per CU.
// k_matvec_f64 reads the p chunks a wave multiplies through L1/L2: with one
// row per wave (the plan for rows of 4096-8192 columns) that is as many
// bytes as A itself (n waves x 8n bytes), and the folded form above reads r
// and p_{k-1} instead, twice that.  Here each block first loads the whole
// vector into LDS -- p, or (FOLD) r and p_{k-1} combined into
// p_k = r + beta p_{k-1} (k_update_xp_f64's expression, so the same bits) --
// and its waves multiply their rows against it: the vector crosses L2 once
// per CU.  The first two steps of A loads are issued before the staging, so
// the stream starts at once.
// Wave w of the grid owns rows w, w + W, ... (W waves in all) and walks
// them as one stream of steps (U chunks of a row each; the next step's
// loads, possibly the next row's, go out before this step's FMAs).  A row
// is summed exactly as k_matvec_f64<1, U> sums it (per lane, chunks in
// order, then the wave sum), so Ap is bit for bit the same; the owner lane
// stores Ap[i] (FOLD: and p_k[i] into the other p buffer) and adds
// p[i] Ap[i] to the fused p.Ap, which therefore adds in this kernel's own
// order -- every form of the iteration at these sizes uses this kernel.
// The LDS array is static (cdna_hip_programming.md Guideline 17: a dynamic
// region behind grid_sum's statics would start misaligned for ds_read_b128).
constexpr int kSmallMaxCols = 8192;
template <bool FOLD, int NTB, int U, int NTA = 1>
__global__ __launch_bounds__(NTB) void k_matvec_small_f64(
    const double *__restrict__ A, int64_t lda, int64_t rows, const double *__restrict__ v,
    const double *__restrict__ pold, double *__restrict__ pnew, const double *rr_new, const double *rr_old,
    const double *__restrict__ pown, double *__restrict__ out, double *dot_out, double *partials,
    unsigned *ticket, const int64_t *gate, int64_t *ts) {
    __shared__ __attribute__((aligned(16))) d2 sp[kSmallMaxCols / 2];
    if (gate && *gate) return;
    ts_start(ts);
    constexpr int WPB = NTB / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double beta = FOLD ? cg_ratio(*rr_new, *rr_old) : 0.0;
    const int64_t W = (int64_t)gridDim.x * WPB;
    const int64_t i0 = (int64_t)blockIdx.x * WPB + wid;
    const int64_t spr = (lda >> 7) / U;                               // steps per row
    const int64_t nrw = i0 < rows ? (rows - i0 + W - 1) / W : 0;      // this wave's rows
    const int64_t nsteps = nrw * spr;
    const d2 *A2 = reinterpret_cast<const d2 *>(A) + lane;
    const int64_t ld2 = lda >> 1;
    // load state: row k_l, step c_l of it
    int64_t kl = 0, cl = 0;
    auto load = [&](d2 (&av)[U]) {
        const d2 *ar = A2 + (i0 + kl * W) * ld2 + cl * (U * 64);
#pragma unroll
        for (int u = 0; u < U; ++u) av[u] = load_a<NTA>(ar + u * 64);
        if (++cl == spr) {
            cl = 0;
            ++kl;
        }
    };
    d2 aa[U], ab[U];
    if (nsteps > 0) load(aa);
    if (nsteps > 1) load(ab);
    {  // stage the vector (FOLD: form p_k) while the first two steps of A are in flight
        constexpr int KS = 4;
        const d2 *v2 = reinterpret_cast<const d2 *>(v);
        const d2 *q2 = reinterpret_cast<const d2 *>(pold);
        for (int64_t k0 = threadIdx.x; k0 < ld2; k0 += KS * NTB) {
            d2 rv[KS], qv[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int64_t k = k0 + s * NTB;
                rv[s] = k < ld2 ? v2[k] : (d2)(0.0);
                if constexpr (FOLD) qv[s] = k < ld2 ? q2[k] : (d2)(0.0);
            }
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int64_t k = k0 + s * NTB;
                if (k < ld2) {
                    if constexpr (FOLD) sp[k] = rv[s] + beta * qv[s];  // p = r + beta p
                    else sp[k] = rv[s];
                }
            }
        }
    }
    __syncthreads();
    const double *spd = reinterpret_cast<const double *>(sp);
    double dacc = 0.0;
    d2 acc = (d2)(0.0);
    int64_t kf = 0, cf = 0;  // FMA state
    auto fma_step = [&](const d2 (&av)[U]) {
        const d2 *pr = sp + cf * (U * 64) + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const d2 pv = pr[u * 64];
            acc.x = __builtin_fma(av[u].x, pv.x, acc.x);
            acc.y = __builtin_fma(av[u].y, pv.y, acc.y);
        }
        if (++cf == spr) {  // the row is complete
            const double y = wave_sum(acc.x + acc.y);
            const int64_t i = i0 + kf * W;
            if (lane == 0) {
                out[i] = y;
                if constexpr (FOLD) {
                    const double pi = spd[i];
                    pnew[i] = pi;
                    dacc += pi * y;
                } else if (pown) {
                    dacc += pown[i] * y;
                }
            }
            acc = (d2)(0.0);
            cf = 0;
            ++kf;
        }
    };
    for (int64_t s = 0; s < nsteps; s += 2) {  // one step's loads in flight behind each step's FMAs
        fma_step(aa);
        if (s + 2 < nsteps) load(aa);
        if (s + 1 >= nsteps) break;
        fma_step(ab);
        if (s + 3 < nsteps) load(ab);
    }
    if (dot_out) grid_sum_last_block<NTB>(dacc, partials, ticket, dot_out);
    ts_end(ts);
}

template <bool FOLD>
using SmallFn = decltype(&k_matvec_small_f64<FOLD, 1024, 4>);
template <bool FOLD, int NTA>
SmallFn<FOLD> pick_small_u(int ntb, int U) {
    if (ntb == 512) return U == 8 ? k_matvec_small_f64<FOLD, 512, 8, NTA> : k_matvec_small_f64<FOLD, 512, 4, NTA>;
    return U == 8 ? k_matvec_small_f64<FOLD, 1024, 8, NTA> : k_matvec_small_f64<FOLD, 1024, 4, NTA>;
}
// nt: the plan's A load policy (0: default policy, A may stay in the 256 MB
// MALL between iterations; otherwise non-temporal)
template <bool FOLD>
SmallFn<FOLD> pick_small(int ntb, int U, int nt) {
    return nt == 0 ? pick_small_u<FOLD, 0>(ntb, U) : pick_small_u<FOLD, 1>(ntb, U);
}

using FoldFn = decltype(&k_matvec_fold_f64<1, 8>);
template <int NTA>
FoldFn pick_fold_u(int R, int U) {
    if (R == 1)
        return U == 2 ? k_matvec_fold_f64<1, 2, NTA> : U == 4 ? k_matvec_fold_f64<1, 4, NTA> : k_matvec_fold_f64<1, 8, NTA>;
    return U == 2 ? k_matvec_fold_f64<2, 2, NTA> : U == 4 ? k_matvec_fold_f64<2, 4, NTA> : k_matvec_fold_f64<2, 8, NTA>;
}
// the plan's A policy: 0 / 2 default-policy loads, otherwise non-temporal
FoldFn pick_fold(int R, int U, int nt) {
    return (nt == 0 || nt == 2) ? pick_fold_u<0>(R, U) : pick_fold_u<1>(R, U);
}

using MvFn = void (*)(const double *, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int,
                      const double *, double *, const double *, double *, double *, unsigned *, const int64_t *,
                      int64_t *);

template <int R, int U, bool ROT>
MvFn pick_nt(int nt) {
    switch (nt) {
        case 0: return k_matvec_f64<R, U, 0, false, ROT>;
        case 2: return k_matvec_f64<R, U, 0, true, ROT>;  // pipelined, default-policy loads
        case 8: return k_matvec_f64<R, U, 1, true, ROT>;  // pipelined, global nt (the default)
        default: return k_matvec_f64<R, U, 1, false, ROT>;
    }
}
template <int R, bool ROT>
MvFn pick_u(int U, int nt) {
    switch (U) {
        case 2: return pick_nt<R, 2, ROT>(nt);
        case 8: return pick_nt<R, 8, ROT>(nt);
        default: return pick_nt<R, 4, ROT>(nt);
    }
}
template <bool ROT>
MvFn pick_r(int R, int U, int nt) {
    switch (R) {
        case 1: return pick_u<1, ROT>(U, nt);
        case 2: return pick_u<2, ROT>(U, nt);
        case 8: return pick_u<8, ROT>(U, nt);
        default: return pick_u<4, ROT>(U, nt);
    }
}
MvFn pick_mv(int R, int U, int nt, bool rot = false) {
    return rot ? pick_r<true>(R, U, nt) : pick_r<false>(R, U, nt);
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
    // an A of up to 64 MiB with default-policy loads (2), so it stays in the
    // 256 MB MALL between iterations (profiles/r03_iteration_floor_mall_l2.jsonl)
    pl.nt = (cols > 0 && rows * cols * 8 <= (int64_t(64) << 20)) ? 2 : 8;
    pl.R = env_opt("CGX_MV_PLAN", "R", pl.R);
    pl.U = env_opt("CGX_MV_PLAN", "U", pl.U);
    pl.nt = env_opt("CGX_MV_PLAN", "nt", pl.nt);
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
    per_cu = env_opt("CGX_MV_PLAN", "bpc", per_cu);
    if (blocks_per_cu > 0) per_cu = blocks_per_cu;
    const int64_t groups = (rows + pl.R - 1) / pl.R;
    const int64_t need = (groups + (kNT / 64) - 1) / (kNT / 64);
    int64_t cap = (int64_t)per_cu * cus;
    if (cap > kMaxRedBlocks) cap = kMaxRedBlocks;
    pl.blocks = (int)std::max<int64_t>(1, std::min(need, cap));
    return pl;
}

MatvecPlan plan_matvec_small_f64(int device, int64_t rows, int64_t lda) {
    MatvecPlan pl;
    if (env_int("CGX_MV_SMALL", 1) == 0 || rows <= 0 || lda < 2048 || lda > kSmallMaxCols || (lda & 127))
        return pl;
    const int cus = cu_count(device);
    const int64_t chunks = lda >> 7;
    // One 512-thread block per CU, 8 chunks per step (64 KiB of A in flight
    // per CU), the first two steps issued before the staging.  Per iteration
    // (folded, device clock) at n = 2048 / 4096 / 8192: 13.8 / 30.0-30.1 /
    // 91.0 us against 14.3 / 30.8 / 92.1 for round 2's two-launch form on
    // the same box; 1024 threads x 4 chunks: 14.6-14.8 / 30.9-33.3 / 92.2-92.4,
    // x 8: 15.2 / 31.0 / 91.1-91.4 (profiles/r03_iteration_floor_small*.jsonl).
    pl.small = env_opt("CGX_SMALL_PLAN", "threads", 512);
    pl.U = env_opt("CGX_SMALL_PLAN", "U", chunks % 8 ? 4 : 8);
    if ((pl.small != 512 && pl.small != 1024) || (pl.U != 4 && pl.U != 8) || chunks % pl.U) {
        pl.small = 0;
        return pl;
    }
    pl.R = 1;
    // A of up to 64 MiB read with default-policy loads stays in the 256 MB
    // MALL between iterations: 13.4 vs 13.9 us per iteration at n = 2048 (33.5
    // MB); at 4096 (134 MB) 30.6 vs 30.2, at 8192 (537 MB) 103 vs 90
    // (profiles/r03_iteration_floor_small_mall.jsonl)
    pl.nt = env_opt("CGX_SMALL_PLAN", "nt", rows * lda * 8 <= (int64_t(64) << 20) ? 0 : 1) ? 8 : 0;
    const int64_t need = (rows + pl.small / 64 - 1) / (pl.small / 64);
    pl.blocks = (int)std::max<int64_t>(1, std::min<int64_t>(need, std::min<int64_t>(cus, kMaxRedBlocks)));
    return pl;
}

hipError_t matvec_f64(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                      const double *v, double *out, const double *pown, double *dot_out,
                      const RedWs &ws, hipStream_t s, const int64_t *gate, int64_t *ts) {
    if (rows <= 0) return hipSuccess;
    if (pl.small) {  // every column to lda (A and v zero past n), vector in LDS
        if (cols != lda || (lda & 127) || lda > kSmallMaxCols ||
            ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(pick_small<false>(pl.small, pl.U, pl.nt), dim3(pl.blocks), dim3(pl.small), 0, s, A, lda, rows, v,
                           nullptr, nullptr, nullptr, nullptr, pown, out, dot_out, ws.partials,
                           ws.tickets + T_MATVEC, gate, ts);
        return hipGetLastError();
    }
    // The vector path needs 16-B-aligned rows and p; otherwise every column
    // goes through the scalar tail loop.
    const bool aligned = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15) == 0 &&
                         (lda & 1) == 0;
    const int64_t vec_cols = aligned ? (cols & ~int64_t(127)) : 0;
    MvFn fn = pick_mv(pl.R, pl.U, pl.nt);
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, vec_cols, int64_t(0),
                       vec_cols >> 7, int64_t(0), 1, 0, v, out, pown, dot_out, ws.partials, ws.tickets + T_MATVEC,
                       gate, ts);
    return hipGetLastError();
}

hipError_t matvec_f64_cols(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t col_first, int64_t col_count, bool accumulate, const double *v, double *out,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate, int64_t *ts, int64_t col_seg) {
    if (rows <= 0) return hipSuccess;
    if ((cols & 127) || (col_first & 127) || (col_count & 127) || (col_seg & 127) || (lda & 1) ||
        col_first >= cols || col_count > cols || col_seg < 0 || col_seg > col_count || (col_seg && accumulate) ||
        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15))
        return hipErrorInvalidValue;
    const bool rot = col_seg > 0 && col_seg < col_count;
    MvFn fn = pick_mv(pl.R, pl.U, pl.nt, rot);
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, cols, col_first >> 7,
                       col_count >> 7, rot ? col_seg >> 7 : int64_t(0), 0, accumulate ? 1 : 0, v, out, pown,
                       dot_out, ws.partials, ws.tickets + T_MATVEC, gate, ts);
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
    if (pl.small) {
        if (cols != lda || (lda & 127) || lda > kSmallMaxCols) return hipErrorInvalidValue;
        hipLaunchKernelGGL(pick_small<true>(pl.small, pl.U, pl.nt), dim3(pl.blocks), dim3(pl.small), 0, s, A, lda, rows, r,
                           pold, pnew, rr_new, rr_old, nullptr, out, dot_out, ws.partials, ws.tickets + T_MATVEC,
                           gate, ts);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(pick_fold(pl.R == 1 ? 1 : 2, pl.U, pl.nt), dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols,
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
