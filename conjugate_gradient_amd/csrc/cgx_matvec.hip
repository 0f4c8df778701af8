// cgx_matvec.hip -- the dense fp64 matVec (the CG hot path's HBM-bound kernel).
//
// The reference's matVec (serialConjugate.c:109-120, parallel_cg.c:172-184)
// becomes k_matvec_f64 (+ the p.Ap vecVec fused into its epilogue) and its
// load-policy variants (flat, SGPR-base, LDS-staged p).  The other kernels of
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
//   0 plain global_load, 1 global_load ... nt,
//   2..6: buffer_load with cache-policy bits aux = kBufAux[POL] (2 nt,
//   18 nt sc1, 19 sc0 nt sc1, 16 sc1, 0 none) through a per-row descriptor;
//   7 / 8: software-pipelined, buffer / global nt (8 = the default plan);
//   9 / 10 flattened pipeline; 11 LDS-staged p; 12 / 13 SGPR row bases
//   (+ LDS p).  All give the same row sums bit for bit.
constexpr int kBufAux[7] = {0, 0, 2, 18, 19, 16, 0};
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ d2 load_a(const d2 *p) {
    if constexpr (POL == 1) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int POL>
__device__ __forceinline__ d2 load_a_buf(__amdgpu_buffer_rsrc_t rs, int64_t chunk, int lane) {
    // loop-invariant voffset, the chunk in soffset (wave-uniform): no per-step
    // VGPR address arithmetic, which the register allocator otherwise places
    // in registers the previous step's loads still write (forcing a wait)
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (int)(chunk * 1024), kBufAux[POL]);
    return __builtin_bit_cast(d2, v);
}

// ---------------------------------------------------------------------------
// matVec (serialConjugate.c:109-120 / parallel_cg.c:172-184), fp64.
// Wave w owns row groups g = w, w + waves, ...; a group is R consecutive rows.
// Per step a lane holds U 16-B chunks of p and R*U 16-B chunks of A.
// ---------------------------------------------------------------------------
// Accumulate 128-column chunks [c0, c1) of R rows into acc (U chunks per step).
template <int R, int U, int NT>
__device__ __forceinline__ void mv_chunks(const d2 *const (&arow)[R], const __amdgpu_buffer_rsrc_t (&rs)[R],
                                          int lane, const d2 *v2, int64_t c0, int64_t c1, d2 (&acc)[R]) {
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
                if constexpr (NT >= 2) av[r][u] = load_a_buf<NT>(rs[r], c + u, lane);
                else av[r][u] = load_a<NT>(arow[r] + (c + u) * 64);
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
            d2 a;
            if constexpr (NT >= 2) a = load_a_buf<NT>(rs[r], c, lane);
            else a = load_a<NT>(arow[r] + c * 64);
            acc[r].x = __builtin_fma(a.x, pv.x, acc[r].x);
            acc[r].y = __builtin_fma(a.y, pv.y, acc[r].y);
        }
    }
}

// Software-pipelined variant: the loads of step c+U are issued before the
// FMAs of step c (two register sets, ping-pong), so a wave always has a
// step's loads in flight.
template <int R, int U, int NT>
__device__ __forceinline__ void mv_load_step(const d2 *const (&arow)[R], const __amdgpu_buffer_rsrc_t (&rs)[R], int lane,
                                             const d2 *v2, int64_t c, d2 (&pv)[U], d2 (&av)[R][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) pv[u] = v2[(c + u) * 64];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (NT >= 2) av[r][u] = load_a_buf<NT>(rs[r], c + u, lane);
            else av[r][u] = load_a<NT>(arow[r] + (c + u) * 64);
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
__device__ __forceinline__ void mv_chunks_pipe(const d2 *const (&arow)[R], const __amdgpu_buffer_rsrc_t (&rs)[R],
                                               int lane, const d2 *v2, int64_t c0, int64_t c1, d2 (&acc)[R]) {
    d2 pa[U], aa[R][U], pb[U], ab[R][U];
    int64_t c = c0;
    if (c + U <= c1) mv_load_step<R, U, NT>(arow, rs, lane, v2, c, pa, aa);
    while (c + U <= c1) {
        const bool more = c + 2 * U <= c1;
        if (more) mv_load_step<R, U, NT>(arow, rs, lane, v2, c + U, pb, ab);
        mv_fma_step<R, U>(pa, aa, acc);
        c += U;
        if (!more) break;
        const bool more2 = c + 2 * U <= c1;
        if (more2) mv_load_step<R, U, NT>(arow, rs, lane, v2, c + U, pa, aa);
        mv_fma_step<R, U>(pb, ab, acc);
        c += U;
        if (!more2) break;
    }
    // remaining single chunks
    for (; c < c1; ++c) {
        const d2 pv = v2[c * 64];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            d2 a;
            if constexpr (NT >= 2) a = load_a_buf<NT>(rs[r], c, lane);
            else a = load_a<NT>(arow[r] + c * 64);
            acc[r].x = __builtin_fma(a.x, pv.x, acc[r].x);
            acc[r].y = __builtin_fma(a.y, pv.y, acc[r].y);
        }
    }
}

// Column range: the `ccount` 128-column chunks starting at chunk `cfirst`,
// wrapping modulo the vec_cols/128 aligned chunks; `tail` adds the scalar
// columns [vec_cols, cols).  `accumulate` adds the existing out[i] (the
// overlap path computes the shard's own column block first, then the rest).
// Flattened pipelined matVec: a wave walks (row group, step) pairs as one
// stream, so the loads of the next group's first step are already in flight
// while the current group's last FMAs, row sums and stores run (mv_chunks_pipe
// drains at every group boundary: 1/16 of the steps at N=16384).  Row bases
// are wave-uniform (readfirstlane), so each A load is an SGPR base plus a
// 32-bit lane offset.  Requires both column pieces to be multiples of U
// chunks (the host picks the plain kernel otherwise).
template <int R, int U, int NT>
__device__ __forceinline__ void mv_flat_load(const double *const (&base)[R], const __amdgpu_buffer_rsrc_t (&rs)[R],
                                             __amdgpu_buffer_rsrc_t prs, int lane, const d2 *v2, int64_t c,
                                             d2 (&pv)[U], d2 (&av)[R][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if constexpr (NT >= 2)
            pv[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(prs, lane * 16, (int)((c + u) * 1024), 0));
        else
            pv[u] = v2[(c + u) * 64];
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (NT >= 2) {
                av[r][u] = load_a_buf<NT>(rs[r], c + u, lane);
            } else {
                const uint32_t off = (uint32_t)(((c + u) * 64 + lane) * 16);
                av[r][u] = load_a<NT>(reinterpret_cast<const d2 *>(reinterpret_cast<const char *>(base[r]) + off));
            }
        }
}

template <int R, int U, int NT>
__global__ __launch_bounds__(kNT) void k_matvec_f64_flat(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
    const double *__restrict__ pown, double *dot_out, double *partials, unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // group / step / chunk counters are 32-bit (rows, chunks < 2^31): their
    // compares stay on the scalar unit; 64-bit ones went through VGPRs that
    // the allocator took from in-flight load destinations (a wait each step)
    const int ngroups = (int)((rows + R - 1) / R);
    const int wstride = (int)gridDim.x * (kNT / 64);
    const int nchunk = (int)(vec_cols >> 7);
    const int64_t ctail = (int64_t)nchunk << 7;
    const int ca = (int)cfirst, cb = (cfirst + ccount < nchunk) ? (int)(cfirst + ccount) : nchunk;
    const int piece1 = cb - ca;
    const int S = (int)((piece1 + (cfirst + ccount - cb)) / U);  // steps per row group
    const d2 *v2 = reinterpret_cast<const d2 *>(v) + lane;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc((void *)v, 0, (int)(nchunk * 1024), 0x00020000);
    double dacc = 0.0;

    // load cursor (group lg, step ls) and its row bases
    int lg = (int)blockIdx.x * (kNT / 64) + wid, ls = 0;
    const double *lbase[R];
    __amdgpu_buffer_rsrc_t lrs[R];
    auto set_rows = [&](int g) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = (g * R + r < (int)rows) ? g * R + r : (int)rows - 1;
            lbase[r] = A + (int64_t)row * lda;
            if constexpr (NT >= 2)
                lrs[r] = __builtin_amdgcn_make_buffer_rsrc((void *)lbase[r], 0, (int)(lda * 8), 0x00020000);
        }
    };
    auto col_of = [&](int s) -> int {
        const int o = s * U;
        return o < piece1 ? ca + o : o - piece1;
    };
    // compute cursor (group cg, step cs)
    int cg = lg, cs = 0;
    d2 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = (d2)(0.0);
    auto finish_group = [&]() {
        const int64_t r0 = (int64_t)cg * R;
        if (tail)
            for (int64_t j = ctail + lane; j < cols; j += 64) {
                const double vj = v[j];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int64_t row = (r0 + r < rows) ? r0 + r : rows - 1;
                    acc[r].x = __builtin_fma(A[row * lda + j], vj, acc[r].x);
                }
            }
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double s = wave_sum(acc[r].x + acc[r].y);
            if (lane == r) mine = s;
            acc[r] = (d2)(0.0);
        }
        if (lane < R && r0 + lane < rows) {
            if (accumulate) mine = out[r0 + lane] + mine;
            out[r0 + lane] = mine;
            if (pown) dacc += pown[r0 + lane] * mine;
        }
    };

    if (lg < ngroups && S > 0) {
        d2 pa[U], aa[R][U], pb[U], ab[R][U];
        set_rows(lg);
        mv_flat_load<R, U, NT>(lbase, lrs, prs, lane, v2, col_of(0), pa, aa);
        // The load cursor stops at the wave's last step, which is then loaded
        // again (16 KiB per wave, once): every step issues the same loads, so
        // the compiler's wait counts never assume the next set is absent (a
        // conditional load made them drain it before each step's FMAs).
        bool loading = true;
        auto advance = [&]() {
            if (loading && ++ls == S) {
                if (lg + wstride < ngroups) {
                    ls = 0;
                    lg += wstride;
                    set_rows(lg);
                } else {
                    ls = S - 1;
                    loading = false;
                }
            }
        };
        for (;;) {
            // ---- set A is in flight: issue B = next step, then consume A
            advance();
            mv_flat_load<R, U, NT>(lbase, lrs, prs, lane, v2, col_of(ls), pb, ab);
            mv_fma_step<R, U>(pa, aa, acc);
            if (++cs == S) {
                finish_group();
                cs = 0;
                cg += wstride;
                if (cg >= ngroups) break;
            }
            // ---- set B is in flight: issue A = next step, then consume B
            advance();
            mv_flat_load<R, U, NT>(lbase, lrs, prs, lane, v2, col_of(ls), pa, aa);
            mv_fma_step<R, U>(pb, ab, acc);
            if (++cs == S) {
                finish_group();
                cs = 0;
                cg += wstride;
                if (cg >= ngroups) break;
            }
        }
    } else if (lg < ngroups) {  // no full chunks (vec_cols < 128): tail columns only
        for (; cg < ngroups; cg += wstride) finish_group();
    }
    if (pown) grid_sum_last_block(dacc, partials, ticket, dot_out);
}

// Policies 12 / 13: the pipelined matVec with wave-uniform row bases.  The
// wave id is readfirstlane'd, so a row group's row addresses live in SGPRs;
// every A and p load is `global_load ... v_off, s[base]` with one 32-bit lane
// offset kept opaque to loop strength reduction (which otherwise builds a
// 64-bit per-lane pointer per row).  13 also stages each step's p chunks in a
// double-buffered LDS tile shared by the block's waves (one barrier a step);
// every wave of a block then walks the same number of row groups.
__device__ __forceinline__ d2 ldg_nt(const double *base, uint32_t off) {
    asm volatile("" : "+v"(off));
    return __builtin_nontemporal_load(reinterpret_cast<const d2 *>(reinterpret_cast<const char *>(base) + off));
}
__device__ __forceinline__ d2 ldg(const double *base, uint32_t off) {
    asm volatile("" : "+v"(off));
    return *reinterpret_cast<const d2 *>(reinterpret_cast<const char *>(base) + off);
}

template <int R, int U, bool LDSP>
__global__ __launch_bounds__(kNT) void k_matvec_f64_sb(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
    const double *__restrict__ pown, double *dot_out, double *partials, unsigned *ticket, const int64_t *gate) {
    constexpr int W = kNT / 64, UW = LDSP ? U / W : 1;
    static_assert(!LDSP || U % W == 0, "U chunks shared by the block's waves");
    __shared__ d2 sp[LDSP ? 2 : 1][LDSP ? U : 1][64];
    if (gate && *gate) return;
    const int lane = threadIdx.x & 63;
    const uint32_t loff = (uint32_t)lane * 16;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t ngroups = (rows + R - 1) / R;
    const int64_t nchunk = vec_cols >> 7;
    const int64_t ctail = nchunk << 7;
    const int64_t ca = cfirst, cb = (cfirst + ccount < nchunk) ? cfirst + ccount : nchunk;
    const int64_t piece1 = cb - ca;
    const int64_t S = (piece1 + (cfirst + ccount - cb)) / U;  // whole steps (host guarantees no remainder)
    auto col_of = [&](int64_t s) -> int64_t {
        const int64_t o = s * U;
        return o < piece1 ? ca + o : o - piece1;
    };
    double dacc = 0.0;
    // LDSP: block-uniform loop (all waves take part in every barrier)
    const int64_t gstep = (int64_t)gridDim.x * W;
    for (int64_t gb = (int64_t)blockIdx.x * W + (LDSP ? 0 : wid); LDSP ? gb < ngroups : gb < ngroups; gb += gstep) {
        const int64_t g = LDSP ? gb + wid : gb;
        const bool live = g < ngroups;
        const int64_t r0 = (live ? g : ngroups - 1) * R;
        const double *rb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) rb[r] = A + ((r0 + r < rows) ? r0 + r : rows - 1) * lda;
        d2 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = (d2)(0.0);
        if (S > 0) {
            d2 aa[R][U], ab[R][U], pa[LDSP ? 1 : U], pb[LDSP ? 1 : U], pt[UW];
            int buf = 0;
            auto load_step = [&](int64_t c, d2 (&av)[R][U], d2 (&pv)[LDSP ? 1 : U]) {
                if constexpr (LDSP) {
#pragma unroll
                    for (int q = 0; q < UW; ++q) pt[q] = ldg(v + (c + wid * UW + q) * 128, loff);
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) pv[u] = ldg(v + (c + u) * 128, loff);
                }
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) av[r][u] = ldg_nt(rb[r] + (c + u) * 128, loff);
            };
            auto fma_step = [&](const d2 (&av)[R][U], const d2 (&pv)[LDSP ? 1 : U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    d2 p;
                    if constexpr (LDSP) p = sp[buf][u][lane];
                    else p = pv[u];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        acc[r].x = __builtin_fma(av[r][u].x, p.x, acc[r].x);
                        acc[r].y = __builtin_fma(av[r][u].y, p.y, acc[r].y);
                    }
                }
            };
            load_step(col_of(0), aa, pa);
            if constexpr (LDSP) {
#pragma unroll
                for (int q = 0; q < UW; ++q) sp[0][wid * UW + q][lane] = pt[q];
                __syncthreads();
            }
            for (int64_t s = 0;;) {
                // set A in flight: issue B (step s+1), consume A
                bool more = s + 1 < S;
                if (more) load_step(col_of(s + 1), ab, pb);
                fma_step(aa, pa);
                if constexpr (LDSP) {
                    if (more) {
#pragma unroll
                        for (int q = 0; q < UW; ++q) sp[buf ^ 1][wid * UW + q][lane] = pt[q];
                    }
                    __syncthreads();
                    buf ^= 1;
                }
                if (!more) break;
                ++s;
                // set B in flight: issue A (step s+1), consume B
                more = s + 1 < S;
                if (more) load_step(col_of(s + 1), aa, pa);
                fma_step(ab, pb);
                if constexpr (LDSP) {
                    if (more) {
#pragma unroll
                        for (int q = 0; q < UW; ++q) sp[buf ^ 1][wid * UW + q][lane] = pt[q];
                    }
                    __syncthreads();
                    buf ^= 1;
                }
                if (!more) break;
                ++s;
            }
        }
        if (tail)
            for (int64_t j = ctail + lane; j < cols; j += 64) {
                const double vj = v[j];
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r].x = __builtin_fma(rb[r][j], vj, acc[r].x);
            }
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double sr = wave_sum(acc[r].x + acc[r].y);
            if (lane == r) mine = sr;
        }
        if (live && lane < R && r0 + lane < rows) {
            if (accumulate) mine = out[r0 + lane] + mine;
            out[r0 + lane] = mine;
            if (pown) dacc += pown[r0 + lane] * mine;
        }
    }
    if (pown) grid_sum_last_block(dacc, partials, ticket, dot_out);
}

// LDS-staged p (policy 11; the north star's "LDS staging of the p-vector
// tile"): per step the block's 4 waves load the step's U p chunks once
// (U/4 chunks each) into a double-buffered LDS tile, one barrier, and every
// wave reads its p from LDS, so p costs one global load per block per chunk
// instead of one per wave.  A is software-pipelined as in policy 8 (the next
// step's A loads are issued before this step's FMAs).  All waves of a block
// walk the same number of row groups (waves past the last group keep loading
// and synchronising but store nothing).  Both column pieces must be whole
// steps of U chunks (the host falls back to policy 8 otherwise).
template <int R, int U>
__global__ __launch_bounds__(kNT) void k_matvec_f64_lds(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
    const double *__restrict__ pown, double *dot_out, double *partials, unsigned *ticket, const int64_t *gate) {
    static_assert(U % (kNT / 64) == 0, "U chunks shared by the block's waves");
    constexpr int W = kNT / 64, UW = U / W;
    __shared__ d2 sp[2][U][64];
    if (gate && *gate) return;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t ngroups = (rows + R - 1) / R;
    const int64_t nchunk = vec_cols >> 7;
    const int64_t ctail = nchunk << 7;
    const int64_t ca = cfirst, cb = (cfirst + ccount < nchunk) ? cfirst + ccount : nchunk;
    const int64_t piece1 = cb - ca;
    const int64_t S = (piece1 + (cfirst + ccount - cb)) / U;
    const d2 *v2 = reinterpret_cast<const d2 *>(v) + lane;
    auto col_of = [&](int64_t s) -> int64_t {
        const int64_t o = s * U;
        return o < piece1 ? ca + o : o - piece1;
    };
    double dacc = 0.0;
    for (int64_t gb = (int64_t)blockIdx.x * W; gb < ngroups; gb += (int64_t)gridDim.x * W) {
        const int64_t g = gb + wid;
        const bool live = g < ngroups;
        const int64_t r0 = (live ? g : ngroups - 1) * R;
        const d2 *arow[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t row = (r0 + r < rows) ? r0 + r : rows - 1;
            arow[r] = reinterpret_cast<const d2 *>(A + row * lda) + lane;
        }
        d2 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = (d2)(0.0);
        if (S > 0) {
            d2 aa[R][U], ab[R][U], pt[UW];
            int buf = 0;
            // prologue: A and this wave's share of p for step 0
            {
                const int64_t c = col_of(0);
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int u = 0; u < U; ++u) aa[r][u] = load_a<1>(arow[r] + (c + u) * 64);
#pragma unroll
                for (int q = 0; q < UW; ++q) sp[0][wid * UW + q][lane] = v2[(c + wid * UW + q) * 64];
            }
            __syncthreads();
            for (int64_t s = 0; s < S; ++s) {
                const bool more = s + 1 < S;
                if (more) {  // next step: A into the other register set, p share into registers
                    const int64_t c = col_of(s + 1);
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int u = 0; u < U; ++u) ab[r][u] = load_a<1>(arow[r] + (c + u) * 64);
#pragma unroll
                    for (int q = 0; q < UW; ++q) pt[q] = v2[(c + wid * UW + q) * 64];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const d2 pv = sp[buf][u][lane];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        acc[r].x = __builtin_fma(aa[r][u].x, pv.x, acc[r].x);
                        acc[r].y = __builtin_fma(aa[r][u].y, pv.y, acc[r].y);
                    }
                }
                if (more) {
#pragma unroll
                    for (int q = 0; q < UW; ++q) sp[buf ^ 1][wid * UW + q][lane] = pt[q];
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int u = 0; u < U; ++u) aa[r][u] = ab[r][u];
                }
                __syncthreads();
                buf ^= 1;
            }
        }
        if (tail)
            for (int64_t j = ctail + lane; j < cols; j += 64) {
                const double vj = v[j];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int64_t row = (r0 + r < rows) ? r0 + r : rows - 1;
                    acc[r].x = __builtin_fma(A[row * lda + j], vj, acc[r].x);
                }
            }
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double sr = wave_sum(acc[r].x + acc[r].y);
            if (lane == r) mine = sr;
        }
        if (live && lane < R && r0 + lane < rows) {
            if (accumulate) mine = out[r0 + lane] + mine;
            out[r0 + lane] = mine;
            if (pown) dacc += pown[r0 + lane] * mine;
        }
    }
    if (pown) grid_sum_last_block(dacc, partials, ticket, dot_out);
}

template <int R, int U, int NT, bool PIPE = false>
__global__ __launch_bounds__(kNT) void k_matvec_f64(
    const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols, int64_t vec_cols, int64_t cfirst,
    int64_t ccount, int tail, int accumulate, const double *__restrict__ v, double *__restrict__ out,
    const double *__restrict__ pown, double *dot_out, double *partials, unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;  // the solve converged in an earlier iteration (device-side gating)
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
        __amdgpu_buffer_rsrc_t rs[R];
        d2 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            ridx[r] = (r0 + r < rows) ? (r0 + r) : (rows - 1);
            arow[r] = reinterpret_cast<const d2 *>(A + ridx[r] * lda) + lane;
            if constexpr (NT >= 2) {  // wave-uniform row base -> scalar descriptor, no waterfall
                const int64_t row = (int64_t)__builtin_amdgcn_readfirstlane((int)ridx[r]);
                rs[r] = __builtin_amdgcn_make_buffer_rsrc((void *)(A + row * lda), 0, (int)(lda * 8), 0x00020000);
            }
            acc[r] = (d2)(0.0);
        }
        if constexpr (PIPE) {
            mv_chunks_pipe<R, U, NT>(arow, rs, lane, v2, ca, cb, acc);
            if (wrap > 0) mv_chunks_pipe<R, U, NT>(arow, rs, lane, v2, 0, wrap, acc);
        } else {
            mv_chunks<R, U, NT>(arow, rs, lane, v2, ca, cb, acc);
            if (wrap > 0) mv_chunks<R, U, NT>(arow, rs, lane, v2, 0, wrap, acc);
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
}

using MvFn = void (*)(const double *, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int,
                      const double *, double *, const double *, double *, double *, unsigned *, const int64_t *);

template <int R, int U>
MvFn pick_nt(int nt) {
    switch (nt) {
        case 0: return k_matvec_f64<R, U, 0>;
        case 2: return k_matvec_f64<R, U, 2>;
        case 3: return k_matvec_f64<R, U, 3>;
        case 4: return k_matvec_f64<R, U, 4>;
        case 5: return k_matvec_f64<R, U, 5>;
        case 6: return k_matvec_f64<R, U, 6>;
        case 7: return k_matvec_f64<R, U, 2, true>;  // pipelined, buffer nt
        case 8: return k_matvec_f64<R, U, 1, true>;  // pipelined, global nt
        case 9: return k_matvec_f64_flat<R, U, 1>;    // flattened pipeline, global nt
        case 10: return k_matvec_f64_flat<R, U, 2>;   // flattened pipeline, buffer nt
        case 11: return k_matvec_f64_lds<R, U>;       // LDS-staged p, pipelined A
        case 12: return k_matvec_f64_sb<R, U, false>;  // pipelined, SGPR row bases
        case 13: return k_matvec_f64_sb<R, U, true>;   // + LDS-staged p
        default: return k_matvec_f64<R, U, 1>;
    }
}
template <int R, int U>
MvFn pick_nt_basic(int nt) {
    return nt == 0 ? k_matvec_f64<R, U, 0> : k_matvec_f64<R, U, 1>;
}
template <int R>
MvFn pick_u(int U, int nt) {
    switch (U) {
        case 2: return pick_nt_basic<R, 2>(nt);
        case 8: return pick_nt<R, 8>(nt);
        default: return pick_nt<R, 4>(nt);
    }
}
// The flattened kernels need both column pieces to be whole steps of U
// chunks; otherwise the per-group pipelined kernel takes the launch.
int mv_policy(const MatvecPlan &pl, int64_t nchunk, int64_t cfirst, int64_t ccount) {
    if (pl.nt < 9) return pl.nt;
    const int64_t cb = std::min(cfirst + ccount, nchunk);
    const int64_t p1 = cb - cfirst, p2 = cfirst + ccount - cb;
    if (p1 % pl.U || p2 % pl.U) return pl.nt == 10 ? 7 : 8;  // 9, 11-13 need whole steps
    return pl.nt;
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

MatvecPlan plan_matvec_f64(int device, int64_t rows, int R, int U, int nt, int blocks_per_cu) {
    MatvecPlan pl;
    const int cus = cu_count(device);
    // Software-pipelined (loads of step c+U issued before the FMAs of step c),
    // 2 rows per wave, U=8, global_load ... nt: 256 VGPRs, one wave per SIMD,
    // 32 KiB of A in flight per wave.  Measured on MI355X, interleaved against
    // every (R, U, policy) of the unpipelined kernel (profiles/r01_sweep_pipe*):
    // 7.24 TB/s at 65536^2 (unpipelined best R=8,U=8,buffer-nt: 7.09),
    // 7.21 TB/s on an 8192 x 65536 row block (7.05), 6.81 TB/s at 16384^2 (6.60).
    // R=1 when there are fewer than 2 rows per resident wave.
    const int64_t want_waves = (int64_t)cus * 4;
    pl.R = rows >= 2 * want_waves ? 2 : 1;
    pl.U = 8;
    pl.nt = 8;
    pl.R = env_int("CGX_MV_R", pl.R);
    pl.U = env_int("CGX_MV_U", pl.U);
    pl.nt = env_int("CGX_MV_NT", pl.nt);
    if (R > 0) pl.R = R;
    if (U > 0) pl.U = U;
    if (nt >= 0) pl.nt = nt;
    if (pl.R != 1 && pl.R != 2 && pl.R != 4 && pl.R != 8) pl.R = 4;
    if (pl.U != 2 && pl.U != 4 && pl.U != 8) pl.U = 4;
    if (pl.nt < 0 || pl.nt > 13) pl.nt = 1;
    if (pl.U == 2 && pl.nt >= 2) pl.nt = 1;  // buffer variants exist for U = 4, 8
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(pick_mv(pl.R, pl.U, pl.nt)),
                                                     kNT, 0) != hipSuccess || per_cu <= 0)
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
                      const RedWs &ws, hipStream_t s, const int64_t *gate) {
    if (rows <= 0) return hipSuccess;
    // The vector path needs 16-B-aligned rows and p; otherwise every column
    // goes through the scalar tail loop.
    const bool aligned = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15) == 0 &&
                         (lda & 1) == 0;
    const int64_t vec_cols = aligned ? (cols & ~int64_t(127)) : 0;
    MvFn fn = pick_mv(pl.R, pl.U, mv_policy(pl, vec_cols >> 7, 0, vec_cols >> 7));
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, vec_cols, int64_t(0),
                       vec_cols >> 7, 1, 0, v, out, pown, dot_out, ws.partials, ws.tickets + T_MATVEC, gate);
    return hipGetLastError();
}

hipError_t matvec_f64_cols(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t col_first, int64_t col_count, bool accumulate, const double *v, double *out,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate) {
    if (rows <= 0) return hipSuccess;
    if ((cols & 127) || (col_first & 127) || (col_count & 127) || (lda & 1) ||
        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15))
        return hipErrorInvalidValue;
    MvFn fn = pick_mv(pl.R, pl.U, mv_policy(pl, cols >> 7, col_first >> 7, col_count >> 7));
    hipLaunchKernelGGL(fn, dim3(pl.blocks), dim3(kNT), 0, s, A, lda, rows, cols, cols, col_first >> 7,
                       col_count >> 7, 0, accumulate ? 1 : 0, v, out, pown, dot_out, ws.partials,
                       ws.tickets + T_MATVEC, gate);
    return hipGetLastError();
}

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_matvec() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_f64<2, 8, 1, true>));
}

}  // namespace cgx
