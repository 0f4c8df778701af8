// cgx_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the CG hot path.
//
// The reference's BLAS-1/2 loops (serialConjugate.c:109-177, parallel_cg.c:
// 172-245) become:
//   k_matvec_f64      matVec (+ the p.Ap vecVec fused into its epilogue)
//   k_residual_f64    residual x2 + r.r      (serialConjugate.c:209-212)
//   k_update_r_f64    scalarVec+vecSub (r), r.r       (serialConjugate.c:226-234)
//   k_update_xp_f64   scalarVec+vecAdd (x, deferred) and (p) (:221-225, :239-243),
//                     with the device-side stop decision
//   k_update_xr_f64 / k_update_p_f64   the same split as the reference (kernel-level ABI)
//   k_poisson_p_f64 / k_poisson_xr_f64 the fused matrix-free Poisson iteration
// and, for CGX_F32_REF, kernels that keep the reference's exact fp32
// operation order (sequential per-row and per-dot accumulation, every
// multiply and add rounded separately: `#pragma clang fp contract(off)`).
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
#include "cgx_kernels.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace cgx {
namespace {

typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kNT = 256;  // threads per block for the fp64 kernels

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum `v` over all threads of the grid.  Each block stores its total in
// partials[blockIdx.x]; the last block to arrive sums the partials in index
// order and writes *out.  Deterministic for a fixed grid.
//
// Hand-off (cdna_hip_programming.md Guideline 16, the write-through form):
// the partial is stored write-through (8-B agent-scope atomic store = sc1),
// the storing lane drains it (s_waitcnt vmcnt(0)) before its relaxed
// agent-scope ticket add, and the block whose add returns gridDim-1 reads
// every partial with sc1 loads (agent-scope atomic loads) -- no release /
// acquire fence, so no per-block write-back of the L2's dirty lines (which
// cost the r-update ~35 % of its time with a buffer_wbl2 per block).
__device__ __forceinline__ void grid_sum_last_block(double v, double *partials, unsigned *ticket,
                                                    double *out, bool add_to_out = false) {
    __shared__ double red[kNT / 64];
    __shared__ int is_last;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < kNT / 64; ++w) t += red[w];
        __hip_atomic_store(partials + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!is_last) return;
    // all of this thread's partials in flight at once (grid <= 8192 = 32 * kNT)
    double s = 0.0;
    for (unsigned i0 = threadIdx.x; i0 < gridDim.x; i0 += 8 * kNT) {
        double pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned i = i0 + u * kNT;
            pv[u] = (i < gridDim.x) ? __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * kNT < gridDim.x) s += pv[u];
    }
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = red[0];
#pragma unroll
        for (int w = 1; w < kNT / 64; ++w) t += red[w];
        *out = add_to_out ? *out + t : t;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

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

__device__ __forceinline__ d2 ld2(const double *p) { return *reinterpret_cast<const d2 *>(p); }
__device__ __forceinline__ void st2(double *p, d2 v) { *reinterpret_cast<d2 *>(p) = v; }
// Stream policy of the vector kernels (VP): 0 plain, 1 non-temporal stores,
// 2 non-temporal loads and stores (default: -8 % time on the Poisson
// vectors, 537 MB each; profiles/r01_vector_policy.txt).
template <int VP>
__device__ __forceinline__ d2 ldv(const double *p) {
    if constexpr (VP >= 2) return __builtin_nontemporal_load(reinterpret_cast<const d2 *>(p));
    else return *reinterpret_cast<const d2 *>(p);
}
template <int VP>
__device__ __forceinline__ void stv(double *p, d2 v) {
    if constexpr (VP >= 1) __builtin_nontemporal_store(v, reinterpret_cast<d2 *>(p));
    else *reinterpret_cast<d2 *>(p) = v;
}

// Vector kernels.  VEC (every pointer 16-B aligned): a block step covers
// kVU * kNT consecutive element pairs; each thread loads its kVU pairs of
// every input (16-B loads, all issued before any store), computes, stores.
// Otherwise a scalar grid-stride loop.  The odd tail element of the VEC
// path is done by thread 0 of block 0.  Per-thread sums run in a fixed
// order, then the deterministic grid reduction.
constexpr int kVU = 4;

#define CGX_VEC_LOOP_BEGIN                                                                   \
    const int64_t npairs = n >> 1;                                                           \
    const int64_t step = (int64_t)gridDim.x * kNT * kVU;                                     \
    for (int64_t base = (int64_t)blockIdx.x * kNT * kVU + threadIdx.x; base < npairs; base += step) { \
        bool ok[kVU];                                                                        \
        _Pragma("unroll") for (int u = 0; u < kVU; ++u) ok[u] = base + u * kNT < npairs;
#define CGX_VEC_LOOP_END }

// residual x2 + vecVec (serialConjugate.c:210-212)
template <bool VEC>
__global__ __launch_bounds__(kNT) void k_residual_f64(int64_t n, const double *__restrict__ b,
                                                      const double *__restrict__ Ax,
                                                      double *__restrict__ r, double *__restrict__ p,
                                                      double *rr_out, double *partials,
                                                      unsigned *ticket) {
    double acc = 0.0;
    if constexpr (VEC) {
        CGX_VEC_LOOP_BEGIN
        d2 bv[kVU], av[kVU];
#pragma unroll
        for (int u = 0; u < kVU; ++u)
            if (ok[u]) { const int64_t i = 2 * (base + u * kNT); bv[u] = ld2(b + i); av[u] = ld2(Ax + i); }
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
            const double ri = b[n - 1] - Ax[n - 1];
            r[n - 1] = ri;
            if (p) p[n - 1] = ri;
            acc += ri * ri;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
            const double ri = b[i] - Ax[i];
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
    const double alpha = *rsold / *pAp;
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
    const double beta = *rr / *rsold;
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

// The solver's split of the x/r/p updates (fp64): x's update moves into the
// p update, which reads p anyway -- 24 + 40 B per element instead of 48 + 24.
// r -= alpha Ap; r.r   (alpha = rsold / pAp)
template <bool VEC, int VP = 2>
__global__ __launch_bounds__(kNT) void k_update_r_f64(int64_t n, double *__restrict__ r, const double *__restrict__ Ap,
                                                      const double *rsold, const double *pAp, double *rr_out,
                                                      double *partials, unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;
    const double alpha = *rsold / *pAp;
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
}

// x += alpha p (alpha = rsold / pAp); then, if rr != nullptr, p = r + (rr / rsold) p.
// With cv.kdone != nullptr (device-side gating) the kernel also makes the
// reference's stopping decision, `sqrt(r.r) < EPSILON` (serialConjugate.c:235):
// on convergence it does only the x update and records k+1 and r.r; in a
// later iteration (kdone in (0, k]) it does nothing.
struct ConvArgs {
    double eps = -1.0;
    int64_t k = 0;
    int64_t *kdone = nullptr;   // 0 = not converged, else the loop-iteration count
    double *rrfinal = nullptr;
    int64_t *hrec = nullptr;    // host-mapped copy of {kdone, rrfinal}: read by the host without a copy
};

// The convergence record: device slots for later launches' gates, and the
// host-mapped copy the host reads after an event (no per-iteration D2H copy).
__device__ __forceinline__ void record_convergence(const ConvArgs &cv, int64_t kdone, double rr) {
    *cv.rrfinal = rr;
    *cv.kdone = kdone;
    if (cv.hrec) {
        __hip_atomic_store(cv.hrec + 1, __double_as_longlong(rr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(cv.hrec, kdone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool VEC, int VP = 2>
__global__ __launch_bounds__(kNT) void k_update_xp_f64(int64_t n, double *__restrict__ x, double *__restrict__ p,
                                                       const double *__restrict__ r, const double *rsold,
                                                       const double *pAp, const double *rr, ConvArgs cv) {
    bool upd_p = rr != nullptr;
    if (cv.kdone) {
        const int64_t kd = *cv.kdone;
        if (kd != 0 && kd <= cv.k) return;
        const double rrn = *rr;
        if (cv.eps >= 0.0 && sqrt(rrn) < cv.eps) {
            upd_p = false;
            if (blockIdx.x == 0 && threadIdx.x == 0) record_convergence(cv, cv.k + 1, rrn);
        }
    }
    const double alpha = *rsold / *pAp;
    const double beta = upd_p ? *rr / *rsold : 0.0;
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

// ---------------------------------------------------------------------------
// counter-hash SPD generator (generateSPDmatrix.m:4-17 distribution)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double u01(uint64_t salt, uint64_t i, uint64_t j) {
    const uint64_t h = mix64(((i << 32) | (j & 0xffffffffull)) ^ salt);
    return (double)(h >> 11) * 0x1.0p-53;
}

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

// Scalars combined in rank order: ((in0 + in1) + in2) + ...  Inputs sit in
// 8-byte slots (a float at the slot start for F32_REF): element q at in[q*stride].
// ---------------------------------------------------------------------------
// matrix-free 5-point Poisson A.p on a slab (configs[4]; no reference
// counterpart).  ph = p with one halo row above and below: rows 0 and
// mloc+1 are the neighbours' boundary rows (zero at the domain boundary).
// Each block owns a contiguous run of grid rows and sweeps them in order so
// the rows above/below are L2/MALL hits; a thread handles column pairs
// (16-B loads of the centre/up/down rows, 8-B loads of the two side points).
// Fused: *dot_out = p . Ap (same last-block reduction as the matVec).
// ---------------------------------------------------------------------------
// Even m: column-strip marching.  A block owns a strip of 2*kNT columns and a
// run of rows; each thread holds a column pair and walks down the rows with
// the up/centre rows in registers, so every p element is loaded once (plus
// two halo rows per run).  The left/right neighbours come from the adjacent
// lanes by wave shuffle; only lanes 0 / 63 load them (L1 hits).  The next
// row is prefetched one step ahead.
__global__ __launch_bounds__(kNT) void k_stencil5_strip_f64(const double *__restrict__ ph, int64_t mloc, int64_t m,
                                                            int64_t nstrips, int64_t rows_per_block,
                                                            double *__restrict__ Ap, double *dot_out,
                                                            double *partials, unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;
    const int lane = threadIdx.x & 63;
    const int64_t strip = blockIdx.x % nstrips, chunk = blockIdx.x / nstrips;
    const int64_t j = strip * (2 * kNT) + 2 * threadIdx.x;
    const bool valid = j < m;
    const int64_t i0 = chunk * rows_per_block;
    const int64_t i1 = (i0 + rows_per_block < mloc) ? i0 + rows_per_block : mloc;
    double acc = 0.0;
    if (i0 < i1) {
        const d2 zero = (d2)(0.0);
        const double *col = ph + j;
        d2 up = valid ? ld2(col + i0 * m) : zero;
        d2 ce = valid ? ld2(col + (i0 + 1) * m) : zero;
        d2 dn = valid ? ld2(col + (i0 + 2) * m) : zero;
        for (int64_t i = i0; i < i1; ++i) {
            // prefetch the row after next while this row is computed
            const d2 nx = (valid && i + 1 < i1) ? ld2(col + (i + 3) * m) : zero;
            double l = __shfl_up(ce.y, 1, 64);
            double r = __shfl_down(ce.x, 1, 64);
            const double *crow = ph + (i + 1) * m;
            if (lane == 0) l = (j > 0 && valid) ? crow[j - 1] : 0.0;
            if (lane == 63) r = (j + 2 < m) ? crow[j + 2] : 0.0;
            d2 o;
            o.x = 4.0 * ce.x - up.x - dn.x - l - ce.y;
            o.y = 4.0 * ce.y - up.y - dn.y - ce.x - r;
            if (valid) {
                st2(Ap + i * m + j, o);
                if (dot_out) acc += ce.x * o.x + ce.y * o.y;
            }
            up = ce;
            ce = dn;
            dn = nx;
        }
    }
    if (dot_out) grid_sum_last_block(acc, partials, ticket, dot_out);
}

// Odd m (rows not 16-B aligned): a block walks a run of rows, one column per thread.
// Fused Poisson iteration (even m): two strip-marching kernels per CG
// iteration instead of stencil + r update + x/p update, so no Ap vector
// exists.  A p_k is recomputed by the second kernel from p_k (5 flops per
// point against 16 B of an Ap round trip).  Bytes per grid point per
// iteration: 24 (k_poisson_p: r, p_{k-1} -> p_k) + 40 (k_poisson_xr: p_k,
// x, r -> x, r) = 64, against 80 for the three-kernel split.
//
// k_poisson_p_f64 (iteration k):  p_k = r_k + beta p_{k-1} (p_0 = r_0) into
// the other p buffer (the window reads p_{k-1} rows owned by neighbouring
// blocks, so the update cannot be in place), including the slab's halo rows
// (computed from the exchanged r halo and the p_{k-1} halo this kernel wrote
// one iteration earlier; zero at the domain boundary), and
// *dot_out = p_k . A p_k.  With cv.kdone it first decides the previous
// iteration's sqrt(r.r) < eps (device-side gating): on convergence it stores
// *kdone = k, *rrfinal = r.r and does nothing else; x is already final.

// Work items are (strip of 2*kNT columns, run of `rpi` rows), numbered strip-
// fastest, and blocks take them grid-stride: the items in flight at any time
// are consecutive, i.e. a narrow band of grid rows, so the vectors are
// streamed roughly in address order instead of from ~2048 places at once.
// Each item's run is walked RB rows per step: all loads of a step (RB new p
// rows, RB rows of each streamed vector, the lane-0/63 side points) are
// issued before its arithmetic.  Streamed vectors use non-temporal loads and
// stores (NT), as the vector kernels do.
// Addresses: a wave-uniform row base plus the lane's 32-bit byte offset
// (lanes past the last column load column 0 and their values are zeroed),
// so a step of RB rows is straight-line code: no per-row or per-lane branch
// between its loads and its arithmetic except around the stores.  The side
// points j-1 of lane 0 and j+2 of lane 63 are wave-uniform addresses.
// Row base + lane offset with the offset made opaque to the optimiser (an
// empty asm on the VGPR), so loop strength reduction cannot fold it into a
// per-lane 64-bit pointer induction variable: every access keeps the
// `global_load ... vOff, s[base]` form, with the row stepping in SGPRs.
template <bool NT>
__device__ __forceinline__ d2 lds2(const double *row, uint32_t off) {
    asm volatile("" : "+v"(off));
    const d2 *p = reinterpret_cast<const d2 *>(reinterpret_cast<const char *>(row) + off);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void sts2(double *row, uint32_t off, d2 v) {
    asm volatile("" : "+v"(off));
    d2 *p = reinterpret_cast<d2 *>(reinterpret_cast<char *>(row) + off);
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// One lane's view of a work item: column pair j, j+1 (byte offset `off`,
// 0 for lanes past the grid), its wave wv and the wave's first column jw.
// Side points: lane 0 needs column j-1, lane 63 column j+2.  Inside a block
// they come from the neighbouring wave through LDS (one barrier per step);
// only the block's outer edges (wave 0 left, wave 3 right) load them, from
// wave-uniform addresses.  Loading every wave's side points from memory
// costs a 64-128 B line per 8-B value: +25 % of the fetched bytes (PMC).
struct StripLane {
    bool valid, has_l, has_r;
    int wv;
    uint32_t off;
    int64_t jw;
};
constexpr int kWaves = kNT / 64;
__device__ __forceinline__ StripLane strip_lane(int64_t w, int64_t nstrips, int64_t m) {
    StripLane L;
    L.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    L.jw = (w % nstrips) * (2 * kNT) + L.wv * 128;
    const int64_t j = L.jw + 2 * (threadIdx.x & 63);
    L.valid = j < m;
    L.off = L.valid ? (uint32_t)(j * 8) : 0u;
    L.has_l = L.wv == 0 && L.jw > 0;
    L.has_r = L.wv == kWaves - 1 && L.jw + 128 < m;
    return L;
}
__device__ __forceinline__ d2 keep(bool valid, d2 v) {
    d2 o;
    o.x = valid ? v.x : 0.0;
    o.y = valid ? v.y : 0.0;
    return o;
}

// LDS edge exchange: eb[(wave * 2 + side) * 8 + t], side 0 = the wave's first
// value (lane 0's .x), side 1 = its last (lane 63's .y); two halves by step
// parity so one barrier per step suffices.
constexpr int kEdgeRB = 8;
template <int RBn>
__device__ __forceinline__ void edges_put(double *eb, const StripLane &L, const d2 (&ce)[RBn]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        if (lane == 0) eb[(L.wv * 2 + 0) * kEdgeRB + t] = ce[t].x;
        if (lane == 63) eb[(L.wv * 2 + 1) * kEdgeRB + t] = ce[t].y;
    }
}
__device__ __forceinline__ double edge_l(const double *eb, const StripLane &L, int t, double outer) {
    return L.wv > 0 ? eb[((L.wv - 1) * 2 + 1) * kEdgeRB + t] : outer;
}
__device__ __forceinline__ double edge_r(const double *eb, const StripLane &L, int t, double outer) {
    return L.wv < kWaves - 1 ? eb[((L.wv + 1) * 2 + 0) * kEdgeRB + t] : outer;
}

// p_k rows (FIRST: p_0 = r_0)
template <bool NT, bool FIRST>
__device__ __forceinline__ d2 pnv(const double *rrow, const double *prow, const StripLane &L, double beta) {
    const d2 rv = lds2<NT>(rrow, L.off);
    if constexpr (FIRST) return keep(L.valid, rv);
    const d2 pv = lds2<NT>(prow, L.off);
    d2 o;
    o.x = __builtin_fma(beta, pv.x, rv.x);
    o.y = __builtin_fma(beta, pv.y, rv.y);
    return keep(L.valid, o);
}
template <bool FIRST>
__device__ __forceinline__ double pns(const double *rrow, const double *prow, int64_t col, double beta) {
    if constexpr (FIRST) return rrow[col];
    else return __builtin_fma(beta, prow[col], rrow[col]);
}

// RBn output rows starting at interior row i: pm, pc carry p_k rows h = i, i+1.
template <int RBn, bool NT, bool FIRST, bool HT>
__device__ __forceinline__ void poisson_p_step(const double *__restrict__ rh, const double *__restrict__ poh,
                                               double *__restrict__ pnh, int64_t mloc, int64_t m, int64_t i,
                                               const StripLane &L, double beta, d2 &pm, d2 &pc, double &acc,
                                               double *eb) {
    const int lane = threadIdx.x & 63;
    d2 pr[RBn], ce[RBn];
    double el[RBn], er[RBn];
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const int64_t hc = (i + t + 1) * m;  // centre row (halo coordinates) of output row i+t
        // HT: the last two rows are the next item's first two (its halo):
        // default-policy loads keep them in L2 for the block that reads them next
        pr[t] = (HT && t >= RBn - 2) ? pnv<false, FIRST>(rh + hc + m, poh + hc + m, L, beta)
                                     : pnv<NT, FIRST>(rh + hc + m, poh + hc + m, L, beta);
        el[t] = L.has_l ? pns<FIRST>(rh + hc, poh + hc, L.jw - 1, beta) : 0.0;
        er[t] = L.has_r ? pns<FIRST>(rh + hc, poh + hc, L.jw + 128, beta) : 0.0;
    }
#pragma unroll
    for (int t = 0; t < RBn; ++t) ce[t] = t == 0 ? pc : pr[t - 1];
    edges_put<RBn>(eb, L, ce);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const d2 up = t == 0 ? pm : (t == 1 ? pc : pr[t - 2]);
        const d2 dn = pr[t];
        const double lw = edge_l(eb, L, t, el[t]), rw = edge_r(eb, L, t, er[t]);
        double l = __shfl_up(ce[t].y, 1, 64);
        double r = __shfl_down(ce[t].x, 1, 64);
        l = lane == 0 ? lw : l;
        r = lane == 63 ? rw : r;
        d2 o;
        o.x = 4.0 * ce[t].x - up.x - dn.x - l - ce[t].y;
        o.y = 4.0 * ce[t].y - up.y - dn.y - ce[t].x - r;
        acc += ce[t].x * o.x + ce[t].y * o.y;  // zero on lanes past the grid
        if (L.valid) {
            sts2<NT>(pnh + (i + t + 1) * m, L.off, ce[t]);
            if (i + t == mloc - 1) sts2<NT>(pnh + (mloc + 1) * m, L.off, dn);  // bottom halo row of p_k
        }
    }
    if constexpr (RBn >= 2) {
        pm = pr[RBn - 2];
        pc = pr[RBn - 1];
    } else {
        pm = pc;
        pc = pr[0];
    }
}

// Work items [w0, w0+cnt1) then [w2, w2+cnt2) (the whole slab, or, when
// the r halo exchange overlaps the kernel, the slab's interior runs first
// and its two edge runs after the exchange).
struct ItemRanges {
    int64_t w0, cnt1, w2, cnt2;
};

template <int RB, bool NT, bool FIRST, bool HT>
__device__ __forceinline__ double poisson_p_body(const double *__restrict__ rh, const double *__restrict__ poh,
                                                 double *__restrict__ pnh, int64_t mloc, int64_t m, int64_t nstrips,
                                                 int64_t rpi, ItemRanges ir, double beta, double *edge) {
    double acc = 0.0;
    int par = 0;
    for (int64_t v = blockIdx.x; v < ir.cnt1 + ir.cnt2; v += gridDim.x) {
        const int64_t w = v < ir.cnt1 ? ir.w0 + v : ir.w2 + (v - ir.cnt1);
        const StripLane L = strip_lane(w, nstrips, m);
        const int64_t i0 = (w / nstrips) * rpi;
        const int64_t i1 = (i0 + rpi < mloc) ? i0 + rpi : mloc;
        d2 pm = pnv<NT && !HT, FIRST>(rh + i0 * m, poh + i0 * m, L, beta);
        d2 pc = pnv<NT && !HT, FIRST>(rh + (i0 + 1) * m, poh + (i0 + 1) * m, L, beta);
        if (L.valid && i0 == 0) sts2<NT>(pnh, L.off, pm);  // top halo row of p_k
        int64_t i = i0;
        for (; i + RB <= i1; i += RB, par ^= 1)
            poisson_p_step<RB, NT, FIRST, HT>(rh, poh, pnh, mloc, m, i, L, beta, pm, pc, acc,
                                          edge + par * (kWaves * 2 * kEdgeRB));
        for (; i < i1; ++i, par ^= 1)
            poisson_p_step<1, NT, FIRST, HT>(rh, poh, pnh, mloc, m, i, L, beta, pm, pc, acc,
                                         edge + par * (kWaves * 2 * kEdgeRB));
    }
    return acc;
}

template <int RB, bool NT, bool HT>
__global__ __launch_bounds__(kNT) void k_poisson_p_f64(const double *__restrict__ rh, const double *__restrict__ poh,
                                                       double *__restrict__ pnh, int64_t mloc, int64_t m,
                                                       int64_t nstrips, int64_t rpi, ItemRanges ir, const double *rr,
                                                       const double *rsold, int first, ConvArgs cv, double *dot_out,
                                                       int add_to_out, double *partials, unsigned *ticket) {
    static_assert(RB <= kEdgeRB, "edge buffer");
    __shared__ double edge[2 * kWaves * 2 * kEdgeRB];
    if (cv.kdone) {
        if (*cv.kdone != 0) return;
        if (!first && cv.eps >= 0.0 && sqrt(*rr) < cv.eps) {  // the same decision in every block
            if (blockIdx.x == 0 && threadIdx.x == 0) record_convergence(cv, cv.k, *rr);
            return;
        }
    }
    // p_0 = r_0 (first) has its own instantiation: no p_{k-1} loads
    const double acc = first ? poisson_p_body<RB, NT, true, HT>(rh, poh, pnh, mloc, m, nstrips, rpi, ir, 0.0, edge)
                             : poisson_p_body<RB, NT, false, HT>(rh, poh, pnh, mloc, m, nstrips, rpi, ir,
                                                                 *rr / *rsold, edge);
    grid_sum_last_block(acc, partials, ticket, dot_out, add_to_out != 0);
}

// k_poisson_xr_f64 (iteration k): alpha = *rsold / *pAp; x += alpha p_k and
// r -= alpha A p_k with A p_k recomputed from p_k (halo included);
// *rr_out = r.r.  Skipped once *gate != 0.
template <int RBn, bool NT, bool HT>
__device__ __forceinline__ void poisson_xr_step(const double *__restrict__ pnh, double *__restrict__ x,
                                                double *__restrict__ r, int64_t m, int64_t i, const StripLane &L,
                                                double alpha, d2 &pm, d2 &pc, double &acc, double *eb) {
    const int lane = threadIdx.x & 63;
    d2 pr[RBn], xv[RBn], rv[RBn], ce[RBn];
    double el[RBn], er[RBn];
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const int64_t hc = (i + t + 1) * m, ic = (i + t) * m;
        pr[t] = keep(L.valid, (HT && t >= RBn - 2) ? lds2<false>(pnh + hc + m, L.off) : lds2<NT>(pnh + hc + m, L.off));
        xv[t] = lds2<NT>(x + ic, L.off);
        rv[t] = lds2<NT>(r + ic, L.off);
        el[t] = L.has_l ? pnh[hc + L.jw - 1] : 0.0;
        er[t] = L.has_r ? pnh[hc + L.jw + 128] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < RBn; ++t) ce[t] = t == 0 ? pc : pr[t - 1];
    edges_put<RBn>(eb, L, ce);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const d2 up = t == 0 ? pm : (t == 1 ? pc : pr[t - 2]);
        const d2 dn = pr[t];
        const double lw = edge_l(eb, L, t, el[t]), rw = edge_r(eb, L, t, er[t]);
        double l = __shfl_up(ce[t].y, 1, 64);
        double rt = __shfl_down(ce[t].x, 1, 64);
        l = lane == 0 ? lw : l;
        rt = lane == 63 ? rw : rt;
        d2 o;
        o.x = 4.0 * ce[t].x - up.x - dn.x - l - ce[t].y;
        o.y = 4.0 * ce[t].y - up.y - dn.y - ce[t].x - rt;
        d2 xn, rn;
        xn.x = __builtin_fma(alpha, ce[t].x, xv[t].x);
        xn.y = __builtin_fma(alpha, ce[t].y, xv[t].y);
        rn.x = __builtin_fma(-alpha, o.x, rv[t].x);
        rn.y = __builtin_fma(-alpha, o.y, rv[t].y);
        acc += L.valid ? rn.x * rn.x + rn.y * rn.y : 0.0;
        if (L.valid) {
            sts2<NT>(x + (i + t) * m, L.off, xn);
            sts2<NT>(r + (i + t) * m, L.off, rn);
        }
    }
    if constexpr (RBn >= 2) {
        pm = pr[RBn - 2];
        pc = pr[RBn - 1];
    } else {
        pm = pc;
        pc = pr[0];
    }
}

template <int RB, bool NT, bool HT>
__global__ __launch_bounds__(kNT) void k_poisson_xr_f64(const double *__restrict__ pnh, double *__restrict__ x,
                                                        double *__restrict__ r, int64_t mloc, int64_t m,
                                                        int64_t nstrips, int64_t rpi, int64_t nitems, int reverse,
                                                        const double *rsold, const double *pAp, double *rr_out,
                                                        double *partials, unsigned *ticket, const int64_t *gate) {
    static_assert(RB <= kEdgeRB, "edge buffer");
    __shared__ double edge[2 * kWaves * 2 * kEdgeRB];
    if (gate && *gate) return;
    const double alpha = *rsold / *pAp;
    double acc = 0.0;
    int par = 0;
    for (int64_t v = blockIdx.x; v < nitems; v += gridDim.x) {
        // reverse: walk the slab from its end, where the previous kernel
        // (k_poisson_p, forward) last wrote p_k, so the first bytes read may
        // still sit in the 256 MB MALL
        const int64_t w = reverse ? nitems - 1 - v : v;
        const StripLane L = strip_lane(w, nstrips, m);
        const int64_t i0 = (w / nstrips) * rpi;
        const int64_t i1 = (i0 + rpi < mloc) ? i0 + rpi : mloc;
        d2 pm = keep(L.valid, lds2<NT && !HT>(pnh + i0 * m, L.off));
        d2 pc = keep(L.valid, lds2<NT && !HT>(pnh + (i0 + 1) * m, L.off));
        int64_t i = i0;
        for (; i + RB <= i1; i += RB, par ^= 1)
            poisson_xr_step<RB, NT, HT>(pnh, x, r, m, i, L, alpha, pm, pc, acc, edge + par * (kWaves * 2 * kEdgeRB));
        for (; i < i1; ++i, par ^= 1)
            poisson_xr_step<1, NT, HT>(pnh, x, r, m, i, L, alpha, pm, pc, acc, edge + par * (kWaves * 2 * kEdgeRB));
    }
    grid_sum_last_block(acc, partials, ticket, rr_out);
}

__global__ __launch_bounds__(kNT) void k_stencil5_rows_f64(const double *__restrict__ ph, int64_t mloc, int64_t m,
                                                           double *__restrict__ Ap, double *dot_out, double *partials,
                                                           unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;
    const int64_t rows_per_block = (mloc + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t i1 = (i0 + rows_per_block < mloc) ? i0 + rows_per_block : mloc;
    double acc = 0.0;
    for (int64_t i = i0; i < i1; ++i) {
        const double *up = ph + i * m, *ce = up + m, *dn = ce + m;
        double *out = Ap + i * m;
        for (int64_t j = threadIdx.x; j < m; j += kNT) {
            const double c = ce[j];
            const double o = 4.0 * c - up[j] - dn[j] - ((j > 0) ? ce[j - 1] : 0.0) - ((j + 1 < m) ? ce[j + 1] : 0.0);
            out[j] = o;
            if (dot_out) acc += c * o;
        }
    }
    if (dot_out) grid_sum_last_block(acc, partials, ticket, dot_out);
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_fill(T *p, int64_t n, T v) {
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) p[i] = v;
}

template <typename T>
__global__ void k_sum_ordered(const T *in, int cnt, int stride, T *out) {
#pragma clang fp contract(off)
    T s = in[0];
    for (int q = 1; q < cnt; ++q) s = s + in[q * stride];
    *out = s;
}

// ---------------------------------------------------------------------------
// fp32 kernels in serialConjugate.c's exact operation order (CGX_F32_REF)
// ---------------------------------------------------------------------------
// matVec: one lane per row, columns in ascending order, out = ((0 + a0 v0) + a1 v1) + ...
// A 64x64 tile is staged through LDS so the global reads stay coalesced.
// One lane per row keeps the reference's order: out[i] = ((0 + a_i0 v_0) +
// a_i1 v_1) + ..., every product and sum rounded to float.  A wave owns 64
// rows and walks 64 x 128 tiles: the next tile is loaded into registers
// (32 float4 loads per lane, coalesced 512-B row pieces, all issued at once)
// while the current one is consumed from LDS, then written to the other LDS
// buffer (row stride 129 floats: conflict-free when lane t walks row t).
constexpr int kRefTC = 128;  // tile columns
__global__ __launch_bounds__(64) void k_matvec_ref_f32(const float *__restrict__ A, int64_t lda,
                                                       int64_t rows, int64_t cols,
                                                       const float *__restrict__ v,
                                                       float *__restrict__ out) {
#pragma clang fp contract(off)
    __shared__ float tile[2][64][kRefTC + 1];
    __shared__ float pv[2][kRefTC];
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * 64;
    const int q = t & 31;          // column quad of this lane within a tile row
    const int rsub = t >> 5;       // 0/1: which of two rows this lane loads per step
    const bool vec_ok = (lda & 3) == 0 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    const int64_t ntiles = (cols + kRefTC - 1) / kRefTC;
    f4 nx[32];
    float pn[2];
    auto load_tile = [&](int64_t c0) {
        const int w = (cols - c0 < kRefTC) ? (int)(cols - c0) : kRefTC;
        if (vec_ok && row0 + 64 <= rows && w == kRefTC) {  // whole tile: 32 unconditional 16-B loads
            const float *base = A + (row0 + rsub) * lda + c0 + 4 * q;
#pragma unroll
            for (int k = 0; k < 32; ++k) nx[k] = *reinterpret_cast<const f4 *>(base + (int64_t)(2 * k) * lda);
            pn[0] = v[c0 + t];
            pn[1] = v[c0 + t + 64];
            return;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const int64_t rr = row0 + 2 * k + rsub;
            const int c = 4 * q;
            f4 val = (f4)(0.0f);
            if (rr < rows) {
                if (vec_ok && c + 4 <= w) {
                    val = *reinterpret_cast<const f4 *>(A + rr * lda + c0 + c);
                } else {
                    for (int e = 0; e < 4; ++e)
                        if (c + e < w) val[e] = A[rr * lda + c0 + c + e];
                }
            }
            nx[k] = val;
        }
        pn[0] = (t < w) ? v[c0 + t] : 0.0f;
        pn[1] = (t + 64 < w) ? v[c0 + t + 64] : 0.0f;
    };
    auto store_tile = [&](int b) {
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            float *dst = &tile[b][2 * k + rsub][4 * q];
            dst[0] = nx[k][0];
            dst[1] = nx[k][1];
            dst[2] = nx[k][2];
            dst[3] = nx[k][3];
        }
        pv[b][t] = pn[0];
        pv[b][t + 64] = pn[1];
    };
    float acc = 0.0f;
    if (ntiles > 0) {
        load_tile(0);
        store_tile(0);
        __syncthreads();
    }
    for (int64_t tt = 0; tt < ntiles; ++tt) {
        const int b = (int)(tt & 1);
        const int64_t c0 = tt * kRefTC;
        const int w = (cols - c0 < kRefTC) ? (int)(cols - c0) : kRefTC;
        if (tt + 1 < ntiles) load_tile(c0 + kRefTC);  // in flight during the chain below
        if (w == kRefTC) {
#pragma unroll 16
            for (int j = 0; j < kRefTC; ++j) {
                const float prod = tile[b][t][j] * pv[b][j];
                acc = acc + prod;
            }
        } else {
            for (int j = 0; j < w; ++j) {
                const float prod = tile[b][t][j] * pv[b][j];
                acc = acc + prod;
            }
        }
        if (tt + 1 < ntiles) store_tile(b ^ 1);
        __syncthreads();
    }
    if (row0 + t < rows) out[row0 + t] = acc;
}

// The same float arithmetic with more of the chip in flight.  k_matvec_ref_f32
// above has every row of the system progressing through the columns at the
// same pace, so the bytes in flight chip-wide are rows x 128 columns x 4 B
// (4 MiB at N=8192, about 2 TB/s at HBM latency) on 128 waves.  Here a wave
// owns 16 rows and walks 16 x 512 tiles: all 64 lanes load the next tile
// (32 coalesced 16-B loads each, 32 KiB per wave, 16 MiB chip-wide at
// N=8192) while lanes 0-15 run their rows' sequential sums over the current
// one.  The products A[i][j] * x[j] (each rounded to float, as
// serialConjugate.c:117 forms them) are made by all 64 lanes when a tile is
// stored, so a row's chain is one LDS read per 4 columns and 4 dependent
// adds.  Rows are padded to 516 floats: 16-B aligned, and lanes 0-15 reading
// columns 4j..4j+3 hit banks 4*lane + 4j .. +3, all distinct.
// Measured at N=8192: 62 us per matVec (the 64-row kernel: 166 us); an
// 8-row x 1024-column variant (32 MiB in flight) measured 64 us.
constexpr int kRef2Rows = 16, kRef2TC = 512, kRef2Ld = kRef2TC + 4;
__global__ __launch_bounds__(64) void k_matvec_ref_f32_r16(const float *__restrict__ A, int64_t lda,
                                                           int64_t rows, int64_t cols,
                                                           const float *__restrict__ v,
                                                           float *__restrict__ out) {
#pragma clang fp contract(off)
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int kLd4 = kRef2Ld / 4, kTC4 = kRef2TC / 4;  // f4 per padded row / per tile row
    constexpr int kK = kRef2Rows * kTC4 / 64;              // f4 loads per lane per tile (32)
    static_assert(kTC4 == 128, "lane t's A loads cover columns 4*((k&1)*64+t): pn[k&1]");
    __shared__ f4 prod[2][kRef2Rows * kLd4];
    const int t = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * kRef2Rows;
    const bool vec_ok = (lda & 3) == 0 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0) &&
                        ((reinterpret_cast<uintptr_t>(v) & 15) == 0);
    const int64_t ntiles = (cols + kRef2TC - 1) / kRef2TC;
    f4 nx[kK];
    f4 pn[2];
    // A[row0 + r][c0 + 4*c4 ..] for idx = k*64 + t, r = idx / 128, c4 = idx % 128 = (k&1)*64 + t
    auto load_tile = [&](int64_t c0) {
        const int w = (cols - c0 < kRef2TC) ? (int)(cols - c0) : kRef2TC;
        if (vec_ok && row0 + kRef2Rows <= rows && w == kRef2TC) {  // whole tile: unconditional 16-B loads
#pragma unroll
            for (int k = 0; k < kK; ++k)
                nx[k] = __builtin_nontemporal_load(
                    reinterpret_cast<const f4 *>(A + (row0 + (k >> 1)) * lda + c0 + 4 * ((k & 1) * 64 + t)));
#pragma unroll
            for (int u = 0; u < 2; ++u) pn[u] = *reinterpret_cast<const f4 *>(v + c0 + 4 * (u * 64 + t));
            return;
        }
#pragma unroll
        for (int k = 0; k < kK; ++k) {
            const int c = 4 * ((k & 1) * 64 + t);
            const int64_t rr = row0 + (k >> 1);
            f4 val = (f4)(0.0f);
            if (rr < rows)
                for (int e = 0; e < 4; ++e)
                    if (c + e < w) val[e] = A[rr * lda + c0 + c + e];
            nx[k] = val;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = 4 * (u * 64 + t);
            f4 val = (f4)(0.0f);
            for (int e = 0; e < 4; ++e)
                if (c + e < w) val[e] = v[c0 + c + e];
            pn[u] = val;
        }
    };
    auto store_tile = [&](int b) {
#pragma unroll
        for (int k = 0; k < kK; ++k) prod[b][(k >> 1) * kLd4 + (k & 1) * 64 + t] = nx[k] * pn[k & 1];
    };
    float acc = 0.0f;  // matvec[i] = 0.0  (serialConjugate.c:114)
    if (ntiles > 0) {
        load_tile(0);
        store_tile(0);
        __syncthreads();
    }
    for (int64_t tt = 0; tt < ntiles; ++tt) {
        const int b = (int)(tt & 1);
        const int64_t c0 = tt * kRef2TC;
        const int w = (cols - c0 < kRef2TC) ? (int)(cols - c0) : kRef2TC;
        if (tt + 1 < ntiles) load_tile(c0 + kRef2TC);  // in flight during the sums below
        if (t < kRef2Rows) {  // matvec[i] += A[i][j] * x[j], j ascending (:117)
            const f4 *trow = &prod[b][t * kLd4];
            if (w == kRef2TC) {
                constexpr int G = 8;  // LDS reads of the next G quads in flight while adding these
                f4 q[G], qn[G];
#pragma unroll
                for (int u = 0; u < G; ++u) q[u] = trow[u];
                for (int j4 = 0; j4 < kTC4; j4 += G) {
                    if (j4 + G < kTC4) {
#pragma unroll
                        for (int u = 0; u < G; ++u) qn[u] = trow[j4 + G + u];
                    }
#pragma unroll
                    for (int u = 0; u < G; ++u) {
                        acc = acc + q[u].x;
                        acc = acc + q[u].y;
                        acc = acc + q[u].z;
                        acc = acc + q[u].w;
                    }
#pragma unroll
                    for (int u = 0; u < G; ++u) q[u] = qn[u];
                }
            } else {
                const float *tf = reinterpret_cast<const float *>(trow);
                for (int j = 0; j < w; ++j) acc = acc + tf[j];
            }
        }
        if (tt + 1 < ntiles) store_tile(b ^ 1);
        __syncthreads();
    }
    if (t < kRef2Rows && row0 + t < rows) out[row0 + t] = acc;
}

// vecVec: one wave; products in parallel, the sum strictly sequential in
// index order (s = s + a_i b_i), broadcast lane by lane with v_readlane.
__global__ __launch_bounds__(64) void k_dot_ref_f32(int64_t n, const float *__restrict__ a,
                                                    const float *__restrict__ b, float *out) {
#pragma clang fp contract(off)
    // One wave.  The products of 8 chunks of 64 (each rounded to float, as
    // serialConjugate.c:150 forms them) go to LDS; then every lane walks them
    // in index order with 16-B broadcast reads and adds them one by one, the
    // reference's single sequential sum (all lanes hold the same s).
    constexpr int B = 8;
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ f4 sp[B * 64 / 4];
    float *spf = reinterpret_cast<float *>(sp);
    const int lane = threadIdx.x;
    float s = 0.0f;
    for (int64_t c0 = 0; c0 < n; c0 += 64 * B) {
        float pr[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int64_t i = c0 + u * 64 + lane;
            pr[u] = i < n ? a[i] * b[i] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < B; ++u) spf[u * 64 + lane] = pr[u];
        __syncthreads();
        const int64_t left = n - c0;
        if (left >= 64 * B) {
#pragma unroll 8
            for (int q = 0; q < B * 16; ++q) {
                const f4 v = sp[q];
                s = s + v.x;
                s = s + v.y;
                s = s + v.z;
                s = s + v.w;
            }
        } else {
            for (int i = 0; i < (int)left; ++i) s = s + spf[i];
        }
        __syncthreads();
    }
    if (lane == 0) *out = s;
}

// The same single sequential sum with its loads off the chain: 4 waves load
// the next 4096-element chunk (raw a and b, 16 of each per thread) while wave
// 0 adds up the current chunk's products from LDS; the products are formed
// (rounded to float, serialConjugate.c:150) when the chunk is stored.
constexpr int kDotChunk = 4096;
__global__ __launch_bounds__(256) void k_dot_ref_f32_blk(int64_t n, const float *__restrict__ a,
                                                         const float *__restrict__ b, float *out) {
#pragma clang fp contract(off)
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int U = kDotChunk / 256;
    __shared__ f4 sp[2][kDotChunk / 4];
    const int t = threadIdx.x;
    float av[U], bv[U];
    auto load = [&](int64_t c0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = c0 + u * 256 + t;
            av[u] = i < n ? a[i] : 0.0f;
            bv[u] = i < n ? b[i] : 0.0f;
        }
    };
    auto store = [&](int buf) {
        float *spf = reinterpret_cast<float *>(sp[buf]);
#pragma unroll
        for (int u = 0; u < U; ++u) spf[u * 256 + t] = av[u] * bv[u];
    };
    const int64_t nch = (n + kDotChunk - 1) / kDotChunk;
    float s = 0.0f;  // sum = 0.0  (:149)
    if (nch > 0) {
        load(0);
        store(0);
        __syncthreads();
    }
    for (int64_t ch = 0; ch < nch; ++ch) {
        const int buf = (int)(ch & 1);
        if (ch + 1 < nch) load((ch + 1) * kDotChunk);
        if (t < 64) {  // wave 0: sum += v1[i] * v2[i], i ascending (:152)
            const int64_t left = n - ch * kDotChunk;
            if (left >= kDotChunk) {
#pragma unroll 8
                for (int q = 0; q < kDotChunk / 4; ++q) {
                    const f4 v = sp[buf][q];
                    s = s + v.x;
                    s = s + v.y;
                    s = s + v.z;
                    s = s + v.w;
                }
            } else {
                const float *spf = reinterpret_cast<const float *>(sp[buf]);
                for (int i = 0; i < (int)left; ++i) s = s + spf[i];
            }
        }
        if (ch + 1 < nch) store(buf ^ 1);
        __syncthreads();
    }
    if (t == 0) *out = s;
}

// residual(r) and residual(p): r = b - Ax; p = b - Ax  (serialConjugate.c:210-211)
__global__ __launch_bounds__(kNT) void k_residual_ref_f32(int64_t n, const float *__restrict__ b,
                                                          const float *__restrict__ Ax,
                                                          float *__restrict__ r, float *__restrict__ p) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
        r[i] = b[i] - Ax[i];
        if (p) p[i] = b[i] - Ax[i];
    }
}

// alpha = rsold / pAp (:220); x = x + p*alpha (:221,225); r = r - Ap*alpha (:226,230)
__global__ __launch_bounds__(kNT) void k_update_xr_ref_f32(int64_t n, float *__restrict__ x,
                                                           float *__restrict__ r,
                                                           const float *__restrict__ p,
                                                           const float *__restrict__ Ap,
                                                           const float *rsold, const float *pAp) {
#pragma clang fp contract(off)
    const float alpha = *rsold / *pAp;
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
        const float tx = p[i] * alpha;
        x[i] = x[i] + tx;
        const float tr = Ap[i] * alpha;
        r[i] = r[i] - tr;
    }
}

// p = r + p*(beta/rsold)  (:239,243)
__global__ __launch_bounds__(kNT) void k_update_p_ref_f32(int64_t n, float *__restrict__ p,
                                                          const float *__restrict__ r,
                                                          const float *rr, const float *rsold) {
#pragma clang fp contract(off)
    const float ratio = *rr / *rsold;
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
        const float t = p[i] * ratio;
        p[i] = r[i] + t;
    }
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
struct DevInfo {
    int cus = 0;
};
std::mutex g_mu;
DevInfo g_dev[64];

int cu_count(int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (device < 0 || device >= 64) return 256;
    if (g_dev[device].cus == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0)
            v = 256;
        g_dev[device].cus = v;
    }
    return g_dev[device].cus;
}

// ---------------------------------------------------------------------------
// CGX_SYMMETRIC: A stored as the upper triangle of 128 x 128 tiles (CG's
// matrix is symmetric by contract; the generator's is exactly), so a matVec
// reads N^2/2 doubles instead of N^2.
//
// Layout: tile (I, J), J >= I, at index sym_off(I) + J - I (row-major over
// the upper triangle); a diagonal tile is stored whole.  Inside a tile the
// doubles are in the order the 512-thread block loads them: d2 number
// k * 512 + t holds (row, col) = (8 tr + rr, 4 tc + 2 cc + {0, 1}) with
// t = 32 tr + tc, k = 2 rr + cc, so every load step reads 8 KiB contiguous.
// (kSymNT = 1024, 4 rows per thread, measured 6-7 % slower.)
//
// k_symv_f64: a block streams a contiguous range of `per` tiles (the next
// tile's loads in flight during the current one's arithmetic).  Per tile
// (I, J), off the diagonal, it writes the 128 column partials A_IJ^T p_I to
// pcol[tile]; the row partials A_IJ p_J are summed over the block's run of
// tiles in tile row I and written once per run, at prow[first tile of the
// run] (a run starts at sym_off(I) or at a multiple of `per`).
// k_symv_reduce_f64 sums row i's run partials and column partials in a fixed
// order, so the result is deterministic, and fuses p.Ap.
// ---------------------------------------------------------------------------
constexpr int kSymT = 128, kSymNT = 512;
constexpr int kSymRPT = kSymT * kSymT / (4 * kSymNT);  // rows per thread (4 columns each)
constexpr int kSymK = 2 * kSymRPT;                      // d2 loads per thread per tile
constexpr int kSymTR = kSymT / kSymRPT;                 // thread rows per tile (32)
constexpr int64_t kSymTileD2 = kSymT * kSymT / 2;
static_assert((kSymRPT == 8 || kSymRPT == 4) && kSymNT / kSymTR == 32, "row reduction: 8 or 4 rows x 32 lanes");
static_assert(kSymNT == 512 && kSymRPT == 8, "sym_pos_h (cgx_kernels.h) assumes 512 threads, 8 rows per thread");

__host__ __device__ __forceinline__ int64_t sym_off(int64_t I, int64_t nt) { return I * nt - I * (I - 1) / 2; }

__device__ __forceinline__ void sym_tile_ij(int64_t q, int64_t nt, int64_t &I, int64_t &J) {
    int64_t lo = 0, hi = nt - 1;  // the last tile row starting at or before q
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (sym_off(mid, nt) <= q) lo = mid;
        else hi = mid - 1;
    }
    I = lo;
    J = lo + (q - sym_off(lo, nt));
}

// double offset of tile element (r, c) in the load order above
__host__ __device__ __forceinline__ int64_t sym_pos(int r, int c) {
    const int t = (r / kSymRPT) * 32 + (c >> 2), k = (r % kSymRPT) * 2 + ((c >> 1) & 1);
    return ((int64_t)k * kSymNT + t) * 2 + (c & 1);
}

// One tile's loads: its 16 d2 of A per thread and the p values it multiplies.
struct SymSlot {
    d2 a[kSymK], pj[2], pi[kSymRPT / 2];
    int64_t I, J;
};

// Buffer loads with wave-uniform bases (tile q, p): the only per-lane
// address is the loop-invariant t*16 (or tc/tr offsets), so no address
// registers are recomputed per tile -- recomputed ones landed in registers
// the slot loads had just written, and the compiler's wait for them drained
// the loads in flight at the top of every iteration.
// qa: the tile's index in At (At may hold a range of tiles starting at q_base).
template <int NTL>
__device__ __forceinline__ void sym_load(SymSlot &S, const double *At, __amdgpu_buffer_rsrc_t prs, int64_t qa,
                                         int64_t I, int64_t J, int t, int tr, int tc) {
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(At + qa * (int64_t)kSymT * kSymT), 0, kSymT * kSymT * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < kSymK; ++k)
        S.a[k] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(trs, t * 16, k * kSymNT * 16,
                                                                              NTL ? 2 : 0));
    const int jo = (int)(J * kSymT * 8), io = (int)(I * kSymT * 8);
#pragma unroll
    for (int u = 0; u < 2; ++u)
        S.pj[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(prs, tc * 32 + u * 16, jo, 0));
#pragma unroll
    for (int u = 0; u < kSymRPT / 2; ++u)
        S.pi[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(prs, tr * kSymRPT * 8 + u * 16, io, 0));
    S.I = I;
    S.J = J;
}

__device__ __forceinline__ void sym_next(int64_t &I, int64_t &J, int64_t nt) {
    if (++J == nt) J = ++I;
}

// Row partials A_IJ p_J (always) and column partials A_IJ^T p_I (J > I) of
// one tile; `buf` selects the LDS half for the column sums (flipped per use).
// racc: this lane's running row sum over the current run; end_of_run: the
// next tile is in another tile row (or there is none), so write it.
__device__ __forceinline__ void sym_tile(const SymSlot &S, int64_t q, double (*cs)[kSymTR][kSymT], int &buf,
                                         double *__restrict__ prow, double *__restrict__ pcol, int t, int tr, int tc,
                                         double &racc, int64_t &qrun, bool end_of_run) {
    // row partials over this thread's 4 columns, then over the 32 lanes of
    // its thread-row group: a halving exchange (the lane pairs 16, 8, (4)
    // apart swap half their rows) until one row per lane, then the rest
    double rs[kSymRPT];
#pragma unroll
    for (int rr = 0; rr < kSymRPT; ++rr) {
        double v = S.a[2 * rr].x * S.pj[0].x;
        v = __builtin_fma(S.a[2 * rr].y, S.pj[0].y, v);
        v = __builtin_fma(S.a[2 * rr + 1].x, S.pj[1].x, v);
        rs[rr] = __builtin_fma(S.a[2 * rr + 1].y, S.pj[1].y, v);
    }
    int row = 0;  // which of the thread's rows the lane ends up holding
    double k1;
    {
        constexpr int H = kSymRPT / 2;
        const bool h = tc & 16;
        double k[H];
#pragma unroll
        for (int u = 0; u < H; ++u) k[u] = (h ? rs[u + H] : rs[u]) + __shfl_xor(h ? rs[u] : rs[u + H], 16, 64);
        row += h ? H : 0;
        const bool h2 = tc & 8;
        double m[H / 2];
#pragma unroll
        for (int u = 0; u < H / 2; ++u) m[u] = (h2 ? k[u + H / 2] : k[u]) + __shfl_xor(h2 ? k[u] : k[u + H / 2], 8, 64);
        row += h2 ? H / 2 : 0;
        if constexpr (kSymRPT == 8) {
            const bool h3 = tc & 4;
            k1 = (h3 ? m[1] : m[0]) + __shfl_xor(h3 ? m[0] : m[1], 4, 64);
            row += h3 ? 1 : 0;
        } else {
            k1 = m[0] + __shfl_xor(m[0], 4, 64);
        }
    }
    k1 += __shfl_xor(k1, 2, 64);
    k1 += __shfl_xor(k1, 1, 64);
    racc += k1;
    if (end_of_run) {
        if ((tc & (32 / kSymRPT - 1)) == 0) prow[qrun * kSymT + tr * kSymRPT + row] = racc;
        racc = 0.0;
        qrun = q + 1;
    }
    if (S.J > S.I) {  // column partials A_IJ^T p_I (the diagonal tile has none)
        double c[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int rr = 0; rr < kSymRPT; ++rr) {
            const double pr = (rr & 1) ? S.pi[rr >> 1].y : S.pi[rr >> 1].x;
            c[0] = __builtin_fma(S.a[2 * rr].x, pr, c[0]);
            c[1] = __builtin_fma(S.a[2 * rr].y, pr, c[1]);
            c[2] = __builtin_fma(S.a[2 * rr + 1].x, pr, c[2]);
            c[3] = __builtin_fma(S.a[2 * rr + 1].y, pr, c[3]);
        }
        *reinterpret_cast<d2 *>(&cs[buf][tr][tc * 4]) = d2{c[0], c[1]};
        *reinterpret_cast<d2 *>(&cs[buf][tr][tc * 4 + 2]) = d2{c[2], c[3]};
        // LDS-only barrier: __syncthreads()' fence would also wait vmcnt(0)
        // (stores and loads share the counter on gfx9), draining the next
        // tile's loads that are in flight across this point
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (t < kSymT) {
            double sum = cs[buf][0][t];
#pragma unroll
            for (int g = 1; g < kSymTR; ++g) sum += cs[buf][g][t];
            pcol[q * kSymT + t] = sum;
        }
        buf ^= 1;
    }
}

// Two slots alternate: the loads of tile q+1 go out before tile q's
// arithmetic.  Measured against a one-slot loop that copies the prefetched
// slot in (the wait lands at the copy) and against __syncthreads(): all
// within 1 % (tools/sym_ab.py).
template <int NTL>
// Tiles [q_base, q_base + count) of the triangle, At holding exactly those
// (a streamed chunk) or all of them (q_base = 0).  tile_runs: every tile is
// its own run (its row partials written per tile): chunk boundaries then do
// not matter to the reduce, which is told per = 1.
__global__ __launch_bounds__(kSymNT) void k_symv_f64(const double *__restrict__ At, int64_t nt, int64_t q_base,
                                                     int64_t count, int64_t per, int tile_runs,
                                                     const double *__restrict__ p, double *__restrict__ prow,
                                                     double *__restrict__ pcol, const int64_t *gate) {
    if (gate && *gate) return;
    __shared__ double cs[2][kSymTR][kSymT];
    const int t = threadIdx.x, tr = t >> 5, tc = t & 31;
    const int64_t q0 = q_base + (int64_t)blockIdx.x * per;
    const int64_t q1 = (q0 + per < q_base + count) ? q0 + per : q_base + count;
    if (q0 >= q1) return;
    int64_t Ic, Jc;  // tile q
    sym_tile_ij(q0, nt, Ic, Jc);
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(nt * kSymT * 8), 0x00020000);
    int buf = 0;
    double racc = 0.0;
    int64_t qrun = q0;
    SymSlot S0, S1;
    sym_load<NTL>(S0, At, prs, q0 - q_base, Ic, Jc, t, tr, tc);
    // Every load is issued unconditionally (past the range end a slot
    // reloads the last tile): with a conditional load block the compiler's
    // wait counts at the merge assume no newer loads and drain the next
    // tile's loads before the current tile is used.
    for (int64_t q = q0; q < q1; q += 2) {
        int64_t I1 = Ic, J1 = Jc;
        sym_next(I1, J1, nt);
        const bool va = q + 1 < q1;
        sym_load<NTL>(S1, At, prs, (va ? q + 1 : q) - q_base, va ? I1 : Ic, va ? J1 : Jc, t, tr, tc);
        __builtin_amdgcn_sched_barrier(0);  // the loads go out before this tile's arithmetic
        if (tile_runs) qrun = q;
        sym_tile(S0, q, cs, buf, prow, pcol, t, tr, tc, racc, qrun, tile_runs || !va || I1 != Ic);
        if (!va) break;
        int64_t I2 = I1, J2 = J1;
        sym_next(I2, J2, nt);
        const bool vb = q + 2 < q1;
        sym_load<NTL>(S0, At, prs, (vb ? q + 2 : q + 1) - q_base, vb ? I2 : I1, vb ? J2 : J1, t, tr, tc);
        __builtin_amdgcn_sched_barrier(0);
        if (tile_runs) qrun = q + 1;
        sym_tile(S1, q + 1, cs, buf, prow, pcol, t, tr, tc, racc, qrun, tile_runs || !vb || I2 != I1);
        Ic = I2;
        Jc = J2;
    }
}

// y_i = sum over the runs of tile row I of prow[run][i % 128]
//     + sum_{I' < I} pcol[(I', I)][i % 128], rows [0, n);
// *dot_out = pown . y when pown != nullptr.  A block owns 64 consecutive
// rows (one lane each, so every partial read is 512 B contiguous); its 4
// waves take every 4th entry of the rows' list (runs, then column partials),
// 8 loads in flight, and the 4 wave sums are added in wave order.
__global__ __launch_bounds__(kNT) void k_symv_reduce_f64(int64_t n, int64_t nt, int64_t per,
                                                         const double *__restrict__ prow,
                                                         const double *__restrict__ pcol, double *__restrict__ y,
                                                         const double *__restrict__ pown, double *dot_out,
                                                         double *partials, unsigned *ticket, const int64_t *gate) {
    if (gate && *gate) return;
    __shared__ double ws4[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double dacc = 0.0;
    for (int64_t g = blockIdx.x; g * 64 < n; g += gridDim.x) {
        const int64_t i = g * 64 + lane;
        const int64_t I = (g * 64) >> 7, o = i & (kSymT - 1);
        const int64_t first = sym_off(I, nt), last = sym_off(I + 1, nt) - 1;
        const int64_t k0 = first / per, R = 1 + last / per - k0;  // runs of tile row I
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int64_t j = w;
        for (; j < R; j += 4) acc[0] += prow[(j == 0 ? first : (k0 + j) * per) * kSymT + o];
        int64_t Ip = j - R;  // continue the stride into the column partials
        for (; Ip + 28 < I; Ip += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t c = Ip + 4 * u;
                acc[u] += pcol[(sym_off(c, nt) + I - c) * kSymT + o];
            }
        }
        for (; Ip < I; Ip += 4) acc[0] += pcol[(sym_off(Ip, nt) + I - Ip) * kSymT + o];
        ws4[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        __syncthreads();
        if (w == 0 && i < n) {
            const double yi = (ws4[0][lane] + ws4[1][lane]) + (ws4[2][lane] + ws4[3][lane]);
            y[i] = yi;
            if (pown) dacc += pown[i] * yi;
        }
        __syncthreads();
    }
    if (pown) grid_sum_last_block(dacc, partials, ticket, dot_out);
}

// Pack rows [row0, row0 + nrows) (row-major, leading dimension ld, n valid
// columns) into the tiles: row i supplies columns 128*(i/128) .. lda-1.
__global__ __launch_bounds__(kNT) void k_sym_pack_f64(const double *__restrict__ rows, int64_t ld, int64_t row0,
                                                      int64_t nrows, int64_t n, int64_t lda, int64_t nt,
                                                      double *__restrict__ At) {
    for (int64_t rr = blockIdx.x; rr < nrows; rr += gridDim.x) {
        const int64_t i = row0 + rr, I = i >> 7;
        const int r = (int)(i & (kSymT - 1));
        for (int64_t j = I * kSymT + threadIdx.x; j < lda; j += kNT) {
            const int64_t J = j >> 7;
            At[(sym_off(I, nt) + J - I) * (int64_t)kSymT * kSymT + sym_pos(r, (int)(j & (kSymT - 1)))] =
                j < n ? rows[rr * ld + j] : 0.0;
        }
    }
}

// The counter-hash SPD system (k_gen_spd's values) straight into the tiles.
// Tiles [q_base, q_base + count) into At (At[0] = tile q_base).
__global__ __launch_bounds__(kSymNT) void k_gen_spd_sym(int64_t n, int64_t nt, int64_t q_base, int64_t count,
                                                        uint64_t salt, double *__restrict__ At) {
#pragma clang fp contract(off)
    for (int64_t qi = blockIdx.x; qi < count; qi += gridDim.x) {
        int64_t I, J;
        sym_tile_ij(q_base + qi, nt, I, J);
        d2 *tile = reinterpret_cast<d2 *>(At) + qi * kSymTileD2;
        const int t = threadIdx.x, tr = t >> 5, tc = t & 31;
        for (int k = 0; k < kSymK; ++k) {
            const uint64_t i = (uint64_t)(I * kSymT + tr * kSymRPT + (k >> 1));
            d2 v;
            for (int e = 0; e < 2; ++e) {
                const uint64_t j = (uint64_t)(J * kSymT + tc * 4 + (k & 1) * 2 + e);
                double val = 0.0;
                if (i < (uint64_t)n && j < (uint64_t)n) {
                    val = 0.5 * (u01(salt, i, j) + u01(salt, j, i));
                    if (i == j) val = val + (double)n;
                }
                v[e] = val;
            }
            tile[k * kSymNT + t] = v;
        }
    }
}

__global__ __launch_bounds__(kNT) void k_gen_b(int64_t row0, int64_t nrows, uint64_t salt_b, double *b) {
    for (int64_t rr = (int64_t)blockIdx.x * kNT + threadIdx.x; rr < nrows; rr += (int64_t)gridDim.x * kNT) {
        const uint64_t h = mix64((uint64_t)(row0 + rr) ^ salt_b);
        b[rr] = (double)(h >> 11) * 0x1.0p-53;
    }
}

int env_int(const char *name, int dflt) {
    const char *s = std::getenv(name);
    return (s && *s) ? std::atoi(s) : dflt;
}

unsigned grid_1d(int64_t n, int per_block, unsigned cap) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (int64_t)cap) g = cap;
    return (unsigned)g;
}

// Grid of the vector kernels: <= kMaxRedBlocks (the partial slots), <= 8 blocks/CU.
unsigned grid_vec(int64_t n) { return grid_1d((n + 1) / 2, kNT * kVU, 2048); }

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

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

hipError_t residual_f64(int64_t n, const double *b, const double *Ax, double *r, double *p,
                        double *rr_out, const RedWs &ws, hipStream_t s) {
    const bool vec = al16(b) && al16(Ax) && al16(r) && al16(p);
    hipLaunchKernelGGL(vec ? k_residual_f64<true> : k_residual_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, b,
                       Ax, r, p, rr_out, ws.partials, ws.tickets + T_RESID);
    return hipGetLastError();
}

hipError_t update_xr_f64(int64_t n, double *x, double *r, const double *p, const double *Ap,
                         const double *rsold, const double *pAp, double *rr_out, const RedWs &ws,
                         hipStream_t s) {
    const bool vec = al16(x) && al16(r) && al16(p) && al16(Ap);
    const int vp = env_int("CGX_VEC_POLICY", 2);
    auto fn = !vec ? k_update_xr_f64<false> : vp == 1 ? k_update_xr_f64<true, 1>
                                            : vp == 2 ? k_update_xr_f64<true, 2> : k_update_xr_f64<true, 0>;
    hipLaunchKernelGGL(fn, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x, r, p, Ap, rsold, pAp, rr_out, ws.partials,
                       ws.tickets + T_XR);
    return hipGetLastError();
}

hipError_t update_p_f64(int64_t n, double *p, const double *r, const double *rr, const double *rsold,
                        hipStream_t s) {
    const bool vec = al16(p) && al16(r);
    const int vp = env_int("CGX_VEC_POLICY", 2);
    auto fn = !vec ? k_update_p_f64<false> : vp == 1 ? k_update_p_f64<true, 1>
                                           : vp == 2 ? k_update_p_f64<true, 2> : k_update_p_f64<true, 0>;
    hipLaunchKernelGGL(fn, dim3(grid_vec(n)), dim3(kNT), 0, s, n, p, r, rr, rsold);
    return hipGetLastError();
}

hipError_t update_r_f64(int64_t n, double *r, const double *Ap, const double *rsold, const double *pAp,
                        double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate) {
    const bool vec = al16(r) && al16(Ap);
    hipLaunchKernelGGL(vec ? k_update_r_f64<true> : k_update_r_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, r,
                       Ap, rsold, pAp, rr_out, ws.partials, ws.tickets + T_XR, gate);
    return hipGetLastError();
}

hipError_t update_xp_f64(int64_t n, double *x, double *p, const double *r, const double *rsold, const double *pAp,
                         const double *rr, hipStream_t s, double eps, int64_t k, int64_t *kdone, double *rrfinal,
                         int64_t *hrec) {
    const bool vec = al16(x) && al16(p) && al16(r);
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(vec ? k_update_xp_f64<true> : k_update_xp_f64<false>, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x,
                       p, r, rsold, pAp, rr, cv);
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

hipError_t stencil5_f64(const double *ph, int64_t mloc, int64_t m, double *Ap, double *dot_out, const RedWs &ws,
                        hipStream_t s, const int64_t *gate) {
    if (mloc <= 0) return hipSuccess;
    if ((m & 1) == 0 && al16(ph) && al16(Ap)) {
        const int64_t nstrips = (m + 2 * kNT - 1) / (2 * kNT);
        int64_t chunks = std::max<int64_t>(1, 2048 / nstrips);
        chunks = std::min<int64_t>(chunks, mloc);
        const int64_t rpb = (mloc + chunks - 1) / chunks;
        chunks = (mloc + rpb - 1) / rpb;
        int64_t grid = nstrips * chunks;
        if (grid > kMaxRedBlocks) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_stencil5_strip_f64, dim3((unsigned)grid), dim3(kNT), 0, s, ph, mloc, m, nstrips, rpb, Ap,
                           dot_out, ws.partials, ws.tickets + T_MATVEC, gate);
    } else {
        const unsigned grid = (unsigned)std::min<int64_t>(mloc, 2048);
        hipLaunchKernelGGL(k_stencil5_rows_f64, dim3(grid), dim3(kNT), 0, s, ph, mloc, m, Ap, dot_out, ws.partials,
                           ws.tickets + T_MATVEC, gate);
    }
    return hipGetLastError();
}

// Fused Poisson kernels: rows per step RB (CGX_STENCIL_RB: 1, 2, 4, 8), rows
// per work item (CGX_STENCIL_ROWS), resident blocks (CGX_STENCIL_BLOCKS), NT
// streams (CGX_STENCIL_NT=0: default-policy loads/stores).  Defaults RB=8,
// 8-row items, occupancy-sized grid: measured at m=8192 over RB 2..8, items
// of 8..128 rows and 1024..4096 blocks (profiles/r01_sweep_poisson*.jsonl);
// short items keep the rows in flight in a narrow band (64- and 128-row items
// are 7-20 % slower).
struct PoissonPlan {
    int rb, nt, ht;
    int64_t nstrips, rpi, nitems, grid;
};
static PoissonPlan poisson_plan(int64_t mloc, int64_t m) {
    PoissonPlan p;
    p.rb = env_int("CGX_STENCIL_RB", 8);
    p.nt = env_int("CGX_STENCIL_NT", 1);
    p.ht = env_int("CGX_STENCIL_HALO_T", 1);
    p.nstrips = (m + 2 * kNT - 1) / (2 * kNT);
    p.rpi = std::max(1, env_int("CGX_STENCIL_ROWS", 8));
    p.nitems = p.nstrips * ((mloc + p.rpi - 1) / p.rpi);
    p.grid = 0;  // set per kernel from its occupancy (resident_grid)
    return p;
}

// Every block resident at once (occupancy x CUs), capped by the work items
// and the reduction slots; CGX_STENCIL_BLOCKS overrides.
static int64_t resident_grid(const void *fn, int64_t nitems) {
    int dev = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    static std::mutex mu;
    static std::vector<std::pair<std::pair<const void *, int>, int>> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto &e : cache)
            if (e.first.first == fn && e.first.second == dev) per_cu = e.second;
        if (per_cu == 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, 0) != hipSuccess || per_cu <= 0)
                per_cu = 4;
            cache.push_back({{fn, dev}, per_cu});
        }
    }
    int64_t g = (int64_t)per_cu * cu_count(dev);
    g = env_int("CGX_STENCIL_BLOCKS", (int)g);
    return std::max<int64_t>(1, std::min<int64_t>({g, nitems, kMaxRedBlocks}));
}

bool poisson_fusable(int64_t mloc, int64_t m) { return mloc > 0 && m > 0 && (m & 1) == 0; }

template <int RB>
static void launch_poisson_p(const PoissonPlan &pl, hipStream_t s, const double *rh, const double *poh, double *pnh,
                             int64_t mloc, int64_t m, const double *rr, const double *rsold, int first, ConvArgs cv,
                             double *pap_out, const RedWs &ws, ItemRanges ir, int add_to_out) {
    auto fn = pl.nt ? (pl.ht ? k_poisson_p_f64<RB, true, true> : k_poisson_p_f64<RB, true, false>)
                    : k_poisson_p_f64<RB, false, false>;
    const int64_t grid = resident_grid(reinterpret_cast<const void *>(fn), ir.cnt1 + ir.cnt2);
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kNT), 0, s, rh, poh, pnh, mloc, m, pl.nstrips, pl.rpi, ir, rr,
                       rsold, first, cv, pap_out, add_to_out, ws.partials, ws.tickets + T_MATVEC);
}
template <int RB>
static void launch_poisson_xr(const PoissonPlan &pl, hipStream_t s, const double *pnh, double *x, double *r,
                              int64_t mloc, int64_t m, const double *rsold, const double *pAp, double *rr_out,
                              const RedWs &ws, const int64_t *gate) {
    auto fn = pl.nt ? (pl.ht ? k_poisson_xr_f64<RB, true, true> : k_poisson_xr_f64<RB, true, false>)
                    : k_poisson_xr_f64<RB, false, false>;
    const int64_t grid = resident_grid(reinterpret_cast<const void *>(fn), pl.nitems);
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kNT), 0, s, pnh, x, r, mloc, m, pl.nstrips, pl.rpi,
                       pl.nitems, env_int("CGX_STENCIL_REVERSE", 1), rsold, pAp, rr_out, ws.partials,
                       ws.tickets + T_XR, gate);
}

hipError_t poisson_p_f64(const double *rh, const double *poh, double *pnh, int64_t mloc, int64_t m, const double *rr,
                         const double *rsold, bool first, double *pap_out, const RedWs &ws, hipStream_t s, double eps,
                         int64_t k, int64_t *kdone, double *rrfinal, int part, int64_t *hrec) {
    if (!poisson_fusable(mloc, m) || !al16(rh) || !al16(pnh) || (!first && !al16(poh))) return hipErrorInvalidValue;
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    const PoissonPlan pl = poisson_plan(mloc, m);
    const int64_t nruns = pl.nitems / pl.nstrips, ns = pl.nstrips;
    // part 0: every item; 1: runs 1..nruns-2 (no halo row read); 2: runs 0 and
    // nruns-1, adding to part 1's p.Ap when part 1 had items
    ItemRanges ir{0, pl.nitems, 0, 0};
    int add = 0;
    if (part == 1) {
        if (nruns <= 2) return hipSuccess;
        ir = ItemRanges{ns, (nruns - 2) * ns, 0, 0};
    } else if (part == 2) {
        ir = ItemRanges{0, ns, (nruns - 1) * ns, nruns > 1 ? ns : 0};
        add = nruns > 2;
    }
    switch (pl.rb) {
        case 1: launch_poisson_p<1>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add); break;
        case 2: launch_poisson_p<2>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add); break;
        case 8: launch_poisson_p<8>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add); break;
        default: launch_poisson_p<4>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add); break;
    }
    return hipGetLastError();
}

hipError_t poisson_xr_f64(const double *pnh, double *x, double *r, int64_t mloc, int64_t m, const double *rsold,
                          const double *pAp, double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate) {
    if (!poisson_fusable(mloc, m) || !al16(pnh) || !al16(x) || !al16(r)) return hipErrorInvalidValue;
    const PoissonPlan pl = poisson_plan(mloc, m);
    switch (pl.rb) {
        case 1: launch_poisson_xr<1>(pl, s, pnh, x, r, mloc, m, rsold, pAp, rr_out, ws, gate); break;
        case 2: launch_poisson_xr<2>(pl, s, pnh, x, r, mloc, m, rsold, pAp, rr_out, ws, gate); break;
        case 8: launch_poisson_xr<8>(pl, s, pnh, x, r, mloc, m, rsold, pAp, rr_out, ws, gate); break;
        default: launch_poisson_xr<4>(pl, s, pnh, x, r, mloc, m, rsold, pAp, rr_out, ws, gate); break;
    }
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
    hipLaunchKernelGGL(k_sum_ordered<double>, dim3(1), dim3(1), 0, s, in, cnt, 1, out);
    return hipGetLastError();
}

hipError_t sum_ordered_f32(const float *in, int cnt, float *out, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_ordered<float>, dim3(1), dim3(1), 0, s, in, cnt, 2, out);
    return hipGetLastError();
}

hipError_t matvec_ref_f32(const float *A, int64_t lda, int64_t rows, int64_t cols, const float *v,
                          float *out, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    if (env_int("CGX_REF_MV", 2) == 1)  // the 64-row, 128-column-tile kernel (kept for A/B)
        hipLaunchKernelGGL(k_matvec_ref_f32, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, s, A, lda, rows,
                           cols, v, out);
    else
        hipLaunchKernelGGL(k_matvec_ref_f32_r16, dim3((unsigned)((rows + kRef2Rows - 1) / kRef2Rows)), dim3(64), 0,
                           s, A, lda, rows, cols, v, out);
    return hipGetLastError();
}

hipError_t dot_ref_f32(int64_t n, const float *a, const float *b, float *out, hipStream_t s) {
    if (env_int("CGX_REF_DOT", 2) == 1)  // the one-wave kernel (kept for A/B)
        hipLaunchKernelGGL(k_dot_ref_f32, dim3(1), dim3(64), 0, s, n, a, b, out);
    else
        hipLaunchKernelGGL(k_dot_ref_f32_blk, dim3(1), dim3(256), 0, s, n, a, b, out);
    return hipGetLastError();
}

hipError_t residual_ref_f32(int64_t n, const float *b, const float *Ax, float *r, float *p,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_residual_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, b, Ax, r, p);
    return hipGetLastError();
}

hipError_t update_xr_ref_f32(int64_t n, float *x, float *r, const float *p, const float *Ap,
                             const float *rsold, const float *pAp, hipStream_t s) {
    hipLaunchKernelGGL(k_update_xr_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x, r, p, Ap, rsold, pAp);
    return hipGetLastError();
}

hipError_t update_p_ref_f32(int64_t n, float *p, const float *r, const float *rr, const float *rsold,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_update_p_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, p, r, rr, rsold);
    return hipGetLastError();
}

// ---- CGX_SYMMETRIC --------------------------------------------------------------
int64_t sym_tiles(int64_t lda) {
    const int64_t nt = lda / kSymT;
    return nt * (nt + 1) / 2;
}

int sym_grid(int device) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(k_symv_f64<1>), kSymNT,
                                                     0) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    return cus * per_cu;
}

hipError_t symv_f64(const double *At, int64_t n, int64_t lda, int grid, const double *p, double *prow, double *pcol,
                    double *y, const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                    const int64_t *gate) {
    const int64_t ntiles = sym_tiles(lda);
    if (grid <= 0) return hipErrorInvalidValue;
    const int64_t per = (ntiles + grid - 1) / grid;
    hipError_t e = symv_tiles_f64(At, 0, ntiles, lda, grid, false, p, prow, pcol, s, gate);
    if (e != hipSuccess) return e;
    return symv_reduce_f64(n, lda, per, prow, pcol, y, pown, dot_out, ws, s, gate);
}

hipError_t symv_tiles_f64(const double *At, int64_t q_base, int64_t count, int64_t lda, int grid, bool tile_runs,
                          const double *p, double *prow, double *pcol, hipStream_t s, const int64_t *gate) {
    if (lda % kSymT || grid <= 0 || count <= 0 ||
        ((reinterpret_cast<uintptr_t>(At) | reinterpret_cast<uintptr_t>(p)) & 15))
        return hipErrorInvalidValue;
    const int64_t per = (count + grid - 1) / grid;
    auto fn = env_int("CGX_SYM_NT", 1) ? k_symv_f64<1> : k_symv_f64<0>;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kSymNT), 0, s, At, lda / kSymT, q_base, count, per, tile_runs ? 1 : 0, p,
                       prow, pcol, gate);
    return hipGetLastError();
}

hipError_t symv_reduce_f64(int64_t n, int64_t lda, int64_t per, const double *prow, const double *pcol, double *y,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s, const int64_t *gate) {
    hipLaunchKernelGGL(k_symv_reduce_f64, dim3(grid_1d(n, 64, kMaxRedBlocks)), dim3(kNT), 0, s, n, lda / kSymT, per,
                       prow, pcol, y, pown, dot_out, ws.partials, ws.tickets + T_MATVEC, gate);
    return hipGetLastError();
}

hipError_t sym_pack_f64(const double *rows, int64_t ld, int64_t row0, int64_t nrows, int64_t n, int64_t lda,
                        double *At, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sym_pack_f64, dim3(grid_1d(nrows, 1, 65536)), dim3(kNT), 0, s, rows, ld, row0, nrows, n, lda,
                       lda / kSymT, At);
    return hipGetLastError();
}

hipError_t gen_spd_sym_f64(int64_t n, int64_t lda, uint64_t seed, double *At, double *b, hipStream_t s) {
    hipError_t e = gen_spd_sym_tiles_f64(n, lda, seed, 0, sym_tiles(lda), At, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gen_b, dim3(grid_vec(n)), dim3(kNT), 0, s, 0, n, mix64(seed + 1), b);
    return hipGetLastError();
}

hipError_t gen_spd_sym_tiles_f64(int64_t n, int64_t lda, uint64_t seed, int64_t q_base, int64_t count, double *At,
                                 hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_spd_sym, dim3((unsigned)std::min<int64_t>(count, 65536)), dim3(kSymNT), 0, s, n,
                       lda / kSymT, q_base, count, mix64(seed), At);
    return hipGetLastError();
}

hipError_t gen_b_f64(int64_t n, uint64_t seed, double *b, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_b, dim3(grid_vec(n)), dim3(kNT), 0, s, 0, n, mix64(seed + 1), b);
    return hipGetLastError();
}

}  // namespace cgx
