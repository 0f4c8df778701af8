// matvec_variants.hip -- the dense fp64 matVec load policies that were
// measured and NOT adopted, kept out of libcgx and runnable
// here against libcgx's default (policy 8: software-pipelined, R=2, U=8,
// global_load ... nt) on the same rows, interleaved, with HIP events:
//   2..6  unpipelined buffer_load through a per-row scalar descriptor with the
//         cache bits kBufAux[POL] (nt / nt sc1 / sc0 nt sc1 / sc1 / none)
//   7     software-pipelined buffer_load nt
//   9/10  flattened pipeline (global / buffer nt): (row group, step) walked as
//         one stream, row bases in SGPRs
//   11    LDS-staged p (the north star's "LDS staging of the p-vector tile")
//   12/13 SGPR row bases (+ LDS-staged p)
// Every variant must give libcgx's row sums bit for bit (checked per run).
// Results of the round-1 sweeps: profiles/r01_sweep_*.jsonl.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/matvec_variants tools/microbench/matvec_variants.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,$PWD/conjugate_gradient_amd/lib
//   tools/microbench/matvec_variants [rows=8192] [cols=65536] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cgx_device.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

using namespace cgx;

namespace {

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
__global__ __launch_bounds__(kNT) void k_matvec_f64_var(
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

template <int R>
MvFn variant(int pol) {
    constexpr int U = 8;
    switch (pol) {
        case 2: return k_matvec_f64_var<R, U, 2>;
        case 3: return k_matvec_f64_var<R, U, 3>;
        case 4: return k_matvec_f64_var<R, U, 4>;
        case 5: return k_matvec_f64_var<R, U, 5>;
        case 6: return k_matvec_f64_var<R, U, 6>;
        case 7: return k_matvec_f64_var<R, U, 2, true>;
        case 9: return k_matvec_f64_flat<R, U, 1>;
        case 10: return k_matvec_f64_flat<R, U, 2>;
        case 11: return k_matvec_f64_lds<R, U>;
        case 12: return k_matvec_f64_sb<R, U, false>;
        case 13: return k_matvec_f64_sb<R, U, true>;
        default: return nullptr;
    }
}

}  // namespace

int main(int argc, char **argv) {
    const int64_t rows = argc > 1 ? std::atoll(argv[1]) : 8192, cols = argc > 2 ? std::atoll(argv[2]) : 65536;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
    if (cols % 1024) {
        std::fprintf(stderr, "cols must be a multiple of 1024 (whole U=8 steps)\n");
        return 2;
    }
    double *A, *b, *v, *ref, *out, *dot;
    RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * cols * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&v, (size_t)cols * 8));
    CK(hipMalloc(&ref, (size_t)rows * 8));
    CK(hipMalloc(&out, (size_t)rows * 8));
    CK(hipMalloc(&dot, 8));
    CK(hipMalloc(&ws.partials, kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, kTickets * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(gen_spd_f64(cols, cols, 0, rows, 42, A, b, s));  // rows [0, rows) of the N=cols system
    CK(gen_b_f64(cols, 7, v, s));                       // v: uniform [0, 1), another seed
    const MatvecPlan pl = plan_matvec_f64(0, rows);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(matvec_f64(pl, A, cols, rows, cols, v, ref, nullptr, nullptr, ws, s));
    std::vector<double> href(rows), hout(rows);
    CK(hipMemcpyAsync(href.data(), ref, rows * 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 8.0 * rows * cols + 8.0 * cols + 8.0 * rows;
    for (int R : {1, 2}) {
        for (int pol : {2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 13}) {
            MvFn fn = R == 1 ? variant<1>(pol) : variant<2>(pol);
            int per_cu = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(fn), kNT, 0));
            const int64_t need = ((rows + R - 1) / R + 3) / 4;
            const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)std::max(1, per_cu) * cus));
            auto launch_var = [&] {
                hipLaunchKernelGGL(fn, dim3(blocks), dim3(kNT), 0, s, A, cols, rows, cols, cols, int64_t(0),
                                   cols >> 7, 1, 0, v, out, nullptr, nullptr, ws.partials, ws.tickets + T_MATVEC,
                                   nullptr);
                CK(hipGetLastError());
            };
            auto launch_def = [&] { CK(matvec_f64(pl, A, cols, rows, cols, v, ref, nullptr, nullptr, ws, s)); };
            launch_var();
            CK(hipMemcpyAsync(hout.data(), out, rows * 8, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            const bool same = std::memcmp(hout.data(), href.data(), rows * 8) == 0;
            double tv = 0, td = 0;
            for (int rep = 0; rep < reps; ++rep) {
                for (int which = 0; which < 2; ++which) {
                    CK(hipEventRecord(e0, s));
                    if (which) launch_def(); else launch_var();
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep) (which ? td : tv) += ms;
                }
            }
            tv /= reps - 1;
            td /= reps - 1;
            std::printf("{\"rows\": %lld, \"cols\": %lld, \"R\": %d, \"U\": 8, \"policy\": %d, \"blocks\": %d, "
                        "\"ms\": %.4f, \"gbps\": %.1f, \"default_ms\": %.4f, \"default_gbps\": %.1f, "
                        "\"bitwise_equal_to_default\": %s}\n",
                        (long long)rows, (long long)cols, R, pol, blocks, tv, bytes / tv / 1e6, td, bytes / td / 1e6,
                        same ? "true" : "false");
            std::fflush(stdout);
        }
    }
    return 0;
}
