// cgx_ref_f32.hip -- CGX_F32_REF: fp32 kernels in serialConjugate.c's exact
// operation order (bit-identical to the reference build).
#include "cgx_device.h"

namespace cgx {
namespace {

// ---------------------------------------------------------------------------
// fp32 kernels in serialConjugate.c's exact operation order (CGX_F32_REF)
// ---------------------------------------------------------------------------
// matVec: one lane per row keeps the reference's order, out[i] = ((0 +
// a_i0 v_0) + a_i1 v_1) + ..., every product and sum rounded to float.  Round
// 1's kernel had a wave own 64 rows and walk 64 x 128 tiles through LDS, so
// the bytes in flight chip-wide were rows x 128 columns x 4 B (4 MiB at
// N=8192, about 2 TB/s at HBM latency) on 128 waves.  Here a wave owns 16
// rows and walks 16 x 512 tiles: all 64 lanes load the next tile (32
// coalesced 16-B loads each, 32 KiB per wave, 16 MiB chip-wide at
// N=8192) while lanes 0-15 run their rows' sequential sums over the current
// one.  The products A[i][j] * x[j] (each rounded to float, as
// serialConjugate.c:117 forms them) are made by all 64 lanes when a tile is
// stored, so a row's chain is one LDS read per 4 columns and 4 dependent
// adds.  Rows are padded to 516 floats: 16-B aligned, and lanes 0-15 reading
// columns 4j..4j+3 hit banks 4*lane + 4j .. +3, all distinct.
// Measured at N=8192: 62 us per matVec (the 64-row kernel, removed: 166 us); an
// 8-row x 1024-column variant (32 MiB in flight) measured 64 us.
constexpr int kRef2Rows = 16, kRef2TC = 512, kRef2Ld = kRef2TC + 4;
__global__ __launch_bounds__(64) void k_matvec_ref_f32_r16(const float *__restrict__ A, int64_t lda,
                                                           int64_t rows, int64_t cols,
                                                           const float *__restrict__ v,
                                                           float *__restrict__ out,
                                                           const int64_t *gate) {
#pragma clang fp contract(off)
    if (gate && *gate) return;  // converged in an earlier iteration (device-side gating)
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

// The same single sequential sum with its loads off the chain: 4 waves load
// the next 4096-element chunk while wave 0 adds up the current chunk's
// products from LDS; the products are formed (rounded to float,
// serialConjugate.c:150) when the chunk is stored.  The element-wise step
// that produces the summed vector can ride along (one launch instead of two,
// the same float operations in the same order):
//   kDotPlain  sum a_i b_i                                 (vecVec, :145-155)
//   kDotXR     x += p alpha; r -= Ap alpha; sum r_i r_i    (:219-234)
//   kDotResid  r = p = b - Ax; sum r_i r_i                 (:209-212)
//   kDotXRP    kDotXR, then the stopping test (:235-238) and, unless the
//              loop ends, p = r + p (rr / rsold)            (:239,243)
// dot_ref_body is the one block's work, shared by k_dot_ref_f32_blk and the
// last block of k_matvec_ref_f32_w5<.., true>: threads t < 256 load and
// store (a 320-thread block's fifth wave only passes the barriers), wave 0
// holds the sum.  SC1B: b was stored write-through by other blocks of the
// same launch and is read with sc1 loads (the one-counter hand-off).
constexpr int kDotChunk = 4096;
enum { kDotPlain = 0, kDotXR = 1, kDotResid = 2, kDotXRP = 3 };
typedef float f4v __attribute__((ext_vector_type(4)));
struct DotArgs {
    const float *a = nullptr, *b = nullptr;  // plain: the two vectors; resid: b, Ax
    float *x = nullptr, *r = nullptr, *p = nullptr;
    const float *Ap = nullptr, *rsold = nullptr, *pAp = nullptr;
    // kDotXR, several row blocks in one process: p.Ap from the blocks'
    // partials (MPICH order) instead of *pAp; cnt = 0: *pAp
    PeerSumF32 pap_sum{};
};
// ONE: n <= kDotChunk (one chunk, no next-chunk registers live during the
// chain); then keep_p / keep_r (kDotXR) hold this thread's p and new r values
// for the caller's p update (element u*256 + t in [u]).
template <int MODE, bool SC1B, bool ONE = false>
__device__ __forceinline__ float dot_ref_body(int64_t n, const DotArgs &d, f4v (*sp)[kDotChunk / 4], int t,
                                              float *keep_p = nullptr, float *keep_r = nullptr) {
#pragma clang fp contract(off)
    typedef f4v f4;
    constexpr int U = kDotChunk / 256;
    const bool act = t < 256;
    float av[U], bv[U], cv[U], dv[U];
    float alpha = 0.0f;
    if constexpr (MODE == kDotXR) {  // alpha = rsold / pAp  (:220)
        const float pap = d.pap_sum.cnt ? peer_sum_mpich_f32(d.pap_sum) : *d.pAp;
        alpha = *d.rsold / pap;
    }
    auto load = [&](int64_t c0) {
        if (!act) return;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = c0 + u * 256 + t;
            if (MODE == kDotXR) {
                av[u] = i < n ? d.x[i] : 0.0f;
                bv[u] = i < n ? d.p[i] : 0.0f;
                cv[u] = i < n ? d.r[i] : 0.0f;
                dv[u] = i < n ? d.Ap[i] : 0.0f;
            } else {
                av[u] = i < n ? d.a[i] : 0.0f;
                if (SC1B)
                    bv[u] = i < n ? __hip_atomic_load(d.b + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
                else
                    bv[u] = i < n ? d.b[i] : 0.0f;
            }
        }
    };
    auto store = [&](int buf, int64_t c0) {
        if (!act) return;
        float *spf = reinterpret_cast<float *>(sp[buf]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = c0 + u * 256 + t;
            if (MODE == kDotPlain) {
                spf[u * 256 + t] = av[u] * bv[u];
            } else if (MODE == kDotXR) {
                const float tx = bv[u] * alpha;  // x = x + p*alpha  (:221,225)
                const float xn = av[u] + tx;
                const float tr = dv[u] * alpha;  // r = r - Ap*alpha  (:226,230)
                const float rn = cv[u] - tr;
                if (i < n) {
                    d.x[i] = xn;
                    d.r[i] = rn;
                }
                if (ONE && keep_p) {
                    keep_p[u] = bv[u];
                    keep_r[u] = rn;
                }
                spf[u * 256 + t] = i < n ? rn * rn : 0.0f;
            } else {
                const float rn = av[u] - bv[u];  // r = b - Ax; p = b - Ax  (:210-211)
                if (i < n) {
                    d.r[i] = rn;
                    d.p[i] = rn;
                }
                spf[u * 256 + t] = i < n ? rn * rn : 0.0f;
            }
        }
    };
    const int64_t nch = ONE ? (n > 0 ? 1 : 0) : (n + kDotChunk - 1) / kDotChunk;
    float s = 0.0f;  // sum = 0.0  (:149)
    if (nch > 0) {
        load(0);
        store(0, 0);
        __syncthreads();
    }
    for (int64_t ch = 0; ch < nch; ++ch) {
        const int buf = (int)(ch & 1);
        if (!ONE && ch + 1 < nch) load((ch + 1) * kDotChunk);
        if (t < 64) {  // wave 0: sum += v1[i] * v2[i], i ascending (:152)
            // two register sets of G quads: one read from LDS while the other
            // is added (G = 16: 2.9-3.3 ns per dependent add against 3.2-3.6
            // at G = 8, tools/microbench/add_chain.hip).  A short last chunk
            // runs the same loop up to the next 2G quads: store() wrote +0.0f
            // past n, and s + 0.0f == s exactly (s starts at +0 and a
            // round-to-nearest sum never makes -0 from it), so at most 127
            // no-op adds replace a one-element-per-step LDS loop.
            constexpr int G = 16;
            const int64_t left = n - ch * kDotChunk;
            const int nq = left >= kDotChunk ? kDotChunk / 4 : (int)((left + 8 * G - 1) / (8 * G)) * (2 * G);
            f4 q[G], qn[G];
            auto add = [&](const f4 (&w)[G]) {
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    s = s + w[u].x;
                    s = s + w[u].y;
                    s = s + w[u].z;
                    s = s + w[u].w;
                }
            };
#pragma unroll
            for (int u = 0; u < G; ++u) q[u] = sp[buf][u];
#pragma unroll 1
            for (int j = 0; j < nq; j += 2 * G) {
#pragma unroll
                for (int u = 0; u < G; ++u) qn[u] = sp[buf][j + G + u];
                add(q);
                if (j + 2 * G < nq) {
#pragma unroll
                    for (int u = 0; u < G; ++u) q[u] = sp[buf][j + 2 * G + u];
                }
                add(qn);
            }
        }
        if (!ONE && ch + 1 < nch) store(buf ^ 1, (ch + 1) * kDotChunk);
        __syncthreads();
    }
    return s;
}

// The same float arithmetic at the HBM rate: loads decoupled from the chains.
// k_matvec_ref_f32_r16 issues one tile per wave and then waits for it, so
// every step costs an HBM round trip (62 us at N=8192, ~4.1 TB/s).  Here a
// 256-thread block owns 32 rows and keeps two 32 x 512 tiles of A in flight
// (16 nt 16-B buffer loads per lane per tile, two register sets).  Per step
// (one barrier) wave 0's lanes 0-31 add up tile t from LDS, one row each,
// while every lane waits for its share of tile t+1 (issued two steps
// earlier), forms the products A[i][j] * x[j] (rounded to float, as
// serialConjugate.c:117 forms them) into the other LDS slot and issues its
// loads of tile t+3.
//  - Buffer loads: one VGPR offset per lane, the row and tile in the SGPR
//    offset, so the two register sets fit without copies through AGPRs.
//    Every step issues the same loads whatever the tile (tiles past the end
//    read past the buffer's range: zeros, no memory access), and the loads of
//    a set stay together (sched_barrier), so the wait before the products is
//    "all but the newer set" (vmcnt 17), not 0.
//  - FULL: rows % 32 == 0 and cols % 512 == 0 (the reference's sizes).
//    Otherwise rows past `rows` are out of the buffer's range (zeros) and
//    columns past `cols` are zeroed: their products are +0.0f, and
//    acc + 0.0f == acc exactly (acc starts at +0, and a round-to-nearest sum
//    never makes -0 from it), so the chains still run whole tiles.
//  - Needs 16-B aligned A and x and lda % 4 == 0.
constexpr int kRef3Rows = 32, kRef3TC = 512, kRef3Q = kRef3TC / 4, kRef3Ld4 = kRef3Q + 1;
constexpr int kRef3K = kRef3Rows * kRef3Q / 256;
static_assert(kRef3K == 16, "lane t: column quad t % 128 of rows t / 128 + 2k");
// With a dedicated adding wave: 5 waves, wave 0 only runs the chains and
// waves 1-4 only load and form products, so a step costs max(chain, loads)
// rather than chain + wave 0's own share of the loads.  Measured at N=8192
// (rocprofv3, profiles/r02_kernel_stats_ref_f32_n8192.csv): 49.6 us against
// 53.9 for the 4-wave form in which wave 0 also loads (removed in round 5) and
// 62.3 for the 16-row kernel; a third register set (192 KiB in flight per CU)
// measured 51.9.
//
// DOT (the single-GPU two-launch iteration): the rows go out write-through
// (sc1) and the last block to arrive (ticket) runs vecVec(p, Ap) over all
// `rows` -- dot_ref_body, the separate dot kernel's code -- so the matVec and
// p.Ap are one launch (serialConjugate.c:215,219), the same bits.
template <bool FULL, bool DOT>
__global__ __launch_bounds__(320) void k_matvec_ref_f32_w5(const float *__restrict__ A, int64_t lda,
                                                           int64_t rows, int64_t cols,
                                                           const float *__restrict__ v,
                                                           float *__restrict__ out,
                                                           const int64_t *gate, const float *pown,
                                                           float *dot_out, unsigned *ticket) {
#pragma clang fp contract(off)
    if (gate && *gate) return;  // converged in an earlier iteration (device-side gating)
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ f4 prod[2][kRef3Rows * kRef3Ld4];
    const int t = threadIdx.x;
    const int l = t >= 64 ? t - 64 : 0;  // loader lane (waves 1-4); wave 0 only adds
    const int64_t row0 = (int64_t)blockIdx.x * kRef3Rows;
    const int64_t ntiles = (cols + kRef3TC - 1) / kRef3TC;
    const int quad = l % kRef3Q, rsub = l / kRef3Q;
    const int64_t brows = rows - row0 < kRef3Rows ? rows - row0 : kRef3Rows;
    const __amdgpu_buffer_rsrc_t ars =
        __builtin_amdgcn_make_buffer_rsrc((void *)(A + row0 * lda), 0, (int)(brows * lda * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void *)v, 0, (int)(cols * 4), 0x00020000);
    const int voff = (int)((rsub * lda + 4 * quad) * 4);
    const int end_off = (int)(brows * lda * 4);  // a tile past the end: every load out of range
    f4 a0[kRef3K], a1[kRef3K];
    f4 p0, p1;
    auto issue = [&](f4 (&a)[kRef3K], f4 &pv, int64_t tile) {
        const bool real = tile < ntiles;
        const int c4 = (int)(tile * kRef3TC * 4);
#pragma unroll
        for (int k = 0; k < kRef3K; ++k)
            a[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                              ars, voff, real ? (int)(2 * k * lda * 4) + c4 : end_off, 2));
        pv = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(vrs, quad * 16, real ? c4 : (int)(cols * 4), 0));
    };
    auto store = [&](f4 (&a)[kRef3K], f4 &pv, int slot, int64_t tile) {
        if (!FULL) {  // columns past `cols`: +0 products whatever A's padding holds
            const int64_t cq = tile * kRef3TC + 4 * quad;
            for (int e = 0; e < 4; ++e)
                if (cq + e >= cols) {
                    pv[e] = 0.0f;
#pragma unroll
                    for (int k = 0; k < kRef3K; ++k) a[k][e] = 0.0f;
                }
        }
#pragma unroll
        for (int k = 0; k < kRef3K; ++k) prod[slot][(rsub + 2 * k) * kRef3Ld4 + quad] = a[k] * pv;
    };
    float acc = 0.0f;  // matvec[i] = 0.0  (serialConjugate.c:114)
    auto chain = [&](int slot) {  // matvec[i] += A[i][j] * x[j], j ascending (:117)
        const f4 *trow = &prod[slot][t * kRef3Ld4];
        constexpr int G = 8;  // two register sets of G quads: one read from LDS while the other is added
        f4 q[G], qn[G];
        auto add = [&](const f4 (&w)[G]) {
#pragma unroll
            for (int u = 0; u < G; ++u) {
                acc = acc + w[u].x;
                acc = acc + w[u].y;
                acc = acc + w[u].z;
                acc = acc + w[u].w;
            }
        };
#pragma unroll
        for (int u = 0; u < G; ++u) q[u] = trow[u];
#pragma unroll 1
        for (int j4 = 0; j4 < kRef3Q; j4 += 2 * G) {
#pragma unroll
            for (int u = 0; u < G; ++u) qn[u] = trow[j4 + G + u];
            add(q);
            if (j4 + 2 * G < kRef3Q) {
#pragma unroll
                for (int u = 0; u < G; ++u) q[u] = trow[j4 + 2 * G + u];
            }
            add(qn);
        }
    };
    // DOT: every wave (both roles) arrives here after the last barrier.
    __shared__ int is_last;
    auto dot_epilogue = [&](int64_t n, const float *Ap, const float *pv, float *dst, unsigned *tk, int tid) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's Ap stores have landed
        __syncthreads();
        if (tid == 0)
            is_last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        __syncthreads();
        if (!is_last) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        DotArgs d;
        d.a = pv;
        d.b = Ap;
        const float sum = dot_ref_body<kDotPlain, true>(n, d, reinterpret_cast<f4v (*)[kDotChunk / 4]>(&prod[0][0]), tid);
        if (tid == 0) {
            *dst = sum;
            __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // Role by wave (a scalar branch: each role's loop is straight-line code,
    // so the loaders' waits stay "all but the newer set"); both roles pass
    // the same barriers, one per step.
    const int64_t nsteps = (ntiles + 1) / 2 * 2;  // the loaders' steps, whole pairs
    if (__builtin_amdgcn_readfirstlane(t >> 6) == 0) {
        __syncthreads();
        for (int64_t tt = 0; tt < nsteps; ++tt) {
            if (t < kRef3Rows && tt < ntiles) chain((int)(tt & 1));
            __syncthreads();
        }
        if (t < kRef3Rows && row0 + t < rows) {
            if (DOT)
                __hip_atomic_store(out + row0 + t, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
            else
                out[row0 + t] = acc;
        }
        if (DOT) dot_epilogue(rows, out, pown, dot_out, ticket, t);
        return;
    }
    // at step tt the loaders store tile tt + 1 into slot (tt + 1) & 1 and
    // reuse its register set for tile tt + 3 (unrolled by two so the sets
    // are static; steps past the last tile store zeros into a slot nobody
    // reads)
    issue(a0, p0, 0);
    __builtin_amdgcn_sched_barrier(0);
    issue(a1, p1, 1);
    __builtin_amdgcn_sched_barrier(0);
    store(a0, p0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    issue(a0, p0, 2);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    for (int64_t tt = 0; tt < nsteps; tt += 2) {
        store(a1, p1, 1, tt + 1);
        __builtin_amdgcn_sched_barrier(0);
        issue(a1, p1, tt + 3);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        store(a0, p0, 0, tt + 2);
        __builtin_amdgcn_sched_barrier(0);
        issue(a0, p0, tt + 4);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
    if (DOT) dot_epilogue(rows, out, pown, dot_out, ticket, t);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_dot_ref_f32_blk(int64_t n, DotArgs d, float *out, const int64_t *gate,
                                                         ConvArgs cv) {
#pragma clang fp contract(off)
    if (gate && *gate) return;  // converged in an earlier iteration (device-side gating)
    __shared__ f4v sp[2][kDotChunk / 4];
    __shared__ float rr_b;
    const int t = threadIdx.x;
    if constexpr (MODE == kDotResid) {  // the solve's start: reset the convergence record (no memset launch)
        if (cv.kdone && t == 0) {
            *cv.kdone = 0;
            *cv.rrfinal = 0.0;
        }
    }
    constexpr int U = 16;  // every load of a step issued before its stores: one round trip per 4096
    static_assert(U * 256 == kDotChunk, "one chunk of the body is one step of the p update");
    float kp[U], kr[U];  // n <= kDotChunk: p and the new r of this thread's elements, kept from the body
    constexpr int BODY = MODE == kDotXRP ? (int)kDotXR : MODE;
    const bool keep = MODE == kDotXRP && n <= kDotChunk;
    const float s = keep ? dot_ref_body<BODY, false, true>(n, d, sp, t, kp, kr) : dot_ref_body<BODY, false>(n, d, sp, t);
    if (t == 0) *out = s;
    if constexpr (MODE == kDotXRP) {
        // The single-GPU two-launch iteration's update: this block also makes
        // the stopping decision (:235-238, the float r.r widened to double as
        // C's sqrt takes it) and, unless the loop ends there, forms
        // p = r + p*(rr/rsold) (:239,243) -- k_update_p_ref_f32's arithmetic.
        // Element i is stored by thread i % 256 in the body and read back by
        // the same thread here.
        if (t == 0) rr_b = s;
        __syncthreads();
        const float rr = rr_b;
        if (cv.kdone && cv.eps >= 0.0 && sqrt((double)rr) < cv.eps) {
            if (t == 0) record_convergence(cv, cv.k + 1, (double)rr);
            return;
        }
        const float ratio = rr / *d.rsold;
        if (keep) {  // one chunk: no reload of p and r
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = u * 256 + t;
                const float tp = kp[u] * ratio;
                if (i < n) d.p[i] = kr[u] + tp;
            }
            return;
        }
        for (int64_t c0 = 0; c0 < n; c0 += 256 * U) {
            float pv[U], rv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = c0 + u * 256 + t;
                pv[u] = i < n ? d.p[i] : 0.0f;
                rv[u] = i < n ? d.r[i] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = c0 + u * 256 + t;
                const float tp = pv[u] * ratio;
                if (i < n) d.p[i] = rv[u] + tp;
            }
        }
    }
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
                                                           const float *rsold, const float *pAp,
                                                           const int64_t *gate) {
#pragma clang fp contract(off)
    if (gate && *gate) return;  // converged in an earlier iteration (device-side gating)
    const float alpha = *rsold / *pAp;
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
        const float tx = p[i] * alpha;
        x[i] = x[i] + tx;
        const float tr = Ap[i] * alpha;
        r[i] = r[i] - tr;
    }
}

// p = r + p*(beta/rsold)  (:239,243).  With cv.kdone (device-side gating)
// the kernel first makes the reference's stopping decision,
// `if (sqrt(rsnew) < EPSILON) break;` (:235-238: the float r.r widened to
// double, as C's sqrt takes it): on convergence it records k+1 and r.r and
// leaves p alone (the loop has ended); in a later iteration it does nothing.
// rr_sum.cnt > 0 (several row blocks in one process): r.r from the blocks'
// partials in MPICH order (PeerSumF32) instead of *rr, block 0 storing it.
__global__ __launch_bounds__(kNT) void k_update_p_ref_f32(int64_t n, float *__restrict__ p,
                                                          const float *__restrict__ r,
                                                          const float *rr, const float *rsold, ConvArgs cv,
                                                          PeerSumF32 rr_sum) {
#pragma clang fp contract(off)
    if (cv.kdone) {
        const int64_t kd = *cv.kdone;
        if (kd != 0 && kd <= cv.k) return;
    }
    const float rrv = rr_sum.cnt ? peer_sum_mpich_f32(rr_sum) : *rr;
    if (cv.kdone) {
        const double rrn = (double)rrv;
        if (cv.eps >= 0.0 && sqrt(rrn) < cv.eps) {
            if (blockIdx.x == 0 && threadIdx.x == 0) record_convergence(cv, cv.k + 1, rrn);
            return;
        }
    }
    const float ratio = rrv / *rsold;
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
        const float t = p[i] * ratio;
        p[i] = r[i] + t;
    }
}

}  // namespace

hipError_t matvec_ref_f32(const float *A, int64_t lda, int64_t rows, int64_t cols, const float *v,
                          float *out, hipStream_t s, const int64_t *gate) {
    if (rows <= 0) return hipSuccess;
    // 16-B aligned rows and x; the buffer offsets (32 rows of lda floats) fit in 31 bits
    const bool vec_ok = (lda & 3) == 0 && lda < (int64_t(1) << 23) &&
                        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
    if (vec_ok) {
        const bool full = rows % kRef3Rows == 0 && cols % kRef3TC == 0;
        const dim3 grid((unsigned)((rows + kRef3Rows - 1) / kRef3Rows));
        hipLaunchKernelGGL((full ? k_matvec_ref_f32_w5<true, false> : k_matvec_ref_f32_w5<false, false>), grid,
                           dim3(320), 0, s, A, lda, rows, cols, v, out, gate, nullptr, nullptr, nullptr);
    } else {  // unaligned rows: the 16-row kernel (scalar loads)
        hipLaunchKernelGGL(k_matvec_ref_f32_r16, dim3((unsigned)((rows + kRef2Rows - 1) / kRef2Rows)), dim3(64), 0,
                           s, A, lda, rows, cols, v, out, gate);
    }
    return hipGetLastError();
}

hipError_t dot_ref_f32(int64_t n, const float *a, const float *b, float *out, hipStream_t s, const int64_t *gate) {
    DotArgs d;
    d.a = a;
    d.b = b;
    hipLaunchKernelGGL(k_dot_ref_f32_blk<kDotPlain>, dim3(1), dim3(256), 0, s, n, d, out, gate, ConvArgs{});
    return hipGetLastError();
}

bool matvec_dot_ref_f32_fusable(const float *A, int64_t lda, const float *v) {
    return (lda & 3) == 0 && lda < (int64_t(1) << 23) && ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
}

hipError_t matvec_dot_ref_f32(const float *A, int64_t lda, int64_t rows, int64_t cols, const float *v, float *out,
                              const float *pown, float *dot_out, unsigned *ticket, hipStream_t s,
                              const int64_t *gate) {
    if (rows <= 0) return hipSuccess;
    if (!matvec_dot_ref_f32_fusable(A, lda, v)) {  // two launches, the same bits
        const hipError_t e = matvec_ref_f32(A, lda, rows, cols, v, out, s, gate);
        return e != hipSuccess ? e : dot_ref_f32(rows, pown, out, dot_out, s, gate);
    }
    const bool full = rows % kRef3Rows == 0 && cols % kRef3TC == 0;
    hipLaunchKernelGGL((full ? k_matvec_ref_f32_w5<true, true> : k_matvec_ref_f32_w5<false, true>),
                       dim3((unsigned)((rows + kRef3Rows - 1) / kRef3Rows)), dim3(320), 0, s, A, lda, rows, cols, v,
                       out, gate, pown, dot_out, ticket);
    return hipGetLastError();
}

hipError_t update_xrp_dot_ref_f32(int64_t n, float *x, float *r, float *p, const float *Ap, const float *rsold,
                                  const float *pAp, float *rr, hipStream_t s, const int64_t *gate, double eps,
                                  int64_t k, int64_t *kdone, double *rrfinal, int64_t *hrec) {
    DotArgs d;
    d.x = x;
    d.r = r;
    d.p = p;
    d.Ap = Ap;
    d.rsold = rsold;
    d.pAp = pAp;
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(k_dot_ref_f32_blk<kDotXRP>, dim3(1), dim3(256), 0, s, n, d, rr, gate, cv);
    return hipGetLastError();
}

hipError_t update_xr_dot_ref_f32(int64_t n, float *x, float *r, const float *p, const float *Ap, const float *rsold,
                                 const float *pAp, float *rr, hipStream_t s, const int64_t *gate,
                                 const PeerSumF32 *pap_sum) {
    DotArgs d;
    d.x = x;
    d.r = r;
    d.p = const_cast<float *>(p);
    d.Ap = Ap;
    d.rsold = rsold;
    d.pAp = pAp;
    if (pap_sum) {
        if (pap_sum->cnt < 0 || pap_sum->cnt > kMaxPeers) return hipErrorInvalidValue;
        d.pap_sum = *pap_sum;
    }
    hipLaunchKernelGGL(k_dot_ref_f32_blk<kDotXR>, dim3(1), dim3(256), 0, s, n, d, rr, gate, ConvArgs{});
    return hipGetLastError();
}

hipError_t residual_dot_ref_f32(int64_t n, const float *b, const float *Ax, float *r, float *p, float *rr,
                                hipStream_t s, int64_t *clear2) {
    DotArgs d;
    d.a = b;
    d.b = Ax;
    d.r = r;
    d.p = p;
    ConvArgs cv;
    cv.kdone = clear2;
    cv.rrfinal = clear2 ? reinterpret_cast<double *>(clear2 + 1) : nullptr;
    hipLaunchKernelGGL(k_dot_ref_f32_blk<kDotResid>, dim3(1), dim3(256), 0, s, n, d, rr, nullptr, cv);
    return hipGetLastError();
}

hipError_t residual_ref_f32(int64_t n, const float *b, const float *Ax, float *r, float *p,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_residual_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, b, Ax, r, p);
    return hipGetLastError();
}

hipError_t update_xr_ref_f32(int64_t n, float *x, float *r, const float *p, const float *Ap,
                             const float *rsold, const float *pAp, hipStream_t s, const int64_t *gate) {
    hipLaunchKernelGGL(k_update_xr_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, x, r, p, Ap, rsold, pAp, gate);
    return hipGetLastError();
}

hipError_t update_p_ref_f32(int64_t n, float *p, const float *r, const float *rr, const float *rsold,
                            hipStream_t s, double eps, int64_t k, int64_t *kdone, double *rrfinal, int64_t *hrec,
                            const PeerSumF32 *rr_sum) {
    PeerSumF32 rs{};
    if (rr_sum) {
        if (rr_sum->cnt < 0 || rr_sum->cnt > kMaxPeers) return hipErrorInvalidValue;
        rs = *rr_sum;
    }
    ConvArgs cv;
    cv.eps = eps;
    cv.k = k;
    cv.kdone = kdone;
    cv.rrfinal = rrfinal;
    cv.hrec = hrec;
    hipLaunchKernelGGL(k_update_p_ref_f32, dim3(grid_vec(n)), dim3(kNT), 0, s, n, p, r, rr, rsold, cv, rs);
    return hipGetLastError();
}

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_ref_f32() {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_ref_f32_r16));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_dot_ref_f32_blk<kDotXR>));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_ref_f32_w5<true, false>));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_ref_f32_w5<true, true>));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_dot_ref_f32_blk<kDotXRP>));
    return e != hipSuccess ? e : hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_ref_f32_w5<false, false>));
}

}  // namespace cgx
