// cgx_ref_f32.hip -- CGX_F32_REF: fp32 kernels in serialConjugate.c's exact
// operation order (bit-identical to the reference build).
#include "cgx_device.h"

namespace cgx {
namespace {

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

}  // namespace

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

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_ref_f32() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_matvec_ref_f32_r16));
}

}  // namespace cgx
