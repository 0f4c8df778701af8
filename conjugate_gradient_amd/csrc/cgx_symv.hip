// cgx_symv.hip -- CGX_SYMMETRIC: the matVec over the upper triangle of
// 128 x 128 tiles (half of A's bytes per iteration).
#include "cgx_device.h"

#include <algorithm>

namespace cgx {
namespace {

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

}  // namespace

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

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_symv() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_symv_f64<1>));
}

}  // namespace cgx
