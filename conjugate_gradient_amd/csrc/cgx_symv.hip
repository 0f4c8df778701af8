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
// Layout: tile (I, J), J >= I, at index q = sym_off(I) + J - I (row-major over
// the upper triangle); a diagonal tile is stored whole.  A tile is two
// column halves ("units" u = 2q + h: columns 64h .. 64h + 63, all 128 rows,
// 64 KiB each), and inside a unit the doubles are in the order a 256-thread
// block loads them: d2 number k * 256 + t holds (row, col) =
// (8 tr + rr, 64 h + 4 tc + 2 cc + {0, 1}) with t = 16 tr + tc, k = 2 rr + cc,
// so every load step reads 4 KiB contiguous.
//
// Why units of half a tile: the tile stream is bound by how HBM serves the
// CUs' read streams.  tools/microbench/hbm_region_read.hip measured a
// 512-thread block streaming one contiguous region per CU (round 2's
// layout, one block per CU) at 6.96-6.99 TB/s, and two 256-thread blocks per
// CU, each streaming its own region, at 7.12-7.17 TB/s.  A unit gives a
// 256-thread block the same 8 x 4 patch per thread (16 d2 loads, 8 rows x 4
// columns) the 512-thread block had per tile, so registers, the two
// prefetch slots and the arithmetic per load are unchanged; only the row
// reduction spans 16 lanes instead of 32.  The column partials of a tile are
// its two units' 64 columns each, the same 128 per tile (pcol's indexing is
// unchanged); row partials are per run of units.
//
// k_symv_f64: a block streams a contiguous range of `per` units (the next
// unit's loads in flight during the current one's arithmetic).  Per unit of
// tile (I, J), off the diagonal, it writes its 64 column partials
// A_IJ^T p_I to pcol[q * 128 + 64 h ..]; the row partials A_IJ p_J are summed
// over the block's run of units in tile row I and written once per run, at
// prow[first unit of the run] (a run starts at 2 sym_off(I) or at a multiple
// of `per`).  k_symv_reduce_f64 sums row i's run partials and column
// partials in a fixed order, so the result is deterministic, and fuses p.Ap.
// ---------------------------------------------------------------------------
constexpr int kSymT = 128, kSymNT = 256, kSymH = 64;
constexpr int kSymRPT = 8;                                // rows per thread (4 columns each)
constexpr int kSymK = 2 * kSymRPT;                        // d2 loads per thread per unit
constexpr int kSymTR = kSymT / kSymRPT;                   // thread rows per unit (16)
constexpr int kSymTC = kSymNT / kSymTR;                   // thread columns per unit (16)
constexpr int64_t kSymUnit = (int64_t)kSymT * kSymH;      // doubles per unit
static_assert(kSymTC * 4 == kSymH && kSymTR * kSymRPT == kSymT, "unit = 16 x 16 threads of 8 x 4 doubles");
static_assert(kSymNT == 256 && kSymRPT == 8, "sym_pos_h (cgx_kernels.h) assumes 256 threads, 8 rows per thread");

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
    const int h = c / kSymH, cc = c % kSymH;
    const int t = (r / kSymRPT) * kSymTC + (cc >> 2), k = (r % kSymRPT) * 2 + ((cc >> 1) & 1);
    return h * kSymUnit + ((int64_t)k * kSymNT + t) * 2 + (c & 1);
}

// One unit's loads: its 16 d2 of A per thread and the p values it multiplies.
struct SymSlot {
    d2 a[kSymK], pj[2], pi[kSymRPT / 2];
    int64_t I, J;
    int h;
};

// Buffer loads with wave-uniform bases (unit u, p): the only per-lane
// address is the loop-invariant t*16 (or tc/tr offsets), so no address
// registers are recomputed per unit -- recomputed ones landed in registers
// the slot loads had just written, and the compiler's wait for them drained
// the loads in flight at the top of every iteration.
// ua: the unit's index in At (At may hold a range of tiles starting at q_base).
template <int NTL>
__device__ __forceinline__ void sym_load(SymSlot &S, const double *At, __amdgpu_buffer_rsrc_t prs, int64_t ua,
                                         int64_t I, int64_t J, int h, int t, int tr, int tc) {
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(At + ua * kSymUnit), 0, (int)(kSymUnit * 8), 0x00020000);
#pragma unroll
    for (int k = 0; k < kSymK; ++k)
        S.a[k] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(trs, t * 16, k * kSymNT * 16,
                                                                              NTL ? 2 : 0));
    const int jo = (int)((J * kSymT + h * kSymH) * 8), io = (int)(I * kSymT * 8);
#pragma unroll
    for (int u = 0; u < 2; ++u)
        S.pj[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(prs, tc * 32 + u * 16, jo, 0));
#pragma unroll
    for (int u = 0; u < kSymRPT / 2; ++u)
        S.pi[u] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(prs, tr * kSymRPT * 8 + u * 16, io, 0));
    S.I = I;
    S.J = J;
    S.h = h;
}

// the unit after (I, J, h)
__device__ __forceinline__ void sym_next(int64_t &I, int64_t &J, int &h, int64_t nt) {
    if (h == 0) {
        h = 1;
        return;
    }
    h = 0;
    if (++J == nt) J = ++I;
}

// Row partials A_IJ p_J (always) and column partials A_IJ^T p_I (J > I) of
// one unit; `buf` selects the LDS half for the column sums (flipped per use).
// racc: this lane's running row sum over the current run; end_of_run: the
// next unit is in another tile row (or there is none), so write it.
__device__ __forceinline__ void sym_unit(const SymSlot &S, int64_t u, double (*cs)[kSymTR][kSymH], int &buf,
                                         double *__restrict__ prow, double *__restrict__ pcol, int t, int tr, int tc,
                                         double &racc, int64_t &urun, bool end_of_run) {
    // row partials over this thread's 4 columns, then over the 16 lanes of
    // its thread-row group: a halving exchange (the lane pairs 8, 4, 2 apart
    // swap half their rows) until one row per lane pair, then the pair's sum
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
        const bool h1 = tc & 8;
        double k[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) k[q] = (h1 ? rs[q + 4] : rs[q]) + __shfl_xor(h1 ? rs[q] : rs[q + 4], 8, 64);
        row += h1 ? 4 : 0;
        const bool h2 = tc & 4;
        double m[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) m[q] = (h2 ? k[q + 2] : k[q]) + __shfl_xor(h2 ? k[q] : k[q + 2], 4, 64);
        row += h2 ? 2 : 0;
        const bool h3 = tc & 2;
        k1 = (h3 ? m[1] : m[0]) + __shfl_xor(h3 ? m[0] : m[1], 2, 64);
        row += h3 ? 1 : 0;
    }
    k1 += __shfl_xor(k1, 1, 64);
    racc += k1;
    if (end_of_run) {
        if ((tc & 1) == 0) prow[urun * kSymT + tr * kSymRPT + row] = racc;
        racc = 0.0;
        urun = u + 1;
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
        // unit's loads that are in flight across this point
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (t < kSymH) {
            double sum = cs[buf][0][t];
#pragma unroll
            for (int g = 1; g < kSymTR; ++g) sum += cs[buf][g][t];
            pcol[(u >> 1) * kSymT + S.h * kSymH + t] = sum;
        }
        buf ^= 1;
    }
}

// Two slots alternate: the loads of unit u+1 go out before unit u's
// arithmetic.
// Tiles [q_base, q_base + count) of the triangle, At holding exactly those
// (a streamed chunk) or all of them (q_base = 0); per = units per block.
// tile_runs: every unit is its own run (its row partials written per unit):
// chunk boundaries then do not matter to the reduce, which is told per = 1.
template <int NTL>
__global__ __launch_bounds__(kSymNT) void k_symv_f64(const double *__restrict__ At, int64_t nt, int64_t q_base,
                                                     int64_t count, int64_t per, int tile_runs,
                                                     const double *__restrict__ p, double *__restrict__ prow,
                                                     double *__restrict__ pcol, const int64_t *gate) {
    if (gate && *gate) return;
    __shared__ double cs[2][kSymTR][kSymH];
    const int t = threadIdx.x, tr = t / kSymTC, tc = t % kSymTC;
    const int64_t u_base = 2 * q_base, u_end = 2 * (q_base + count);
    const int64_t u0 = u_base + (int64_t)blockIdx.x * per;
    const int64_t u1 = (u0 + per < u_end) ? u0 + per : u_end;
    if (u0 >= u1) return;
    int64_t Ic, Jc;  // unit u
    sym_tile_ij(u0 >> 1, nt, Ic, Jc);
    int hc = (int)(u0 & 1);
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(nt * kSymT * 8), 0x00020000);
    int buf = 0;
    double racc = 0.0;
    int64_t urun = u0;
    SymSlot S0, S1;
    sym_load<NTL>(S0, At, prs, u0 - u_base, Ic, Jc, hc, t, tr, tc);
    // Every load is issued unconditionally (past the range end a slot
    // reloads the last unit): with a conditional load block the compiler's
    // wait counts at the merge assume no newer loads and drain the next
    // unit's loads before the current unit is used.
    for (int64_t u = u0; u < u1; u += 2) {
        int64_t I1 = Ic, J1 = Jc;
        int h1 = hc;
        sym_next(I1, J1, h1, nt);
        const bool va = u + 1 < u1;
        sym_load<NTL>(S1, At, prs, (va ? u + 1 : u) - u_base, va ? I1 : Ic, va ? J1 : Jc, va ? h1 : hc, t, tr, tc);
        __builtin_amdgcn_sched_barrier(0);  // the loads go out before this unit's arithmetic
        if (tile_runs) urun = u;
        sym_unit(S0, u, cs, buf, prow, pcol, t, tr, tc, racc, urun, tile_runs || !va || I1 != Ic);
        if (!va) break;
        int64_t I2 = I1, J2 = J1;
        int h2 = h1;
        sym_next(I2, J2, h2, nt);
        const bool vb = u + 2 < u1;
        sym_load<NTL>(S0, At, prs, (vb ? u + 2 : u + 1) - u_base, vb ? I2 : I1, vb ? J2 : J1, vb ? h2 : h1, t, tr,
                      tc);
        __builtin_amdgcn_sched_barrier(0);
        if (tile_runs) urun = u + 1;
        sym_unit(S1, u + 1, cs, buf, prow, pcol, t, tr, tc, racc, urun, tile_runs || !vb || I2 != I1);
        Ic = I2;
        Jc = J2;
        hc = h2;
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
        const int64_t first = 2 * sym_off(I, nt), last = 2 * sym_off(I + 1, nt) - 1;  // the units of tile row I
        const int64_t k0 = first / per, R = 1 + last / per - k0;                    // its runs
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
// Tiles [q_base, q_base + count) into At (At[0] = tile q_base); a 512-thread
// block fills one tile, threads 256 h + t the patch thread t loads in unit h.
constexpr int kSymGenNT = 2 * kSymNT;
__global__ __launch_bounds__(kSymGenNT) void k_gen_spd_sym(int64_t n, int64_t nt, int64_t q_base, int64_t count,
                                                           uint64_t salt, double *__restrict__ At) {
#pragma clang fp contract(off)
    for (int64_t qi = blockIdx.x; qi < count; qi += gridDim.x) {
        int64_t I, J;
        sym_tile_ij(q_base + qi, nt, I, J);
        const int h = threadIdx.x / kSymNT, t = threadIdx.x % kSymNT, tr = t / kSymTC, tc = t % kSymTC;
        d2 *unit = reinterpret_cast<d2 *>(At) + (qi * 2 + h) * (kSymUnit / 2);
        for (int k = 0; k < kSymK; ++k) {
            const uint64_t i = (uint64_t)(I * kSymT + tr * kSymRPT + (k >> 1));
            d2 v;
            for (int e = 0; e < 2; ++e) {
                const uint64_t j = (uint64_t)(J * kSymT + h * kSymH + tc * 4 + (k & 1) * 2 + e);
                double val = 0.0;
                if (i < (uint64_t)n && j < (uint64_t)n) {
                    val = 0.5 * (u01(salt, i, j) + u01(salt, j, i));
                    if (i == j) val = val + (double)n;
                }
                v[e] = val;
            }
            unit[k * kSymNT + t] = v;
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
    // One 256-thread block per CU, streaming its own range of units: 388.1
    // it/s at N=65536 against 384.8-386.4 with two per CU (and 367-377 for
    // round 2's one 512-thread block per CU), interleaved on one box
    // (profiles/r03_symmetric_blocks_ab.jsonl).  Never more than are resident
    // at once -- each block owns a fixed range, so a block that had to wait
    // for a free CU would run its whole range after the others.  (The
    // occupancy query can over-report by a block for 256-thread kernels:
    // cdna_hip_programming.md.)
    per_cu = std::min(per_cu, env_opt("CGX_SYM_PLAN", "bpc", 1));
    return cus * per_cu;
}

// Units per block (each block streams one contiguous range), rounded up to an
// odd count: the 256 ranges then start at 32 different offsets modulo 2 MiB
// (64-KiB units) instead of all at one offset modulo 128 KiB (N=65536: 1026
// units per block), so the streams spread over the HBM channels however the
// pages land.  N=65536: 399.5-399.7 it/s (6.91 TB/s on the stored bytes)
// against 387.6-388.6 with 1026, four processes each, alternating
// (profiles/r03_symmetric_per_odd_ab.jsonl).  CGX_SYM_PLAN=odd=0: the plain count.
static int64_t sym_units_per_block(int64_t units, int grid) {
    int64_t per = (units + grid - 1) / grid;
    if (env_opt("CGX_SYM_PLAN", "odd", 1) && per > 1) per |= 1;
    return per;
}

hipError_t symv_f64(const double *At, int64_t n, int64_t lda, int grid, const double *p, double *prow, double *pcol,
                    double *y, const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                    const int64_t *gate) {
    const int64_t ntiles = sym_tiles(lda);
    if (grid <= 0) return hipErrorInvalidValue;
    const int64_t per = sym_units_per_block(2 * ntiles, grid);
    hipError_t e = symv_tiles_f64(At, 0, ntiles, lda, grid, false, p, prow, pcol, s, gate);
    if (e != hipSuccess) return e;
    return symv_reduce_f64(n, lda, per, prow, pcol, y, pown, dot_out, ws, s, gate);
}

hipError_t symv_tiles_f64(const double *At, int64_t q_base, int64_t count, int64_t lda, int grid, bool tile_runs,
                          const double *p, double *prow, double *pcol, hipStream_t s, const int64_t *gate) {
    if (lda % kSymT || grid <= 0 || count <= 0 ||
        ((reinterpret_cast<uintptr_t>(At) | reinterpret_cast<uintptr_t>(p)) & 15))
        return hipErrorInvalidValue;
    const int64_t per = sym_units_per_block(2 * count, grid);
    auto fn = env_opt("CGX_SYM_PLAN", "nt", 1) ? k_symv_f64<1> : k_symv_f64<0>;
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
    hipLaunchKernelGGL(k_gen_spd_sym, dim3((unsigned)std::min<int64_t>(count, 65536)), dim3(kSymGenNT), 0, s, n,
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
