// cgx_kernels.h -- host-side launchers for the CDNA4 (gfx950) CG kernels.
// Internal to libcgx.so; the public boundary is include/cgx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace cgx {

// Scratch needed by the last-block reductions (one set per stream in use).
struct RedWs {
    double *partials;      // >= kMaxRedBlocks doubles
    unsigned *tickets;     // kTickets counters, zero at rest
};
constexpr int kMaxRedBlocks = 8192;
// Most partials a scalar combine takes (>= kMaxShards, the rank limit).
constexpr int kMaxCombine = 64;
constexpr int kTickets = 8;
enum Ticket { T_MATVEC = 0, T_RESID = 1, T_XR = 2, T_DOT = 3, T_REF_MV = 4 };

// ---- the multi-shard exchange in one process (several row blocks, LOCAL) ---
// Pointers to every shard's copy of something (its p slice, its scalar slot),
// in shard order; passed by value.  On distinct devices they are peer
// pointers (access enabled at context creation): the kernels below run on the
// CONSUMING shard's stream and only read peers' memory -- the same pull a
// hipMemcpyPeerAsync on that stream does -- after the stream has waited for
// the producers' events.
constexpr int kMaxPeers = 32;
struct PeerTable {
    const char *p[kMaxPeers];
};
// dst[q * slice_bytes ...] = src.p[q][0 .. slice_bytes) for every q < cnt
// except q == skip (the consumer's own slice, already in place; skip < 0
// copies every slice): the allgather of p (or of x) in one launch instead of
// cnt - 1 peer copies.
hipError_t gather_slices(const PeerTable &src, int cnt, int skip, int64_t slice_bytes, char *dst, hipStream_t s);
// *out = the cnt partials src.p[q] (fp64), summed in q order: the rank-order
// combine of exchange_scalar read straight from each shard's slot.
hipError_t combine_peers_f64(const PeerTable &src, int cnt, double *out, hipStream_t s);
// F32_REF: the float partials in rank order or (mpich) MPICH's MPI_Allreduce order.
hipError_t combine_peers_f32(const PeerTable &src, int cnt, float *out, hipStream_t s, bool mpich);
// The fp64 combine folded into the kernel that consumes the scalar (no
// launch of its own): every block sums the cnt partials src.p[q] in q order
// (k_combine_peers' sum, so the same bits) and uses it in place of the
// global slot; block 0 also stores it to *out (the global slot) for later
// kernels and the host.  cnt = 0: none (the kernel reads the slot).
struct PeerSum {
    PeerTable src;
    int cnt;
    double *out;
};
// The F32_REF counterpart: the cnt float partials combined in MPICH's
// MPI_Allreduce order (k_combine_peers<float>'s mpich form, the same adds),
// folded into k_dot_ref_f32_blk<kDotXR> (p.Ap) and k_update_p_ref_f32 (r.r).
struct PeerSumF32 {
    PeerTable src;
    int cnt;
    float *out;
};

// CGX_PHASES in-kernel timestamps: a kernel given `ts` stores block 0's entry
// time in ts[0] and block b's exit time in ts[1 + b] (b < kTsMaxBlocks), on
// the device's constant wall clock (hipDeviceAttributeWallClockRate).  No
// event packets between the kernels, so the timeline being measured is the
// one that runs without CGX_PHASES.
constexpr int kTsMaxBlocks = 2047;
constexpr int kTsSlot = kTsMaxBlocks + 1;  // int64 per kernel slot

// Geometry of the fp64 row-streaming matVec, chosen once per (device, rows).
struct MatvecPlan {
    int R = 4;        // rows per wave
    int U = 4;        // 128-column chunks in flight per row
    int nt = 1;       // non-temporal loads of A
    int blocks = 0;   // grid (256-thread blocks), grid-stride over row groups
    int small = 0;    // > 0: k_matvec_small_f64 with this many threads per block (vector in LDS)
};
// R/U/nt/blocks_per_cu <= 0 pick the defaults (env CGX_MV_PLAN="R=..,U=..,nt=..,bpc=.."
// may override).
// cols > 0 (the row length): fewer than 8 whole 128-column chunks per row
// take U = 4 or 2, so all of a row's loads are issued at once.
MatvecPlan plan_matvec_f64(int device, int64_t rows, int R = 0, int U = 0, int nt = -1,
                           int blocks_per_cu = 0, int64_t cols = 0);
// The LDS-staged matVec of small systems (cgx_matvec.hip k_matvec_small_f64):
// rows of lda columns, 2048 <= lda <= 8192; small = 0 (not applicable)
// otherwise.  CGX_MV_SMALL=0 turns it off; CGX_SMALL_PLAN="threads=..,U=..,nt=.."
// picks the block size (512, 1024), chunks per step (4, 8) and A's load policy.
MatvecPlan plan_matvec_small_f64(int device, int64_t rows, int64_t lda);

// ---- fp64 -------------------------------------------------------------------
// out[i] = sum_j A[i*lda+j] v[j]; if pown != nullptr also *dot_out = pown . out
// (last-block reduction, fixed order).
// gate (optional): device word; when non-zero the kernel returns at once
// (device-side convergence gating of queued iterations).
hipError_t matvec_f64(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows,
                      int64_t cols, const double *v, double *out, const double *pown,
                      double *dot_out, const RedWs &ws, hipStream_t s, const int64_t *gate = nullptr,
                      int64_t *ts = nullptr);
// Columns [col_first, col_first+col_count) mod cols (all multiples of 128,
// cols = the padded width): out[i] = (accumulate ? out[i] : 0) + partial row
// sum; optional fused dot as above.  Used to overlap the p exchange with the
// shard's own column block.  col_seg > 0 (not with accumulate): the first
// col_seg columns of the range and the rest are summed separately and added
// (own + rest) -- the bits of a col_seg launch followed by an accumulating
// launch of the rest, in one launch (the unoverlapped iteration of an
// aligned row block, so both forms give the same x).
hipError_t matvec_f64_cols(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t col_first, int64_t col_count, bool accumulate, const double *v, double *out,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate = nullptr, int64_t *ts = nullptr, int64_t col_seg = 0);
// r = b - Ax; p = r (if p); *rr_out = r.r (if rr_out).  Ax == nullptr: Ax = 0
// (r = b - 0.0).  clear2: two int64 the kernel zeroes (the convergence record).
hipError_t residual_f64(int64_t n, const double *b, const double *Ax, double *r, double *p,
                        double *rr_out, const RedWs &ws, hipStream_t s, int64_t *clear2 = nullptr);
// alpha = *rsold / *pAp; x += alpha p; r -= alpha Ap; *rr_out = r.r
hipError_t update_xr_f64(int64_t n, double *x, double *r, const double *p, const double *Ap,
                         const double *rsold, const double *pAp, double *rr_out,
                         const RedWs &ws, hipStream_t s);
// p = r + (*rr / *rsold) p
hipError_t update_p_f64(int64_t n, double *p, const double *r, const double *rr,
                        const double *rsold, hipStream_t s);
// Solver split of the updates: r -= alpha Ap with *rr_out = r.r; then
// x += alpha p and (rr != nullptr) p = r + (*rr / *rsold) p; alpha = *rsold / *pAp.
// With kdone != nullptr update_xp also decides sqrt(*rr) < eps on the device:
// on convergence it skips the p update and stores *kdone = k+1, *rrfinal = *rr
// (and the same pair into hrec[0..1], host-mapped memory, when hrec != nullptr);
// once *kdone is in (0, k] both kernels (update_r via gate) do nothing.
hipError_t update_r_f64(int64_t n, double *r, const double *Ap, const double *rsold, const double *pAp,
                        double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate = nullptr,
                        int64_t *ts = nullptr, const PeerSum *pap_sum = nullptr);
// The two-launch iteration's update (one GPU, small n): x += alpha p;
// r -= alpha Ap; *rr_out = r.r; then (last block) the stopping decision as
// update_xp's, and unless stopped p = r + (*rr_out / *rsold) p.
hipError_t update_xrp_f64(int64_t n, double *x, double *r, double *p, const double *Ap, const double *rsold,
                          const double *pAp, double *rr_out, const RedWs &ws, hipStream_t s, const int64_t *gate,
                          double eps, int64_t k, int64_t *kdone, double *rrfinal, int64_t *hrec,
                          int64_t *ts = nullptr);
// The folded two-launch iteration (one GPU, small n): the matVec forms
// p_k = r + (*rr_new / *rr_old) p_{k-1} for the chunks it multiplies, stores
// p_k's own rows into pnew and fuses *dot_out = p_k . out; then update_xr_stop
// does x += alpha p_k, r -= alpha Ap, *rr_out = r.r and the stopping decision.
hipError_t matvec_fold_f64(const MatvecPlan &pl, const double *A, int64_t lda, int64_t rows, int64_t cols,
                           const double *r, const double *pold, double *pnew, const double *rr_new,
                           const double *rr_old, double *out, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate = nullptr, int64_t *ts = nullptr);
hipError_t update_xr_stop_f64(int64_t n, double *x, double *r, const double *p, const double *Ap,
                              const double *rsold, const double *pAp, double *rr_out, const RedWs &ws, hipStream_t s,
                              const int64_t *gate, double eps, int64_t k, int64_t *kdone, double *rrfinal,
                              int64_t *hrec, int64_t *ts = nullptr);
hipError_t update_xp_f64(int64_t n, double *x, double *p, const double *r, const double *rsold, const double *pAp,
                         const double *rr, hipStream_t s, double eps = -1.0, int64_t k = 0,
                         int64_t *kdone = nullptr, double *rrfinal = nullptr, int64_t *hrec = nullptr,
                         int64_t *ts = nullptr, const PeerSum *rr_sum = nullptr);
hipError_t dot_f64(int64_t n, const double *a, const double *b, double *out,
                   const RedWs &ws, hipStream_t s);
// Rows [row0, row0+nrows) of the counter-hash SPD system; pad columns zeroed.
hipError_t gen_spd_f64(int64_t n, int64_t lda, int64_t row0, int64_t nrows, uint64_t seed,
                       double *A, double *b, hipStream_t s);
// out = sum_{q<cnt} (8-byte slot q of in), in q order (one thread): rank-ordered combine.
hipError_t sum_ordered_f64(const double *in, int cnt, double *out, hipStream_t s);


// 5-point Poisson A.p on a slab of mloc grid rows of width m; ph has one halo
// row above and below.  *dot_out = ph[m..] . Ap when dot_out != nullptr.
hipError_t stencil5_f64(const double *ph, int64_t mloc, int64_t m, double *Ap, double *dot_out, const RedWs &ws,
                        hipStream_t s, const int64_t *gate = nullptr);
// Fused Poisson CG iteration (even m, 16-B-aligned buffers; see the kernels).
// rh, poh, pnh: r, p_{k-1}, p_k slabs with one halo row above and below.
bool poisson_fusable(int64_t mloc, int64_t m);
// part: 0 all rows; 1 interior runs; 2 the two edge runs (+= part 1's p.Ap).
// r_up / r_dn (one process, several slabs): r's top / bottom halo row is read
// in place from the neighbouring slab's boundary row (system-scope loads)
// instead of from rh's halo rows.  rr_sum: *rr is the rank-order sum of the
// slabs' r.r partials, formed by the kernel (block 0 stores it to rr_sum->out).
hipError_t poisson_p_f64(const double *rh, const double *poh, double *pnh, int64_t mloc, int64_t m, const double *rr,
                         const double *rsold, bool first, double *pap_out, const RedWs &ws, hipStream_t s,
                         double eps = -1.0, int64_t k = 0, int64_t *kdone = nullptr, double *rrfinal = nullptr,
                         int part = 0, int64_t *hrec = nullptr, const double *r_up = nullptr,
                         const double *r_dn = nullptr, const PeerSum *rr_sum = nullptr);
// xmode: 1 x += alpha p_k; 0 x untouched, alpha_k to *xalpha; 2 x += alpha_{k-1}
// p_{k-1} (poh, xalpha[0]) then += alpha_k p_k (x every other iteration);
// 3 x += alpha_{k-2} p_{k-2} (pqh, xalpha[0]), alpha_{k-1} p_{k-1} (poh,
// xalpha[1]), alpha_k p_k (x every third iteration).  pap_sum: p.Ap from the
// slabs' partials, as poisson_p_f64's rr_sum.
hipError_t poisson_xr_f64(const double *pnh, const double *poh, const double *pqh, double *x, double *r,
                          int64_t mloc, int64_t m, const double *rsold, const double *pAp, double *rr_out, int xmode,
                          double *xalpha, const RedWs &ws, hipStream_t s, const int64_t *gate = nullptr,
                          const PeerSum *pap_sum = nullptr);
// x += xalpha[0] p (pnh) [then += xalpha[1] p (pbh) when pbh != nullptr] over the
// slab interior: the x updates the last iterations left out.
hipError_t poisson_xflush_f64(const double *pnh, const double *pbh, double *x, int64_t mloc, int64_t m,
                              const double *xalpha, hipStream_t s);
hipError_t fill_f64(double *p, int64_t n, double v, hipStream_t s);
hipError_t fill_f32(float *p, int64_t n, float v, hipStream_t s);

// ---- CGX_SYMMETRIC: A as the upper triangle of 128 x 128 tiles ---------------
// (layout: cgx_symv.hip).  lda is a multiple of 128; At holds sym_tiles(lda)
// tiles of 128*128 doubles; prow 2*sym_tiles(lda)*128 doubles (one row
// partial per unit = half tile, at most), pcol sym_tiles(lda)*128.
int64_t sym_tiles(int64_t lda);
int sym_grid(int device);
// y = A p (rows [0, n)), *dot_out = pown . y when pown != nullptr
hipError_t symv_f64(const double *At, int64_t n, int64_t lda, int grid, const double *p, double *prow, double *pcol,
                    double *y, const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                    const int64_t *gate = nullptr);
// rows [row0, row0+nrows) of A (row-major, leading dimension ld) into the tiles
hipError_t sym_pack_f64(const double *rows, int64_t ld, int64_t row0, int64_t nrows, int64_t n, int64_t lda,
                        double *At, hipStream_t s);
// the counter-hash SPD system of gen_spd_f64, packed; b for all n rows
hipError_t gen_spd_sym_f64(int64_t n, int64_t lda, uint64_t seed, double *At, double *b, hipStream_t s);
// Streamed pieces (CGX_SYMMETRIC | CGX_HOST_STREAM): tiles [q_base, q_base+count)
// held in At (At[0] = tile q_base).  tile_runs: row partials per tile (then
// reduce with per = 1).
hipError_t gen_spd_sym_tiles_f64(int64_t n, int64_t lda, uint64_t seed, int64_t q_base, int64_t count, double *At,
                                 hipStream_t s);
hipError_t gen_b_f64(int64_t n, uint64_t seed, double *b, hipStream_t s);
hipError_t symv_tiles_f64(const double *At, int64_t q_base, int64_t count, int64_t lda, int grid, bool tile_runs,
                          const double *p, double *prow, double *pcol, hipStream_t s, const int64_t *gate = nullptr);
hipError_t symv_reduce_f64(int64_t n, int64_t lda, int64_t per, const double *prow, const double *pcol, double *y,
                           const double *pown, double *dot_out, const RedWs &ws, hipStream_t s,
                           const int64_t *gate = nullptr);
// host copies of the layout helpers (tile index, element offset in a tile)
inline int64_t sym_off_h(int64_t I, int64_t nt) { return I * nt - I * (I - 1) / 2; }
inline int64_t sym_pos_h(int r, int c) {  // kSymNT = 256: unit c / 64, (8 tr + rr, 4 tc + 2 cc + e)
    const int h = c / 64, cc = c % 64;
    const int t = (r / 8) * 16 + (cc >> 2), k = (r % 8) * 2 + ((cc >> 1) & 1);
    return (int64_t)h * 128 * 64 + ((int64_t)k * 256 + t) * 2 + (c & 1);
}

// ---- fp32, serialConjugate.c operation order ---------------------------------
// gate: the device-side convergence record (kernels of an iteration after the
// converged one do nothing); update_p_ref_f32 with kdone makes the stopping
// decision (see k_update_p_ref_f32).
hipError_t matvec_ref_f32(const float *A, int64_t lda, int64_t rows, int64_t cols,
                          const float *v, float *out, hipStream_t s, const int64_t *gate = nullptr);
hipError_t dot_ref_f32(int64_t n, const float *a, const float *b, float *out, hipStream_t s,
                       const int64_t *gate = nullptr);
hipError_t residual_ref_f32(int64_t n, const float *b, const float *Ax, float *r, float *p,
                            hipStream_t s);
hipError_t update_xr_ref_f32(int64_t n, float *x, float *r, const float *p, const float *Ap,
                             const float *rsold, const float *pAp, hipStream_t s, const int64_t *gate = nullptr);
// one launch each: x += p alpha, r -= Ap alpha, *rr = r.r (serialConjugate.c:219-234) /
// r = p = b - Ax, *rr = r.r (:209-212); the same float operations as the separate kernels
// pap_sum (several row blocks in one process): p.Ap summed from the blocks'
// partials in MPICH order instead of read from *pAp, which block 0 stores.
hipError_t update_xr_dot_ref_f32(int64_t n, float *x, float *r, const float *p, const float *Ap, const float *rsold,
                                 const float *pAp, float *rr, hipStream_t s, const int64_t *gate = nullptr,
                                 const PeerSumF32 *pap_sum = nullptr);
hipError_t residual_dot_ref_f32(int64_t n, const float *b, const float *Ax, float *r, float *p, float *rr,
                                hipStream_t s, int64_t *clear2 = nullptr);  // clear2: as residual_f64
// The single-GPU two-launch F32_REF iteration (the same float operations as
// matvec_ref_f32 + dot_ref_f32 + update_xr_dot_ref_f32 + update_p_ref_f32):
// out = A v with *dot_out = pown . out from the matVec's last block (ticket:
// a zeroed counter), then x, r, *rr = r.r, the stopping decision and (unless
// stopped) p = r + p (*rr / *rsold) in one single-block launch.
bool matvec_dot_ref_f32_fusable(const float *A, int64_t lda, const float *v);
hipError_t matvec_dot_ref_f32(const float *A, int64_t lda, int64_t rows, int64_t cols, const float *v, float *out,
                              const float *pown, float *dot_out, unsigned *ticket, hipStream_t s,
                              const int64_t *gate = nullptr);
hipError_t update_xrp_dot_ref_f32(int64_t n, float *x, float *r, float *p, const float *Ap, const float *rsold,
                                  const float *pAp, float *rr, hipStream_t s, const int64_t *gate, double eps,
                                  int64_t k, int64_t *kdone, double *rrfinal, int64_t *hrec);
// rr_sum: likewise for r.r (stored to *rr by block 0)
hipError_t update_p_ref_f32(int64_t n, float *p, const float *r, const float *rr,
                            const float *rsold, hipStream_t s, double eps = -1.0, int64_t k = 0,
                            int64_t *kdone = nullptr, double *rrfinal = nullptr, int64_t *hrec = nullptr,
                            const PeerSumF32 *rr_sum = nullptr);
hipError_t gen_spd_f32(int64_t n, int64_t lda, int64_t row0, int64_t nrows, uint64_t seed,
                       float *A, float *b, hipStream_t s);
// F32_REF combine: rank order (allSum) or, with mpich, MPICH's MPI_Allreduce order.
hipError_t sum_ordered_f32(const float *in, int cnt, float *out, hipStream_t s, bool mpich);

// Each kernel file is its own code object, which HIP loads on a device at
// the first use of one of its kernels.  preload_kernels() loads the ones a
// context will launch from on the current device at context creation
// (overlapped with the CLI's file parsing), so no first launch inside a
// timed solve pays for a load.
hipError_t preload_matvec();
hipError_t preload_vector();
hipError_t preload_poisson();
hipError_t preload_ref_f32();
hipError_t preload_symv();
enum PreloadSet : unsigned { PL_MATVEC = 1, PL_VECTOR = 2, PL_POISSON = 4, PL_REF_F32 = 8, PL_SYMV = 16 };
inline hipError_t preload_kernels(unsigned set) {
    const struct { unsigned bit; hipError_t (*fn)(); } all[] = {
        {PL_MATVEC, preload_matvec}, {PL_VECTOR, preload_vector}, {PL_POISSON, preload_poisson},
        {PL_REF_F32, preload_ref_f32}, {PL_SYMV, preload_symv}};
    for (const auto &e : all)
        if (set & e.bit) {
            const hipError_t r = e.fn();
            if (r != hipSuccess) return r;
        }
    return hipSuccess;
}

}  // namespace cgx
