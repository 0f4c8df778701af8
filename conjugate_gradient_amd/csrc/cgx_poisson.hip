// cgx_poisson.hip -- matrix-free 5-point Poisson operator (configs[4]) and
// the fused two-kernel Poisson CG iteration.
#include "cgx_device.h"

#include <algorithm>
#include <type_traits>

namespace cgx {
namespace {

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
// k_poisson_p_f64 passes the array base and the row's byte offset plus the
// lane's in one 32-bit VGPR (OT = uint32_t; slabs of 4 GiB or more: a 64-bit
// VGPR pair), so its rows step with one VALU add per row shared by the three
// arrays, not a 64-bit scalar add per row and array.
template <bool NT, typename OT = uint32_t>
__device__ __forceinline__ d2 lds2(const double *row, OT off) {
    asm volatile("" : "+v"(off));
    const d2 *p = reinterpret_cast<const d2 *>(reinterpret_cast<const char *>(row) + off);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename OT = uint32_t>
__device__ __forceinline__ void sts2(double *row, OT off, d2 v) {
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

// The fused kernels stream with non-temporal loads and stores, except an
// item's last two rows: those are the next item's first two (its halo) and
// are loaded with default policy so the block that reads them next finds them
// in L2 (profiles/r01_sweep_poisson*.jsonl).
constexpr bool NT = true, HT = true;

// p_k rows (FIRST: p_0 = r_0).  sys: r's row is a neighbouring row block's
// boundary row, read where it lies (the one-process halo pull): system-scope
// 8-B loads, so no line this device's L2 kept from an earlier iteration is
// used (the same loads as the other pull kernels, cgx_device.h load_sys).
// rbase + roff: r's row (byte offset, the lane's included), pbase + poff p_{k-1}'s.
template <bool NTL, bool FIRST, typename OT>
__device__ __forceinline__ d2 pnv(const double *rbase, OT roff, const double *pbase, OT poff, const StripLane &L,
                                  double beta, bool sys = false) {
    d2 rv;
    if (sys) {
        const double *q = reinterpret_cast<const double *>(reinterpret_cast<const char *>(rbase) + roff);
        rv.x = load_sys(q);
        rv.y = load_sys(q + 1);
    } else {
        rv = lds2<NTL>(rbase, roff);
    }
    if constexpr (FIRST) return keep(L.valid, rv);
    // NTL for both rows: an item's last two rows (default policy) are the next item's first two,
    // p_{k-1}'s as well as r's (round 5 briefly streamed p's past L2: 8 % more DRAM reads, 268 -> 283 us)
    const d2 pv = lds2<NTL>(pbase, poff);
    d2 o;
    o.x = __builtin_fma(beta, pv.x, rv.x);
    o.y = __builtin_fma(beta, pv.y, rv.y);
    return keep(L.valid, o);
}
// One side point: byte offset `off` into r and p_{k-1} (wave-uniform: a scalar load).
template <bool FIRST, typename OT>
__device__ __forceinline__ double pns(const double *rbase, const double *pbase, OT off, double beta) {
    const double rv = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(rbase) + off);
    if constexpr (FIRST) return rv;
    else return __builtin_fma(beta, *reinterpret_cast<const double *>(reinterpret_cast<const char *>(pbase) + off), rv);
}

// RBn output rows starting at interior row i: pm, pc carry p_k rows h = i, i+1.
// rdn (one process, several row blocks): r's bottom halo row is the next
// block's first row, read in place instead of from rh's halo row.
template <int RBn, bool FIRST, typename OT>
__device__ __forceinline__ void poisson_p_step(const double *__restrict__ rh, const double *__restrict__ poh,
                                               double *__restrict__ pnh, int64_t mloc, int64_t m, int64_t i,
                                               const StripLane &L, double beta, d2 &pm, d2 &pc, double &acc,
                                               double *eb, const double *rdn) {
    const int lane = threadIdx.x & 63;
    const OT mb = (OT)m * 8, oc0 = (OT)((i + 1) * m) * 8, lo = (OT)L.off;
    d2 pr[RBn], ce[RBn];
    double el[RBn], er[RBn];
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const OT oc = oc0 + (OT)t * mb, od = oc + mb;  // centre row (halo coordinates) of output row i+t, the row below
        const bool pull = rdn && i + t + 1 == mloc;  // the row below is the bottom halo row
        // HT: the last two rows are the next item's first two (its halo):
        // default-policy loads keep them in L2 for the block that reads them next
        pr[t] = (HT && t >= RBn - 2) ? pnv<false, FIRST>(pull ? rdn : rh, pull ? lo : od + lo, poh, od + lo, L, beta, pull)
                                     : pnv<NT, FIRST>(pull ? rdn : rh, pull ? lo : od + lo, poh, od + lo, L, beta, pull);
        el[t] = L.has_l ? pns<FIRST>(rh, poh, oc + (OT)(L.jw - 1) * 8, beta) : 0.0;
        er[t] = L.has_r ? pns<FIRST>(rh, poh, oc + (OT)(L.jw + 128) * 8, beta) : 0.0;
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
            sts2<NT>(pnh, oc0 + (OT)t * mb + lo, ce[t]);
            if (i + t == mloc - 1) sts2<NT>(pnh, (OT)((mloc + 1) * m) * 8 + lo, dn);  // bottom halo row of p_k
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

// XCD bands (CGX_POISSON_BANDS=1, one item range of whole runs): the
// blocks of XCD x (blockIdx % 8, the dispatcher's round-robin) take the
// items of the x-th eighth of the runs, strip-fastest, so an item's left and
// right neighbours (whose edge columns it loads as side points) and the item
// below (whose first two rows are its last two) are fetched through the same
// L2 at about the same time.  Without bands those neighbours are taken by
// blocks of other XCDs.  The v-th item of this block within its band, or -1.
// bands = 1 + rot: band x walks its items starting rot * x items in (mod its
// count), so the eight XCDs' streams (bands 64 MiB apart at m = 8192) sit at
// different offsets (CGX_POISSON_BAND_ROT; an experiment, as for k_symv_f64).
struct Band {
    int64_t first, count, stride, start, rot;
};
__device__ __forceinline__ Band band_of(int64_t w0, int64_t nitems, int64_t nstrips, int bands) {
    Band b;
    const int64_t nruns = nitems / nstrips, x = blockIdx.x % 8;
    const int64_t r0 = nruns * x / 8, r1 = nruns * (x + 1) / 8;
    b.first = w0 + r0 * nstrips;
    b.count = (r1 - r0) * nstrips;
    b.stride = gridDim.x / 8;
    b.start = blockIdx.x / 8;
    b.rot = b.count > 0 ? (int64_t)(bands - 1) * x % b.count : 0;
    return b;
}
__device__ __forceinline__ int64_t band_item(const Band &b, int64_t v) {
    const int64_t q = v + b.rot;
    return b.first + (q >= b.count ? q - b.count : q);
}

// Work items [w0, w0+cnt1) then [w2, w2+cnt2) (the whole slab, or, when
// the r halo exchange overlaps the kernel, the slab's interior runs first
// and its two edge runs after the exchange).
struct ItemRanges {
    int64_t w0, cnt1, w2, cnt2;
};

// The halo pull (one process, several row blocks; rank mode and one block:
// both null): r's top halo row is the previous block's last row (rup), its
// bottom halo row the next block's first (rdn), read where they lie.  The
// producers' r updates are ordered before this kernel by the r.r combine's
// cross-stream events; the copies into rh's halo rows that did this before
// round 5 moved the same bytes, so p_k is the same bits.
struct HaloPull {
    const double *up, *dn;
};

template <int RB, bool FIRST, typename OT>
__device__ __forceinline__ double poisson_p_body(const double *__restrict__ rh, const double *__restrict__ poh,
                                                 double *__restrict__ pnh, int64_t mloc, int64_t m, int64_t nstrips,
                                                 int64_t rpi, ItemRanges ir, double beta, double *edge, int bands,
                                                 HaloPull hp) {
    double acc = 0.0;
    int par = 0;
    const Band bd = bands ? band_of(ir.w0, ir.cnt1, nstrips, bands) : Band{0, 0, 0, 0, 0};
    const int64_t vend = bands ? bd.count : ir.cnt1 + ir.cnt2;
    for (int64_t v = bands ? bd.start : blockIdx.x; v < vend; v += bands ? bd.stride : gridDim.x) {
        const int64_t w = bands ? band_item(bd, v) : v < ir.cnt1 ? ir.w0 + v : ir.w2 + (v - ir.cnt1);
        const StripLane L = strip_lane(w, nstrips, m);
        const int64_t i0 = (w / nstrips) * rpi;
        const int64_t i1 = (i0 + rpi < mloc) ? i0 + rpi : mloc;
        const bool pull = hp.up && i0 == 0;  // the top halo row
        const OT lo = (OT)L.off, o0 = (OT)(i0 * m) * 8 + lo, o1 = (OT)((i0 + 1) * m) * 8 + lo;
        d2 pm = pnv<NT && !HT, FIRST>(pull ? hp.up : rh, pull ? lo : o0, poh, o0, L, beta, pull);
        d2 pc = pnv<NT && !HT, FIRST>(rh, o1, poh, o1, L, beta);
        if (L.valid && i0 == 0) sts2<NT>(pnh, lo, pm);  // top halo row of p_k
        int64_t i = i0;
        for (; i + RB <= i1; i += RB, par ^= 1)
            poisson_p_step<RB, FIRST, OT>(rh, poh, pnh, mloc, m, i, L, beta, pm, pc, acc,
                                          edge + par * (kWaves * 2 * kEdgeRB), hp.dn);
        for (; i < i1; ++i, par ^= 1)
            poisson_p_step<1, FIRST, OT>(rh, poh, pnh, mloc, m, i, L, beta, pm, pc, acc,
                                         edge + par * (kWaves * 2 * kEdgeRB), hp.dn);
    }
    return acc;
}

// The one-process pull's arguments (several row blocks): the halo pull above,
// and rr_sum.cnt > 0: r.r_k is the rank-order sum of the blocks' partials,
// formed here (k_combine_peers' sum, the same bits) instead of by a combine
// kernel of its own; block 0 stores it.  One block and rank mode launch the
// NoPull instantiation, which has neither the arguments nor the pull tests
// (its code is the pre-pull kernel's; profiles/r05_poisson_regression.json).
struct NoPull {};
struct PullArgs {
    HaloPull hp;
    PeerSum rr_sum;
};
// p.Ap for the xr kernels: the slot, or the blocks' partials summed in rank order
__device__ __forceinline__ double pap_of(const NoPull &, const double *pAp) { return *pAp; }
__device__ __forceinline__ double pap_of(const PeerSum &ps, const double *pAp) {
    return ps.cnt ? peer_sum_wave(ps) : *pAp;
}
template <int RB, class PA, typename OT>
__global__ __launch_bounds__(kNT) void k_poisson_p_f64(const double *__restrict__ rh, const double *__restrict__ poh,
                                                       double *__restrict__ pnh, int64_t mloc, int64_t m,
                                                       int64_t nstrips, int64_t rpi, ItemRanges ir, const double *rr,
                                                       const double *rsold, int first, ConvArgs cv, double *dot_out,
                                                       int add_to_out, double *partials, unsigned *ticket, int bands,
                                                       PA pa) {
    static_assert(RB <= kEdgeRB, "edge buffer");
    constexpr bool PULL = std::is_same<PA, PullArgs>::value;
    __shared__ double edge[2 * kWaves * 2 * kEdgeRB];
    // a launch after the stop returns before it reads anything (the slabs'
    // r.r partials included, which the folded combine would read over xGMI and
    // store again)
    if (cv.kdone && *cv.kdone != 0) return;
    double rrk = 0.0;  // r.r_k (not read when first)
    if (!first) {
        if constexpr (PULL) rrk = pa.rr_sum.cnt ? peer_sum_wave(pa.rr_sum) : *rr;
        else rrk = *rr;
    }
    if (cv.kdone) {
        if (!first && cv.eps >= 0.0 && sqrt(rrk) < cv.eps) {  // the same decision in every block
            if (blockIdx.x == 0 && threadIdx.x == 0) record_convergence(cv, cv.k, rrk);
            return;
        }
    }
    HaloPull h{nullptr, nullptr};
    if constexpr (PULL) h = pa.hp;
    // p_0 = r_0 (first) has its own instantiation: no p_{k-1} loads
    const double acc = first ? poisson_p_body<RB, true, OT>(rh, poh, pnh, mloc, m, nstrips, rpi, ir, 0.0, edge, bands, h)
                             : poisson_p_body<RB, false, OT>(rh, poh, pnh, mloc, m, nstrips, rpi, ir,
                                                             cg_ratio(rrk, *rsold), edge, bands, h);
    grid_sum_last_block(acc, partials, ticket, dot_out, add_to_out != 0);
}

// k_poisson_xr_f64 (iteration k): alpha = *rsold / *pAp; x += alpha p_k and
// r -= alpha A p_k with A p_k recomputed from p_k (halo included);
// *rr_out = r.r.  Skipped once *gate != 0.
//
// x's update every other iteration (XM, the solver's CGX_POISSON_XDEFER):
//   XM = 1: x += alpha_k p_k (every iteration: 40 B per point);
//   XM = 0: x is not touched; alpha_k goes to *xalpha (24 B per point);
//   XM = 2: x += alpha_{k-1} p_{k-1} (p_{k-1} = the other slab, which the next
//           k_poisson_p overwrites only after this kernel; alpha_{k-1} from
//           *xalpha), then x += alpha_k p_k (48 B per point).
// The two FMAs are XM = 1's two iterations' own, in the same order, so x is
// bit for bit the every-iteration update's; a solve that ends after an XM = 0
// iteration finishes x with k_poisson_xflush_f64.  60 instead of 64 B per
// point per iteration over a pair of iterations.
template <int RBn, int XM>
__device__ __forceinline__ void poisson_xr_step(const double *__restrict__ pnh, const double *__restrict__ poh,
                                                const double *__restrict__ pqh, double *__restrict__ x,
                                                double *__restrict__ r, int64_t m, int64_t i, const StripLane &L,
                                                double alpha, double alpha_prev, double alpha_prev2, d2 &pm, d2 &pc,
                                                double &acc, double *eb) {
    const int lane = threadIdx.x & 63;
    d2 pr[RBn], xv[RBn], rv[RBn], ce[RBn], po[RBn], pq[RBn];
    double el[RBn], er[RBn];
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const int64_t hc = (i + t + 1) * m, ic = (i + t) * m;
        pr[t] = keep(L.valid, (HT && t >= RBn - 2) ? lds2<false>(pnh + hc + m, L.off) : lds2<NT>(pnh + hc + m, L.off));
        if constexpr (XM != 0) xv[t] = lds2<NT>(x + ic, L.off);
        if constexpr (XM >= 2) po[t] = lds2<NT>(poh + hc, L.off);
        if constexpr (XM == 3) pq[t] = lds2<NT>(pqh + hc, L.off);
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
        if constexpr (XM == 3) {  // alpha_{k-2} p_{k-2}, alpha_{k-1} p_{k-1}, alpha_k p_k: their order
            xn.x = __builtin_fma(alpha_prev2, pq[t].x, xv[t].x);
            xn.y = __builtin_fma(alpha_prev2, pq[t].y, xv[t].y);
            xn.x = __builtin_fma(alpha_prev, po[t].x, xn.x);
            xn.y = __builtin_fma(alpha_prev, po[t].y, xn.y);
            xn.x = __builtin_fma(alpha, ce[t].x, xn.x);
            xn.y = __builtin_fma(alpha, ce[t].y, xn.y);
        } else if constexpr (XM == 2) {
            xn.x = __builtin_fma(alpha_prev, po[t].x, xv[t].x);
            xn.y = __builtin_fma(alpha_prev, po[t].y, xv[t].y);
            xn.x = __builtin_fma(alpha, ce[t].x, xn.x);
            xn.y = __builtin_fma(alpha, ce[t].y, xn.y);
        } else if constexpr (XM == 1) {
            xn.x = __builtin_fma(alpha, ce[t].x, xv[t].x);
            xn.y = __builtin_fma(alpha, ce[t].y, xv[t].y);
        }
        rn.x = __builtin_fma(-alpha, o.x, rv[t].x);
        rn.y = __builtin_fma(-alpha, o.y, rv[t].y);
        acc += L.valid ? rn.x * rn.x + rn.y * rn.y : 0.0;
        if (L.valid) {
            if constexpr (XM != 0) sts2<NT>(x + (i + t) * m, L.off, xn);
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

// Every x mode runs on XM = 1's grid (launch_poisson_xr), so the r.r
// partials add in the same order whichever variant runs (a thread adds its
// rows in row order whatever RB is): x is the same bits with and without the
// deferral.
// PS: PeerSum (one process, several row blocks: p.Ap summed here from the
// blocks' partials, as k_poisson_p_f64's r.r) or NoPull (read *pAp).
template <int RB, int XM, class PS>
__global__ __launch_bounds__(kNT) void k_poisson_xr_f64(const double *__restrict__ pnh, const double *__restrict__ poh,
                                                        const double *__restrict__ pqh, double *__restrict__ x,
                                                        double *__restrict__ r, int64_t mloc,
                                                        int64_t m, int64_t nstrips, int64_t rpi, int64_t nitems,
                                                        int reverse, const double *rsold, const double *pAp,
                                                        double *rr_out, double *xalpha, double *partials,
                                                        unsigned *ticket, const int64_t *gate, int bands,
                                                        PS pap_sum) {
    static_assert(RB <= kEdgeRB, "edge buffer");
    __shared__ double edge[2 * kWaves * 2 * kEdgeRB];
    if (gate && *gate) return;
    const double alpha = cg_ratio(*rsold, pap_of(pap_sum, pAp));
    // XM = 2: alpha_{k-1} = xalpha[0]; XM = 3: alpha_{k-2} = xalpha[0], alpha_{k-1} = xalpha[1]
    const double alpha_prev = XM == 2 ? xalpha[0] : XM == 3 ? xalpha[1] : 0.0;
    const double alpha_prev2 = XM == 3 ? xalpha[0] : 0.0;
    double acc = 0.0;
    int par = 0;
    const Band bd = bands ? band_of(0, nitems, nstrips, bands)
                          : Band{0, nitems, (int64_t)gridDim.x, (int64_t)blockIdx.x, 0};
    for (int64_t v = bd.start; v < bd.count; v += bd.stride) {
        // reverse: walk the slab (each band) from its end, where the previous
        // kernel (k_poisson_p, forward) last wrote p_k, so the first bytes read
        // may still sit in the 256 MB MALL
        const int64_t w = band_item(bd, reverse ? bd.count - 1 - v : v);
        const StripLane L = strip_lane(w, nstrips, m);
        const int64_t i0 = (w / nstrips) * rpi;
        const int64_t i1 = (i0 + rpi < mloc) ? i0 + rpi : mloc;
        d2 pm = keep(L.valid, lds2<NT && !HT>(pnh + i0 * m, L.off));
        d2 pc = keep(L.valid, lds2<NT && !HT>(pnh + (i0 + 1) * m, L.off));
        int64_t i = i0;
        for (; i + RB <= i1; i += RB, par ^= 1)
            poisson_xr_step<RB, XM>(pnh, poh, pqh, x, r, m, i, L, alpha, alpha_prev, alpha_prev2, pm, pc, acc,
                                            edge + par * (kWaves * 2 * kEdgeRB));
        for (; i < i1; ++i, par ^= 1)
            poisson_xr_step<1, XM>(pnh, poh, pqh, x, r, m, i, L, alpha, alpha_prev, alpha_prev2, pm, pc, acc,
                                           edge + par * (kWaves * 2 * kEdgeRB));
    }
    // XM = 0: alpha_k for the next iteration's (or the flush's) x update.  Read
    // by a later kernel on this stream only (kernel boundary = ordering).
    if (XM == 0 && blockIdx.x == 0 && threadIdx.x == 0) *xalpha = alpha;
    grid_sum_last_block(acc, partials, ticket, rr_out);
}

// The x update an XM = 0 iteration left out: x += alpha p_k over the slab's
// interior (p_k's slab pnh, alpha from *xalpha).  The same FMA as the xr
// kernel's, so x is bit for bit the every-iteration update's.
// Even m: npts is even and both slabs 16-B aligned, so it runs on pairs.
// With a second slab pbh (x every third iteration, two updates left out):
// x += xalpha[0] pnh, then += xalpha[1] pbh, in that order.
__global__ __launch_bounds__(kNT) void k_poisson_xflush_f64(const double *__restrict__ pnh,
                                                            const double *__restrict__ pbh, double *__restrict__ x,
                                                            int64_t npts, const double *xalpha) {
    const double alpha = xalpha[0], alpha_b = pbh ? xalpha[1] : 0.0;
    const d2 *p = reinterpret_cast<const d2 *>(pnh), *pb = reinterpret_cast<const d2 *>(pbh);
    d2 *xv = reinterpret_cast<d2 *>(x);
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < npts / 2; i += (int64_t)gridDim.x * kNT) {
        const d2 pv = __builtin_nontemporal_load(p + i), xo = __builtin_nontemporal_load(xv + i);
        d2 o;
        o.x = __builtin_fma(alpha, pv.x, xo.x);
        o.y = __builtin_fma(alpha, pv.y, xo.y);
        if (pbh) {
            const d2 qv = __builtin_nontemporal_load(pb + i);
            o.x = __builtin_fma(alpha_b, qv.x, o.x);
            o.y = __builtin_fma(alpha_b, qv.y, o.y);
        }
        __builtin_nontemporal_store(o, xv + i);
    }
}

// ---- the software-pipelined x catch-up kernel -------------------------------
// Side-point addresses of one row (row base `row`) for the pipelined kernel,
// whose loads are unconditional.  Only the block's outer waves use them (the
// inner waves take their neighbours' edges from LDS); with `hot` set, every
// other wave loads that one L2-resident double instead, so the only side loads
// that reach memory are the outer waves' (as in the plain kernels).  Without
// it every wave loads its neighbours' edge columns: lines the neighbouring
// wave streams with non-temporal loads.
struct SidePts {
    const double *l, *r;
};
__device__ __forceinline__ SidePts side_pts(const double *row, const StripLane &L, int64_t m, const double *__restrict__ hot) {
    SidePts s;
    s.l = (L.has_l || !hot) ? row + (L.jw > 0 ? L.jw - 1 : 0) : hot;
    s.r = (L.has_r || !hot) ? row + (L.jw + 128 < m ? L.jw + 128 : m - 1) : hot;
    return s;
}

// ---- k_poisson_xr_f64, software-pipelined (the x catch-up, XM = 2 / 3) --------
// The same arithmetic, row by row and item by item in the same order as
// k_poisson_xr_f64 (so r, x and every r.r partial are the same bits), with
// the loads of the next step -- or, at an item's last step, of the next
// item's first step and its two prefix rows -- issued before this step's
// arithmetic and stores.  In the plain kernel a step's loads go out only
// after the previous step's stores, and the wait for its own last loads then
// also waits for those stores (loads and stores share vmcnt on gfx9-class
// parts): one store round trip per step.  Here every load and store is
// unconditional, so the compiler's counts stay exact and no wait covers a
// store.  For full strips only (m a multiple of 2 * kNT: every lane valid),
// items of exactly NS * RBn rows (mloc a multiple of that), NT and HT on (the
// defaults); the launcher falls back to k_poisson_xr_f64 otherwise.
// Side points are loaded by every wave (wave-uniform addresses, clamped to
// the grid): lanes 0 / 63 of waves 1-2 read them from LDS as before, so the
// values used are unchanged; the extra loads hit lines the neighbouring wave
// fetches anyway.
template <int RBn, int XM>
struct XrSet {
    d2 pr[RBn], xv[RBn], po[RBn], pq[RBn], rv[RBn];
    double el[RBn], er[RBn];
};
template <int RBn, int XM>
__device__ __forceinline__ void xr_pipe_load(XrSet<RBn, XM> &S, const double *__restrict__ pnh,
                                             const double *__restrict__ poh, const double *__restrict__ pqh,
                                             const double *__restrict__ x, const double *__restrict__ r, int64_t m,
                                             int64_t i, const StripLane &L, bool last, const double *__restrict__ hot) {
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const int64_t hc = (i + t + 1) * m, ic = (i + t) * m;
        // the item's last two rows are the next item's first two (HT): default policy, kept in L2
        S.pr[t] = (last && t >= RBn - 2) ? lds2<false>(pnh + hc + m, L.off) : lds2<true>(pnh + hc + m, L.off);
        if constexpr (XM != 0) S.xv[t] = lds2<true>(x + ic, L.off);
        if constexpr (XM >= 2) S.po[t] = lds2<true>(poh + hc, L.off);
        if constexpr (XM == 3) S.pq[t] = lds2<true>(pqh + hc, L.off);
        S.rv[t] = lds2<true>(r + ic, L.off);
        const SidePts sp = side_pts(pnh + hc, L, m, hot);
        S.el[t] = *sp.l;
        S.er[t] = *sp.r;
    }
}
template <int RBn, int XM>
__device__ __forceinline__ void xr_pipe_step(const XrSet<RBn, XM> &S, double *__restrict__ x,
                                             double *__restrict__ r, int64_t m, int64_t i, const StripLane &L,
                                             double alpha, double alpha_prev, double alpha_prev2, d2 &pm, d2 &pc,
                                             double &acc, double *eb) {
    const int lane = threadIdx.x & 63;
    d2 ce[RBn];
#pragma unroll
    for (int t = 0; t < RBn; ++t) ce[t] = t == 0 ? pc : S.pr[t - 1];
    edges_put<RBn>(eb, L, ce);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RBn; ++t) {
        const d2 up = t == 0 ? pm : (t == 1 ? pc : S.pr[t - 2]);
        const d2 dn = S.pr[t];
        const double lw = edge_l(eb, L, t, L.has_l ? S.el[t] : 0.0), rw = edge_r(eb, L, t, L.has_r ? S.er[t] : 0.0);
        double l = __shfl_up(ce[t].y, 1, 64);
        double rt = __shfl_down(ce[t].x, 1, 64);
        l = lane == 0 ? lw : l;
        rt = lane == 63 ? rw : rt;
        d2 o;
        o.x = 4.0 * ce[t].x - up.x - dn.x - l - ce[t].y;
        o.y = 4.0 * ce[t].y - up.y - dn.y - ce[t].x - rt;
        d2 xn, rn;
        if constexpr (XM == 3) {
            xn.x = __builtin_fma(alpha_prev2, S.pq[t].x, S.xv[t].x);
            xn.y = __builtin_fma(alpha_prev2, S.pq[t].y, S.xv[t].y);
            xn.x = __builtin_fma(alpha_prev, S.po[t].x, xn.x);
            xn.y = __builtin_fma(alpha_prev, S.po[t].y, xn.y);
            xn.x = __builtin_fma(alpha, ce[t].x, xn.x);
            xn.y = __builtin_fma(alpha, ce[t].y, xn.y);
        } else if constexpr (XM == 2) {
            xn.x = __builtin_fma(alpha_prev, S.po[t].x, S.xv[t].x);
            xn.y = __builtin_fma(alpha_prev, S.po[t].y, S.xv[t].y);
            xn.x = __builtin_fma(alpha, ce[t].x, xn.x);
            xn.y = __builtin_fma(alpha, ce[t].y, xn.y);
        } else if constexpr (XM == 1) {
            xn.x = __builtin_fma(alpha, ce[t].x, S.xv[t].x);
            xn.y = __builtin_fma(alpha, ce[t].y, S.xv[t].y);
        }
        rn.x = __builtin_fma(-alpha, o.x, S.rv[t].x);
        rn.y = __builtin_fma(-alpha, o.y, S.rv[t].y);
        acc += rn.x * rn.x + rn.y * rn.y;
        if constexpr (XM != 0) sts2<true>(x + (i + t) * m, L.off, xn);
        sts2<true>(r + (i + t) * m, L.off, rn);
    }
    if constexpr (RBn >= 2) {
        pm = S.pr[RBn - 2];
        pc = S.pr[RBn - 1];
    } else {
        pm = pc;
        pc = S.pr[0];
    }
}
template <int RBn, int NS, int XM, class PS>
__global__ __launch_bounds__(kNT) void k_poisson_xr_pipe_f64(const double *__restrict__ pnh,
                                                             const double *__restrict__ poh,
                                                             const double *__restrict__ pqh, double *__restrict__ x,
                                                             double *__restrict__ r, int64_t m, int64_t nstrips,
                                                             int64_t nitems, int reverse, const double *rsold,
                                                             const double *pAp, double *rr_out, double *xalpha,
                                                             double *partials, unsigned *ticket, const int64_t *gate,
                                                             int bands, const double *__restrict__ hot,
                                                             PS pap_sum) {
    static_assert(RBn <= kEdgeRB && NS % 2 == 0, "edge buffer / set parity");
    constexpr int64_t kRpi = RBn * NS;
    __shared__ double edge[2 * kWaves * 2 * kEdgeRB];
    if (gate && *gate) return;
    const double alpha = cg_ratio(*rsold, pap_of(pap_sum, pAp));
    const double alpha_prev = XM == 2 ? xalpha[0] : XM == 3 ? xalpha[1] : 0.0;
    const double alpha_prev2 = XM == 3 ? xalpha[0] : 0.0;
    double acc = 0.0;
    const Band bd = bands ? band_of(0, nitems, nstrips, bands)
                          : Band{0, nitems, (int64_t)gridDim.x, (int64_t)blockIdx.x, 0};
    if (bd.start < bd.count) {
        auto item_of = [&](int64_t v) { return band_item(bd, reverse ? bd.count - 1 - v : v); };
        int64_t v = bd.start, w = item_of(v);
        StripLane L = strip_lane(w, nstrips, m);
        int64_t i0 = (w / nstrips) * kRpi;
        d2 pm = lds2<false>(pnh + i0 * m, L.off), pc = lds2<false>(pnh + (i0 + 1) * m, L.off);
        XrSet<RBn, XM> S[2];
        xr_pipe_load<RBn, XM>(S[0], pnh, poh, pqh, x, r, m, i0, L, NS == 1, hot);
        for (;;) {
            // the next item (the last one again when there is none: loaded, never used)
            const int64_t vn = v + bd.stride < bd.count ? v + bd.stride : v;
            const int64_t wn = item_of(vn);
            const StripLane Ln = strip_lane(wn, nstrips, m);
            const int64_t i0n = (wn / nstrips) * kRpi;
            d2 pmn, pcn;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if (s + 1 < NS) {
                    xr_pipe_load<RBn, XM>(S[(s + 1) & 1], pnh, poh, pqh, x, r, m, i0 + (s + 1) * RBn, L,
                                          s + 2 == NS, hot);
                } else {
                    pmn = lds2<false>(pnh + i0n * m, Ln.off);
                    pcn = lds2<false>(pnh + (i0n + 1) * m, Ln.off);
                    xr_pipe_load<RBn, XM>(S[(s + 1) & 1], pnh, poh, pqh, x, r, m, i0n, Ln, NS == 1, hot);
                }
                xr_pipe_step<RBn, XM>(S[s & 1], x, r, m, i0 + s * RBn, L, alpha, alpha_prev, alpha_prev2, pm, pc, acc,
                                      edge + (s & 1) * (kWaves * 2 * kEdgeRB));
            }
            if (vn == v) break;
            v = vn;
            L = Ln;
            i0 = i0n;
            pm = pmn;
            pc = pcn;
        }
    }
    if (XM == 0 && blockIdx.x == 0 && threadIdx.x == 0) *xalpha = alpha;
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

}  // namespace

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

// Fused Poisson kernels: the plan.  Rows per step RB (1, 2, 4, 8), rows per
// work item, XCD bands, the xr kernels' walk direction and the grid, from
// CGX_POISSON_PLAN="rb=..,rows=..,bands=..,reverse=..,blocks=.." (keys
// optional).  Defaults RB=8, 8-row items, XCD bands on, the xr kernels walking
// backwards, an occupancy-sized grid: measured at m=8192 over RB 2..8, items
// of 8..128 rows and 1024..4096 blocks (profiles/r01_sweep_poisson*.jsonl;
// short items keep the rows in flight in a narrow band, 64- and 128-row items
// are 7-20 % slower), re-checked on round 4's final tree
// (profiles/r04_poisson_knobs_ab.jsonl, profiles/r04_poisson_rows_ab.jsonl).
struct PoissonPlan {
    int rb, bands, reverse, blocks, pipe;
    int64_t nstrips, rpi, nitems;
};
static PoissonPlan poisson_plan(int64_t mloc, int64_t m) {
    PoissonPlan p;
    p.rb = env_opt("CGX_POISSON_PLAN", "rb", 8);
    // XCD bands: 1341 vs 1288 it/s at m = 8192, two interleaved rounds
    // (profiles/r03_poisson_bands_ab.jsonl)
    p.bands = env_opt("CGX_POISSON_PLAN", "bands", 1);
    p.reverse = env_opt("CGX_POISSON_PLAN", "reverse", 1);
    p.blocks = env_opt("CGX_POISSON_PLAN", "blocks", 0);
    p.pipe = env_opt("CGX_POISSON_PLAN", "pipe", 1);  // 0: the x catch-up on the plain kernel (the same bits)
    p.nstrips = (m + 2 * kNT - 1) / (2 * kNT);
    p.rpi = std::max(1, env_opt("CGX_POISSON_PLAN", "rows", 8));
    p.nitems = p.nstrips * ((mloc + p.rpi - 1) / p.rpi);
    return p;
}

// Every block resident at once (occupancy x CUs), capped by the work items
// and the reduction slots; the plan's `blocks` overrides.
static int64_t resident_grid(const PoissonPlan &pl, const void *fn, int64_t nitems) {
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
    const int64_t g = pl.blocks > 0 ? pl.blocks : (int64_t)per_cu * cu_count(dev);
    return std::max<int64_t>(1, std::min<int64_t>({g, nitems, kMaxRedBlocks}));
}

bool poisson_fusable(int64_t mloc, int64_t m) { return mloc > 0 && m > 0 && (m & 1) == 0; }

static PeerSum no_sum() {
    PeerSum z{};
    z.cnt = 0;
    return z;
}

template <int RB, class PA, typename OT>
static void launch_p(const PoissonPlan &pl, hipStream_t s, const double *rh, const double *poh, double *pnh,
                     int64_t mloc, int64_t m, const double *rr, const double *rsold, int first, ConvArgs cv,
                     double *pap_out, const RedWs &ws, ItemRanges ir, int add_to_out, const PA &pa) {
    auto fn = k_poisson_p_f64<RB, PA, OT>;
    int64_t grid = resident_grid(pl, reinterpret_cast<const void *>(fn), ir.cnt1 + ir.cnt2);
    const int bands = pl.bands && ir.cnt2 == 0 && ir.cnt1 % pl.nstrips == 0 && grid >= 8 ? 1 : 0;
    if (bands) grid &= ~int64_t(7);
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kNT), 0, s, rh, poh, pnh, mloc, m, pl.nstrips, pl.rpi, ir, rr,
                       rsold, first, cv, pap_out, add_to_out, ws.partials, ws.tickets + T_MATVEC, bands, pa);
}
template <int RB>
static void launch_poisson_p(const PoissonPlan &pl, hipStream_t s, const double *rh, const double *poh, double *pnh,
                             int64_t mloc, int64_t m, const double *rr, const double *rsold, int first, ConvArgs cv,
                             double *pap_out, const RedWs &ws, ItemRanges ir, int add_to_out, HaloPull hp,
                             const PeerSum &rr_sum) {
    // every byte offset into a slab (halo rows included) fits 32 bits: the one-VGPR offsets
    const bool o32 = (mloc + 2) * m * 8 <= (int64_t)UINT32_MAX;
    if (hp.up || hp.dn || rr_sum.cnt) {
        const PullArgs pa{hp, rr_sum};
        if (o32) launch_p<RB, PullArgs, uint32_t>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir,
                                                  add_to_out, pa);
        else launch_p<RB, PullArgs, uint64_t>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir,
                                              add_to_out, pa);
    } else if (o32) {
        launch_p<RB, NoPull, uint32_t>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add_to_out,
                                       NoPull{});
    } else {
        launch_p<RB, NoPull, uint64_t>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add_to_out,
                                       NoPull{});
    }
}
template <int XM, class PS>
using XrFn = void (*)(const double *, const double *, const double *, double *, double *, int64_t, int64_t, int64_t,
                      int64_t, int64_t, int, const double *, const double *, double *, double *, double *, unsigned *,
                      const int64_t *, int, PS);
template <int XM, class PS>
static XrFn<XM, PS> xr_fn_rb(int rb) {
    switch (rb) {
        case 1: return k_poisson_xr_f64<1, XM, PS>;
        case 2: return k_poisson_xr_f64<2, XM, PS>;
        case 8: return k_poisson_xr_f64<8, XM, PS>;
        default: return k_poisson_xr_f64<4, XM, PS>;
    }
}
// Every x mode runs on the grid of the every-iteration kernel at the plan's
// RB (its occupancy), so the r.r partials add in the same order whichever
// variant runs.  XM = 2 / 3 carry p_{k-1} (and p_{k-2}): RB / 2 rows per step
// (XM = 3 at RB = 8: 130 VGPRs).  The x catch-up (XM = 2 / 3) runs the
// software-pipelined kernel where it applies (full strips, 8-row items):
// 1489-1496 vs 1471-1480 it/s at m = 8192, three interleaved rounds, the same
// bits (profiles/r04_poisson_catchup_ab.jsonl).  The pipelined form of the
// other kernels measured no better (XM = 0: 283 vs 276 us in the kernel trace;
// k_poisson_p: 1346-1464 vs 1475 it/s) and was removed in round 5.
template <int XM, class PS>
static void launch_poisson_xr(const PoissonPlan &pl, hipStream_t s, const double *pnh, const double *poh,
                              const double *pqh, double *x, double *r, int64_t mloc, int64_t m, const double *rsold,
                              const double *pAp, double *rr_out, double *xalpha, const RedWs &ws,
                              const int64_t *gate, const PS &pap_sum) {
    const int rb = XM >= 2 && pl.rb > 1 ? pl.rb / 2 : pl.rb;
    const XrFn<XM, PS> fn = xr_fn_rb<XM, PS>(rb);
    int64_t grid = resident_grid(pl, reinterpret_cast<const void *>(xr_fn_rb<1, PS>(pl.rb)), pl.nitems);
    const int bands = pl.bands && grid >= 8 ? 1 : 0;
    if (bands) grid &= ~int64_t(7);
    if (XM >= 2 && pl.pipe && m % (2 * kNT) == 0 && pl.rpi == 8 && mloc % 8 == 0) {
        auto fp = k_poisson_xr_pipe_f64<4, 2, XM, PS>;
        hipLaunchKernelGGL(fp, dim3((unsigned)grid), dim3(kNT), 0, s, pnh, poh, pqh, x, r,
                           m, pl.nstrips, pl.nitems, pl.reverse, rsold, pAp, rr_out, xalpha, ws.partials,
                           ws.tickets + T_XR, gate, bands, rsold, pap_sum);
        return;
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(kNT), 0, s, pnh, poh, pqh, x, r, mloc, m, pl.nstrips, pl.rpi,
                       pl.nitems, pl.reverse, rsold, pAp, rr_out, xalpha, ws.partials, ws.tickets + T_XR, gate, bands,
                       pap_sum);
}
template <int XM>
static void launch_poisson_xr_any(const PoissonPlan &pl, hipStream_t s, const double *pnh, const double *poh,
                                  const double *pqh, double *x, double *r, int64_t mloc, int64_t m,
                                  const double *rsold, const double *pAp, double *rr_out, double *xalpha,
                                  const RedWs &ws, const int64_t *gate, const PeerSum *pap_sum) {
    if (pap_sum && pap_sum->cnt > 0)
        launch_poisson_xr<XM, PeerSum>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate,
                                       *pap_sum);
    else
        launch_poisson_xr<XM, NoPull>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate,
                                      NoPull{});
}

hipError_t poisson_p_f64(const double *rh, const double *poh, double *pnh, int64_t mloc, int64_t m, const double *rr,
                         const double *rsold, bool first, double *pap_out, const RedWs &ws, hipStream_t s, double eps,
                         int64_t k, int64_t *kdone, double *rrfinal, int part, int64_t *hrec, const double *r_up,
                         const double *r_dn, const PeerSum *rr_sum) {
    if (!poisson_fusable(mloc, m) || !al16(rh) || !al16(pnh) || (!first && !al16(poh))) return hipErrorInvalidValue;
    if ((r_up && !al16(r_up)) || (r_dn && !al16(r_dn)) || (rr_sum && (rr_sum->cnt < 0 || rr_sum->cnt > kMaxPeers)))
        return hipErrorInvalidValue;
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
    const HaloPull hp{r_up, r_dn};
    const PeerSum rs = rr_sum ? *rr_sum : no_sum();
    switch (pl.rb) {
        case 1: launch_poisson_p<1>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add, hp, rs); break;
        case 2: launch_poisson_p<2>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add, hp, rs); break;
        case 8: launch_poisson_p<8>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add, hp, rs); break;
        default: launch_poisson_p<4>(pl, s, rh, poh, pnh, mloc, m, rr, rsold, first, cv, pap_out, ws, ir, add, hp, rs); break;
    }
    return hipGetLastError();
}

hipError_t poisson_xr_f64(const double *pnh, const double *poh, const double *pqh, double *x, double *r,
                          int64_t mloc, int64_t m, const double *rsold, const double *pAp, double *rr_out, int xmode,
                          double *xalpha, const RedWs &ws, hipStream_t s, const int64_t *gate,
                          const PeerSum *pap_sum) {
    if (!poisson_fusable(mloc, m) || !al16(pnh) || !al16(x) || !al16(r)) return hipErrorInvalidValue;
    if (xmode < 0 || xmode > 3 || (xmode != 1 && !xalpha) || (xmode >= 2 && !al16(poh)) ||
        (xmode == 3 && !al16(pqh)) || (pap_sum && (pap_sum->cnt < 0 || pap_sum->cnt > kMaxPeers)))
        return hipErrorInvalidValue;
    const PoissonPlan pl = poisson_plan(mloc, m);
    switch (xmode) {
        case 0: launch_poisson_xr_any<0>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate, pap_sum); break;
        case 2: launch_poisson_xr_any<2>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate, pap_sum); break;
        case 3: launch_poisson_xr_any<3>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate, pap_sum); break;
        default: launch_poisson_xr_any<1>(pl, s, pnh, poh, pqh, x, r, mloc, m, rsold, pAp, rr_out, xalpha, ws, gate, pap_sum); break;
    }
    return hipGetLastError();
}

hipError_t poisson_xflush_f64(const double *pnh, const double *pbh, double *x, int64_t mloc, int64_t m,
                              const double *xalpha, hipStream_t s) {
    const int64_t npts = mloc * m;
    if (npts <= 0) return hipSuccess;
    if (!poisson_fusable(mloc, m) || !al16(pnh) || !al16(x) || (pbh && !al16(pbh))) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<int64_t>((npts / 2 + kNT - 1) / kNT, 8192);
    hipLaunchKernelGGL(k_poisson_xflush_f64, dim3(grid), dim3(kNT), 0, s, pnh + m, pbh ? pbh + m : nullptr, x, npts,
                       xalpha);
    return hipGetLastError();
}

// Load this file's code object on the current device now (see preload_kernels).
hipError_t preload_poisson() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k_stencil5_strip_f64));
}

}  // namespace cgx
