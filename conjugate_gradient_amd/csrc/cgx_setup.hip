// cgx_setup.hip -- contexts and shards (cgx_ctx.h): creation in the three
// modes (one GPU, several shards in this process, one rank of an RCCL job),
// device and pinned allocations, and the data in and out of a context
// (cgx_set_rows / cgx_set_system: parallel_cg.c:109-117's MPI_Bcast and
// MPI_Scatter; cgx_generate_spd; cgx_get_x).
#include <condition_variable>
#include <memory>
#include <thread>

#include "cgx_ctx.h"

namespace cgxh {

int set_dev(const Shard &s) {
    HIPT(hipSetDevice(s.dev));
    return CGX_OK;
}

int alloc_shard(cgx_ctx *c, Shard &s) {
    TRY(set_dev(s));
    {  // the code objects this context launches from (fp64 residual checks use the vector kernels too)
        unsigned set = PL_VECTOR;
        if (c->op == OP_POISSON) set |= PL_POISSON;
        else if (f32ref(c)) set |= PL_REF_F32;
        else if (c->flags & CGX_SYMMETRIC) set |= PL_SYMV;
        else set |= PL_MATVEC;
        HIPT(preload_kernels(set));
    }
    const size_t es = (size_t)c->es;
    HIPT(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIPT(hipEventCreateWithFlags(&s.ev_sync, hipEventDisableTiming));
    HIPT(hipEventCreateWithFlags(&s.ev_sync2, hipEventDisableTiming));
    HIPT(hipEventCreateWithFlags(&s.ev_root, hipEventDisableTiming));
    if (!s.ev_pready) HIPT(hipEventCreateWithFlags(&s.ev_pready, hipEventDisableTiming));
    const size_t abytes = (size_t)s.nloc * (size_t)c->lda * es;
    auto dmalloc = [&](char **p, size_t bytes) -> int {
        if (bytes == 0) bytes = 16;
        hipError_t e = hipMalloc(p, bytes);
        if (e != hipSuccess)
            return fail(CGX_ERR_NOMEM, "hipMalloc(%zu bytes) on device %d: %s", bytes, s.dev,
                        hipGetErrorString(e));
        return CGX_OK;
    };
    if (c->op == OP_POISSON) {
        // matrix-free: no A
    } else if ((c->flags & CGX_SYMMETRIC) && (c->flags & CGX_HOST_STREAM)) {
        // the upper-triangle tiles in pinned host memory, streamed in chunks of
        // whole tiles through kStreamBufs device buffers (tile_rows = tiles per chunk)
        const int64_t ntiles = sym_tiles(c->lda), tb = 128 * 128 * 8;
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&s.A_host), (size_t)ntiles * tb, hipHostMallocDefault);
        if (e != hipSuccess)
            return fail(CGX_ERR_NOMEM, "hipHostMalloc(%lld bytes) for streamed tiles: %s", (long long)(ntiles * tb),
                        hipGetErrorString(e));
        const char *tmb = std::getenv("CGX_STREAM_TILE_MB");
        const int64_t chunk_bytes = (int64_t)((tmb && *tmb) ? std::atoll(tmb) : 256) << 20;
        s.tile_rows = std::max<int64_t>(1, std::min<int64_t>(ntiles, chunk_bytes / tb));
        const char *nc = std::getenv("CGX_STREAM_COPIES");
        s.ncopy = std::max(1, std::min(kMaxCopyStreams, (nc && *nc) ? std::atoi(nc) : 2));
        for (int b = 0; b < kStreamBufs; ++b) {
            TRY(dmalloc(&s.tile[b], (size_t)s.tile_rows * tb));
            HIPT(hipEventCreateWithFlags(&s.ev_free[b], hipEventDisableTiming));
            for (int q = 0; q < s.ncopy; ++q) HIPT(hipEventCreateWithFlags(&s.ev_loaded[b][q], hipEventDisableTiming));
        }
        for (int q = 0; q < s.ncopy; ++q) HIPT(hipStreamCreateWithFlags(&s.copy[q], hipStreamNonBlocking));
        TRY(dmalloc(&s.sym_prow, (size_t)ntiles * 2 * 128 * 8));  // a row partial per unit (half tile), at most
        TRY(dmalloc(&s.sym_pcol, (size_t)ntiles * 128 * 8));
        s.sym_grid = sym_grid(s.dev);
        // CGX_STREAM_RESIDENT_MB: the first tiles (res_rows counts tiles here) stay in HBM
        const char *rmb = std::getenv("CGX_STREAM_RESIDENT_MB");
        const int64_t res_bytes = (int64_t)((rmb && *rmb) ? std::atoll(rmb) : 0) << 20;
        s.res_rows = std::max<int64_t>(0, std::min<int64_t>(ntiles, res_bytes / tb));
        if (s.res_rows > 0) TRY(dmalloc(&s.A, (size_t)s.res_rows * tb));
    } else if (c->flags & CGX_HOST_STREAM) {
        // A in pinned host memory, kStreamBufs device tiles of ~CGX_STREAM_TILE_MB.
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&s.A_host), abytes ? abytes : 16, hipHostMallocDefault);
        if (e != hipSuccess)
            return fail(CGX_ERR_NOMEM, "hipHostMalloc(%zu bytes) for streamed A: %s", abytes, hipGetErrorString(e));
        const int64_t row_bytes = c->lda * (int64_t)es;
        const char *tmb = std::getenv("CGX_STREAM_TILE_MB");
        const int64_t tile_bytes = (int64_t)((tmb && *tmb) ? std::atoll(tmb) : 256) << 20;
        s.tile_rows = std::max<int64_t>(1, std::min<int64_t>(s.nloc, tile_bytes / row_bytes));
        const char *nc = std::getenv("CGX_STREAM_COPIES");
        s.ncopy = std::max(1, std::min(kMaxCopyStreams, (nc && *nc) ? std::atoi(nc) : 2));
        for (int b = 0; b < kStreamBufs; ++b) {
            TRY(dmalloc(&s.tile[b], (size_t)s.tile_rows * row_bytes));
            HIPT(hipMemsetAsync(s.tile[b], 0, (size_t)s.tile_rows * row_bytes, s.stream));
            HIPT(hipEventCreateWithFlags(&s.ev_free[b], hipEventDisableTiming));
            for (int q = 0; q < s.ncopy; ++q) HIPT(hipEventCreateWithFlags(&s.ev_loaded[b][q], hipEventDisableTiming));
        }
        for (int q = 0; q < s.ncopy; ++q) HIPT(hipStreamCreateWithFlags(&s.copy[q], hipStreamNonBlocking));
        if (!f32ref(c)) s.tile_plan = plan_matvec_f64(s.dev, s.tile_rows, 0, 0, -1, 0, c->lda);
        // an HBM budget for A (out-of-core sizes: keep what fits, stream the rest)
        const char *rmb = std::getenv("CGX_STREAM_RESIDENT_MB");
        const int64_t res_bytes = (int64_t)((rmb && *rmb) ? std::atoll(rmb) : 0) << 20;
        s.res_rows = std::max<int64_t>(0, std::min<int64_t>(s.nloc, res_bytes / row_bytes));
        if (s.res_rows > 0) {
            TRY(dmalloc(&s.A, (size_t)s.res_rows * row_bytes));
            HIPT(hipMemsetAsync(s.A, 0, (size_t)s.res_rows * row_bytes, s.stream));
            if (!f32ref(c)) s.res_plan = plan_matvec_f64(s.dev, s.res_rows, 0, 0, -1, 0, c->lda);
        }
    } else if (c->flags & CGX_SYMMETRIC) {
        const int64_t ntiles = sym_tiles(c->lda);
        const size_t tbytes = (size_t)ntiles * 128 * 128 * 8;
        TRY(dmalloc(&s.A, tbytes));
        HIPT(hipMemsetAsync(s.A, 0, tbytes, s.stream));  // padding rows / columns stay zero
        TRY(dmalloc(&s.sym_prow, (size_t)ntiles * 2 * 128 * 8));  // a row partial per unit (half tile), at most
        TRY(dmalloc(&s.sym_pcol, (size_t)ntiles * 128 * 8));
        s.sym_grid = sym_grid(s.dev);
    } else {
        TRY(dmalloc(&s.A, abytes));
        HIPT(hipMemsetAsync(s.A, 0, abytes, s.stream));  // zero padding columns
    }
    TRY(dmalloc(&s.b, s.nloc * es));
    TRY(dmalloc(&s.x, s.nloc * es));
    if (c->op == OP_POISSON) {  // r with halo rows (the fused iteration exchanges r, not p)
        TRY(dmalloc(&s.rh, (s.nloc + 2 * c->m) * es));
        HIPT(hipMemsetAsync(s.rh, 0, (s.nloc + 2 * c->m) * es, s.stream));
        s.r = s.rh + c->m * es;
        TRY(dmalloc(&s.p2, (s.nloc + 2 * c->m) * es));
        HIPT(hipMemsetAsync(s.p2, 0, (s.nloc + 2 * c->m) * es, s.stream));
        if (c->xd == 3) {
            TRY(dmalloc(&s.p3, (s.nloc + 2 * c->m) * es));
            HIPT(hipMemsetAsync(s.p3, 0, (s.nloc + 2 * c->m) * es, s.stream));
        }
    } else if (c->fold_p) {  // the folded matVec reads r over all lda columns: zero past n
        TRY(dmalloc(&s.r, c->lda * es));
        HIPT(hipMemsetAsync(s.r, 0, c->lda * es, s.stream));
    } else {
        TRY(dmalloc(&s.r, s.nloc * es));
    }
    TRY(dmalloc(&s.Ap, s.nloc * es));
    // full-length p (dense) or the slab with one halo row above and below (Poisson)
    const int64_t plen = (c->op == OP_POISSON) ? s.nloc + 2 * c->m : c->lda;
    const int64_t xlen = (c->op == OP_POISSON) ? c->n : c->lda;
    TRY(dmalloc(&s.pfull, plen * es));
    if (c->fold_p) {
        TRY(dmalloc(&s.p_alt, plen * es));
        HIPT(hipMemsetAsync(s.p_alt, 0, plen * es, s.stream));
    }
    s.pown = (c->op == OP_POISSON) ? s.pfull + c->m * es : s.pfull + s.row0 * es;
    TRY(dmalloc(&s.scal, kScalSlots * 8));
    if (c->mode == M_RCCL && c->nranks > 1) TRY(dmalloc(&s.xfull, xlen * es));
    char *part = nullptr, *tick = nullptr;
    TRY(dmalloc(&part, kMaxRedBlocks * sizeof(double)));
    s.ws.partials = reinterpret_cast<double *>(part);  // owned by the shard from here (free_shard)
    TRY(dmalloc(&tick, kTickets * sizeof(unsigned)));
    s.ws.tickets = reinterpret_cast<unsigned *>(tick);
    if (es == 4) HIPT(fill_f32(reinterpret_cast<float *>(s.b), s.nloc, 0.0f, s.stream));
    else HIPT(fill_f64(reinterpret_cast<double *>(s.b), s.nloc, 0.0, s.stream));
    HIPT(hipMemsetAsync(s.x, 0, s.nloc * es, s.stream));
    HIPT(hipMemsetAsync(s.r, 0, s.nloc * es, s.stream));
    HIPT(hipMemsetAsync(s.Ap, 0, s.nloc * es, s.stream));
    HIPT(hipMemsetAsync(s.pfull, 0, plen * es, s.stream));
    HIPT(hipMemsetAsync(s.scal, 0, kScalSlots * 8, s.stream));
    HIPT(hipMemsetAsync(s.ws.tickets, 0, kTickets * sizeof(unsigned), s.stream));
    if (s.xfull) HIPT(hipMemsetAsync(s.xfull, 0, xlen * es, s.stream));
    HIPT(hipHostMalloc(reinterpret_cast<void **>(&s.h_pin), 8 * (8 + kLookRing), hipHostMallocDefault));
    {
        const size_t xb = (size_t)(s.xfull ? xlen : s.nloc) * es;
        if (xb <= kXStageMax) {
            HIPT(hipHostMalloc(reinterpret_cast<void **>(&s.h_x), xb ? xb : 16, hipHostMallocDefault));
            // one device-to-host copy now: the first one of a process sets up
            // the copy path (~8 ms, measured in cg_hip's get_x), which would
            // otherwise land on the first cgx_get_x
            HIPT(hipMemcpyAsync(s.h_x, s.pfull, std::min<size_t>(xb, (size_t)plen * es), hipMemcpyDeviceToHost,
                                s.stream));
        }
    }
    HIPT(hipHostMalloc(reinterpret_cast<void **>(&s.h_rec), 16, hipHostMallocMapped | hipHostMallocCoherent));
    HIPT(hipHostGetDevicePointer(reinterpret_cast<void **>(&s.d_rec), s.h_rec, 0));
    s.h_rec[0] = s.h_rec[1] = 0;
    {  // The host paces the gated loop on these and then reads the convergence
        // record, which the deciding kernel stores with system-scope atomics
        // itself, so the events need no system-scope release of their own: a
        // convergence-tested solve 2-10 % faster at N = 512-8192
        // (profiles/r03_look_ab.jsonl).
        const unsigned lflags = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
        for (int q = 0; q < kLookRing; ++q) HIPT(hipEventCreateWithFlags(&s.ev_look[q], lflags));
    }
    // Timing-only events (the matVec brackets) skip the system-scope release
    // an event does by default when it completes: that fence writes back and
    // invalidates the caches; an event costs 3.3 us on the stream without it,
    // 4.4 us with it (profiles/r03_event_fence_ab.jsonl).  Nothing reads memory
    // through these events; they only time.
    const unsigned tflags = hipEventDisableSystemFence;
    if (c->flags & CGX_TIMING) {
        s.ev_t.resize(2 * kEvPairs);
        for (auto &e : s.ev_t) HIPT(hipEventCreateWithFlags(&e, tflags));
    }
    if ((c->flags & CGX_PHASES) && &s == &c->sh[0]) {
        const size_t tsb = (size_t)kTsIters * kTsKern * kTsSlot * 8;
        TRY(dmalloc(reinterpret_cast<char **>(&s.ts_dev), tsb));
        HIPT(hipMemsetAsync(s.ts_dev, 0, tsb, s.stream));
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev) == hipSuccess && khz > 0)
            c->ts_khz = khz;
    }
    if (c->mode == M_RCCL)
        for (auto &e : s.ev_prog)  // liveness only: the host asks whether the stream got this far
            HIPT(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    if (!f32ref(c) && c->op == OP_DENSE && !(c->flags & CGX_SYMMETRIC)) {
        s.plan = plan_matvec_f64(s.dev, s.nloc, 0, 0, -1, 0, c->lda);
        if (small_matvec(c)) s.plan = plan_matvec_small_f64(s.dev, s.nloc, c->lda);
    }
    if (c->fold_p) {
        // The folded matVec keeps the plain plan's rows per wave and grid: the
        // fused p.Ap partials then add in the same order (x bit for bit the
        // other forms').  At n = 2048 (R = 2) four chunks in flight beat eight.
        s.fold_plan = plan_matvec_f64(s.dev, s.nloc, s.plan.R, c->n == 2048 ? 4 : s.plan.U, -1, 0, c->lda);
        if (s.fold_plan.blocks != s.plan.blocks || s.plan.small) s.fold_plan = s.plan;
    }
    HIPT(hipStreamSynchronize(s.stream));
    return CGX_OK;
}

void free_shard(Shard &s) {
    (void)hipSetDevice(s.dev);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.comm) ncclCommDestroy(s.comm);
    for (char *p : {s.A, s.b, s.x, s.rh ? s.rh : s.r, s.p2, s.p3, s.Ap, s.pfull, s.p_alt, s.xfull, s.scal, s.sym_prow,
                    s.sym_pcol, s.sym_stage})
        if (p) (void)hipFree(p);
    if (s.ws.partials) (void)hipFree(s.ws.partials);
    if (s.ws.tickets) (void)hipFree(s.ws.tickets);
    if (s.h_pin) (void)hipHostFree(s.h_pin);
    if (s.h_x) (void)hipHostFree(s.h_x);
    if (s.h_rec) (void)hipHostFree(s.h_rec);
    for (auto e : s.ev_t) (void)hipEventDestroy(e);
    if (s.ts_dev) (void)hipFree(s.ts_dev);
    if (s.ts_host) (void)hipHostFree(s.ts_host);
    for (auto e : s.ev_prog)
        if (e) (void)hipEventDestroy(e);
    if (s.ev_sync) (void)hipEventDestroy(s.ev_sync);
    if (s.ev_sync2) (void)hipEventDestroy(s.ev_sync2);
    if (s.ev_root) (void)hipEventDestroy(s.ev_root);
    for (int q = 0; q < kMaxCopyStreams; ++q)
        if (s.copy[q]) {
            (void)hipStreamSynchronize(s.copy[q]);
            (void)hipStreamDestroy(s.copy[q]);
        }
    for (int b = 0; b < kStreamBufs; ++b) {
        if (s.tile[b]) (void)hipFree(s.tile[b]);
        if (s.ev_free[b]) (void)hipEventDestroy(s.ev_free[b]);
        for (int q = 0; q < kMaxCopyStreams; ++q)
            if (s.ev_loaded[b][q]) (void)hipEventDestroy(s.ev_loaded[b][q]);
    }
    if (s.A_host) (void)hipHostFree(s.A_host);
    if (s.cstream) {
        (void)hipStreamSynchronize(s.cstream);
        (void)hipStreamDestroy(s.cstream);
    }
    if (s.ev_pready) (void)hipEventDestroy(s.ev_pready);
    for (auto e : s.ev_look)
        if (e) (void)hipEventDestroy(e);
    if (s.ev_gathered) (void)hipEventDestroy(s.ev_gathered);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Shard();
}

int check_n(int64_t n, int nranks) {
    if (n < 1) return fail(CGX_ERR_ARG, "n must be >= 1 (got %lld)", (long long)n);
    if (nranks < 1) return fail(CGX_ERR_ARG, "nranks must be >= 1");
    if (n % nranks != 0)  // parallel_cg.c:86-90
        return fail(CGX_ERR_SHAPE, "%lld is not divisible by %d", (long long)n, nranks);
    if (n > (int64_t)0xffffffffLL) return fail(CGX_ERR_ARG, "n too large");
    return CGX_OK;
}

cgx_ctx *new_ctx(int64_t n, int nranks, int flags) {
    cgx_ctx *c = new (std::nothrow) cgx_ctx();
    if (!c) return nullptr;
    c->n = n;
    c->lda = round_up(n, 128);
    c->nranks = nranks;
    c->flags = flags;
    c->es = (flags & CGX_F32_REF) ? 4 : 8;
    return c;
}

// The rotated column order (cgx_ctx::rot), which makes the overlapped
// exchange possible and bit-neutral: dense fp64 resident row-major A, more
// than one row block, every block aligned to the matVec's 128-column chunks
// (also with CGX_COMM_P2P, which never overlaps: the same bits as the
// collective exchange).  CGX_OVERLAP=force also takes it at world size 1
// in rank mode (the in-place allgather on the comm stream and the event
// hand-offs run with nothing to exchange), so one GPU can execute the
// rank-mode overlap path.
bool can_rotate(const cgx_ctx *c) {
    if (c->op != OP_DENSE || f32ref(c) || (c->flags & (CGX_HOST_STREAM | CGX_SYMMETRIC))) return false;
    const char *e = std::getenv("CGX_OVERLAP");
    const bool force = e && std::strcmp(e, "force") == 0;
    if (c->mode == M_SINGLE || (c->mode == M_RCCL && c->nranks == 1 && !force)) return false;
    for (const auto &s : c->sh)
        if ((s.row0 & 127) || (s.nloc & 127)) return false;
    return true;
}

int alloc_overlap(cgx_ctx *c) {
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipStreamCreateWithFlags(&s.cstream, hipStreamNonBlocking));
        if (!s.ev_pready) HIPT(hipEventCreateWithFlags(&s.ev_pready, hipEventDisableTiming));
        HIPT(hipEventCreateWithFlags(&s.ev_gathered, hipEventDisableTiming));
    }
    return CGX_OK;
}

// The two-launch dense iteration (do_iteration_fused_p): one GPU, fp64,
// resident row-major A, n up to kFusePMax by default (the p update then runs
// in one block: n doubles read twice and written once by one CU, a few us at
// n = 8192); CGX_FUSE_P=0 keeps three launches, =1 uses two at any n.
constexpr int64_t kFusePMax = 8192;
// ... and the p update is folded into the next matVec (do_iteration_fold_p)
// up to kFoldPMax with k_matvec_fold_f64 -- measured per iteration
// (profiles/r03_iteration_floor.jsonl, device clock) 9.6 vs 10.2 us at
// n = 512, 11.8 vs 12.0 at 1024, 13.9-14.0 vs 14.2 at 2048 -- and wherever
// the LDS-staged matVec applies (small_matvec: 2048 <= lda <= 8192), which
// forms p_k once per CU instead of once per wave: 13.8 / 30.0-30.1 / 91.0 us
// at 2048 / 4096 / 8192 against 14.3 / 30.8 / 92.1 for the two-launch form
// with round 2's matVec (profiles/r03_iteration_floor_small_prefetch2.jsonl).
// With k_matvec_fold_f64 above 2048 the fold's extra reads of r and p_{k-1}
// per chunk of A cost more than the single-block pass saves (37.4 vs 31.1 us
// at 4096), so without the LDS-staged matVec k_update_xrp_f64 stays.
constexpr int64_t kFoldPMax = 2048;
// One GPU, one resident row-major shard of 2048 <= lda <= 8192 columns: the
// matVec stages p in LDS (k_matvec_small_f64, every form of the iteration).
bool small_matvec(const cgx_ctx *c) {
    if (c->mode != M_SINGLE || c->sh.size() != 1 || c->op != OP_DENSE || f32ref(c)) return false;
    if (c->flags & (CGX_SYMMETRIC | CGX_HOST_STREAM)) return false;
    return plan_matvec_small_f64(c->sh[0].dev, c->sh[0].nloc, c->lda).small > 0;
}

static bool can_fuse_p(const cgx_ctx *c) {
    if (c->mode != M_SINGLE || c->op != OP_DENSE || f32ref(c)) return false;
    if (c->flags & (CGX_SYMMETRIC | CGX_HOST_STREAM)) return false;
    if (c->n * 8 > INT32_MAX) return false;
    const char *e = std::getenv("CGX_FUSE_P");
    if (e && *e == '0') return false;
    if (e && *e == '1') return true;
    return c->n <= kFusePMax;
}

// The F32_REF counterparts: with resident row-major A the matVec's last
// block runs vecVec(p, Ap) over the shard's rows (the shard's partial in
// row-block modes), and on one GPU the iteration is two launches
// (do_iteration_ref_fused).  CGX_REF_FUSE=0 keeps the separate launches
// (matVec, p.Ap, x/r + r.r, p).  The same float operations in the same order
// either way.
static bool can_fuse_ref_dot(const cgx_ctx *c) {
    if (c->op != OP_DENSE || !f32ref(c)) return false;
    if (c->flags & (CGX_SYMMETRIC | CGX_HOST_STREAM)) return false;
    const char *e = std::getenv("CGX_REF_FUSE");
    return !(e && *e == '0');
}

int finish_create(cgx_ctx *c, cgx_ctx **out) {
    {
        const char *e = std::getenv("CGX_LOCAL_XCHG");
        c->xchg_kernels = !(e && !std::strcmp(e, "copy"));
        const char *f = std::getenv("CGX_LOCAL_FUSE");
        c->fuse_combine = c->mode == M_LOCAL && c->xchg_kernels && !(f && *f == '0') && !(c->flags & CGX_F32_REF) &&
                          !(c->flags & CGX_COMM_P2P) && (int)c->sh.size() <= kMaxPeers;
        c->fuse_f32 = c->mode == M_LOCAL && c->xchg_kernels && !(f && *f == '0') && (c->flags & CGX_F32_REF) &&
                      !(c->flags & CGX_COMM_P2P) && (int)c->sh.size() <= kMaxPeers && c->op == OP_DENSE;
    }
    c->rot = can_rotate(c);
    c->overlap = false;  // choose_overlap below, once the row blocks exist
    c->fused_p = can_fuse_p(c);
    {  // the folded form of the two-launch iteration (CGX_FOLD_P=0 / 1: never / at any fused n)
        const char *e = std::getenv("CGX_FOLD_P");
        c->fold_p = c->fused_p && (e && *e ? *e == '1' : c->n <= kFoldPMax || small_matvec(c));
    }
    c->ref_mv_dot = can_fuse_ref_dot(c);
    c->ref_fused = c->ref_mv_dot && c->mode == M_SINGLE;
    if (c->op == OP_POISSON) {  // CGX_POISSON_FUSED=0: the three-kernel split (stencil, r, x/p)
        const char *e = std::getenv("CGX_POISSON_FUSED");
        c->fused = !(e && *e == '0') && poisson_fusable(c->sh[0].nloc / c->m, c->m);
        // one process, several slabs: the next k_poisson_p reads r's halo rows
        // in place (no copies, nothing to overlap); CGX_LOCAL_XCHG=copy keeps
        // round 3's peer copies and combine kernels (the same bits)
        c->halo_pull = c->fused && c->mode == M_LOCAL && c->xchg_kernels;
        if (!c->fused || c->mode != M_LOCAL) c->fuse_combine = false;  // dense: decided above; Poisson: fused only
        // rank mode: r's halo rows travel by ncclSend/Recv on the comm stream
        // while k_poisson_p runs the slab's interior (CGX_HALO_OVERLAP=0: before it)
        const char *h = std::getenv("CGX_HALO_OVERLAP");
        const bool force = h && std::strcmp(h, "force") == 0;  // also at world size 1 in rank mode
        c->halo_overlap = c->fused && !(h && *h == '0') && !c->halo_pull && c->mode != M_SINGLE &&
                          !(c->mode == M_RCCL && c->nranks == 1 && !force);
        const char *xd = std::getenv("CGX_POISSON_XDEFER");
        c->xdefer = c->fused && !(xd && *xd == '0');
        // x every third iteration by default (1478-1479 vs 1447-1457 it/s every
        // other, 1330-1344 every iteration at m = 8192, interleaved:
        // profiles/r03_poisson_xdefer3_ab.jsonl); CGX_POISSON_XDEFER=2: every other
        c->xd = !c->xdefer ? 1 : (xd && *xd == '2') ? 2 : 3;
    }
    auto undo = [c](int rc) {
        std::string keep = g_err;
        for (auto &t : c->sh) free_shard(t);
        delete c;
        snprintf(g_err, sizeof g_err, "%s", keep.c_str());
        return rc;
    };
    for (auto &s : c->sh) {
        int rc = alloc_shard(c, s);
        if (rc == CGX_OK && (c->rot || c->halo_overlap) && &s == &c->sh.back()) rc = alloc_overlap(c);
        if (rc != CGX_OK) return undo(rc);
    }
    if (c->rot) {  // overlapped or plain exchange, by measurement (rank mode: a collective decision)
        const int rc = choose_overlap(c);
        if (rc != CGX_OK) return undo(rc);
    }
    // one enqueuing thread per row block (cgx_local_mt.hip); without it the
    // iteration is enqueued by the calling thread, the same launches
    if (local_mt_eligible(c) && local_mt_start(c) != CGX_OK) c->pool = nullptr;
    if (warm_eligible(c)) {
        const int rc = warm_solve_kernels(c);
        if (rc != CGX_OK) return undo(rc);
    }
    *out = c;
    return CGX_OK;
}

}  // namespace cgxh

extern "C" {

static int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(CGX_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(CGX_ERR_ARG, "device %d out of range (%d visible)", device, n);
    return CGX_OK;
}

// Operator-generic constructors.  Dense: n unknowns, row blocks of n/P rows.
// Poisson: n = m*m unknowns, slabs of m/P grid rows (n/P unknowns).
static int check_op(int op, int64_t n, int64_t m, int parts, int flags) {
    if ((flags & CGX_PHASES) && (op != OP_DENSE || (flags & (CGX_F32_REF | CGX_HOST_STREAM | CGX_SYMMETRIC))))
        return fail(CGX_ERR_ARG, "CGX_PHASES: the dense fp64 operator with A resident (row-major) only");
    if (op == OP_POISSON) {
        if (m < 1) return fail(CGX_ERR_ARG, "m must be >= 1");
        if (m % parts != 0) return fail(CGX_ERR_SHAPE, "%lld is not divisible by %d", (long long)m, parts);
        if (flags & (CGX_F32_REF | CGX_HOST_STREAM | CGX_COMM_P2P))
            return fail(CGX_ERR_ARG, "the Poisson operator supports CGX_F64 (+CGX_TIMING) only");
        return CGX_OK;
    }
    if ((flags & CGX_SYMMETRIC) && (parts != 1 || (flags & CGX_F32_REF)))
        return fail(CGX_ERR_ARG, "CGX_SYMMETRIC: fp64 on one GPU only (no CGX_F32_REF)");
    return check_n(n, parts);
}

static cgx_ctx *new_ctx_op(int op, int64_t n, int64_t m, int parts, int flags) {
    cgx_ctx *c = new_ctx(n, parts, flags);
    if (!c) return nullptr;
    c->op = op;
    c->m = m;
    if (op == OP_POISSON) c->lda = m;
    return c;
}

static int create_single(cgx_ctx **ctx, int op, int64_t n, int64_t m, int device, int flags) {
    if (!ctx) return fail(CGX_ERR_ARG, "ctx is NULL");
    *ctx = nullptr;
    TRY(check_op(op, n, m, 1, flags));
    TRY(check_device(device));
    cgx_ctx *c = new_ctx_op(op, n, m, 1, flags);
    if (!c) return fail(CGX_ERR_NOMEM, "host allocation failed");
    c->mode = M_SINGLE;
    c->sh.resize(1);
    c->sh[0].dev = device;
    c->sh[0].index = 0;
    c->sh[0].row0 = 0;
    c->sh[0].nloc = n;
    return finish_create(c, ctx);
}

static int create_multi(cgx_ctx **ctx, int op, int64_t n, int64_t m, int nshards, const int *devices, int flags) {
    if (!ctx || !devices) return fail(CGX_ERR_ARG, "ctx/devices is NULL");
    *ctx = nullptr;
    if (nshards < 1 || nshards > kMaxShards) return fail(CGX_ERR_ARG, "nshards must be in [1, %d]", kMaxShards);
    TRY(check_op(op, n, m, nshards, flags));
    for (int i = 0; i < nshards; ++i) TRY(check_device(devices[i]));
    cgx_ctx *c = new_ctx_op(op, n, m, nshards, flags);
    if (!c) return fail(CGX_ERR_NOMEM, "host allocation failed");
    c->mode = nshards == 1 ? M_SINGLE : M_LOCAL;
    c->sh.resize(nshards);
    const int64_t loc = n / nshards;
    for (int i = 0; i < nshards; ++i) {
        c->sh[i].dev = devices[i];
        c->sh[i].index = i;
        c->sh[i].row0 = (int64_t)i * loc;
        c->sh[i].nloc = loc;
    }
    // Peer access between distinct devices (xGMI), which parallel_cg.c's
    // MPI_Scatter / MPI_Allgather (:109-117, :290) become here: every ordered
    // pair must be able to reach the other's memory (hipDeviceCanAccessPeer),
    // and access is enabled once per pair.  A pair that cannot is an error
    // naming it -- the copies would otherwise be staged through host memory
    // without a word.  Every failed HIP call's error is consumed here, so the
    // thread's last HIP error is clean when the context is handed out
    // (test_create_multi_leaves_no_hip_error).  Repeated devices need nothing.
    bool distinct = false;
    for (int i = 0; i < nshards; ++i)
        for (int j = 0; j < nshards; ++j) {
            if (devices[i] == devices[j]) continue;
            distinct = true;
            int can = 0;
            hipError_t e = hipDeviceCanAccessPeer(&can, devices[i], devices[j]);
            if (e != hipSuccess || !can) {
                (void)hipGetLastError();
                delete c;
                return fail(CGX_ERR_HIP, "device %d cannot access device %d's memory (hipDeviceCanAccessPeer: %s, "
                                         "%d): the row blocks need peer access",
                            devices[i], devices[j], hipGetErrorString(e), can);
            }
            if (hipSetDevice(devices[i]) != hipSuccess) {
                (void)hipGetLastError();
                delete c;
                return fail(CGX_ERR_HIP, "hipSetDevice(%d) failed", devices[i]);
            }
            e = hipDeviceEnablePeerAccess(devices[j], 0);
            (void)hipGetLastError();  // hipErrorPeerAccessAlreadyEnabled (an earlier context) is fine
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                delete c;
                return fail(CGX_ERR_HIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", devices[i], devices[j],
                            hipGetErrorString(e));
            }
        }
    c->peer = distinct;
    return finish_create(c, ctx);
}

static int create_rank(cgx_ctx **ctx, int op, int64_t n, int64_t m, int rank, int nranks, const cgx_unique_id *id,
                       int device, int flags) {
    if (!ctx || !id) return fail(CGX_ERR_ARG, "ctx/id is NULL");
    *ctx = nullptr;
    TRY(check_op(op, n, m, nranks, flags));
    if (rank < 0 || rank >= nranks) return fail(CGX_ERR_ARG, "rank %d not in [0, %d)", rank, nranks);
    if (nranks > S_TR - S_GATHER) return fail(CGX_ERR_ARG, "at most %d ranks", S_TR - S_GATHER);
    TRY(check_device(device));
    if (!rccl_load()) return CGX_ERR_RCCL;
    cgx_ctx *c = new_ctx_op(op, n, m, nranks, flags);
    if (!c) return fail(CGX_ERR_NOMEM, "host allocation failed");
    c->mode = M_RCCL;
    c->sh.resize(1);
    Shard &s = c->sh[0];
    s.dev = device;
    s.index = rank;
    s.nloc = n / nranks;
    s.row0 = (int64_t)rank * s.nloc;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return fail(CGX_ERR_HIP, "hipSetDevice(%d) failed", device);
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    // The initialisation runs on a helper thread and this one waits for it
    // with the deadline: ncclCommInitRank blocks in the bootstrap until every
    // rank has joined (RCCL 2.27 does so inside the call even for a
    // nonblocking communicator, measured), so a rank that never joins would
    // hang the others.  On the deadline the call returns CGX_ERR_RCCL and the
    // helper is left behind, detached; should it still finish, it aborts the
    // communicator it made.  The process is expected to exit on the error.
    c->rccl_timeout_s = rccl_timeout_from_env();
    struct InitJob {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclResult_t r = ncclInternalError;
        ncclComm_t comm = nullptr;
    };
    auto job = std::make_shared<InitJob>();
    std::thread([job, nranks, u, rank, device] {
        ncclComm_t comm = nullptr;
        ncclResult_t r = hipSetDevice(device) == hipSuccess ? ncclCommInitRank(&comm, nranks, u, rank)
                                                            : ncclUnhandledCudaError;
        std::lock_guard<std::mutex> lk(job->mu);
        if (job->abandoned) {
            if (comm) (void)ncclCommAbort(comm);
            return;
        }
        job->r = r;
        job->comm = comm;
        job->done = true;
        job->cv.notify_all();
    }).detach();
    ncclResult_t nr;
    {
        std::unique_lock<std::mutex> lk(job->mu);
        auto ready = [&job] { return job->done; };
        if (c->rccl_timeout_s > 0.0)
            job->cv.wait_for(lk, std::chrono::duration<double>(c->rccl_timeout_s), ready);
        else
            job->cv.wait(lk, ready);
        if (!job->done) {
            job->abandoned = true;
            debug_log("rank %d: ncclCommInitRank did not return within %.0f s", rank, c->rccl_timeout_s);
            delete c;
            return fail(CGX_ERR_RCCL, "ncclCommInitRank(rank %d of %d): not every rank joined within %.0f s "
                                      "(CGX_RCCL_TIMEOUT_S)", rank, nranks, rccl_timeout_from_env());
        }
        nr = job->r;
        s.comm = job->comm;
    }
    if (nr != ncclSuccess) {
        if (s.comm) (void)ncclCommAbort(s.comm);
        delete c;
        return fail(CGX_ERR_RCCL, "ncclCommInitRank(rank %d of %d): %s", rank, nranks, ncclGetErrorString(nr));
    }
    return finish_create(c, ctx);
}

int cgx_create(cgx_ctx **ctx, int64_t n, int device, int flags) {
    return create_single(ctx, OP_DENSE, n, 0, device, flags);
}

int cgx_create_multi(cgx_ctx **ctx, int64_t n, int nshards, const int *devices, int flags) {
    return create_multi(ctx, OP_DENSE, n, 0, nshards, devices, flags);
}

int cgx_get_unique_id(cgx_unique_id *id) {
    if (!id) return fail(CGX_ERR_ARG, "id is NULL");
    static_assert(sizeof(ncclUniqueId) == sizeof(cgx_unique_id), "unique id size");
    if (!rccl_load()) return CGX_ERR_RCCL;
    ncclUniqueId u;
    NCCLT(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return CGX_OK;
}

int cgx_rccl_available(void) { return rccl_load() ? CGX_OK : CGX_ERR_RCCL; }

int cgx_create_rank(cgx_ctx **ctx, int64_t n, int rank, int nranks, const cgx_unique_id *id, int device,
                    int flags) {
    return create_rank(ctx, OP_DENSE, n, 0, rank, nranks, id, device, flags);
}

static int check_m(int64_t m) {
    if (m < 1 || m > 46340 * 4) return fail(CGX_ERR_ARG, "grid width m out of range");
    return CGX_OK;
}

int cgx_create_poisson(cgx_ctx **ctx, int64_t m, int device, int flags) {
    TRY(check_m(m));
    return create_single(ctx, OP_POISSON, m * m, m, device, flags);
}

int cgx_create_poisson_multi(cgx_ctx **ctx, int64_t m, int nshards, const int *devices, int flags) {
    TRY(check_m(m));
    return create_multi(ctx, OP_POISSON, m * m, m, nshards, devices, flags);
}

int cgx_create_poisson_rank(cgx_ctx **ctx, int64_t m, int rank, int nranks, const cgx_unique_id *id, int device,
                            int flags) {
    TRY(check_m(m));
    return create_rank(ctx, OP_POISSON, m * m, m, rank, nranks, id, device, flags);
}

int cgx_fill(cgx_ctx *c, double b_value, double x_value) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        if (f32ref(c)) {
            HIPT(fill_f32(reinterpret_cast<float *>(s.b), s.nloc, (float)b_value, s.stream));
            HIPT(fill_f32(reinterpret_cast<float *>(s.x), s.nloc, (float)x_value, s.stream));
        } else {
            HIPT(fill_f64(reinterpret_cast<double *>(s.b), s.nloc, b_value, s.stream));
            HIPT(fill_f64(reinterpret_cast<double *>(s.x), s.nloc, x_value, s.stream));
        }
        s.x_zero = x_value == 0.0;
    }
    TRY(sync_all(c));
    c->state = ST_IDLE;
    return CGX_OK;
}

int cgx_destroy(cgx_ctx *ctx) {
    if (!ctx) return CGX_OK;
    // rank mode: drain with the deadline first, so a job whose peer died is
    // aborted here instead of hanging in the stream syncs below
    const int rc = (ctx->mode == M_RCCL && !ctx->dead) ? sync_all(ctx) : CGX_OK;
    local_mt_stop(ctx);
    for (auto &s : ctx->sh) free_shard(s);
    delete ctx;
    return rc;
}

int cgx_get_info(const cgx_ctx *c, cgx_info *info) {
    if (!c || !info) return fail(CGX_ERR_ARG, "NULL argument");
    info->n = c->n;
    info->lda = c->lda;
    info->nranks = c->nranks;
    info->nshards = (int)c->sh.size();
    info->rank0 = c->sh[0].index;
    info->row0 = c->sh[0].row0;
    info->nrows = 0;
    for (auto &s : c->sh) info->nrows += s.nloc;
    info->flags = c->flags | (c->overlap ? CGX_OVERLAP_ACTIVE : 0) |
                  ((c->fused || c->fused_p || c->ref_fused) ? CGX_FUSED_ACTIVE : 0) | (c->peer ? CGX_PEER_ACTIVE : 0) |
                  (c->sh[0].plan.small ? CGX_SMALL_ACTIVE : 0) | (c->fold_p ? CGX_FOLD_ACTIVE : 0) |
                  (c->xdefer ? CGX_XDEFER_ACTIVE : 0) |
                  (c->xd == 3 ? CGX_XDEFER3_ACTIVE : 0) |
                  ((c->mode == M_LOCAL && c->xchg_kernels) ? CGX_PULL_ACTIVE : 0) |
                  ((c->fuse_combine || c->fuse_f32) ? CGX_FOLDED_ACTIVE : 0) | (c->halo_pull ? CGX_HALO_PULL_ACTIVE : 0) |
                  (c->pool ? CGX_THREADS_ACTIVE : 0) | (c->halo_overlap ? CGX_HALO_OVERLAP_ACTIVE : 0);
    info->elem_bytes = c->es;
    return CGX_OK;
}

int cgx_get_overlap_info(const cgx_ctx *c, cgx_overlap_info *info) {
    if (!c || !info) return fail(CGX_ERR_ARG, "NULL argument");
    info->active = c->overlap ? 1 : 0;
    info->decided_by = c->ov_how;
    info->allgather_us = c->ov_ag_us;
    info->split_us = c->ov_split_us;
    info->one_launch_us = c->ov_one_us;
    info->split_cost_us = c->ov_cost_us;
    info->overlap_form_us = c->ov_form_us;
    info->plain_form_us = c->ov_plain_form_us;
    info->margin = kOverlapMargin;
    info->forms_ms = c->ov_forms_ms;
    return CGX_OK;
}

int cgx_get_comm_info(cgx_ctx *c, cgx_comm_info *info) {
    if (!c || !info) return fail(CGX_ERR_ARG, "NULL argument");
    std::memset(info, 0, sizeof *info);
    const Shard &s = c->sh[0];
    info->device = s.dev;
    info->rccl_nranks = c->nranks;
    info->rccl_device = -1;
    info->rccl_rank = s.index;
    HIPT(hipDeviceGetPCIBusId(info->pci_bus_id, (int)sizeof info->pci_bus_id, s.dev));
    if (c->mode == M_RCCL) {
        if (c->dead || !s.comm) return dead_error(c);
        NCCLT(ncclCommCount(s.comm, &info->rccl_nranks));
        NCCLT(ncclCommCuDevice(s.comm, &info->rccl_device));
        NCCLT(ncclCommUserRank(s.comm, &info->rccl_rank));
    }
    return CGX_OK;
}

int cgx_set_rows(cgx_ctx *c, int64_t row0, int64_t nrows, const void *A_rows, int64_t lda_host,
                 const void *b_rows, const void *x_rows) {
    const Range range_("cgx_set_rows");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    if (row0 < 0 || nrows < 0 || row0 + nrows > c->n)
        return fail(CGX_ERR_SHAPE, "rows [%lld, %lld) outside [0, %lld)", (long long)row0,
                    (long long)(row0 + nrows), (long long)c->n);
    if (A_rows && c->op == OP_POISSON) return fail(CGX_ERR_ARG, "the Poisson operator is matrix-free: A must be NULL");
    if (A_rows && lda_host < c->n) return fail(CGX_ERR_ARG, "lda_host (%lld) < n", (long long)lda_host);
    const size_t es = (size_t)c->es;
    // A host-streamed A is rewritten in place on the host: first let every
    // copy (and kernel) still reading it from enqueued iterations finish.
    if (A_rows && (c->flags & CGX_HOST_STREAM)) TRY(sync_all(c));
    for (auto &s : c->sh) {
        const int64_t lo = std::max(row0, s.row0), hi = std::min(row0 + nrows, s.row0 + s.nloc);
        if (hi <= lo) continue;
        TRY(set_dev(s));
        if (A_rows && s.A_host && (c->flags & CGX_SYMMETRIC)) {
            // pack on the host: row i supplies columns 128*(i/128) .. lda-1 of its tile row
            const int64_t nt = c->lda / 128;
            double *At = reinterpret_cast<double *>(s.A_host);
            for (int64_t i = lo; i < hi; ++i) {
                const double *row = static_cast<const double *>(A_rows) + (size_t)(i - row0) * lda_host;
                const int64_t I = i / 128;
                const int r = (int)(i % 128);
                for (int64_t j = I * 128; j < c->lda; ++j)
                    At[(sym_off_h(I, nt) + j / 128 - I) * 128 * 128 + sym_pos_h(r, (int)(j % 128))] =
                        j < c->n ? row[j] : 0.0;
            }
            if (sym_off_h(lo / 128, nt) < s.res_rows) s.res_dirty = true;
        } else if (A_rows && s.A_host) {
            for (int64_t i = lo; i < hi; ++i) {
                char *dst = s.A_host + (size_t)(i - s.row0) * c->lda * es;
                std::memcpy(dst, static_cast<const char *>(A_rows) + (size_t)(i - row0) * lda_host * es, (size_t)c->n * es);
                if (c->lda > c->n) std::memset(dst + (size_t)c->n * es, 0, (size_t)(c->lda - c->n) * es);
            }
            if (lo - s.row0 < s.res_rows) s.res_dirty = true;
        } else if (A_rows && (c->flags & CGX_SYMMETRIC)) {
            // rows through a staging buffer, then packed into the tiles
            if (!s.sym_stage) {
                s.sym_stage_rows = std::max<int64_t>(1, std::min<int64_t>(c->n, (int64_t)(128 << 20) / (c->lda * 8)));
                HIPT(hipMalloc(&s.sym_stage, (size_t)s.sym_stage_rows * c->lda * 8));
            }
            for (int64_t i0 = lo; i0 < hi; i0 += s.sym_stage_rows) {
                const int64_t k = std::min(s.sym_stage_rows, hi - i0);
                HIPT(hipMemcpy2DAsync(s.sym_stage, (size_t)c->lda * 8,
                                      static_cast<const char *>(A_rows) + (size_t)(i0 - row0) * lda_host * 8,
                                      (size_t)lda_host * 8, (size_t)c->n * 8, (size_t)k, hipMemcpyHostToDevice,
                                      s.stream));
                HIPT(sym_pack_f64(reinterpret_cast<const double *>(s.sym_stage), c->lda, i0, k, c->n, c->lda,
                                  reinterpret_cast<double *>(s.A), s.stream));
            }
        } else if (A_rows && lda_host == c->lda && c->lda == c->n) {
            // same row pitch on both sides: one contiguous copy (a pitched copy
            // of the same bytes ran at a third of the rate from pinned memory)
            HIPT(hipMemcpyAsync(s.A + (size_t)(lo - s.row0) * c->lda * es,
                                static_cast<const char *>(A_rows) + (size_t)(lo - row0) * lda_host * es,
                                (size_t)(hi - lo) * c->lda * es, hipMemcpyHostToDevice, s.stream));
        } else if (A_rows)
            HIPT(hipMemcpy2DAsync(s.A + (size_t)(lo - s.row0) * c->lda * es, (size_t)c->lda * es,
                                  static_cast<const char *>(A_rows) + (size_t)(lo - row0) * lda_host * es,
                                  (size_t)lda_host * es, (size_t)c->n * es, (size_t)(hi - lo), hipMemcpyHostToDevice,
                                  s.stream));
        if (b_rows)
            HIPT(hipMemcpyAsync(s.b + (lo - s.row0) * es, static_cast<const char *>(b_rows) + (lo - row0) * es,
                                (hi - lo) * es, hipMemcpyHostToDevice, s.stream));
        if (x_rows) {
            HIPT(hipMemcpyAsync(s.x + (lo - s.row0) * es, static_cast<const char *>(x_rows) + (lo - row0) * es,
                                (hi - lo) * es, hipMemcpyHostToDevice, s.stream));
            bool zeros = true;  // +0 / -0 only (A x is then exactly zero)
            const char *xs = static_cast<const char *>(x_rows) + (lo - row0) * es;
            for (int64_t i = 0; i < hi - lo && zeros; ++i)
                zeros = es == 4 ? reinterpret_cast<const float *>(xs)[i] == 0.0f
                                : reinterpret_cast<const double *>(xs)[i] == 0.0;
            const bool whole = lo == s.row0 && hi == s.row0 + s.nloc;
            s.x_zero = whole ? zeros : (s.x_zero && zeros);
        }
        TRY(rank_wait_stream(c, s.stream, "the copies of cgx_set_rows"));
    }
    if (x_rows && row0 == 0 && nrows == c->n) c->x_incomplete = c->x_deferred = false;  // x fully defined again
    c->state = ST_IDLE;
    return CGX_OK;
}

int cgx_set_system(cgx_ctx *c, const void *A, const void *b, const void *x0) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    return cgx_set_rows(c, 0, c->n, A, c->n, b, x0);
}

int cgx_generate_spd(cgx_ctx *c, uint64_t seed) {
    const Range range_("cgx_generate_spd");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    if (c->op == OP_POISSON) return fail(CGX_ERR_ARG, "the Poisson operator has no matrix to generate (use cgx_fill)");
    if (c->flags & CGX_HOST_STREAM) TRY(sync_all(c));  // copies of enqueued iterations still read A_host
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        if (s.A_host && (c->flags & CGX_SYMMETRIC)) {
            // the packed tiles chunk by chunk on the device, then to the host copy
            const int64_t ntiles = sym_tiles(c->lda), tb = 128 * 128 * 8;
            for (int64_t q0 = 0; q0 < ntiles; q0 += s.tile_rows) {
                const int64_t cnt = std::min(s.tile_rows, ntiles - q0);
                HIPT(gen_spd_sym_tiles_f64(c->n, c->lda, seed, q0, cnt, reinterpret_cast<double *>(s.tile[0]),
                                           s.stream));
                HIPT(hipMemcpyAsync(s.A_host + (size_t)q0 * tb, s.tile[0], (size_t)cnt * tb, hipMemcpyDeviceToHost,
                                    s.stream));
            }
            HIPT(gen_b_f64(c->n, seed, reinterpret_cast<double *>(s.b), s.stream));
            TRY(rank_wait_stream(c, s.stream, "the tile generation"));
            s.res_dirty = s.res_rows > 0;
        } else if (s.A_host) {
            // Generate each tile on the device and move it to the host copy of A;
            // b is generated for the whole block first (rows are independent).
            const int64_t row_bytes = c->lda * (int64_t)c->es;
            for (int64_t r0 = 0; r0 < s.nloc; r0 += s.tile_rows) {
                const int64_t rows = std::min(s.tile_rows, s.nloc - r0);
                if (f32ref(c))
                    HIPT(gen_spd_f32(c->n, c->lda, s.row0 + r0, rows, seed, reinterpret_cast<float *>(s.tile[0]),
                                     reinterpret_cast<float *>(s.b) + r0, s.stream));
                else
                    HIPT(gen_spd_f64(c->n, c->lda, s.row0 + r0, rows, seed, reinterpret_cast<double *>(s.tile[0]),
                                     reinterpret_cast<double *>(s.b) + r0, s.stream));
                HIPT(hipMemcpyAsync(s.A_host + (size_t)r0 * row_bytes, s.tile[0], (size_t)rows * row_bytes,
                                    hipMemcpyDeviceToHost, s.stream));
            }
            s.res_dirty = s.res_rows > 0;
            TRY(rank_wait_stream(c, s.stream, "the tile generation"));
        } else if (c->flags & CGX_SYMMETRIC) {
            HIPT(gen_spd_sym_f64(c->n, c->lda, seed, reinterpret_cast<double *>(s.A), reinterpret_cast<double *>(s.b),
                                 s.stream));
        } else if (f32ref(c)) {
            HIPT(gen_spd_f32(c->n, c->lda, s.row0, s.nloc, seed, reinterpret_cast<float *>(s.A),
                             reinterpret_cast<float *>(s.b), s.stream));
        } else {
            HIPT(gen_spd_f64(c->n, c->lda, s.row0, s.nloc, seed, reinterpret_cast<double *>(s.A),
                             reinterpret_cast<double *>(s.b), s.stream));
        }
        HIPT(hipMemsetAsync(s.x, 0, s.nloc * c->es, s.stream));
        s.x_zero = true;
    }
    TRY(sync_all(c));
    c->state = ST_IDLE;
    return CGX_OK;
}

int cgx_set_x(cgx_ctx *c, const void *x) {
    if (!c || !x) return fail(CGX_ERR_ARG, "NULL argument");
    return cgx_set_rows(c, 0, c->n, nullptr, c->n, nullptr, x);
}

int cgx_get_x(cgx_ctx *c, void *x) {
    const Range range_("cgx_get_x");
    if (!c || !x) return fail(CGX_ERR_ARG, "NULL argument");
    TRY(check_x_complete(c));
    const size_t es = (size_t)c->es;
    if (c->mode == M_RCCL && c->nranks > 1) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        NCCLC(c, ncclAllGather(s.x, s.xfull, (size_t)s.nloc, f32ref(c) ? ncclFloat : ncclDouble, s.comm, s.stream),
              "ncclAllGather(x) for cgx_get_x");
        HIPT(hipMemcpyAsync(s.h_x ? s.h_x : x, s.xfull, (size_t)c->n * es, hipMemcpyDeviceToHost, s.stream));
        TRY(rank_wait_stream(c, s.stream, "the x allgather"));
        if (s.h_x) std::memcpy(x, s.h_x, (size_t)c->n * es);
        return CGX_OK;
    }
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipMemcpyAsync(s.h_x ? s.h_x : static_cast<char *>(x) + s.row0 * es, s.x, s.nloc * es,
                            hipMemcpyDeviceToHost, s.stream));
    }
    TRY(sync_all(c));
    for (auto &s : c->sh)
        if (s.h_x) std::memcpy(static_cast<char *>(x) + s.row0 * es, s.h_x, s.nloc * es);
    return CGX_OK;
}

}  // extern "C"
