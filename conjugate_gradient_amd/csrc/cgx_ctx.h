// cgx_ctx.h -- internal to libcgx: the context and shard types, the error
// plumbing, and the functions the host-side files share:
//   cgx_setup.hip     contexts and shards: create, destroy, data in and out
//   cgx_exchange.hip  the per-iteration exchanges (RCCL / device copies / p2p)
//   cgx_iterate.hip   the conjugrad loop: begin, iterations, gating, solve
//   cgx_api.hip       errors, devices and the kernel-level entry points
// Not part of the C ABI (include/cgx.h).
//
// Reference mapping:
//   conjugrad()              serialConjugate.c:180-259 / parallel_cg.c:248-345
//       -> cgx_solve = cgx_solve_begin (:209-212) + cgx_iterate (:213-245)
//   MPI_Bcast x0 / MPI_Scatter A,b   parallel_cg.c:109-117 -> cgx_set_rows
//   MPI_Allgather(local_p -> p)      parallel_cg.c:290-291 -> exchange_allgather
//   MPI_Allreduce(p.Ap), (r.r)       parallel_cg.c:287,294,313 -> exchange_scalar
//
// A context holds one or more shards.  A shard = one contiguous row block of
// A (rows [row0, row0+nloc), every column, leading dimension lda = n rounded
// up to 128 with zero padding), its slices of b, x, r, Ap, a full-length p
// (padded, zero tail) whose own slice doubles as the local p, and a small
// device scalar block.  Three exchange modes:
//   SINGLE  one shard, no exchange.
//   LOCAL   several shards in this process (distinct or repeated devices);
//           allgather by device-to-device copies, scalars combined from the
//           gathered partials in a fixed order (fp64: rank order; F32_REF:
//           MPICH's MPI_Allreduce order, parallel_cg.c).
//   RCCL    one shard per process (torchrun / mpirun style), RCCL allgather
//           of p and allreduce of the scalars over xGMI on the shard stream
//           (F32_REF: allgather of the partials + the MPICH-order combine).
// CGX_COMM_P2P (either multi-shard mode) follows point-to-point_cg.c instead:
// gather to rank 0 and send back, scalars summed in rank order (allSum).
//
// Scalar slots (8 bytes each; F32_REF stores a float at the slot start):
//   RR(j)   = r_j.r_j (global)      PAP(k) = p_k.Ap_k (global)   ring of 4
//   LRR(j), LPAP(k): this shard's partials when an exchange follows
//   GATHER+q: the partial of shard q (ordered combine)
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <mutex>
#include <new>
#include <string>
#include <vector>
#include <algorithm>

#include "cgx.h"
#include "cgx_kernels.h"

using namespace cgx;

namespace cgxh {
extern thread_local char g_err[1024];
int fail(int code, const char *fmt, ...);
// CGX_DEBUG=1: one line per rank-mode fail-fast event on stderr.
void debug_log(const char *fmt, ...);

// RCCL, loaded on first use (cgx_rccl.hip): rank mode calls it through these
// pointers (the macros below keep the nccl* names at the call sites).
struct RcclApi {
    decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&::ncclCommInitRank) CommInitRank = nullptr;
    decltype(&::ncclCommDestroy) CommDestroy = nullptr;
    decltype(&::ncclGetErrorString) GetErrorString = nullptr;
    decltype(&::ncclAllGather) AllGather = nullptr;
    decltype(&::ncclAllReduce) AllReduce = nullptr;
    decltype(&::ncclSend) Send = nullptr;
    decltype(&::ncclRecv) Recv = nullptr;
    decltype(&::ncclGroupStart) GroupStart = nullptr;
    decltype(&::ncclGroupEnd) GroupEnd = nullptr;
    // fail-fast: asynchronous error query, abort
    decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&::ncclCommAbort) CommAbort = nullptr;
    // what the communicator reports about itself (cgx_get_comm_info)
    decltype(&::ncclCommCount) CommCount = nullptr;
    decltype(&::ncclCommCuDevice) CommCuDevice = nullptr;
    decltype(&::ncclCommUserRank) CommUserRank = nullptr;
};
extern RcclApi g_rccl;
// Loads librccl.so.1 once; false (with cgx_last_error set) if it cannot.
// Every entry point that reaches RCCL first passes through this.
bool rccl_load();
}  // namespace cgxh

#ifndef CGX_RCCL_LOADER
#define ncclGetUniqueId (cgxh::g_rccl.GetUniqueId)
#define ncclCommInitRank (cgxh::g_rccl.CommInitRank)
#define ncclCommDestroy (cgxh::g_rccl.CommDestroy)
#define ncclGetErrorString (cgxh::g_rccl.GetErrorString)
#define ncclAllGather (cgxh::g_rccl.AllGather)
#define ncclAllReduce (cgxh::g_rccl.AllReduce)
#define ncclSend (cgxh::g_rccl.Send)
#define ncclRecv (cgxh::g_rccl.Recv)
#define ncclGroupStart (cgxh::g_rccl.GroupStart)
#define ncclGroupEnd (cgxh::g_rccl.GroupEnd)
#define ncclCommGetAsyncError (cgxh::g_rccl.CommGetAsyncError)
#define ncclCommAbort (cgxh::g_rccl.CommAbort)
#define ncclCommCount (cgxh::g_rccl.CommCount)
#define ncclCommCuDevice (cgxh::g_rccl.CommCuDevice)
#define ncclCommUserRank (cgxh::g_rccl.CommUserRank)
#endif

#define HIPT(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(CGX_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                              \
    } while (0)

#define NCCLT(expr)                                                                               \
    do {                                                                                          \
        ncclResult_t e_ = (expr);                                                                 \
        if (e_ != ncclSuccess)                                                                    \
            return fail(CGX_ERR_RCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                \
    } while (0)

// An RCCL call on the context's communicator (rank mode): `what` names the
// exchange for the error message; a call that returns ncclInProgress (the
// communicator is nonblocking) is waited for with the context's deadline; a
// context whose communicator was aborted refuses further RCCL calls.
#define NCCLC(c, expr, what)                                                            \
    do {                                                                                \
        if ((c)->dead) return dead_error(c);                                            \
        ncclResult_t e_ = (expr);                                                       \
        TRY(rccl_after(c, e_, what, #expr, __FILE__, __LINE__));                         \
    } while (0)

#define TRY(expr)                          \
    do {                                   \
        int rc_ = (expr);                  \
        if (rc_ != CGX_OK) return rc_;     \
    } while (0)

namespace cgxh {

constexpr int kScalSlots = 138;  // 16 ring slots, up to 112 gathered partials, 10 aux
constexpr int kMaxShards = 32;
// choose_overlap: the overlapped form runs when its measured time is below
// (1 - kOverlapMargin) x the plain form's (cgx_overlap_info.margin)
constexpr double kOverlapMargin = 0.01;
constexpr int S_RR = 0, S_PAP = 4, S_LRR = 8, S_LPAP = 12, S_GATHER = 16;
constexpr int S_TR = 128, S_TB = 129, S_LTR = 130, S_LTB = 131;  // true-residual check
constexpr int S_XNZ = 134;  // rank mode: count of ranks whose x0 is not all zeros
constexpr int S_XALPHA = 135;  // fused Poisson, x every D-th iteration: the alphas of the x updates left out (135, 136)
constexpr int S_KDONE = 132, S_RRFINAL = 133;  // device-side convergence: k+1 at the break, r.r there
constexpr int kLookRing = 8;                    // pinned slots for the host's lagged convergence checks
inline int ring(int64_t j) { return (int)(j & 3); }

enum Mode { M_SINGLE = 0, M_LOCAL = 1, M_RCCL = 2 };
enum Op { OP_DENSE = 0, OP_POISSON = 1 };
enum State { ST_IDLE = 0, ST_BEGUN = 1, ST_CONVERGED = 2 };

constexpr int kEvPairs = 256;
// CGX_PHASES: the kernels of an iteration that stamp their start / end
// (cgx_kernels.h kTsSlot), in the order they run on the first shard's stream.
enum TsKernel { TK_OWN = 0, TK_MV = 1, TK_UR = 2, TK_UXP = 3, kTsKern = 4 };
// iterations stamped before a resolve (1024 x 4 x 16 KiB = 64 MiB of HBM):
// a timed run of up to 1024 iterations never resolves (copies, waits) inside
constexpr int kTsIters = 1024;
constexpr size_t kXStageMax = 64u << 20;
constexpr int kStreamBufs = 3;
constexpr int kMaxCopyStreams = 4;

struct Shard {
    int dev = 0;
    int index = 0;  // global row-block index
    int64_t row0 = 0, nloc = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    char *A = nullptr, *b = nullptr, *x = nullptr, *r = nullptr, *Ap = nullptr, *pfull = nullptr,
         *xfull = nullptr, *scal = nullptr;
    char *pown = nullptr;  // this shard's p: pfull + row0 (dense) or the slab interior (Poisson)
    // fused Poisson iteration: r with halo rows (r = rh + one row) and a
    // second p slab; p_k lives in pfull for even k, in p2 for odd k
    char *rh = nullptr, *p2 = nullptr;
    char *p3 = nullptr;  // fused Poisson, x every third iteration: p_k in {pfull, p2, p3}[k % 3]
    char *p_alt = nullptr;  // the folded two-launch iteration: p_k for odd k (pfull holds even k)
    bool x_zero = true;  // x is known to be all zeros (x0 = 0: the first A x is skipped)
    RedWs ws{nullptr, nullptr};
    double *h_pin = nullptr;
    // pinned staging for cgx_get_x (x of this shard, or all of x in rank
    // mode), allocated with the context so the first D2H of a solve's result
    // does not set up HIP's pageable-copy path (~7 ms); null above kXStageMax
    char *h_x = nullptr;
    // convergence record {kdone, bits of r.r there} in host-mapped coherent
    // memory: the deciding kernel stores it, the host reads it after an event
    int64_t *h_rec = nullptr, *d_rec = nullptr;
    MatvecPlan plan;
    MatvecPlan fold_plan;  // k_matvec_fold_f64's (c->fold_p)
    // CGX_SYMMETRIC: A = the upper-triangle tiles; per-tile row / column
    // partials of a matVec; a staging buffer for rows copied from the host
    char *sym_prow = nullptr, *sym_pcol = nullptr, *sym_stage = nullptr;
    int64_t sym_stage_rows = 0;
    int sym_grid = 0;
    hipEvent_t ev_sync = nullptr;  // cross-shard ordering (LOCAL mode): local_barrier
    hipEvent_t ev_sync2 = nullptr;  // ... the r.r record point of the threaded iteration (cgx_local_mt.hip)
    hipEvent_t ev_root = nullptr;  // CGX_COMM_P2P in LOCAL mode: shard 0's result is ready
    std::vector<hipEvent_t> ev_t;  // timing pairs (CGX_TIMING)
    int ev_used = 0;
    // CGX_HOST_STREAM: A stays in pinned host memory; row tiles are copied
    // into kStreamBufs device buffers on `ncopy` copy streams while the
    // compute stream multiplies the previous tiles.
    char *A_host = nullptr;
    int64_t tile_rows = 0;
    char *tile[kStreamBufs] = {};
    int ncopy = 0;
    hipStream_t copy[kMaxCopyStreams] = {};
    hipEvent_t ev_loaded[kStreamBufs][kMaxCopyStreams] = {};
    hipEvent_t ev_free[kStreamBufs] = {};
    bool buf_used[kStreamBufs] = {};
    int next_buf = 0;
    MatvecPlan tile_plan;
    // CGX_STREAM_RESIDENT_MB: the first res_rows rows (CGX_SYMMETRIC: tiles) also live in HBM (A),
    // copied from A_host when res_dirty; only the rest streams per matVec,
    // and the resident rows are multiplied while the first tiles copy.
    int64_t res_rows = 0;
    bool res_dirty = false;
    MatvecPlan res_plan;
    hipEvent_t ev_look[8] = {};  // lagged convergence checks (kLookRing)
    hipEvent_t ev_prog[8] = {};  // rank mode, host-checked iterations: one per iteration (fail-fast progress)
    int prog_next = 0;
    // CGX_PHASES (shard 0): kTsIters x kTsKern timestamp slots on the device,
    // zero where no kernel stamped; ts_cur = the ring row of the iteration
    // being enqueued (-1 between iterations), ts_used = rows since the resolve
    int64_t *ts_dev = nullptr;
    int64_t *ts_host = nullptr;  // pinned copy for the resolve, allocated at the first one
    int ts_used = 0, ts_cur = -1;
    // overlap of the p exchange with the own-column-block matVec
    hipStream_t cstream = nullptr;
    hipEvent_t ev_pready = nullptr, ev_gathered = nullptr;
};

}  // namespace cgxh

namespace cgxh {
struct LocalPool;  // cgx_local_mt.hip
}

using namespace cgxh;

struct cgx_ctx {
    int64_t n = 0, lda = 0;
    int op = 0;        // OP_DENSE or OP_POISSON
    int64_t m = 0;     // Poisson grid width (n = m*m)
    int nranks = 1;
    int flags = 0;
    int es = 8;
    Mode mode = M_SINGLE;
    std::vector<Shard> sh;
    State state = ST_IDLE;
    int64_t k = 0;  // iterations of the current solve
    double last_rr = 0.0;
    int converged = 0;
    double solve_ms = 0.0, matvec_ms = 0.0;
    int64_t matvec_count = 0, total_iters = 0;
    // Row blocks aligned to the matVec's 128-column chunks (dense fp64,
    // resident A, several blocks): every matVec of the context runs the
    // rotated column order -- the block's own columns first, then the rest --
    // with the own part and the rest summed separately, so the overlapped
    // exchange (own launch beside the allgather, then the rest) and the plain
    // one (allgather, then one launch) give the same bits, and the choice
    // between them (choose_overlap, at creation) is a matter of speed only.
    bool rot = false;
    bool overlap = false;  // own-column-block matVec while p is exchanged
    // what choose_overlap measured (-1: not measured) and how it decided
    double ov_ag_us = -1.0, ov_split_us = -1.0, ov_one_us = -1.0, ov_cost_us = -1.0;
    // ... and the two whole forms, exchange + matVec end to end (the decision)
    double ov_form_us = -1.0, ov_plain_form_us = -1.0;
    double ov_forms_ms = -1.0;  // host wall time of that timing (this rank)
    int ov_how = CGX_OV_NA;
    bool fused = false;    // Poisson: two-kernel fused iteration (k_poisson_p + k_poisson_xr)
    bool fused_p = false;  // dense, one GPU, small n: two launches per iteration (matVec, k_update_xrp_f64)
    bool fold_p = false;   // ... with the p update folded into the matVec (k_matvec_fold_f64, k_update_xr_stop_f64)
    bool ref_mv_dot = false;  // CGX_F32_REF, resident dense: the matVec's last block runs vecVec(p, Ap) (any mode)
    bool ref_fused = false;   // ... and on one GPU: two launches per iteration (matVec + p.Ap, x/r/r.r/p)
    bool halo_overlap = false;  // fused Poisson, several slabs: r's halo exchange overlaps k_poisson_p
    bool halo_pending = false;  // an overlapped r halo exchange is in flight on the comm streams
    // fused Poisson, one process, several slabs (pull kernels): k_poisson_p
    // reads r's halo rows in place from the neighbouring slabs instead of
    // copies into rh's halo rows
    bool halo_pull = false;
    // ... and the r.r of iteration c->k is still partials only (its combine
    // folded into the next k_poisson_p): settle_rr forms it when needed
    bool rr_unsummed = false;
    // fused Poisson: x updated every other iteration (k_poisson_xr_f64's XM;
    // CGX_POISSON_XDEFER=0: every iteration).  Within one cgx_iterate call the
    // iterations k0, k0+2, ... leave x out and k0+1, k0+3, ... catch up; a call
    // that ends after a left-out update finishes x (poisson_x_finish).
    bool xdefer = false;
    int xd = 1;  // the period: 2 (default) or 3 (CGX_POISSON_XDEFER=3, a third p slab)
    int64_t xd_k0 = 0;
    // a cgx_iterate call failed: x may hold part of an iteration, or (x_deferred,
    // xd > 1) lack the alphas left out, which cannot be placed -- x is
    // incomplete until cgx_set_x defines it or the next cgx_solve_begin;
    // cgx_get_x / cgx_iterate / cgx_residual_norm refuse it
    bool x_incomplete = false, x_deferred = false;
    bool xalpha_pending = false;  // fused Poisson: an xr kernel left alpha_k p_k out of x (xmode 0), not yet caught up
    // a cgx_iterate call failed part-way through an iteration (a HIP error, an
    // RCCL deadline, a row block's worker): some blocks may have applied part
    // of iteration k, so repeating it would apply it twice -- cgx_iterate
    // refuses until the next cgx_solve_begin (x: x_incomplete)
    bool iter_failed = false;
    // rank mode fail-fast (cgx_exchange.hip, rank_wait_*): every host wait
    // polls with a deadline of rccl_timeout_s seconds (CGX_RCCL_TIMEOUT_S,
    // default 60, 0 = wait forever) and checks the communicator's asynchronous
    // error; on either the communicator is aborted (ncclCommAbort, which also
    // stops RCCL kernels still waiting on a peer) and the call returns
    // CGX_ERR_RCCL.  `dead` then refuses every later RCCL call.
    double rccl_timeout_s = 60.0;
    bool dead = false;
    char dead_why[400] = "";
    const char *last_coll = "none";  // the last exchange enqueued, and its iteration
    int64_t last_coll_k = -1;
    bool peer = false;  // multi-shard over distinct devices: peer access enabled between every pair
    // LOCAL mode: the allgather and the scalar combines as one pull kernel per
    // consuming shard (gather_slices / combine_peers_*), the default; false
    // (CGX_LOCAL_XCHG=copy): one hipMemcpyPeerAsync per (consumer, producer)
    // pair, round 3's form, kept for A/B runs
    bool xchg_kernels = true;
    // ... and, for the dense fp64 iteration, the two scalar combines folded
    // into the kernels that consume them (k_update_r_f64 sums the p.Ap
    // partials, k_update_xp_f64 the r.r partials: PeerSum), so an iteration
    // launches no combine kernel (CGX_LOCAL_FUSE=0: separate combine kernels)
    bool fuse_combine = false;
    // ... and for CGX_F32_REF: both scalars summed in MPICH order by the
    // kernels that consume them (k_dot_ref_f32_blk<kDotXR>: p.Ap,
    // k_update_p_ref_f32: r.r; PeerSumF32), the same bits as the combine kernels
    bool fuse_f32 = false;
    // LOCAL mode: one host thread per row block enqueues its block's iteration
    // (cgx_local_mt.hip); null when not used
    cgxh::LocalPool *pool = nullptr;
    // CGX_PHASES: resolved per-iteration phase durations (us), cgx_phase_times' order;
    // the wall clock's rate, and the previous stamped iteration's first start /
    // last end (ticks; 0 = none) so the gap across a resolve is still measured
    std::vector<float> ph_samples[CGX_PH_COUNT];
    double ts_khz = 100000.0;
    int64_t ts_prev_start = 0, ts_prev_end = 0;
};

namespace cgxh {

inline bool f32ref(const cgx_ctx *c) { return (c->flags & CGX_F32_REF) != 0; }
inline void *slot(const Shard &s, int i) { return s.scal + 8 * i; }
inline bool p2p(const cgx_ctx *c) { return (c->flags & CGX_COMM_P2P) != 0; }
// Where a kernel writes its (partial) scalar: the global slot directly when
// there is nothing to combine, else the shard-local slot.
inline int out_slot(const cgx_ctx *c, int lslot, int gslot) { return c->mode == M_SINGLE ? gslot : lslot; }
inline int64_t *rec_of(const cgx_ctx *c, const Shard &s, bool gated) {
    return (gated && &s == &c->sh[0]) ? s.d_rec : nullptr;
}

inline const int64_t *gate_of(const Shard &s, bool gated) {
    return gated ? reinterpret_cast<const int64_t *>(slot(s, S_KDONE)) : nullptr;
}

// roctx range over an API call (rocprofv3 --marker-trace shows the solve
// phases on the timeline; a no-op without a tool attached).
struct Range {
    explicit Range(const char *name) { roctxRangePushA(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// cgx_setup.hip
int set_dev(const Shard &s);
int alloc_shard(cgx_ctx *c, Shard &s);
bool small_matvec(const cgx_ctx *c);  // k_matvec_small_f64 applies (cgx_setup.hip)
void free_shard(Shard &s);
int check_n(int64_t n, int nranks);
cgx_ctx *new_ctx(int64_t n, int nranks, int flags);
bool can_rotate(const cgx_ctx *c);
int alloc_overlap(cgx_ctx *c);
int finish_create(cgx_ctx *c, cgx_ctx **out);
// cgx_exchange.hip
int timing_resolve(cgx_ctx *c);
int phase_iter_begin(cgx_ctx *c);
int64_t *ts_of(cgx_ctx *c, const Shard &s, int kern);
void phase_iter_end(cgx_ctx *c);
int phase_resolve(cgx_ctx *c);
int progress_mark(cgx_ctx *c);
int local_barrier(cgx_ctx *c);
int exchange_halo(cgx_ctx *c, bool from_x);
int exchange_halo_of(cgx_ctx *c, char *Shard::*slab);
int p2p_allgather(cgx_ctx *c, bool from_x);
int p2p_scalar(cgx_ctx *c, int lslot, int gslot);
int exchange_allgather(cgx_ctx *c, bool from_x);
int exchange_scalar(cgx_ctx *c, int lslot, int gslot);
PeerSum peer_sum(const cgx_ctx *c, const Shard &d, int lslot, int gslot);
PeerSumF32 peer_sum_f32(const cgx_ctx *c, const Shard &d, int lslot, int gslot);
int overlapped_matvec(cgx_ctx *c, int dot_slot, bool gated, bool timed = true);
int overlap_matvecs(cgx_ctx *c, Shard &d, int dot_slot, bool gated, bool timed = true);
int choose_overlap(cgx_ctx *c);
int exchange_halo_async(cgx_ctx *c);
int settle_halo(cgx_ctx *c);
int sync_all(cgx_ctx *c);
// rank-mode fail-fast (plain blocking waits in the other modes)
int rccl_after(cgx_ctx *c, ncclResult_t r, const char *what, const char *expr, const char *file, int line);
int dead_error(const cgx_ctx *c);
int rank_wait_event(cgx_ctx *c, hipEvent_t ev, const char *what);
int rank_wait_stream(cgx_ctx *c, hipStream_t st, const char *what);
double rccl_timeout_from_env();
// cgx_local_mt.hip
bool local_mt_eligible(const cgx_ctx *c);
int local_mt_start(cgx_ctx *c);
void local_mt_stop(cgx_ctx *c);
int local_mt_iteration(cgx_ctx *c, double eps, bool gated);
PeerTable peer_table(const cgx_ctx *c, char *Shard::*buf, int64_t off);
// cgx_iterate.hip
int matvec_rows(cgx_ctx *c, Shard &s, const MatvecPlan &pl, const char *Arows, int64_t r0, int64_t rows,
                const char *vec, bool fuse_dot, int dot_slot, bool gated = false, int64_t *ts = nullptr);
int matvec_streamed(cgx_ctx *c, Shard &s, const char *vec);
int matvec_sym_streamed(cgx_ctx *c, Shard &s, const char *vec, bool with_dot, int dot_slot, const int64_t *gate);
int launch_matvec(cgx_ctx *c, Shard &s, const char *vec, bool with_dot, int dot_slot, bool gated = false);
int x0_is_zero(cgx_ctx *c, bool *zero);
int do_begin(cgx_ctx *c);
int read_scalar(cgx_ctx *c, int gslot, double *out);
int do_iteration_poisson(cgx_ctx *c, double eps, int *stop, bool gated);
int poisson_x_finish(cgx_ctx *c);
int settle_rr(cgx_ctx *c);
int check_x_complete(const cgx_ctx *c);
int do_iteration(cgx_ctx *c, double eps, int *stop, bool gated = false);
bool warm_eligible(const cgx_ctx *c);
int warm_solve_kernels(cgx_ctx *c);
// cgx_api.hip
int dev_ws(RedWs *out);
int check_dtype(int dtype);

}  // namespace cgxh
