/*
 * cgx.h -- C ABI of the MI355X-native conjugate-gradient hot path (libcgx.so).
 *
 * This is the drop-in boundary for the reference's CG loop
 * (mawunyega/conjugate_gradient).  The reference has no library API of its
 * own: its solvers are self-contained C programs whose functions are
 *
 *   void  matVec(float *out, float *A, float *x [, int local_row]);
 *         serialConjugate.c:109-120, parallel_cg.c:172-184
 *   float vecVec(float *v1, float *v2 [, int local_row]);
 *         serialConjugate.c:145-155, parallel_cg.c:211-221
 *   void  residual(float *out, float *b, float *Ax [, int]);      :124-131
 *   void  scalarVec / vecAdd / vecSub(...)                          :135-177
 *   void  conjugrad(float *A, float *b, float *x
 *                   [, int local_row, int rank, int P]);
 *         serialConjugate.c:180-259, parallel_cg.c:248-345
 *   MPI_Bcast / MPI_Scatter distribution        parallel_cg.c:109-117
 *   MPI_Allgather(p) + 2x MPI_Allreduce(SUM)     parallel_cg.c:287-313
 *
 * and this header maps each of them to an entry point (see INTEGRATION.md for
 * the function-by-function table and the ctypes / C bindings a maintainer
 * adds).  Conventions:
 *   - plain C types only: pointers, sizes, int status codes; nothing aborts;
 *   - host arrays are caller-owned; device buffers, streams, events and RCCL
 *     communicators are owned by the context;
 *   - a context is not thread-safe; one host thread drives it;
 *   - x is in/out exactly like conjugrad's vectorX (x0 in, solution out).
 *
 * Numerics (flags):
 *   CGX_F64      (default) double data and arithmetic; the fp64 reading of
 *                conjgrad.m.  Dots are deterministic fixed-order reductions.
 *                Precondition: A is finite (with x0 = 0 the initial A x0 is
 *                skipped as exactly zero; an Inf/NaN in A would have made it NaN).
 *   CGX_F32_REF  float data, serialConjugate.c's operation order: sequential
 *                fp32 accumulation per row and per dot, no FMA contraction.
 *                Produces the reference's x bit for bit: serialConjugate.c on
 *                one shard; parallel_cg.c on P row blocks (per-rank partials
 *                combined in MPICH 3.3's MPI_Allreduce order, recursive
 *                doubling); point-to-point_cg.c with CGX_COMM_P2P (rank-order
 *                allSum).  Pinned by mpiexec runs of the unmodified programs
 *                (tests/golden/mpi/).
 *
 * Multi-GPU: the matrix is split into contiguous row blocks (parallel_cg.c:83,
 * 97-99; n % nranks == 0 as parallel_cg.c:86-90 requires).  Per iteration
 * the p vector is allgathered and the two scalars p.Ap and r.r are
 * allreduced (RCCL over xGMI in rank mode; in the multi-shard mode one pull
 * kernel per consuming row block reads the other blocks' slices / partials
 * through peer pointers).  x stays distributed and is gathered on demand.
 */
#ifndef CGX_H
#define CGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGX_VERSION 101 /* 0.1.1: cgx_overlap_info gained the end-to-end form times */

/* ---- status codes (0 = OK, negative = error) --------------------------- */
#define CGX_OK            0
#define CGX_ERR_ARG      -1  /* bad argument / unsupported combination        */
#define CGX_ERR_HIP      -2  /* a HIP runtime call failed                      */
#define CGX_ERR_RCCL     -3  /* an RCCL call failed                            */
#define CGX_ERR_SHAPE    -4  /* n not divisible by ranks, rows out of range   */
#define CGX_ERR_NOMEM    -5  /* device or pinned allocation failed            */
#define CGX_ERR_STATE    -6  /* call out of order (iterate before begin, ...) */
#define CGX_ERR_NODEV    -7  /* no usable GPU                                  */

/* ---- flags ---------------------------------------------------------------- */
#define CGX_F64          0x0   /* double data (default)                        */
#define CGX_F32_REF      0x1   /* float data, bit-exact serialConjugate.c order */
#define CGX_TIMING       0x100 /* time every matVec launch with HIP events      */
#define CGX_NO_OVERLAP   0x400 /* multi-shard dense fp64: do not overlap the p
                                  exchange with the own-column-block matVec
                                  (the allgather, then one matVec launch).
                                  Without it the form is chosen at creation
                                  when every row block is a multiple of 128
                                  rows: the overlap runs only if that whole
                                  form (allgather beside the split matVec),
                                  timed end to end at creation, beats the
                                  plain one by 1 % (cgx_get_overlap_info;
                                  env CGX_OVERLAP=0 / 1: never / always).  Both
                                  forms give the same bits. */
#define CGX_OVERLAP_ACTIVE 0x800 /* reported in cgx_info.flags when it is on */
#define CGX_FUSED_ACTIVE 0x2000 /* reported in cgx_info.flags: a fused
                                   iteration is on -- the Poisson operator's
                                   two-kernel iteration (even m; env
                                   CGX_POISSON_FUSED=0 selects the stencil /
                                   r / x,p three-kernel split), or a small
                                   dense fp64 system on one GPU iterating in
                                   two launches instead of three (n <= 8192;
                                   env CGX_FUSE_P=0 / 1: never / any n);
                                   results are the same bits either way */
#define CGX_COMM_P2P     0x1000 /* point-to-point_cg.c's exchange instead of
                                   collectives: gather to rank 0, then rank 0
                                   sends to every rank (ncclSend/Recv; device
                                   copies through shard 0 in multi-shard mode).
                                   Scalars are summed in rank order (allSum,
                                   point-to-point_cg.c:339-359).  For the
                                   p2p-vs-collective comparison of the report. */
#define CGX_DETERMINISTIC 0x4000 /* rank mode, fp64: combine the two scalars by
                                    allgathering the per-rank partials and
                                    summing them in rank order (as multi-shard
                                    mode always does) instead of ncclAllReduce:
                                    results independent of RCCL's algorithm and
                                    bitwise equal to the multi-shard run with the
                                    same partition */
#define CGX_SYMMETRIC    0x8000 /* fp64, one GPU: keep only the upper triangle of
                                   A, in 128 x 128 tiles, and compute A.p from
                                   it (half the bytes per matVec).  CG requires
                                   a symmetric A; this mode reads only
                                   A[i][j] for j >= 128*(i/128) (the lower
                                   triangle outside the diagonal tiles is never
                                   read).  With CGX_HOST_STREAM the tiles stay
                                   in pinned host memory and stream in chunks.
                                   Sums run in a different order than
                                   the row-major kernel: results agree to fp64
                                   rounding, deterministically. */
#define CGX_HOST_STREAM  0x200 /* keep A in pinned host memory and stream row
                                  tiles through the GPU every matVec (out-of-HBM
                                  systems; tile size CGX_STREAM_TILE_MB, default
                                  256, copy streams CGX_STREAM_COPIES, default 2) */
#define CGX_PHASES       0x10000 /* dense fp64 (row-major, resident A): the
                                    kernels of every iteration on the first
                                    shard stamp their start and end on the
                                    device's constant clock -- nothing is
                                    inserted between them -- and
                                    cgx_get_phase_times() turns the stamps into
                                    phase durations after the fact */
#define CGX_PEER_ACTIVE  0x20000 /* reported in cgx_info.flags: a multi-shard
                                    context spans distinct devices and peer
                                    access is enabled between every pair of
                                    them (the exchange kernels then read
                                    peers' memory over xGMI) */
#define CGX_SMALL_ACTIVE 0x40000 /* reported in cgx_info.flags: one GPU, one
                                    resident fp64 row block of 2048..8192
                                    columns -- the matVec stages the vector in
                                    LDS, one block per CU (k_matvec_small_f64;
                                    CGX_MV_SMALL=0 turns it off) */
#define CGX_FOLD_ACTIVE  0x80000 /* reported in cgx_info.flags: the two-launch
                                    iteration folds p = r + beta p into the
                                    next matVec (CGX_FOLD_P) */
#define CGX_XDEFER_ACTIVE 0x100000 /* reported in cgx_info.flags: the fused
                                    Poisson iteration updates x only every
                                    other or every third iteration (60 / 58.7
                                    instead of 64 B per grid point; x the same
                                    bits after every cgx_iterate call;
                                    CGX_POISSON_XDEFER=0: every iteration) */
#define CGX_XDEFER3_ACTIVE 0x200000 /* reported in cgx_info.flags with
                                    CGX_XDEFER_ACTIVE: every third iteration
                                    (the default, a third p slab;
                                    CGX_POISSON_XDEFER=2: every other) */
/* Reported in cgx_info.flags: how a context with several row blocks
 * exchanges, so a caller (bench.py) can say what ran. */
#define CGX_PULL_ACTIVE   0x400000 /* one process: the exchange runs as pull
                                    kernels on each consuming block's stream
                                    (else one hipMemcpyPeerAsync per block pair,
                                    CGX_LOCAL_XCHG=copy) */
#define CGX_FOLDED_ACTIVE 0x800000 /* one process, fp64: both scalar combines
                                    summed in rank order by the kernels that
                                    consume them (else a combine kernel per
                                    block and scalar, CGX_LOCAL_FUSE=0) */
#define CGX_HALO_PULL_ACTIVE 0x1000000 /* one process, fused Poisson: r's halo
                                    rows read in place from the neighbouring
                                    slabs by k_poisson_p (no halo copies) */
#define CGX_THREADS_ACTIVE 0x2000000 /* one process: one host thread per row
                                    block enqueues its work (CGX_LOCAL_THREADS=1) */
#define CGX_HALO_OVERLAP_ACTIVE 0x4000000 /* fused Poisson over slabs in rank
                                    mode (or copies): r's halo exchange runs on
                                    the comm stream beside k_poisson_p's
                                    interior (CGX_HALO_OVERLAP=0: before it) */

typedef struct cgx_ctx cgx_ctx;

/* Opaque RCCL bootstrap id (ncclUniqueId is 128 bytes). */
typedef struct { char bytes[128]; } cgx_unique_id;

typedef struct {
    int64_t n;            /* global system size                               */
    int64_t lda;          /* device leading dimension (n rounded up to 128)   */
    int     nranks;       /* row blocks in the whole job                      */
    int     nshards;      /* row blocks driven by this process                */
    int     rank0;        /* global index of this process's first row block   */
    int64_t row0;         /* first global row owned by this process           */
    int64_t nrows;        /* rows owned by this process                       */
    int     flags;
    int     elem_bytes;   /* 8 (CGX_F64) or 4 (CGX_F32_REF)                   */
} cgx_info;

typedef struct {
    int64_t iterations;    /* loop iterations of the last solve (k+1 at break) */
    int     converged;     /* 1 if sqrt(r.r) < eps ended the loop              */
    double  rr;            /* last r.r (global)                                */
    double  solve_ms;      /* host wall time of the last cgx_solve             */
    double  matvec_ms;     /* sum of timed matVec kernel durations (CGX_TIMING)*/
    int64_t matvec_count;  /* matVec launches timed                            */
    int64_t total_iterations; /* iterations since the context was created     */
} cgx_stats;

/* Per-phase times of the iterations since the last cgx_reset_timing (or since
 * creation), CGX_PHASES contexts: for each phase the median and the mean over
 * the iterations, in microseconds, and the number of samples.  Phases follow
 * parallel_cg.c's loop (:288-323) on the first shard's stream: a kernel's own
 * span (first block's start to last block's end), or the span between two
 * consecutive kernels -- the exchange enqueued between them, or a launch gap.
 * Consecutive phases tile the iteration: MATVEC_OWN + GATHER_EXPOSED + MATVEC
 * + COMBINE_PAP + UPDATE_R + COMBINE_RR + UPDATE_XP + GAP = ITERATION. */
#define CGX_PH_MATVEC_OWN     0 /* overlap: own-column-block matVec (p local)   */
#define CGX_PH_GATHER_EXPOSED 1 /* the compute stream waiting for p's allgather
                                   (overlap: from the end of the own-block
                                   launch to the start of the rest launch,
                                   which waits for the allgather on the same
                                   stream; otherwise the whole allgather,
                                   launch gap included) parallel_cg.c:290-291 */
#define CGX_PH_MATVEC         2 /* the matVec with p.Ap (overlap: the rest
                                   launch, accumulating onto the own block's
                                   row sums, with p.Ap)               :292-293 */
#define CGX_PH_COMBINE_PAP    3 /* MPI_Allreduce(p.Ap) counterpart        :294   */
#define CGX_PH_UPDATE_R       4 /* r -= alpha Ap, r.r                     :304-309 */
#define CGX_PH_COMBINE_RR     5 /* MPI_Allreduce(r.r) counterpart         :313   */
#define CGX_PH_UPDATE_XP      6 /* x += alpha p, p = r + beta p  :299-303,318-322 */
#define CGX_PH_GAP            7 /* end of an iteration to the start of the next
                                   (host launch rate, lookahead waits)          */
#define CGX_PH_ITERATION      8 /* start of an iteration to the start of the next */
#define CGX_PH_MATVEC_BUSY    9 /* not a tile: the time the iteration's matVec
                                   kernels ran, the union of their spans (with
                                   the overlap: the own-block launch and the
                                   rest launch) -- the matVec's duration
                                   without the wait for p */
#define CGX_PH_COUNT         10
typedef struct {
    int64_t samples[CGX_PH_COUNT];
    double  median_us[CGX_PH_COUNT];
    double  mean_us[CGX_PH_COUNT];
} cgx_phase_times;

/* What the exchange runs on (rank mode): the communicator's rank count,
 * device and rank as RCCL reports them (ncclCommCount / ncclCommCuDevice /
 * ncclCommUserRank), and the PCI bus id of the context's device.  Other
 * modes: nranks = row blocks, rccl_device = -1. */
typedef struct {
    int  rccl_nranks;
    int  rccl_device;
    int  rccl_rank;
    int  device;
    char pci_bus_id[32];
} cgx_comm_info;

/* How the p exchange of an aligned multi-shard dense fp64 context was chosen
 * (parallel_cg.c:290-293: allgather p, then the matVec).  At creation the
 * context times both whole forms end to end on its own row blocks: overlap =
 * the real allgather (RCCL in rank mode, the pull kernels in one process) in
 * flight beside the own-column-block launch, then the rest launch; plain =
 * the allgather, then one launch over the whole row block.  The overlapped
 * form runs when overlap_form_us < (1 - margin) * plain_form_us.  In rank
 * mode every number is the max over ranks, so every rank decides alike.  The
 * parts are timed too and reported: the matVec split in two launches against
 * the one launch, and the allgather alone.  Times in microseconds, -1 when
 * not measured. */
#define CGX_OV_MEASURED 0 /* chosen from the measurement                     */
#define CGX_OV_FORCED   1 /* CGX_OVERLAP=1 / force: on                       */
#define CGX_OV_OFF      2 /* CGX_NO_OVERLAP or CGX_OVERLAP=0: off            */
#define CGX_OV_NA       3 /* no choice: one shard, unaligned blocks, fp32,
                             streamed A, p2p exchange                        */
typedef struct {
    int    active;         /* the overlapped form runs (CGX_OVERLAP_ACTIVE) */
    int    decided_by;     /* CGX_OV_*                                      */
    double allgather_us;   /* one allgather of p                            */
    double split_us;       /* own-block launch + rest launch                */
    double one_launch_us;  /* the one launch over the whole row block       */
    double split_cost_us;  /* split_us - one_launch_us (max over blocks)    */
    double overlap_form_us; /* the overlapped form, allgather included (the
                               slowest block, best of 2 passes of 2 forms
                               back to back)                                 */
    double plain_form_us;  /* the plain form: allgather, then one launch     */
    double margin;         /* the hysteresis of the decision (0.01)          */
    double forms_ms;       /* host wall time the end-to-end timing added to
                              the context's creation (this process)         */
} cgx_overlap_info;

/* ---- errors / info ------------------------------------------------------- */
const char *cgx_strerror(int code);
/* Detail message of the last failure on this thread ("" if none). */
const char *cgx_last_error(void);
int cgx_version(void);
int cgx_device_count(int *count);
/* The calling thread's pending HIP error (hipPeekAtLastError; 0 = none).
 * libcgx consumes the errors of the HIP calls it makes and reports them
 * through its own return codes, so this stays 0 across its entry points. */
int cgx_hip_last_error(void);
/* PCI bus id of a visible device ("0000:xx:yy.z"). */
int cgx_device_pci_bus_id(int device, char *buf, int len);
/* The link between two visible devices: *link_type as HSA reports it (4 =
 * xGMI, 2 = PCIe; -1 when HIP cannot tell), *hops, and *peer = 1 when
 * device_a can access device_b's memory directly (hipDeviceCanAccessPeer). */
int cgx_device_link(int device_a, int device_b, int *link_type, int *hops, int *peer);

/* ---- context lifetime ------------------------------------------------------ */
/* One GPU (device `device`).  Replaces serialConjugate.c's single process.
 * Dense n <= 16384 (no CGX_TIMING / CGX_PHASES / CGX_HOST_STREAM /
 * CGX_SYMMETRIC): the solve's kernels are launched once here, as no-ops, so
 * the first solve does not carry the runtime's first-launch cost
 * (CGX_WARM=0: not). */
int cgx_create(cgx_ctx **ctx, int64_t n, int device, int flags);

/* One process driving `nshards` row blocks on devices[0..nshards-1] (a device
 * may repeat: several row blocks on one GPU).  Exchange by pull kernels on
 * each consuming block's stream: one gather of p (k_gather_slices), one
 * rank-order combine per scalar (k_combine_peers); CGX_LOCAL_XCHG=copy:
 * one hipMemcpyPeerAsync per block pair instead (the same bits). */
int cgx_create_multi(cgx_ctx **ctx, int64_t n, int nshards, const int *devices, int flags);

/* One process per GPU (parallel_cg.c's one MPI rank per process): this
 * process owns row block `rank` of `nranks`; `id` comes from
 * cgx_get_unique_id() on rank 0 and is broadcast by the caller.  Exchange by
 * RCCL (allgather p, allreduce p.Ap and r.r) on the context's stream.
 * Fail-fast (the reference stops the job with MPI_Abort, parallel_cg.c:79-94):
 * the communicator's initialisation and every host wait are bounded by a
 * deadline of CGX_RCCL_TIMEOUT_S seconds (environment, default 60; 0 = wait
 * forever), and the waits watch RCCL's asynchronous error.  A rank that never joins,
 * dies, or issues a different collective makes the others' calls return
 * CGX_ERR_RCCL (naming the exchange and iteration) instead of hanging; the
 * communicator is then aborted and the context only accepts cgx_destroy. */
int cgx_get_unique_id(cgx_unique_id *id);
/* Loads RCCL (done on first rank-mode use anyway) and checks that every entry
 * point libcgx calls is present: CGX_OK, or CGX_ERR_RCCL with the reason in
 * cgx_last_error().  Needs no GPU.  A failed load is permanent for the process. */
int cgx_rccl_available(void);
int cgx_create_rank(cgx_ctx **ctx, int64_t n, int rank, int nranks,
                    const cgx_unique_id *id, int device, int flags);

/* Matrix-free 5-point 2D Poisson operator (configs[4]; no reference
 * counterpart): n = m*m unknowns on an m x m interior grid, Dirichlet zero
 * boundary, (A u)_ij = 4u_ij - u_(i-1)j - u_(i+1)j - u_i(j-1) - u_i(j+1),
 * natural row-major order.  Multi-GPU splits the grid into slabs of m/P grid
 * rows (m % P == 0) and exchanges one halo row with each neighbour per
 * iteration (ncclSend/Recv in rank mode) instead of allgathering p.
 * CGX_F64 only; set b / x0 with cgx_fill or cgx_set_rows (A must be NULL). */
int cgx_create_poisson(cgx_ctx **ctx, int64_t m, int device, int flags);
int cgx_create_poisson_multi(cgx_ctx **ctx, int64_t m, int nshards, const int *devices, int flags);
int cgx_create_poisson_rank(cgx_ctx **ctx, int64_t m, int rank, int nranks,
                            const cgx_unique_id *id, int device, int flags);

int cgx_destroy(cgx_ctx *ctx);
int cgx_get_info(const cgx_ctx *ctx, cgx_info *info);
int cgx_get_comm_info(cgx_ctx *ctx, cgx_comm_info *info);
int cgx_get_overlap_info(const cgx_ctx *ctx, cgx_overlap_info *info);

/* ---- data in / out (host arrays; element type per flags) ----------------- */
/* Rows [row0, row0+nrows) of A (row-major, host leading dimension lda_host),
 * of b and of x0.  Any pointer may be NULL.  Rows this process does not own
 * are ignored, so every rank may pass the full system (MPI_Scatter /
 * MPI_Bcast, parallel_cg.c:111-115) or only its own block.  */
int cgx_set_rows(cgx_ctx *ctx, int64_t row0, int64_t nrows, const void *A_rows,
                 int64_t lda_host, const void *b_rows, const void *x_rows);
/* Whole system: A is n x n row-major, b and x0 have n entries. */
int cgx_set_system(cgx_ctx *ctx, const void *A, const void *b, const void *x0);
/* On-device synthetic SPD system (generateSPDmatrix.m style, counter hash):
 *   A_ij = 0.5*(u(i,j)+u(j,i)) + n*[i==j],  b_i = u_b(i),  x0 = 0,
 * u = splitmix64-finalised counter hash -> 53-bit uniform in [0,1). */
int cgx_generate_spd(cgx_ctx *ctx, uint64_t seed);
/* b = b_value and x0 = x_value everywhere (e.g. the Poisson config: b = 1, x0 = 0). */
int cgx_fill(cgx_ctx *ctx, double b_value, double x_value);
/* x (n entries, replicated result like parallel_cg.c's local_vectorX).
 * After a cgx_iterate that failed part-way (a HIP error, an RCCL deadline),
 * x may hold part of an iteration: cgx_get_x and cgx_residual_norm return
 * CGX_ERR_STATE until cgx_set_x defines x again or cgx_solve_begin starts a
 * new solve, and cgx_iterate refuses until cgx_solve_begin. */
int cgx_get_x(cgx_ctx *ctx, void *x);
int cgx_set_x(cgx_ctx *ctx, const void *x);

/* ---- the solve (conjugrad) -------------------------------------------------- */
/* x_inout may be NULL (use / leave the device-resident x).  eps < 0: never
 * stop early; max_iter < 0: n (the reference's `k < ROWS`).  Iterations past
 * exact convergence (p.Ap or the old r.r exactly 0, e.g. after r.r underflows
 * in a long fixed-count run) take alpha = beta = 0 in fp64, so x stays at the
 * solution; CGX_F32_REF divides as serialConjugate.c does (0/0 = NaN). */
int cgx_solve(cgx_ctx *ctx, void *x_inout, double eps, int64_t max_iter, cgx_stats *st);
/* serialConjugate.c's `conjugrad(A, b, x)` (:180-259) in one call, for a
 * literal function-level drop-in: `conjugrad(A, b, x);` becomes
 * `cgx_conjugrad(A, b, x, ROWS, CGX_F32_REF, 1.0e-6, -1, NULL);`.  Host
 * arrays as the reference passes them (A row-major n x n, b, x in / out;
 * float with CGX_F32_REF -- the reference's x bit for bit -- else double),
 * one context on device 0 created, used and destroyed inside the call; st
 * may be NULL.  Repeated solves on one system: the context functions above. */
int cgx_conjugrad(const void *A, const void *b, void *x, int64_t n, int flags, double eps, int64_t max_iter,
                  cgx_stats *st);
/* The same solve in pieces: r0 = p0 = b - A x, then `count` iterations. */
int cgx_solve_begin(cgx_ctx *ctx);
int cgx_iterate(cgx_ctx *ctx, int64_t count, double eps, int64_t *done, int *converged);
int cgx_get_stats(cgx_ctx *ctx, cgx_stats *st);
/* CGX_PHASES: the per-phase times (resolves the recorded events; waits for
 * the work they mark). */
int cgx_get_phase_times(cgx_ctx *ctx, cgx_phase_times *out);
int cgx_reset_timing(cgx_ctx *ctx);
int cgx_synchronize(cgx_ctx *ctx);
/* The context's HIP stream of its first shard (hipStream_t as void*). */
void *cgx_stream(cgx_ctx *ctx);
/* Tuning of the fp64 matVec (k_matvec_f64): rows per wave (1,2,4,8), 128-column
 * chunks in flight per row (2,4,8), the A load policy (0 plain, 1 non-temporal
 * global loads, 2 software-pipelined default-policy loads, 8 software-
 * pipelined non-temporal = default; every R and U goes with each policy --
 * R=8 U=8 pipelined is accepted but spills to scratch, so the default plan
 * never picks it; all give the same row sums bit for bit,
 * test_matvec_f64_every_plan_bitwise_equal; the variants measured and not adopted are
 * in tools/microbench/matvec_variants.hip),
 * resident blocks per CU for the grid (<= 0: occupancy query).  Results do not
 * depend on the plan's R/U/policy; the p.Ap partial order depends on the grid
 * size. */
int cgx_set_matvec_plan(cgx_ctx *ctx, int rows_per_wave, int chunks_in_flight, int nontemporal,
                        int blocks_per_cu);
int cgx_get_matvec_plan(cgx_ctx *ctx, int *rows_per_wave, int *chunks_in_flight, int *nontemporal,
                        int *blocks);
/* True residual of the current x: *rnorm = ||b - A x||_2, *bnorm = ||b||_2
 * (either may be NULL).  Overwrites r and p: ends a solve in progress. */
int cgx_residual_norm(cgx_ctx *ctx, double *rnorm, double *bnorm);

/* ---- kernel-level entry points (device pointers; unit parity) -------------- */
/* dtype: CGX_F64 or CGX_F32_REF.  stream: hipStream_t or NULL.
 * The reducing calls (cgx_dot, cgx_residual, cgx_update_xr) share one
 * reduction workspace per device: issue them on one stream per device (or
 * order the streams), as the reference's single-threaded calls are ordered. */
int cgx_dev_malloc(void **ptr, size_t bytes);
int cgx_dev_free(void *ptr);
int cgx_memcpy_h2d(void *dst, const void *src, size_t bytes);
int cgx_memcpy_d2h(void *dst, const void *src, size_t bytes);
int cgx_dev_synchronize(void);
/* matVec: out[i] = sum_j A[i*lda + j] * v[j], i < rows, j < cols. */
int cgx_matvec(int dtype, const void *A, int64_t lda, int64_t rows, int64_t cols,
               const void *v, void *out, void *stream);
/* vecVec: *out_dev = a . b */
int cgx_dot(int dtype, int64_t n, const void *a, const void *b, void *out_dev, void *stream);
/* residual x2 + vecVec: r = b - Ax; p = b - Ax; *rr_dev = r.r (rr_dev may be NULL) */
int cgx_residual(int dtype, int64_t n, const void *b, const void *Ax, void *r, void *p,
                 void *rr_dev, void *stream);
/* alpha = *rsold_dev / *pAp_dev; x += alpha p; r -= alpha Ap; *rr_dev = r.r */
int cgx_update_xr(int dtype, int64_t n, void *x, void *r, const void *p, const void *Ap,
                  const void *rsold_dev, const void *pAp_dev, void *rr_dev, void *stream);
/* p = r + (*rr_dev / *rsold_dev) p */
int cgx_update_p(int dtype, int64_t n, void *p, const void *r, const void *rr_dev,
                 const void *rsold_dev, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* CGX_H */
