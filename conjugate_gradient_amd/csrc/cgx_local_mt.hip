// cgx_local_mt.hip -- the one-process multi-shard iteration (LOCAL mode,
// cgx_create_multi) enqueued by one host thread per row block.
//
// One thread enqueuing every block's work (cgx_iterate.hip do_iteration)
// pays 5S launches, 4S event records and ~3S^2 stream waits per iteration:
// about 250-290 us at S = 8 (profiles/r04_multishard_floor.jsonl), which at
// small N is the iteration.  Here each block has a worker thread that
// enqueues its own block's work (parallel_cg.c:290-323 for one rank: p's
// gather, the matVec, the r update, the x/p update), and the cross-block
// dependencies are the same events as before.  A stream may wait only on an
// event record that already exists, so the workers meet at a host barrier
// after each record point (three per iteration) -- what MPI's collectives do
// for the reference's ranks.  Distinct events per record point make the
// reuse safe: a block re-records an event only after passing two more
// barriers, by which time every other block has enqueued its wait on it.
//
// Used for the dense fp64 iteration with the folded scalar combines, gated
// or fixed-count (the host-checked form reads r.r between the kernels and
// stays on the single-thread path), when the blocks span distinct devices
// (local_mt_eligible).
#include <atomic>
#include <condition_variable>
#include <thread>

#include "cgx_ctx.h"

namespace cgxh {

static inline void cpu_relax() { __builtin_ia32_pause(); }

// Every worker meets here; false when a worker failed (abort), so nobody
// waits for a worker that will not arrive.
struct SpinBarrier {
    std::atomic<int> count{0};
    std::atomic<unsigned> gen{0};
    int n = 0;
    bool wait(const std::atomic<bool> &abort) {
        const unsigned g = gen.load(std::memory_order_acquire);
        if (count.fetch_add(1, std::memory_order_acq_rel) == n - 1) {
            count.store(0, std::memory_order_relaxed);
            gen.fetch_add(1, std::memory_order_release);
            return true;
        }
        while (gen.load(std::memory_order_acquire) == g) {
            if (abort.load(std::memory_order_relaxed)) return false;
            cpu_relax();
        }
        return true;
    }
};

struct LocalPool {
    cgx_ctx *c = nullptr;
    std::vector<std::thread> th;
    SpinBarrier bar;
    // the job: one iteration k with these arguments
    std::atomic<uint64_t> job{0};
    std::atomic<int> done{0};
    std::atomic<bool> abort{false}, quit{false};
    int64_t k = 0;
    double eps = -1.0;
    bool gated = false;
    // the first failure (code and message: fail() writes a thread-local buffer)
    std::mutex err_mu;
    int err = CGX_OK;
    std::string err_msg;
    // idle workers sleep here after spinning for a while
    std::mutex mu;
    std::condition_variable cv;
};

#define BAR()                                                                          \
    do {                                                                               \
        if (!P.bar.wait(P.abort)) return fail(CGX_ERR_STATE, "another block failed"); \
    } while (0)

// Block d's share of iteration k (do_iteration's dense fp64 LOCAL form with
// fuse_combine): the same launches, in the same order on d's streams, as the
// single-thread path, so the results are bit for bit the same.
static int shard_iteration(LocalPool &P, Shard &d) {
    cgx_ctx *c = P.c;
    const int64_t k = P.k;
    const bool gated = P.gated;
    const int S = (int)c->sh.size();
    const int pg = S_PAP + ring(k), pl = S_LPAP + ring(k);
    const int rg = S_RR + ring(k + 1), rl = S_LRR + ring(k + 1);
    const size_t es = (size_t)c->es;
    auto D = [](void *q) { return reinterpret_cast<double *>(q); };
    auto CD = [](const void *q) { return reinterpret_cast<const double *>(q); };
    TRY(set_dev(d));
    // 1. p_k is in place (the previous x/p update): everyone may read it
    HIPT(hipEventRecord(d.ev_pready, d.stream));
    BAR();
    const PeerTable pown = peer_table(c, &Shard::pown, 0);
    const bool timing = (c->flags & CGX_TIMING) && d.index == 0;
    if (c->overlap) {  // parallel_cg.c:290-293, overlapped (overlapped_matvec)
        for (auto &s : c->sh) HIPT(hipStreamWaitEvent(d.cstream, s.ev_pready, 0));
        HIPT(gather_slices(pown, S, d.index, d.nloc * (int64_t)es, d.pfull, d.cstream));
        TRY(overlap_matvecs(c, d, pl, gated));
    } else {  // MPI_Allgather(local_p -> p), then the matVec (parallel_cg.c:290-293)
        if (timing && d.ev_used >= kEvPairs) TRY(timing_resolve(c));
        if (timing) HIPT(hipEventRecord(d.ev_t[2 * d.ev_used], d.stream));
        for (auto &s : c->sh)
            if (&s != &d) HIPT(hipStreamWaitEvent(d.stream, s.ev_pready, 0));
        HIPT(gather_slices(pown, S, d.index, d.nloc * (int64_t)es, d.pfull, d.stream));
        TRY(matvec_rows(c, d, d.plan, d.A, 0, d.nloc, d.pfull, true, pl, gated, ts_of(c, d, TK_MV)));
        if (timing) {
            HIPT(hipEventRecord(d.ev_t[2 * d.ev_used + 1], d.stream));
            d.ev_used++;
        }
    }
    // 2. MPI_Allreduce(p.Ap) (parallel_cg.c:294): summed by k_update_r_f64 itself
    HIPT(hipEventRecord(d.ev_sync, d.stream));
    BAR();
    for (auto &s : c->sh)
        if (&s != &d) HIPT(hipStreamWaitEvent(d.stream, s.ev_sync, 0));
    const PeerSum pap = peer_sum(c, d, pl, pg);
    HIPT(update_r_f64(d.nloc, D(d.r), CD(d.Ap), CD(slot(d, S_RR + ring(k))), CD(slot(d, pg)), D(slot(d, rl)), d.ws,
                      d.stream, gate_of(d, gated), ts_of(c, d, TK_UR), &pap));
    // 3. MPI_Allreduce(r.r) (parallel_cg.c:313): summed by k_update_xp_f64
    HIPT(hipEventRecord(d.ev_sync2, d.stream));
    BAR();
    for (auto &s : c->sh)
        if (&s != &d) HIPT(hipStreamWaitEvent(d.stream, s.ev_sync2, 0));
    const PeerSum rr = peer_sum(c, d, rl, rg);
    if (gated)
        HIPT(update_xp_f64(d.nloc, D(d.x), D(d.pown), CD(d.r), CD(slot(d, S_RR + ring(k))), CD(slot(d, pg)),
                           CD(slot(d, rg)), d.stream, P.eps, k, reinterpret_cast<int64_t *>(slot(d, S_KDONE)),
                           D(slot(d, S_RRFINAL)), rec_of(c, d, gated), ts_of(c, d, TK_UXP), &rr));
    else
        HIPT(update_xp_f64(d.nloc, D(d.x), D(d.pown), CD(d.r), CD(slot(d, S_RR + ring(k))), CD(slot(d, pg)),
                           CD(slot(d, rg)), d.stream, -1.0, 0, nullptr, nullptr, nullptr, ts_of(c, d, TK_UXP), &rr));
    return CGX_OK;
}

static void worker(LocalPool *P, int index) {
    Shard &d = P->c->sh[index];
    uint64_t seen = 0;
    for (;;) {
        uint64_t j = P->job.load(std::memory_order_acquire);
        for (int spin = 0; j == seen && !P->quit.load(std::memory_order_relaxed); ++spin) {
            if (spin < (1 << 14)) {
                cpu_relax();
            } else {  // idle: sleep until the next job (or the pool's end)
                std::unique_lock<std::mutex> lk(P->mu);
                P->cv.wait_for(lk, std::chrono::milliseconds(50), [&] {
                    return P->job.load(std::memory_order_acquire) != seen || P->quit.load();
                });
                spin = 0;
            }
            j = P->job.load(std::memory_order_acquire);
        }
        if (P->quit.load()) return;
        seen = j;
        const int rc = shard_iteration(*P, d);
        if (rc != CGX_OK) {
            {
                std::lock_guard<std::mutex> lk(P->err_mu);
                if (P->err == CGX_OK) {
                    P->err = rc;
                    P->err_msg = cgx_last_error();
                }
            }
            P->abort.store(true);
        }
        P->done.fetch_add(1, std::memory_order_acq_rel);
    }
}

// Opt-in (CGX_LOCAL_THREADS=1).  With every block on one GPU the runtime
// serialises the threads' launches on that device's queues and the threaded
// enqueue measured no faster (275-345 vs 275-294 us per iteration at 8
// blocks, profiles/r04_multishard_floor_threads.jsonl).  Across distinct
// devices, where each thread would launch onto its own device's queues, it
// has not run on hardware yet (the suite's distinct-device tests run it when
// a box has two GPUs or more), so it is not the default there either.
bool local_mt_eligible(const cgx_ctx *c) {
    const char *e = std::getenv("CGX_LOCAL_THREADS");
    if (!(e && *e == '1')) return false;
    return c->mode == M_LOCAL && c->fuse_combine && c->op == OP_DENSE && !f32ref(c) &&
           !(c->flags & (CGX_HOST_STREAM | CGX_SYMMETRIC | CGX_COMM_P2P)) && c->sh.size() >= 2;
}

int local_mt_start(cgx_ctx *c) {
    LocalPool *P = new (std::nothrow) LocalPool();
    if (!P) return fail(CGX_ERR_NOMEM, "worker pool");
    P->c = c;
    P->bar.n = (int)c->sh.size();
    try {
        for (int i = 0; i < (int)c->sh.size(); ++i) P->th.emplace_back(worker, P, i);
    } catch (...) {
        P->quit.store(true);
        P->cv.notify_all();
        for (auto &t : P->th) t.join();
        delete P;
        return fail(CGX_ERR_STATE, "could not start the row blocks' worker threads");
    }
    c->pool = P;
    return CGX_OK;
}

void local_mt_stop(cgx_ctx *c) {
    LocalPool *P = c->pool;
    if (!P) return;
    P->quit.store(true);
    {
        std::lock_guard<std::mutex> lk(P->mu);
    }
    P->cv.notify_all();
    for (auto &t : P->th) t.join();
    delete P;
    c->pool = nullptr;
}

// Iteration c->k on every block, enqueued by the workers; returns when all
// of it is enqueued (not run).
int local_mt_iteration(cgx_ctx *c, double eps, bool gated) {
    LocalPool *P = c->pool;
    P->k = c->k;
    P->eps = eps;
    P->gated = gated;
    P->done.store(0, std::memory_order_relaxed);
    P->abort.store(false, std::memory_order_relaxed);
    P->bar.count.store(0, std::memory_order_relaxed);
    P->job.fetch_add(1, std::memory_order_release);
    {  // a worker that checked the job under the lock is now waiting: the notify reaches it
        std::lock_guard<std::mutex> lk(P->mu);
    }
    P->cv.notify_all();
    const int S = (int)c->sh.size();
    while (P->done.load(std::memory_order_acquire) < S) cpu_relax();
    if (P->err != CGX_OK) {
        const int rc = P->err;
        const std::string msg = P->err_msg;
        P->err = CGX_OK;
        return fail(rc, "row block worker: %s", msg.c_str());
    }
    return CGX_OK;
}

}  // namespace cgxh
