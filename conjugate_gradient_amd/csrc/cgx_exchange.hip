// cgx_exchange.hip -- the per-iteration exchanges (cgx_ctx.h):
//   MPI_Allgather(local_p -> p)   parallel_cg.c:290-291 -> exchange_allgather
//   MPI_Allreduce(p.Ap), (r.r)    parallel_cg.c:287,294,313 -> exchange_scalar
//   point-to-point_cg.c:239-256,339-394 (CGX_COMM_P2P) -> p2p_allgather / p2p_scalar
// in RCCL rank mode, by device copies in multi-shard mode; the overlap of
// p's exchange with the own-column-block matVec; the Poisson halo rows.
#include <chrono>
#include <thread>

#include "cgx_ctx.h"

namespace cgxh {

// Names of the exchanges in rank-mode error messages (NCCLC).
constexpr const char *kWhatHalo = "the Poisson halo exchange";
constexpr const char *kWhatP2P = "the p2p gather + send of p (allGather, BcastVector)";
constexpr const char *kWhatHaloAsync = "the overlapped r halo exchange";
static const char *scalar_name(int gslot) {
    if (gslot >= S_PAP && gslot < S_PAP + 4) return "the p.Ap combine";
    if (gslot >= S_RR && gslot < S_RR + 4) return "the r.r combine";
    return "the true-residual combine";
}

// ---- timing -------------------------------------------------------------------
int timing_resolve(cgx_ctx *c) {
    if (!(c->flags & CGX_TIMING)) return CGX_OK;
    Shard &s = c->sh[0];
    TRY(set_dev(s));
    for (int i = 0; i < s.ev_used; ++i) {
        float ms = 0.f;
        TRY(rank_wait_event(c, s.ev_t[2 * i + 1], "a timed matVec"));
        HIPT(hipEventElapsedTime(&ms, s.ev_t[2 * i], s.ev_t[2 * i + 1]));
        c->matvec_ms += ms;
        c->matvec_count += 1;
    }
    s.ev_used = 0;
    return CGX_OK;
}

// ---- CGX_PHASES ------------------------------------------------------------------
// The iteration's kernels on the first shard stamp their start and end on the
// device's constant wall clock (cgx_kernels.h kTsSlot); nothing is inserted
// between them, so what is measured is the timeline that runs without
// CGX_PHASES.  (HIP events were tried first: each one put 3.3 us onto the
// stream, 4.4 us with its default system-scope release -- 5-7 % of an 8-GPU
// iteration.)  The stamps are turned into phase durations after the fact
// (phase_resolve): a kernel's own time, and the time between consecutive
// kernels, which is the exchange enqueued between them (RCCL's allgather /
// allreduce kernels, or the device copies) or the launch gap.
int phase_iter_begin(cgx_ctx *c) {
    if (!(c->flags & CGX_PHASES)) return CGX_OK;
    Shard &s = c->sh[0];
    if (s.ts_used >= kTsIters) TRY(phase_resolve(c));
    s.ts_cur = s.ts_used;
    return CGX_OK;
}

int64_t *ts_of(cgx_ctx *c, const Shard &s, int kern) {
    if (!(c->flags & CGX_PHASES) || &s != &c->sh[0] || s.ts_cur < 0) return nullptr;
    return s.ts_dev + ((size_t)s.ts_cur * kTsKern + kern) * kTsSlot;
}

void phase_iter_end(cgx_ctx *c) {
    if (!(c->flags & CGX_PHASES)) return;
    Shard &s = c->sh[0];
    if (s.ts_cur >= 0) s.ts_used = s.ts_cur + 1;
    s.ts_cur = -1;
}

int phase_resolve(cgx_ctx *c) {
    if (c->sh.empty() || !(c->flags & CGX_PHASES)) return CGX_OK;
    Shard &s = c->sh[0];
    if (s.ts_used == 0) return CGX_OK;
    TRY(set_dev(s));
    const size_t words = (size_t)s.ts_used * kTsKern * kTsSlot;
    if (!s.ts_host)
        HIPT(hipHostMalloc(reinterpret_cast<void **>(&s.ts_host), (size_t)kTsIters * kTsKern * kTsSlot * 8,
                           hipHostMallocDefault));
    const int64_t *h = s.ts_host;
    HIPT(hipMemcpyAsync(s.ts_host, s.ts_dev, words * 8, hipMemcpyDeviceToHost, s.stream));
    TRY(rank_wait_stream(c, s.stream, "the phase timestamps"));
    HIPT(hipMemsetAsync(s.ts_dev, 0, words * 8, s.stream));
    s.ts_used = 0;
    const double us_per_tick = 1e3 / c->ts_khz;
    auto add = [&](int seg, int64_t t0, int64_t t1) { c->ph_samples[seg].push_back((float)((t1 - t0) * us_per_tick)); };
    // the phase between two consecutive kernels of an iteration (by slot)
    auto between = [](int a, int b) {
        if (a == TK_OWN) return CGX_PH_GATHER_EXPOSED;  // own block done, waiting for p
        if (a == TK_MV) return CGX_PH_COMBINE_PAP;      // (two-launch form: the kernel boundary)
        return CGX_PH_COMBINE_RR;
    };
    const int kern_seg[kTsKern] = {CGX_PH_MATVEC_OWN, CGX_PH_MATVEC, CGX_PH_UPDATE_R, CGX_PH_UPDATE_XP};
    for (int i = 0; i < (int)(words / ((size_t)kTsKern * kTsSlot)); ++i) {
        int64_t st[kTsKern], en[kTsKern];
        int first = -1, last = -1;
        for (int k = 0; k < kTsKern; ++k) {
            const int64_t *q = h + ((size_t)i * kTsKern + k) * kTsSlot;
            st[k] = q[0];
            en[k] = 0;
            for (int b = 1; b < kTsSlot; ++b) en[k] = std::max(en[k], q[b]);
            if (st[k] == 0 || en[k] == 0) continue;  // not launched, or skipped itself (gated)
            if (first < 0) first = k;
            if (last >= 0) add(between(last, k), en[last], st[k]);
            add(kern_seg[k], st[k], en[k]);
            last = k;
        }
        if (first < 0) {  // an iteration that did nothing (after a device-side stop)
            c->ts_prev_start = c->ts_prev_end = 0;
            continue;
        }
        {  // the matVec kernels' busy time: the union of their spans (the overlap's own block and rest)
            std::pair<int64_t, int64_t> iv[2];
            int niv = 0;
            for (int k : {TK_OWN, TK_MV})
                if (st[k] != 0 && en[k] != 0) iv[niv++] = {st[k], en[k]};
            std::sort(iv, iv + niv);
            int64_t busy = 0, cs = 0, ce = 0;
            for (int j = 0; j < niv; ++j) {
                if (j == 0 || iv[j].first > ce) {
                    busy += ce - cs;
                    cs = iv[j].first;
                    ce = iv[j].second;
                } else {
                    ce = std::max(ce, iv[j].second);
                }
            }
            busy += ce - cs;
            if (niv) add(CGX_PH_MATVEC_BUSY, 0, busy);
        }
        if (c->ts_prev_end) {
            // before the first kernel: p's allgather when it is not overlapped
            // (a non-overlapped exchange between iterations), else the launch gap
            add((first == TK_MV && c->mode != M_SINGLE) ? CGX_PH_GATHER_EXPOSED : CGX_PH_GAP, c->ts_prev_end, st[first]);
            add(CGX_PH_ITERATION, c->ts_prev_start, st[first]);
        }
        c->ts_prev_start = st[first];
        c->ts_prev_end = en[last];
    }
    return CGX_OK;
}

// Rank mode, host-checked iterations: one event per iteration, so a host
// wait can tell a healthy long queue (events completing) from a stall.
int progress_mark(cgx_ctx *c) {
    if (c->mode != M_RCCL) return CGX_OK;
    Shard &s = c->sh[0];
    if (!s.ev_prog[0]) return CGX_OK;
    TRY(set_dev(s));
    HIPT(hipEventRecord(s.ev_prog[s.prog_next], s.stream));
    s.prog_next = (s.prog_next + 1) % 8;
    return CGX_OK;
}

// ---- exchange ---------------------------------------------------------------------
// Make every shard's stream wait for the work already queued on all shards.
int local_barrier(cgx_ctx *c) {
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipEventRecord(s.ev_sync, s.stream));
    }
    for (auto &d : c->sh) {
        TRY(set_dev(d));
        for (auto &s : c->sh)
            if (&s != &d) HIPT(hipStreamWaitEvent(d.stream, s.ev_sync, 0));
    }
    return CGX_OK;
}

// The table of every shard's copy of a buffer at byte offset `off` (+ the
// shard's own row offset when `own_rows`), in shard order, for the pull
// kernels of the LOCAL exchange.
PeerTable peer_table(const cgx_ctx *c, char *Shard::*buf, int64_t off) {
    PeerTable t{};
    for (const auto &s : c->sh) t.p[s.index] = s.*buf + off;
    return t;
}

// Poisson: refresh the two halo rows of every slab from its neighbours
// (ncclSend/Recv of one grid row each way in rank mode, device copies in
// LOCAL mode); from_x first copies x into the slab interior (for A x0).
int exchange_halo_of(cgx_ctx *c, char *Shard::*slab);
int exchange_halo(cgx_ctx *c, bool from_x) {
    const size_t es = (size_t)c->es;
    if (from_x)
        for (auto &s : c->sh) {
            TRY(set_dev(s));
            HIPT(hipMemcpyAsync(s.pown, s.x, s.nloc * es, hipMemcpyDeviceToDevice, s.stream));
        }
    return exchange_halo_of(c, &Shard::pfull);
}

// The halo rows of the slab buffer `slab` (row 0 and row mloc+1 around the
// mloc interior rows) from the neighbouring slabs' boundary rows.
int exchange_halo_of(cgx_ctx *c, char *Shard::*slab) {
    const size_t row = (size_t)c->m * (size_t)c->es;
    if (c->mode == M_SINGLE) return CGX_OK;
    const int64_t mloc = c->sh[0].nloc / c->m;
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        if (c->nranks == 1) return CGX_OK;
        TRY(set_dev(s));
        const int g = s.index;
        char *base = s.*slab, *own = base + row;
        NCCLC(c, ncclGroupStart(), kWhatHalo);
        if (g > 0) {
            NCCLC(c, ncclSend(own, (size_t)c->m, ncclDouble, g - 1, s.comm, s.stream), kWhatHalo);
            NCCLC(c, ncclRecv(base, (size_t)c->m, ncclDouble, g - 1, s.comm, s.stream), kWhatHalo);
        }
        if (g < c->nranks - 1) {
            NCCLC(c, ncclSend(own + (size_t)(mloc - 1) * row, (size_t)c->m, ncclDouble, g + 1, s.comm, s.stream),
                  kWhatHalo);
            NCCLC(c, ncclRecv(own + (size_t)mloc * row, (size_t)c->m, ncclDouble, g + 1, s.comm, s.stream), kWhatHalo);
        }
        NCCLC(c, ncclGroupEnd(), kWhatHalo);
        return CGX_OK;
    }
    TRY(local_barrier(c));
    const int S = (int)c->sh.size();
    for (int q = 0; q < S; ++q) {
        Shard &d = c->sh[q];
        TRY(set_dev(d));
        if (q > 0) {
            const Shard &u = c->sh[q - 1];
            HIPT(hipMemcpyPeerAsync(d.*slab, d.dev, u.*slab + (size_t)mloc * row, u.dev, row, d.stream));
        }
        if (q < S - 1) {
            const Shard &w = c->sh[q + 1];
            HIPT(hipMemcpyPeerAsync(d.*slab + (size_t)(mloc + 1) * row, d.dev, w.*slab + row, w.dev, row, d.stream));
        }
    }
    return CGX_OK;
}

// CGX_COMM_P2P: point-to-point_cg.c's exchange pattern, gather to rank 0 then
// send from rank 0 to every rank (allGather :364-394 + BcastVector :239-256),
// O(P) messages through rank 0.  ncclSend/Recv in rank mode, device copies
// through shard 0 in LOCAL mode.
int p2p_allgather(cgx_ctx *c, bool from_x) {
    const size_t es = (size_t)c->es;
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        const ncclDataType_t t = f32ref(c) ? ncclFloat : ncclDouble;
        const int P = c->nranks;
        if (s.index == 0 && from_x)
            HIPT(hipMemcpyAsync(s.pown, s.x, s.nloc * es, hipMemcpyDeviceToDevice, s.stream));
        NCCLC(c, ncclGroupStart(), kWhatP2P);
        if (s.index != 0) {
            const void *src = from_x ? (const void *)s.x : (const void *)s.pown;
            NCCLC(c, ncclSend(src, (size_t)s.nloc, t, 0, s.comm, s.stream), kWhatP2P);
        } else {
            for (int q = 1; q < P; ++q)
                NCCLC(c, ncclRecv(s.pfull + (size_t)q * s.nloc * es, (size_t)s.nloc, t, q, s.comm, s.stream), kWhatP2P);
        }
        NCCLC(c, ncclGroupEnd(), kWhatP2P);
        NCCLC(c, ncclGroupStart(), kWhatP2P);
        if (s.index == 0) {
            for (int q = 1; q < P; ++q) NCCLC(c, ncclSend(s.pfull, (size_t)c->n, t, q, s.comm, s.stream), kWhatP2P);
        } else {
            NCCLC(c, ncclRecv(s.pfull, (size_t)c->n, t, 0, s.comm, s.stream), kWhatP2P);
        }
        NCCLC(c, ncclGroupEnd(), kWhatP2P);
        return CGX_OK;
    }
    TRY(local_barrier(c));
    Shard &r0 = c->sh[0];
    const int S = (int)c->sh.size();
    const int64_t slice = r0.nloc * (int64_t)es;
    TRY(set_dev(r0));
    // every slice to block 0 (gatherRow), then the whole vector from block 0 to
    // every block (BcastVector): pull kernels on the receiving streams (one
    // launch each instead of one peer copy per slice), or, with
    // CGX_LOCAL_XCHG=copy, the peer copies; the same bytes either way
    if (c->xchg_kernels) {
        HIPT(gather_slices(peer_table(c, from_x ? &Shard::x : &Shard::pown, 0), S, from_x ? -1 : 0, slice, r0.pfull,
                           r0.stream));
    } else {
        for (auto &s : c->sh) {
            if (&s == &r0 && !from_x) continue;
            HIPT(hipMemcpyPeerAsync(r0.pfull + s.row0 * es, r0.dev, from_x ? s.x : s.pown, s.dev, s.nloc * es,
                                    r0.stream));
        }
    }
    HIPT(hipEventRecord(r0.ev_root, r0.stream));
    PeerTable whole{};  // block 0's full vector, slice by slice
    for (int q = 0; q < S; ++q) whole.p[q] = r0.pfull + (int64_t)q * slice;
    for (auto &d : c->sh) {
        if (&d == &r0) continue;
        TRY(set_dev(d));
        HIPT(hipStreamWaitEvent(d.stream, r0.ev_root, 0));
        if (c->xchg_kernels) HIPT(gather_slices(whole, S, -1, slice, d.pfull, d.stream));
        else HIPT(hipMemcpyPeerAsync(d.pfull, d.dev, r0.pfull, r0.dev, (size_t)c->n * es, d.stream));
    }
    // Shard 0 must not touch its pfull again until every shard has copied it:
    // with from_x its very next kernels (matVec, then the residual writing p
    // into pfull) would otherwise race the other streams' copies (seen as
    // wrong x in about 1 solve in 5 before this barrier).
    return local_barrier(c);
}

// allSum (point-to-point_cg.c:339-359): partials to rank 0, summed there in
// rank order, the sum sent back to every rank (BcastVector(&s, 1)).
int p2p_scalar(cgx_ctx *c, int lslot, int gslot) {
    const char *what = scalar_name(gslot);
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        const int P = c->nranks;
        if (s.index == 0) HIPT(hipMemcpyAsync(slot(s, S_GATHER), slot(s, lslot), 8, hipMemcpyDeviceToDevice, s.stream));
        NCCLC(c, ncclGroupStart(), what);
        if (s.index != 0) {
            NCCLC(c, ncclSend(slot(s, lslot), 1, ncclUint64, 0, s.comm, s.stream), what);
        } else {
            for (int q = 1; q < P; ++q) NCCLC(c, ncclRecv(slot(s, S_GATHER + q), 1, ncclUint64, q, s.comm, s.stream),
                                              what);
        }
        NCCLC(c, ncclGroupEnd(), what);
        if (s.index == 0) {
            if (f32ref(c))
                HIPT(sum_ordered_f32(reinterpret_cast<const float *>(slot(s, S_GATHER)), P,
                                     reinterpret_cast<float *>(slot(s, gslot)), s.stream, false));
            else
                HIPT(sum_ordered_f64(reinterpret_cast<const double *>(slot(s, S_GATHER)), P,
                                     reinterpret_cast<double *>(slot(s, gslot)), s.stream));
        }
        NCCLC(c, ncclGroupStart(), what);
        if (s.index == 0) {
            for (int q = 1; q < P; ++q) NCCLC(c, ncclSend(slot(s, gslot), 1, ncclUint64, q, s.comm, s.stream), what);
        } else {
            NCCLC(c, ncclRecv(slot(s, gslot), 1, ncclUint64, 0, s.comm, s.stream), what);
        }
        NCCLC(c, ncclGroupEnd(), what);
        return CGX_OK;
    }
    TRY(local_barrier(c));
    Shard &r0 = c->sh[0];
    const int S = (int)c->sh.size();
    TRY(set_dev(r0));
    // block 0 pulls the partials and sums them in rank order (one kernel, the
    // adds of sum_ordered's rank order), then every block pulls the sum (a
    // "sum" of one value: the value); CGX_LOCAL_XCHG=copy: peer copies
    if (c->xchg_kernels) {
        const PeerTable src = peer_table(c, &Shard::scal, 8 * (int64_t)lslot);
        if (f32ref(c)) HIPT(combine_peers_f32(src, S, reinterpret_cast<float *>(slot(r0, gslot)), r0.stream, false));
        else HIPT(combine_peers_f64(src, S, reinterpret_cast<double *>(slot(r0, gslot)), r0.stream));
    } else {
        for (auto &s : c->sh)
            HIPT(hipMemcpyPeerAsync(slot(r0, S_GATHER + s.index), r0.dev, slot(s, lslot), s.dev, 8, r0.stream));
        if (f32ref(c))
            HIPT(sum_ordered_f32(reinterpret_cast<const float *>(slot(r0, S_GATHER)), S,
                                 reinterpret_cast<float *>(slot(r0, gslot)), r0.stream, false));
        else
            HIPT(sum_ordered_f64(reinterpret_cast<const double *>(slot(r0, S_GATHER)), S,
                                 reinterpret_cast<double *>(slot(r0, gslot)), r0.stream));
    }
    HIPT(hipEventRecord(r0.ev_root, r0.stream));
    PeerTable root{};
    root.p[0] = static_cast<const char *>(slot(r0, gslot));
    for (auto &d : c->sh) {
        if (&d == &r0) continue;
        TRY(set_dev(d));
        HIPT(hipStreamWaitEvent(d.stream, r0.ev_root, 0));
        if (!c->xchg_kernels)
            HIPT(hipMemcpyPeerAsync(slot(d, gslot), d.dev, slot(r0, gslot), r0.dev, 8, d.stream));
        else if (f32ref(c))
            HIPT(combine_peers_f32(root, 1, reinterpret_cast<float *>(slot(d, gslot)), d.stream, false));
        else
            HIPT(combine_peers_f64(root, 1, reinterpret_cast<double *>(slot(d, gslot)), d.stream));
    }
    return local_barrier(c);  // as in p2p_allgather: shard 0's slots stay put until copied
}

// Every shard's pfull gets every shard's slice of `src(shard)` (its own slice
// of a full-length buffer when in_place, else a separate local buffer).
int exchange_allgather(cgx_ctx *c, bool from_x) {
    if (c->op == OP_POISSON) return exchange_halo(c, from_x);
    if (p2p(c) && c->mode != M_SINGLE) return p2p_allgather(c, from_x);
    const size_t es = (size_t)c->es;
    if (c->mode == M_SINGLE) {
        if (from_x) {
            Shard &s = c->sh[0];
            TRY(set_dev(s));
            HIPT(hipMemcpyAsync(s.pown, s.x, s.nloc * es, hipMemcpyDeviceToDevice, s.stream));
        }
        return CGX_OK;
    }
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        const ncclDataType_t t = f32ref(c) ? ncclFloat : ncclDouble;
        const void *send = from_x ? (const void *)s.x : (const void *)s.pown;
        NCCLC(c, ncclAllGather(send, s.pfull, (size_t)s.nloc, t, s.comm, s.stream),
              from_x ? "ncclAllGather(x)" : "ncclAllGather(p)");
        return CGX_OK;
    }
    // LOCAL: after all producers are done, every shard pulls the other
    // slices: one gather kernel per shard (or, CGX_LOCAL_XCHG=copy, a peer
    // copy per pair).
    TRY(local_barrier(c));
    if (c->xchg_kernels) {
        const PeerTable src = peer_table(c, from_x ? &Shard::x : &Shard::pown, 0);
        for (auto &d : c->sh) {
            TRY(set_dev(d));
            HIPT(gather_slices(src, (int)c->sh.size(), from_x ? -1 : d.index, d.nloc * (int64_t)es, d.pfull,
                               d.stream));
        }
        return CGX_OK;
    }
    for (auto &d : c->sh) {
        TRY(set_dev(d));
        for (auto &s : c->sh) {
            char *dst = d.pfull + s.row0 * es;
            const char *src = from_x ? s.x : s.pown;
            if (&s == &d && !from_x) continue;
            HIPT(hipMemcpyPeerAsync(dst, d.dev, src, s.dev, s.nloc * es, d.stream));
        }
    }
    return CGX_OK;
}

// The combine folded into the consuming kernel (c->fuse_combine): the table
// of every shard's partial in `lslot`, summed into shard d's `gslot`.  The
// caller has ordered d's stream after every producer (local_barrier).
PeerSum peer_sum(const cgx_ctx *c, const Shard &d, int lslot, int gslot) {
    PeerSum ps{};
    ps.src = peer_table(c, &Shard::scal, 8 * (int64_t)lslot);
    ps.cnt = (int)c->sh.size();
    ps.out = reinterpret_cast<double *>(slot(d, gslot));
    return ps;
}

PeerSumF32 peer_sum_f32(const cgx_ctx *c, const Shard &d, int lslot, int gslot) {
    PeerSumF32 ps{};
    ps.src = peer_table(c, &Shard::scal, 8 * (int64_t)lslot);
    ps.cnt = (int)c->sh.size();
    ps.out = reinterpret_cast<float *>(slot(d, gslot));
    return ps;
}

// Combine the per-shard partials in slot `lslot` into the global slot `gslot`.
int exchange_scalar(cgx_ctx *c, int lslot, int gslot) {
    if (c->mode == M_SINGLE) return CGX_OK;  // kernels wrote the global slot directly
    if (p2p(c)) return p2p_scalar(c, lslot, gslot);
    const int S = (int)c->sh.size();
    const char *what = scalar_name(gslot);
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        if (f32ref(c)) {
            // parallel_cg.c's MPI_Allreduce, bit for bit: gather the partials and
            // combine them in MPICH's recursive-doubling order on every rank
            NCCLC(c, ncclAllGather(slot(s, lslot), slot(s, S_GATHER), 1, ncclUint64, s.comm, s.stream), what);
            HIPT(sum_ordered_f32(reinterpret_cast<const float *>(slot(s, S_GATHER)), c->nranks,
                                 reinterpret_cast<float *>(slot(s, gslot)), s.stream, true));
        } else if (c->flags & CGX_DETERMINISTIC) {
            // fp64, rank-order sum: the same bits as the multi-shard mode with the
            // same partition, whatever algorithm RCCL would pick for an allreduce
            NCCLC(c, ncclAllGather(slot(s, lslot), slot(s, S_GATHER), 1, ncclUint64, s.comm, s.stream), what);
            HIPT(sum_ordered_f64(reinterpret_cast<const double *>(slot(s, S_GATHER)), c->nranks,
                                 reinterpret_cast<double *>(slot(s, gslot)), s.stream));
        } else {
            NCCLC(c, ncclAllReduce(slot(s, lslot), slot(s, gslot), 1, ncclDouble, ncclSum, s.comm, s.stream), what);
        }
        return CGX_OK;
    }
    TRY(local_barrier(c));
    if (c->xchg_kernels) {  // every shard reads the S partials from their slots: the same sums, no copies
        const PeerTable src = peer_table(c, &Shard::scal, 8 * (int64_t)lslot);
        for (auto &d : c->sh) {
            TRY(set_dev(d));
            if (f32ref(c))  // parallel_cg.c's MPI_Allreduce order (MPICH), as in rank mode
                HIPT(combine_peers_f32(src, S, reinterpret_cast<float *>(slot(d, gslot)), d.stream, true));
            else
                HIPT(combine_peers_f64(src, S, reinterpret_cast<double *>(slot(d, gslot)), d.stream));
        }
        return CGX_OK;
    }
    for (auto &d : c->sh) {
        TRY(set_dev(d));
        for (auto &s : c->sh)
            HIPT(hipMemcpyPeerAsync(slot(d, S_GATHER + s.index), d.dev, slot(s, lslot), s.dev, 8, d.stream));
        if (f32ref(c))  // parallel_cg.c's MPI_Allreduce order (MPICH), as in rank mode
            HIPT(sum_ordered_f32(reinterpret_cast<const float *>(slot(d, S_GATHER)), S,
                                 reinterpret_cast<float *>(slot(d, gslot)), d.stream, true));
        else
            HIPT(sum_ordered_f64(reinterpret_cast<const double *>(slot(d, S_GATHER)), S,
                                 reinterpret_cast<double *>(slot(d, gslot)), d.stream));
    }
    return CGX_OK;
}

// Where a kernel writes its (partial) scalar: the global slot directly when
// there is nothing to combine, else the shard-local slot.

// The overlapped matVec of row block d once p's exchange is enqueued on
// d.cstream (the RCCL allgather, or the pull kernel): the own column block on
// the compute stream (its p is local) while the exchange runs, then, once p
// has landed, the rest of the columns, accumulating, with the fused p.Ap.
// (Round 5 also ran the rest launch on the exchange stream beside the own
// block, with an add kernel after both: 644.9 against 638.7 us per iteration
// at 8 row blocks of N = 65536 -- the matVec's one wave per SIMD leaves no room
// for a second kernel's waves, so the two did not overlap, and the add cost
// its launch; profiles/r05_rank_iteration.jsonl.  Removed.)
int overlap_matvecs(cgx_ctx *c, Shard &d, int dot_slot, bool gated, bool timed) {
    const double *A = reinterpret_cast<const double *>(d.A);
    const double *v = reinterpret_cast<const double *>(d.pfull);
    double *Ap = reinterpret_cast<double *>(d.Ap);
    HIPT(hipEventRecord(d.ev_gathered, d.cstream));
    const bool timing = timed && (c->flags & CGX_TIMING) && (&d == &c->sh[0]);
    if (timing && d.ev_used >= kEvPairs) TRY(timing_resolve(c));
    if (timing) HIPT(hipEventRecord(d.ev_t[2 * d.ev_used], d.stream));
    HIPT(matvec_f64_cols(d.plan, A, c->lda, d.nloc, c->lda, d.row0, d.nloc, false, v, Ap, nullptr, nullptr, d.ws,
                         d.stream, gate_of(d, gated), ts_of(c, d, TK_OWN)));
    HIPT(hipStreamWaitEvent(d.stream, d.ev_gathered, 0));
    HIPT(matvec_f64_cols(d.plan, A, c->lda, d.nloc, c->lda, (d.row0 + d.nloc) % c->lda, c->lda - d.nloc, true, v, Ap,
                         reinterpret_cast<const double *>(d.pown), reinterpret_cast<double *>(slot(d, dot_slot)),
                         d.ws, d.stream, gate_of(d, gated), ts_of(c, d, TK_MV)));
    if (timing) {
        HIPT(hipEventRecord(d.ev_t[2 * d.ev_used + 1], d.stream));
        d.ev_used++;
    }
    return CGX_OK;
}

// Overlapped exchange + matVec (parallel_cg.c:290-293): p is allgathered on
// each shard's exchange stream while the compute stream multiplies the
// shard's own column block; overlap_matvecs does the rest.
int overlapped_matvec(cgx_ctx *c, int dot_slot, bool gated, bool timed) {
    const size_t es = (size_t)c->es;
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipEventRecord(s.ev_pready, s.stream));
    }
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        HIPT(hipStreamWaitEvent(s.cstream, s.ev_pready, 0));
        NCCLC(c, ncclAllGather(s.pown, s.pfull, (size_t)s.nloc, ncclDouble, s.comm, s.cstream),
              "ncclAllGather(p), overlapped");
    } else {
        const PeerTable src = peer_table(c, &Shard::pown, 0);
        for (auto &d : c->sh) {
            TRY(set_dev(d));
            for (auto &s : c->sh) HIPT(hipStreamWaitEvent(d.cstream, s.ev_pready, 0));
            if (c->xchg_kernels)
                HIPT(gather_slices(src, (int)c->sh.size(), d.index, d.nloc * (int64_t)es, d.pfull, d.cstream));
            else
                for (auto &s : c->sh)
                    if (&s != &d)
                        HIPT(hipMemcpyPeerAsync(d.pfull + s.row0 * es, d.dev, s.pown, s.dev, s.nloc * es, d.cstream));
        }
    }
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        TRY(overlap_matvecs(c, s, dot_slot, gated, timed));
    }
    return CGX_OK;
}

// ---- overlapped or plain: the choice at creation ------------------------------
// The two forms of an aligned multi-shard iteration (c->rot) give the same
// bits, so the choice is speed only.  The overlap hides the allgather behind
// the own-block launch but pays for splitting the matVec in two launches (a
// second fill and drain: 15 / 20 / 23 us per iteration at 8 / 4 / 2 row blocks
// of N = 65536, profiles/r05_rank_iteration.jsonl); the plain form exposes
// the allgather.  The exchange and the matVec also compete when they run
// together (the allgather's kernel beside a matVec that holds every CU and
// saturates HBM), which the parts timed alone cannot show.  So the context
// times both WHOLE forms end to end on its own row blocks (zeros at this
// point: the same bytes move) -- the real allgather (RCCL or the pull
// kernels) with the matVec(s) after or beside it -- and overlaps only when
// that form is faster by more than kOverlapMargin (a hysteresis: runs of the
// same configuration do not flip between forms on noise).  The parts (the
// split, the one launch, the allgather alone) are still timed and reported.
// Rank mode: every rank measures and the maxima over ranks decide, so the
// ranks agree (they would pair their collectives either way).
// CGX_NO_OVERLAP / CGX_OVERLAP=0 and CGX_OVERLAP=1 / force override the
// decision (the numbers are still measured and reported).  kOverlapMargin:
// cgx_ctx.h.

static int measure_split(cgx_ctx *c) {
    constexpr int kReps = 3;
    double split = 0.0, one = 0.0, cost = 0.0;
    for (auto &s : c->sh) {  // one block at a time: blocks sharing a GPU would contend
        TRY(set_dev(s));
        hipEvent_t ev[3] = {};
        for (auto &e : ev) HIPT(hipEventCreate(&e));
        const double *A = reinterpret_cast<const double *>(s.A), *v = reinterpret_cast<const double *>(s.pfull);
        double *Ap = reinterpret_cast<double *>(s.Ap), *dot = reinterpret_cast<double *>(slot(s, S_TR));
        const double *pown = reinterpret_cast<const double *>(s.pown);
        float best_split = 1e30f, best_one = 1e30f;
        int rc = CGX_OK;
        for (int rep = 0; rep <= kReps && rc == CGX_OK; ++rep) {  // rep 0 warms up
            rc = [&]() -> int {
                HIPT(hipEventRecord(ev[0], s.stream));
                HIPT(hipStreamWaitEvent(s.cstream, ev[0], 0));  // the overlapped form with nothing to exchange
                TRY(overlap_matvecs(c, s, S_TR, false, false));
                HIPT(hipEventRecord(ev[1], s.stream));
                HIPT(matvec_f64_cols(s.plan, A, c->lda, s.nloc, c->lda, s.row0, c->lda, false, v, Ap, pown, dot, s.ws,
                                     s.stream, nullptr, nullptr, s.nloc));
                HIPT(hipEventRecord(ev[2], s.stream));
                TRY(rank_wait_stream(c, s.stream, "the overlap calibration"));
                float t1 = 0.f, t2 = 0.f;
                HIPT(hipEventElapsedTime(&t1, ev[0], ev[1]));
                HIPT(hipEventElapsedTime(&t2, ev[1], ev[2]));
                if (rep > 0) {
                    best_split = std::min(best_split, t1);
                    best_one = std::min(best_one, t2);
                }
                return CGX_OK;
            }();
        }
        for (auto e : ev) (void)hipEventDestroy(e);
        TRY(rc);
        split = std::max(split, 1e3 * best_split);
        one = std::max(one, 1e3 * best_one);
        cost = std::max(cost, 1e3 * (best_split - best_one));
    }
    c->ov_split_us = split;
    c->ov_one_us = one;
    c->ov_cost_us = cost;
    return CGX_OK;
}

static int measure_allgather(cgx_ctx *c) {
    constexpr int kReps = 8;
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        TRY(set_dev(s));
        hipEvent_t ev[2] = {};
        for (auto &e : ev) HIPT(hipEventCreate(&e));
        int rc = [&]() -> int {
            for (int i = 0; i < 2; ++i)  // warm: the ranks meet, RCCL sets up its channels
                NCCLC(c, ncclAllGather(s.pown, s.pfull, (size_t)s.nloc, ncclDouble, s.comm, s.stream),
                      "ncclAllGather(p), overlap calibration");
            TRY(rank_wait_stream(c, s.stream, "the overlap calibration"));
            HIPT(hipEventRecord(ev[0], s.stream));
            for (int i = 0; i < kReps; ++i)
                NCCLC(c, ncclAllGather(s.pown, s.pfull, (size_t)s.nloc, ncclDouble, s.comm, s.stream),
                      "ncclAllGather(p), overlap calibration");
            HIPT(hipEventRecord(ev[1], s.stream));
            TRY(rank_wait_stream(c, s.stream, "the overlap calibration"));
            float ms = 0.f;
            HIPT(hipEventElapsedTime(&ms, ev[0], ev[1]));
            c->ov_ag_us = 1e3 * ms / kReps;
            return CGX_OK;
        }();
        for (auto e : ev) (void)hipEventDestroy(e);
        return rc;
    }
    // one process: the exchange as the plain iteration runs it (events, then
    // the pull kernels), per block from its stream's start to its gather's end
    const int S = (int)c->sh.size();
    std::vector<hipEvent_t> ev(2 * S, nullptr);
    int rc = [&]() -> int {
        for (int q = 0; q < S; ++q) {
            TRY(set_dev(c->sh[q]));
            HIPT(hipEventCreate(&ev[2 * q]));
            HIPT(hipEventCreate(&ev[2 * q + 1]));
        }
        double best = 1e30;
        for (int rep = 0; rep <= 3; ++rep) {
            TRY(sync_all(c));
            for (int q = 0; q < S; ++q) {
                TRY(set_dev(c->sh[q]));
                HIPT(hipEventRecord(ev[2 * q], c->sh[q].stream));
            }
            TRY(exchange_allgather(c, false));
            for (int q = 0; q < S; ++q) {
                TRY(set_dev(c->sh[q]));
                HIPT(hipEventRecord(ev[2 * q + 1], c->sh[q].stream));
            }
            TRY(sync_all(c));
            double worst = 0.0;
            for (int q = 0; q < S; ++q) {
                float ms = 0.f;
                HIPT(hipEventElapsedTime(&ms, ev[2 * q], ev[2 * q + 1]));
                worst = std::max(worst, 1e3 * (double)ms);
            }
            if (rep > 0) best = std::min(best, worst);
        }
        c->ov_ag_us = best;
        return CGX_OK;
    }();
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

// Both exchange + matVec forms end to end, as the iteration runs them:
// plain = exchange_allgather then one rotated launch per block; overlap =
// overlapped_matvec.  Each timed region holds kBack forms back to back (the
// host runs ahead after the first, as in the iteration, and each form's
// gather waits for every block's previous matVec, as the next iteration's
// does); per pass the slowest block's average, best of kPasses, after one
// warm-up of each.  Rank mode: a one-double allreduce right before each timed
// region lines the ranks up on the device, so host skew between the ranks is
// not timed.
static int measure_forms(cgx_ctx *c) {
    constexpr int kBack = 2, kPasses = 2;
    const int S = (int)c->sh.size();
    std::vector<hipEvent_t> ev(2 * S, nullptr);
    auto one_form = [&](bool overlap) -> int {
        if (overlap) return overlapped_matvec(c, S_TR, false, false);
        TRY(exchange_allgather(c, false));
        for (auto &s : c->sh) {
            TRY(set_dev(s));
            HIPT(matvec_f64_cols(s.plan, reinterpret_cast<const double *>(s.A), c->lda, s.nloc, c->lda, s.row0,
                                 c->lda, false, reinterpret_cast<const double *>(s.pfull),
                                 reinterpret_cast<double *>(s.Ap), reinterpret_cast<const double *>(s.pown),
                                 reinterpret_cast<double *>(slot(s, S_TR)), s.ws, s.stream, nullptr, nullptr,
                                 s.nloc));
        }
        return CGX_OK;
    };
    auto timed = [&](bool overlap, int reps, double *us) -> int {
        TRY(sync_all(c));
        if (c->mode == M_RCCL) {  // line the ranks up
            Shard &s = c->sh[0];
            TRY(set_dev(s));
            NCCLC(c, ncclAllReduce(slot(s, S_GATHER), slot(s, S_GATHER), 1, ncclDouble, ncclMax, s.comm, s.stream),
                  "ncclAllReduce(max), overlap calibration");
        }
        for (int q = 0; q < S; ++q) {
            TRY(set_dev(c->sh[q]));
            HIPT(hipEventRecord(ev[2 * q], c->sh[q].stream));
        }
        for (int r = 0; r < reps; ++r) TRY(one_form(overlap));
        for (int q = 0; q < S; ++q) {
            TRY(set_dev(c->sh[q]));
            HIPT(hipEventRecord(ev[2 * q + 1], c->sh[q].stream));
        }
        TRY(sync_all(c));
        double worst = 0.0;
        for (int q = 0; q < S; ++q) {
            float ms = 0.f;
            HIPT(hipEventElapsedTime(&ms, ev[2 * q], ev[2 * q + 1]));
            worst = std::max(worst, 1e3 * (double)ms / reps);
        }
        *us = worst;
        return CGX_OK;
    };
    int rc = [&]() -> int {
        for (int q = 0; q < S; ++q) {
            TRY(set_dev(c->sh[q]));
            HIPT(hipEventCreate(&ev[2 * q]));
            HIPT(hipEventCreate(&ev[2 * q + 1]));
        }
        double t = 0.0, best_plain = 1e300, best_ov = 1e300;
        TRY(timed(false, 1, &t));  // warm-up of each form
        TRY(timed(true, 1, &t));
        for (int pass = 0; pass < kPasses; ++pass) {
            TRY(timed(false, kBack, &t));
            best_plain = std::min(best_plain, t);
            TRY(timed(true, kBack, &t));
            best_ov = std::min(best_ov, t);
        }
        c->ov_plain_form_us = best_plain;
        c->ov_form_us = best_ov;
        return CGX_OK;
    }();
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

constexpr int kOvNums = 6;  // the numbers choose_overlap takes the max over ranks of

int choose_overlap(cgx_ctx *c) {
    if (p2p(c)) {  // point-to-point_cg.c's exchange: through rank 0, never overlapped
        c->overlap = false;
        c->ov_how = CGX_OV_NA;
        return CGX_OK;
    }
    const char *e = std::getenv("CGX_OVERLAP");
    int forced = -1;  // -1: measure and decide
    if ((c->flags & CGX_NO_OVERLAP) || (e && *e == '0')) forced = 0;
    else if (e && (*e == '1' || std::strcmp(e, "force") == 0)) forced = 1;
    if (c->mode == M_LOCAL || c->nranks > 1) {
        TRY(measure_split(c));
        TRY(measure_allgather(c));
        const auto t0 = std::chrono::steady_clock::now();
        TRY(measure_forms(c));
        c->ov_forms_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (c->mode == M_RCCL) {  // the maxima over ranks, on every rank
            Shard &s = c->sh[0];
            TRY(set_dev(s));
            double *h = s.h_pin;
            double *const v[kOvNums] = {&c->ov_ag_us, &c->ov_split_us, &c->ov_one_us, &c->ov_cost_us,
                                        &c->ov_form_us, &c->ov_plain_form_us};
            for (int i = 0; i < kOvNums; ++i) h[i] = *v[i];
            HIPT(hipMemcpyAsync(slot(s, S_GATHER), h, 8 * kOvNums, hipMemcpyHostToDevice, s.stream));
            NCCLC(c, ncclAllReduce(slot(s, S_GATHER), slot(s, S_GATHER), kOvNums, ncclDouble, ncclMax, s.comm,
                                   s.stream),
                  "ncclAllReduce(max), overlap calibration");
            HIPT(hipMemcpyAsync(h, slot(s, S_GATHER), 8 * kOvNums, hipMemcpyDeviceToHost, s.stream));
            TRY(rank_wait_stream(c, s.stream, "the overlap calibration"));
            for (int i = 0; i < kOvNums; ++i) *v[i] = h[i];
        }
    }
    if (forced >= 0) {
        c->overlap = forced == 1;
        c->ov_how = forced ? CGX_OV_FORCED : CGX_OV_OFF;
    } else {
        c->overlap = c->ov_form_us < (1.0 - kOverlapMargin) * c->ov_plain_form_us;
        c->ov_how = CGX_OV_MEASURED;
    }
    debug_log("overlap %s (overlap form %.1f us, plain form %.1f us; allgather %.1f us, split %.1f us, one launch "
              "%.1f us, cost %.1f us; how %d)",
              c->overlap ? "on" : "off", c->ov_form_us, c->ov_plain_form_us, c->ov_ag_us, c->ov_split_us,
              c->ov_one_us, c->ov_cost_us, c->ov_how);
    return CGX_OK;
}

// Overlapped r halo exchange (several slabs): on the comm streams, after
// everything already on the compute streams (the r update and the r.r
// allreduce, so two RCCL operations never run at once).  The next
// k_poisson_p runs its interior runs meanwhile and waits for ev_gathered
// before its two edge runs.
int exchange_halo_async(cgx_ctx *c) {
    const size_t row = (size_t)c->m * (size_t)c->es;
    const int64_t mloc = c->sh[0].nloc / c->m;
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipEventRecord(s.ev_pready, s.stream));
    }
    if (c->mode == M_RCCL) {
        Shard &s = c->sh[0];
        const int g = s.index;
        char *base = s.rh, *own = base + row;
        HIPT(hipStreamWaitEvent(s.cstream, s.ev_pready, 0));
        NCCLC(c, ncclGroupStart(), kWhatHaloAsync);
        if (g > 0) {
            NCCLC(c, ncclSend(own, (size_t)c->m, ncclDouble, g - 1, s.comm, s.cstream), kWhatHaloAsync);
            NCCLC(c, ncclRecv(base, (size_t)c->m, ncclDouble, g - 1, s.comm, s.cstream), kWhatHaloAsync);
        }
        if (g < c->nranks - 1) {
            NCCLC(c, ncclSend(own + (size_t)(mloc - 1) * row, (size_t)c->m, ncclDouble, g + 1, s.comm, s.cstream),
                  kWhatHaloAsync);
            NCCLC(c, ncclRecv(own + (size_t)mloc * row, (size_t)c->m, ncclDouble, g + 1, s.comm, s.cstream),
                  kWhatHaloAsync);
        }
        NCCLC(c, ncclGroupEnd(), kWhatHaloAsync);
        HIPT(hipEventRecord(s.ev_gathered, s.cstream));
    } else {
        const int S = (int)c->sh.size();
        for (int q = 0; q < S; ++q) {
            Shard &d = c->sh[q];
            TRY(set_dev(d));
            for (auto &s : c->sh) HIPT(hipStreamWaitEvent(d.cstream, s.ev_pready, 0));
            if (q > 0) {
                const Shard &u = c->sh[q - 1];
                HIPT(hipMemcpyPeerAsync(d.rh, d.dev, u.rh + (size_t)mloc * row, u.dev, row, d.cstream));
            }
            if (q < S - 1) {
                const Shard &w = c->sh[q + 1];
                HIPT(hipMemcpyPeerAsync(d.rh + (size_t)(mloc + 1) * row, d.dev, w.rh + row, w.dev, row, d.cstream));
            }
            HIPT(hipEventRecord(d.ev_gathered, d.cstream));
        }
    }
    c->halo_pending = true;
    return CGX_OK;
}

// Order every compute stream after an overlapped halo exchange still in
// flight (before anything else touches r or its halo rows).
int settle_halo(cgx_ctx *c) {
    if (!c->halo_pending) return CGX_OK;
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        HIPT(hipStreamWaitEvent(s.stream, s.ev_gathered, 0));
    }
    c->halo_pending = false;
    return CGX_OK;
}

int sync_all(cgx_ctx *c) {
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        TRY(rank_wait_stream(c, s.stream, "the compute stream"));
        for (int q = 0; q < s.ncopy; ++q) HIPT(hipStreamSynchronize(s.copy[q]));
        if (s.cstream) TRY(rank_wait_stream(c, s.cstream, "the exchange stream"));
    }
    // The timing and phase events are resolved on request (cgx_get_stats,
    // cgx_get_phase_times, cgx_reset_timing), not here: a caller's own timed
    // region ending in a synchronize pays no event queries.
    return CGX_OK;
}

// ---- rank-mode fail-fast ---------------------------------------------------------
// The reference stops the whole job on a failure (MPI_Abort, parallel_cg.c:79,
// 89,94,143).  RCCL has no such global stop: a rank that died or issued a
// different collective leaves its peers' RCCL kernels waiting forever, and a
// plain hipStreamSynchronize with them.  So in rank mode every host wait polls
// with a deadline and watches the communicator's asynchronous error; on either
// the communicator is aborted (its kernels see the abort flag and exit, the
// stream drains) and the call returns CGX_ERR_RCCL naming the exchange and the
// iteration.  The other modes keep plain blocking waits.
double rccl_timeout_from_env() {
    const char *e = std::getenv("CGX_RCCL_TIMEOUT_S");
    if (!e || !*e) return 60.0;
    const double v = std::atof(e);
    return v > 0.0 ? v : 0.0;
}

int dead_error(const cgx_ctx *c) {
    return fail(CGX_ERR_RCCL, "rank %d of %d: the RCCL communicator was aborted earlier (%s)", c->sh[0].index,
                c->nranks, c->dead_why);
}

static int rccl_abort(cgx_ctx *c, const char *fmt, ...) {
    Shard &s = c->sh[0];
    char why[320];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(why, sizeof why, fmt, ap);
    va_end(ap);
    snprintf(c->dead_why, sizeof c->dead_why, "%s; last exchange enqueued: %s at iteration %lld", why, c->last_coll,
             (long long)c->last_coll_k);
    c->dead = true;
    debug_log("rank %d: aborting the communicator: %s", s.index, c->dead_why);
    if (s.comm) {
        (void)ncclCommAbort(s.comm);  // RCCL kernels still waiting on a peer exit
        s.comm = nullptr;
    }
    debug_log("rank %d: ncclCommAbort returned", s.index);
    return fail(CGX_ERR_RCCL, "rank %d of %d: %s", s.index, c->nranks, c->dead_why);
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Which of the shard's per-iteration events (the lookahead ring, the progress
// ring, the newest timing event) have completed, as a bit pattern: when
// it changes the GPU has finished more of the enqueued work, i.e. the job is
// making progress.
static uint64_t progress_sig(const cgx_ctx *c) {
    const Shard &s = c->sh[0];
    uint64_t sig = 0;
    int bit = 0;
    auto probe = [&](hipEvent_t e) {
        if (e && bit < 64 && hipEventQuery(e) == hipSuccess) sig |= uint64_t(1) << bit;
        ++bit;
    };
    for (auto e : s.ev_look) probe(e);
    for (auto e : s.ev_prog) probe(e);
    const int nt = s.ev_used;  // the newest timed matVec's end
    if (nt > 0) probe(s.ev_t[2 * nt - 1]);
    return sig;
}

// Poll `ready` (a hipEventQuery / hipStreamQuery) until it reports success,
// checking the communicator and the deadline in between.  The deadline
// counts time WITHOUT PROGRESS: it restarts whenever one more of the shard's
// per-iteration events completes (progress_sig), so a long healthy wait (a
// fixed-count run of many iterations, ranks reaching their first collective
// at different times while the others still compute) never trips it; only a
// stall does -- a peer that died or issued a different collective.
template <typename F>
static int rank_poll(cgx_ctx *c, F ready, const char *what) {
    double t0 = now_s();
    uint64_t sig = progress_sig(c);
    for (long spins = 0;; ++spins) {
        const hipError_t e = ready();
        if (e == hipSuccess) return CGX_OK;
        if (e != hipErrorNotReady)
            return fail(CGX_ERR_HIP, "waiting for %s: %s", what, hipGetErrorString(e));
        if (spins < 2048) continue;  // the common case: done within microseconds
        ncclResult_t ar = ncclSuccess;
        if (c->sh[0].comm && ncclCommGetAsyncError(c->sh[0].comm, &ar) == ncclSuccess && ar != ncclSuccess &&
            ar != ncclInProgress)
            return rccl_abort(c, "RCCL reported '%s' while waiting for %s", ncclGetErrorString(ar), what);
        if ((spins & 63) == 0) {
            const uint64_t now_sig = progress_sig(c);
            if (now_sig != sig) {
                sig = now_sig;
                t0 = now_s();
            }
        }
        if (c->rccl_timeout_s > 0.0 && now_s() - t0 > c->rccl_timeout_s)
            return rccl_abort(c, "no progress for %.0f s waiting for %s (a rank died, or ranks issued different "
                                 "collectives; CGX_RCCL_TIMEOUT_S sets the limit)",
                              c->rccl_timeout_s, what);
        std::this_thread::sleep_for(std::chrono::microseconds(spins < 20000 ? 20 : 200));
    }
}

int rank_wait_event(cgx_ctx *c, hipEvent_t ev, const char *what) {
    if (c->mode != M_RCCL || c->rccl_timeout_s <= 0.0) {
        HIPT(hipEventSynchronize(ev));
        return CGX_OK;
    }
    if (c->dead) return dead_error(c);
    return rank_poll(c, [ev] { return hipEventQuery(ev); }, what);
}

int rank_wait_stream(cgx_ctx *c, hipStream_t st, const char *what) {
    if (c->mode != M_RCCL || c->rccl_timeout_s <= 0.0 || c->dead) {
        // a dead context's streams drain once the abort has stopped RCCL's kernels
        HIPT(hipStreamSynchronize(st));
        return CGX_OK;
    }
    return rank_poll(c, [st] { return hipStreamQuery(st); }, what);
}

// After an RCCL call (NCCLC): ncclInProgress (a nonblocking communicator's
// asynchronous enqueue) is waited for with the deadline, and the
// communicator's asynchronous error state is checked after every call, so a
// failure the proxy thread saw surfaces at the next exchange.
int rccl_after(cgx_ctx *c, ncclResult_t r, const char *what, const char *expr, const char *file, int line) {
    c->last_coll = what;
    c->last_coll_k = c->k;
    if (r == ncclSuccess || r == ncclInProgress) {
        const double t0 = now_s();
        Shard &s = c->sh[0];
        for (;;) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t q = ncclCommGetAsyncError(s.comm, &st);
            if (q != ncclSuccess) {
                r = q;
                break;
            }
            if (st != ncclInProgress) {
                r = st;
                break;
            }
            if (c->rccl_timeout_s > 0.0 && now_s() - t0 > c->rccl_timeout_s)
                return rccl_abort(c, "%s did not finish enqueueing within %.0f s", what, c->rccl_timeout_s);
            std::this_thread::yield();
        }
    }
    if (r == ncclSuccess) return CGX_OK;
    return rccl_abort(c, "%s: %s (%s:%d)", expr, ncclGetErrorString(r), file, line);
}

}  // namespace cgxh
