// cgx_iterate.hip -- the conjugrad loop (cgx_ctx.h):
//   conjugrad()  serialConjugate.c:180-259 / parallel_cg.c:248-345
//     -> cgx_solve = cgx_solve_begin (:209-212) + cgx_iterate (:213-245)
// the matVec dispatch (resident, host-streamed, symmetric, Poisson), the
// iteration with its stopping test on the host or on the device (gating),
// and the true-residual check.
#include "cgx_ctx.h"

namespace cgxh {

// ---- the iteration pieces ----------------------------------------------------------
// One tile of the matVec: rows [r0, r0+rows) of this shard, A rows at `Arows`.
int matvec_rows(cgx_ctx *c, Shard &s, const MatvecPlan &pl, const char *Arows, int64_t r0, int64_t rows,
                const char *vec, bool fuse_dot, int dot_slot, bool gated, int64_t *ts) {
    if (f32ref(c)) {
        HIPT(matvec_ref_f32(reinterpret_cast<const float *>(Arows), c->lda, rows, c->n,
                            reinterpret_cast<const float *>(vec), reinterpret_cast<float *>(s.Ap) + r0, s.stream,
                            gate_of(s, gated)));
    } else if (c->rot && Arows == s.A && r0 == 0 && rows == s.nloc) {
        // the block's own columns, then the rest, summed apart and added: the
        // overlapped form's bits in one launch (cgx_ctx::rot)
        HIPT(matvec_f64_cols(pl, reinterpret_cast<const double *>(Arows), c->lda, rows, c->lda, s.row0, c->lda, false,
                             reinterpret_cast<const double *>(vec), reinterpret_cast<double *>(s.Ap),
                             fuse_dot ? reinterpret_cast<const double *>(s.pown) : nullptr,
                             fuse_dot ? reinterpret_cast<double *>(slot(s, dot_slot)) : nullptr, s.ws, s.stream,
                             gated ? reinterpret_cast<const int64_t *>(slot(s, S_KDONE)) : nullptr, ts, s.nloc));
    } else {
        HIPT(matvec_f64(pl, reinterpret_cast<const double *>(Arows), c->lda, rows, c->lda,
                        reinterpret_cast<const double *>(vec), reinterpret_cast<double *>(s.Ap) + r0,
                        fuse_dot ? reinterpret_cast<const double *>(s.pown) + r0 : nullptr,
                        fuse_dot ? reinterpret_cast<double *>(slot(s, dot_slot)) : nullptr, s.ws, s.stream,
                        gated ? reinterpret_cast<const int64_t *>(slot(s, S_KDONE)) : nullptr, ts));
    }
    return CGX_OK;
}

// CGX_HOST_STREAM matVec: tile t goes to buffer (next_buf++ % kStreamBufs);
// its copy waits until the kernel that last read that buffer is done (A is
// read-only, so copies of the next iteration's first tiles overlap this
// iteration's vector work); its kernel waits for the copy.
// With resident rows (CGX_STREAM_RESIDENT_MB) their kernel goes first on the
// compute stream, so it runs while the copy streams bring in the first tiles
// of the rest (same row sums: every plan adds a row in the same order).
int matvec_streamed(cgx_ctx *c, Shard &s, const char *vec) {
    const int64_t row_bytes = c->lda * (int64_t)c->es;
    if (s.res_rows > 0) {
        if (s.res_dirty) {  // A changed on the host since the last copy (pinned: async)
            HIPT(hipMemcpyAsync(s.A, s.A_host, (size_t)s.res_rows * row_bytes, hipMemcpyHostToDevice, s.stream));
            s.res_dirty = false;
        }
        TRY(matvec_rows(c, s, s.res_plan, s.A, 0, s.res_rows, vec, false, 0));
    }
    for (int64_t r0 = s.res_rows; r0 < s.nloc; r0 += s.tile_rows) {
        const int64_t rows = std::min(s.tile_rows, s.nloc - r0);
        const int b = s.next_buf;
        s.next_buf = (s.next_buf + 1) % kStreamBufs;
        const int64_t bytes = rows * row_bytes;
        const char *src = s.A_host + (size_t)r0 * row_bytes;
        const int64_t part = (bytes / s.ncopy + 4095) & ~int64_t(4095);
        for (int q = 0; q < s.ncopy; ++q) {
            const int64_t lo = std::min<int64_t>(bytes, q * part), hi = std::min<int64_t>(bytes, lo + part);
            if (s.buf_used[b]) HIPT(hipStreamWaitEvent(s.copy[q], s.ev_free[b], 0));
            if (hi > lo) HIPT(hipMemcpyAsync(s.tile[b] + lo, src + lo, hi - lo, hipMemcpyHostToDevice, s.copy[q]));
            HIPT(hipEventRecord(s.ev_loaded[b][q], s.copy[q]));
            HIPT(hipStreamWaitEvent(s.stream, s.ev_loaded[b][q], 0));
        }
        TRY(matvec_rows(c, s, s.tile_plan, s.tile[b], r0, rows, vec, false, 0));
        HIPT(hipEventRecord(s.ev_free[b], s.stream));
        s.buf_used[b] = true;
    }
    return CGX_OK;
}

// CGX_SYMMETRIC | CGX_HOST_STREAM: the upper-triangle tiles stream from
// pinned host memory in chunks (the same buffer rotation and copy streams as
// matvec_streamed); each chunk's k_symv_f64 writes per-tile row and column
// partials, and one reduce (with the fused p.Ap) follows the last chunk.
int matvec_sym_streamed(cgx_ctx *c, Shard &s, const char *vec, bool with_dot, int dot_slot, const int64_t *gate) {
    const int64_t ntiles = sym_tiles(c->lda), tb = 128 * 128 * 8;
    const double *p = reinterpret_cast<const double *>(vec);
    if (s.res_rows > 0) {  // the resident tiles first, under the copies of the rest (as matvec_streamed)
        if (s.res_dirty) {
            HIPT(hipMemcpyAsync(s.A, s.A_host, (size_t)s.res_rows * tb, hipMemcpyHostToDevice, s.stream));
            s.res_dirty = false;
        }
        HIPT(symv_tiles_f64(reinterpret_cast<const double *>(s.A), 0, s.res_rows, c->lda, s.sym_grid, true, p,
                            reinterpret_cast<double *>(s.sym_prow), reinterpret_cast<double *>(s.sym_pcol), s.stream,
                            gate));
    }
    for (int64_t q0 = s.res_rows; q0 < ntiles; q0 += s.tile_rows) {
        const int64_t cnt = std::min(s.tile_rows, ntiles - q0);
        const int b = s.next_buf;
        s.next_buf = (s.next_buf + 1) % kStreamBufs;
        const int64_t bytes = cnt * tb;
        const char *src = s.A_host + (size_t)q0 * tb;
        const int64_t part = (bytes / s.ncopy + 4095) & ~int64_t(4095);
        for (int q = 0; q < s.ncopy; ++q) {
            const int64_t lo = std::min<int64_t>(bytes, q * part), hi = std::min<int64_t>(bytes, lo + part);
            if (s.buf_used[b]) HIPT(hipStreamWaitEvent(s.copy[q], s.ev_free[b], 0));
            if (hi > lo) HIPT(hipMemcpyAsync(s.tile[b] + lo, src + lo, hi - lo, hipMemcpyHostToDevice, s.copy[q]));
            HIPT(hipEventRecord(s.ev_loaded[b][q], s.copy[q]));
            HIPT(hipStreamWaitEvent(s.stream, s.ev_loaded[b][q], 0));
        }
        HIPT(symv_tiles_f64(reinterpret_cast<const double *>(s.tile[b]), q0, cnt, c->lda, s.sym_grid, true, p,
                            reinterpret_cast<double *>(s.sym_prow), reinterpret_cast<double *>(s.sym_pcol), s.stream,
                            gate));
        HIPT(hipEventRecord(s.ev_free[b], s.stream));
        s.buf_used[b] = true;
    }
    HIPT(symv_reduce_f64(c->n, c->lda, 1, reinterpret_cast<const double *>(s.sym_prow),
                         reinterpret_cast<const double *>(s.sym_pcol), reinterpret_cast<double *>(s.Ap),
                         with_dot ? reinterpret_cast<const double *>(s.pown) : nullptr,
                         with_dot ? reinterpret_cast<double *>(slot(s, dot_slot)) : nullptr, s.ws, s.stream, gate));
    return CGX_OK;
}

// The host-mapped convergence record: written by shard 0's deciding kernel only.

int launch_matvec(cgx_ctx *c, Shard &s, const char *vec, bool with_dot, int dot_slot, bool gated) {
    const bool timing = (c->flags & CGX_TIMING) && (&s == &c->sh[0]);
    if (timing && s.ev_used >= kEvPairs) TRY(timing_resolve(c));
    if (timing) HIPT(hipEventRecord(s.ev_t[2 * s.ev_used], s.stream));
    const bool streamed = (c->flags & CGX_HOST_STREAM) != 0;
    if (c->op == OP_POISSON)
        HIPT(stencil5_f64(reinterpret_cast<const double *>(vec), s.nloc / c->m, c->m, reinterpret_cast<double *>(s.Ap),
                          with_dot ? reinterpret_cast<double *>(slot(s, dot_slot)) : nullptr, s.ws, s.stream,
                          gate_of(s, gated)));
    else if (streamed && (c->flags & CGX_SYMMETRIC))
        TRY(matvec_sym_streamed(c, s, vec, with_dot, dot_slot, gate_of(s, gated)));
    else if (streamed) TRY(matvec_streamed(c, s, vec));
    else if (c->flags & CGX_SYMMETRIC)
        HIPT(symv_f64(reinterpret_cast<const double *>(s.A), c->n, c->lda, s.sym_grid,
                      reinterpret_cast<const double *>(vec), reinterpret_cast<double *>(s.sym_prow),
                      reinterpret_cast<double *>(s.sym_pcol), reinterpret_cast<double *>(s.Ap),
                      with_dot ? reinterpret_cast<const double *>(s.pown) : nullptr,
                      with_dot ? reinterpret_cast<double *>(slot(s, dot_slot)) : nullptr, s.ws, s.stream,
                      gate_of(s, gated)));
    else if (with_dot && c->ref_mv_dot)  // matVec + vecVec(p, Ap) in one launch (serialConjugate.c:215,219)
        HIPT(matvec_dot_ref_f32(reinterpret_cast<const float *>(s.A), c->lda, s.nloc, c->n,
                                reinterpret_cast<const float *>(vec), reinterpret_cast<float *>(s.Ap),
                                reinterpret_cast<const float *>(s.pown), reinterpret_cast<float *>(slot(s, dot_slot)),
                                s.ws.tickets + T_REF_MV, s.stream, gate_of(s, gated)));
    else TRY(matvec_rows(c, s, s.plan, s.A, 0, s.nloc, vec, with_dot && !f32ref(c), dot_slot, gated,
                         f32ref(c) ? nullptr : ts_of(c, s, TK_MV)));
    if (timing) {
        HIPT(hipEventRecord(s.ev_t[2 * s.ev_used + 1], s.stream));
        s.ev_used++;
    }
    if (with_dot && ((f32ref(c) && !c->ref_mv_dot) || (streamed && !(c->flags & CGX_SYMMETRIC)))) {
        if (f32ref(c))  // vecVec(p, Ap) sequential (serialConjugate.c:219)
            HIPT(dot_ref_f32(s.nloc, reinterpret_cast<const float *>(s.pown),
                             reinterpret_cast<const float *>(s.Ap), reinterpret_cast<float *>(slot(s, dot_slot)),
                             s.stream, gate_of(s, gated)));
        else
            HIPT(dot_f64(s.nloc, reinterpret_cast<const double *>(s.pown),
                         reinterpret_cast<const double *>(s.Ap), reinterpret_cast<double *>(slot(s, dot_slot)), s.ws,
                         s.stream));
    }
    return CGX_OK;
}

// Whether x0 is all zeros on every shard (every rank in rank mode: one
// int64 allreduce, so all ranks take the same branch of do_begin).
int x0_is_zero(cgx_ctx *c, bool *zero) {
    bool local = true;
    for (auto &s : c->sh) local = local && s.x_zero;
    if (c->mode != M_RCCL || c->nranks == 1) {
        *zero = local;
        return CGX_OK;
    }
    Shard &s = c->sh[0];
    TRY(set_dev(s));
    int64_t *pin = reinterpret_cast<int64_t *>(s.h_pin);
    pin[0] = local ? 0 : 1;
    HIPT(hipMemcpyAsync(slot(s, S_XNZ), pin, 8, hipMemcpyHostToDevice, s.stream));
    NCCLC(c, ncclAllReduce(slot(s, S_XNZ), slot(s, S_XNZ), 1, ncclInt64, ncclSum, s.comm, s.stream),
          "ncclAllReduce(x0 != 0 count)");
    HIPT(hipMemcpyAsync(pin, slot(s, S_XNZ), 8, hipMemcpyDeviceToHost, s.stream));
    TRY(rank_wait_stream(c, s.stream, "the x0 check"));
    *zero = pin[0] == 0;
    return CGX_OK;
}

int do_begin(cgx_ctx *c) {
    // r0 = p0 = b - A x0; rr0 = r0.r0   (serialConjugate.c:209-212, parallel_cg.c:283-287)
    // With x0 = 0 (the reference's usual initialguess, and the bench's) A x0 is
    // exactly zero for a finite A, so the exchange and the matVec are skipped:
    // r0 = b - 0 = b bit for bit, one matVec fewer per solve.  (An A holding
    // Inf or NaN gives NaN in A x0 at serialConjugate.c:209; cgx.h states the
    // finite-A precondition of the fp64 mode.)  CGX_F32_REF, the mode that
    // promises the reference's bits for any input, always does the matVec.
    TRY(settle_halo(c));
    bool zero = false;  // CGX_F32_REF always does the matVec: no need to ask (in rank mode: a collective)
    if (!f32ref(c)) TRY(x0_is_zero(c, &zero));
    // One GPU, CGX_F32_REF in HBM: the matVec reads x0 where it lies (its
    // vector loads stop at n, where pfull would be zero-padded), so x0 is not
    // copied into pfull first -- one copy fewer per solve.
    const bool x_direct = f32ref(c) && c->mode == M_SINGLE && !(c->flags & CGX_HOST_STREAM);
    if (!zero && !x_direct) TRY(exchange_allgather(c, /*from_x=*/true));  // full x0 into pfull
    const int gs = S_RR + ring(0), ls = S_LRR + ring(0);
    const int os = out_slot(c, ls, gs);
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        if (!zero)
            TRY(launch_matvec(c, s, x_direct ? s.x : s.pfull, false, 0));
        s.x_zero = false;  // the iterations update x
        if (f32ref(c)) {
            HIPT(residual_dot_ref_f32(s.nloc, reinterpret_cast<const float *>(s.b),
                                      reinterpret_cast<const float *>(s.Ap), reinterpret_cast<float *>(s.r),
                                      reinterpret_cast<float *>(s.pown), reinterpret_cast<float *>(slot(s, os)),
                                      s.stream, reinterpret_cast<int64_t *>(slot(s, S_KDONE))));
        } else {
            // x0 = 0: Ax = nullptr (r = b - 0.0, no Ap buffer to clear); the
            // kernel also resets the convergence record (no memset launch)
            double *pown = reinterpret_cast<double *>(s.pown);
            HIPT(residual_f64(s.nloc, reinterpret_cast<const double *>(s.b),
                              zero ? nullptr : reinterpret_cast<const double *>(s.Ap),
                              reinterpret_cast<double *>(s.r), pown, reinterpret_cast<double *>(slot(s, os)), s.ws,
                              s.stream, reinterpret_cast<int64_t *>(slot(s, S_KDONE))));
        }
    }
    TRY(exchange_scalar(c, ls, gs));
    c->rr_unsummed = false;
    // r0's halo rows for k_poisson_p (which reads them in place itself with halo_pull)
    if (c->fused && !c->halo_pull) TRY(exchange_halo_of(c, &Shard::rh));
    // The device-side convergence record {kdone, r.r} was reset by the residual
    // kernel above (k_residual_f64 / k_dot_ref_f32_blk<kDotResid>); the host copy here.
    for (auto &s : c->sh) s.h_rec[0] = s.h_rec[1] = 0;  // no kernel of this solve has run yet (do_begin follows a sync)
    c->k = 0;
    c->converged = 0;
    c->state = ST_BEGUN;
    c->x_incomplete = c->x_deferred = false;
    c->xalpha_pending = false;
    c->iter_failed = false;
    return CGX_OK;
}

int read_scalar(cgx_ctx *c, int gslot, double *out) {
    Shard &s = c->sh[0];
    TRY(set_dev(s));
    HIPT(hipMemcpyAsync(s.h_pin, slot(s, gslot), 8, hipMemcpyDeviceToHost, s.stream));
    TRY(rank_wait_stream(c, s.stream, "a scalar read-back"));
    if (f32ref(c)) {
        float f;
        std::memcpy(&f, s.h_pin, 4);
        *out = (double)f;
    } else {
        *out = s.h_pin[0];
    }
    return CGX_OK;
}

// Fused Poisson iteration k (conjgrad.m's loop, two kernels, 64 B per grid
// point; see k_poisson_p_f64 / k_poisson_xr_f64):
//   p_k = r_k + beta p_{k-1}, p_k . A p_k      (gated: first decides the
//                                               previous iteration's stop)
//   allreduce(p.Ap)
//   x += alpha p_k, r -= alpha A p_k, r.r
//   allreduce(r.r); host-checked stop; r's halo rows for the next iteration.
// x is updated every other iteration (c->xdefer: the left-out iteration's
// alpha is kept in S_XALPHA and p_k stays in its slab until the next
// iteration's xr kernel has read it); poisson_x_finish completes it at the end
// of a cgx_iterate call.
// Where p_k lives: two slabs alternate (pfull for even k), three rotate with x every third iteration.
static char *poisson_slab(const cgx_ctx *c, const Shard &s, int64_t k) {
    if (c->xd == 3) {
        const int64_t q = ((k % 3) + 3) % 3;
        return q == 0 ? s.pfull : q == 1 ? s.p2 : s.p3;
    }
    return (k & 1) ? s.p2 : s.pfull;
}

int do_iteration_poisson(cgx_ctx *c, double eps, int *stop, bool gated) {
    const int64_t k = c->k;
    *stop = 0;
    const int64_t m = c->m;
    const int pg = S_PAP + ring(k), pl = S_LPAP + ring(k);
    const int rk = S_RR + ring(k), rkm1 = S_RR + ring(k + 3);  // r.r of iterations k, k-1
    auto D = [](void *p) { return reinterpret_cast<double *>(p); };
    const bool split = c->halo_pending;  // interior runs while the r halo exchange is in flight
    // x every D-th iteration (D = c->xd): leave it out at the first D-1 of every
    // D iterations from k0 (alpha_k to slot S_XALPHA + j), catch up at the D-th
    const int64_t jx = (k - c->xd_k0) % c->xd;
    const int xmode = c->xd == 1 ? 1 : jx == c->xd - 1 ? c->xd : 0;
    const int xslot = S_XALPHA + (xmode == 0 ? (int)jx : 0);
    // One process, several slabs (c->fuse_combine): the scalar combines are
    // folded into the kernels that consume them -- p.Ap into k_poisson_xr,
    // r.r into the next k_poisson_p (not when the host reads r.r after the
    // iteration: then a combine kernel forms it) -- and r's halo rows are read
    // in place from the neighbouring slabs by k_poisson_p (c->halo_pull).
    // Both wait on the same cross-stream events the combines waited on.
    const bool fold_rr = c->fuse_combine && (gated || eps < 0.0);
    const int S = (int)c->sh.size();
    const int64_t mloc = c->sh[0].nloc / m;
    for (int q = 0; q < S; ++q) {
        Shard &s = c->sh[q];
        TRY(set_dev(s));
        char *pold = poisson_slab(c, s, k - 1), *pnew = poisson_slab(c, s, k);
        // the previous slab's last interior row of r, the next slab's first
        const double *r_up = c->halo_pull && q > 0 ? D(c->sh[q - 1].rh) + mloc * m : nullptr;
        const double *r_dn = c->halo_pull && q < S - 1 ? D(c->sh[q + 1].r) : nullptr;
        const PeerSum rs = c->rr_unsummed ? peer_sum(c, s, S_LRR + ring(k), rk) : PeerSum{};
        for (int part : split ? std::initializer_list<int>{1, 2} : std::initializer_list<int>{0}) {
            if (part == 2) HIPT(hipStreamWaitEvent(s.stream, s.ev_gathered, 0));
            HIPT(poisson_p_f64(D(s.rh), D(pold), D(pnew), mloc, m, D(slot(s, rk)), D(slot(s, rkm1)), k == 0,
                               D(slot(s, out_slot(c, pl, pg))), s.ws, s.stream, gated ? eps : -1.0, k,
                               gated ? reinterpret_cast<int64_t *>(slot(s, S_KDONE)) : nullptr,
                               gated ? D(slot(s, S_RRFINAL)) : nullptr, part, rec_of(c, s, gated), r_up, r_dn,
                               c->rr_unsummed ? &rs : nullptr));
        }
    }
    c->rr_unsummed = false;
    c->halo_pending = false;
    if (c->fuse_combine) TRY(local_barrier(c));  // MPI_Allreduce(p.Ap): summed by k_poisson_xr itself
    else TRY(exchange_scalar(c, pl, pg));
    const int rg = S_RR + ring(k + 1), rl = S_LRR + ring(k + 1);
    const int ro = out_slot(c, rl, rg);
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        const bool timing = (c->flags & CGX_TIMING) && (&s == &c->sh[0]);
        if (timing && s.ev_used >= kEvPairs) TRY(timing_resolve(c));
        if (timing) HIPT(hipEventRecord(s.ev_t[2 * s.ev_used], s.stream));
        char *pnew = poisson_slab(c, s, k), *pold = poisson_slab(c, s, k - 1),
             *pq = c->xd == 3 ? poisson_slab(c, s, k - 2) : nullptr;
        const PeerSum ps = c->fuse_combine ? peer_sum(c, s, pl, pg) : PeerSum{};
        HIPT(poisson_xr_f64(D(pnew), D(pold), D(pq), D(s.x), D(s.r), mloc, m, D(slot(s, rk)), D(slot(s, pg)),
                            D(slot(s, ro)), xmode, D(slot(s, xslot)), s.ws, s.stream, gate_of(s, gated),
                            c->fuse_combine ? &ps : nullptr));
        if (timing) {
            HIPT(hipEventRecord(s.ev_t[2 * s.ev_used + 1], s.stream));
            s.ev_used++;
        }
    }
    c->xalpha_pending = xmode == 0;  // the catch-up (xmode xd) and every-iteration x (1) leave nothing out
    if (fold_rr) {  // MPI_Allreduce(r.r): summed by the next k_poisson_p (or settle_rr)
        TRY(local_barrier(c));
        c->rr_unsummed = true;
    } else {
        TRY(exchange_scalar(c, rl, rg));
    }
    c->k = k + 1;
    c->total_iters += 1;
    if (!gated && eps >= 0.0) {
        double rr = 0.0;
        TRY(read_scalar(c, rg, &rr));
        c->last_rr = rr;
        if (std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
            *stop = 1;
            return CGX_OK;
        }
    }
    if (c->halo_pull) return CGX_OK;  // the next k_poisson_p reads the neighbours' rows itself
    return c->halo_overlap ? exchange_halo_async(c) : exchange_halo_of(c, &Shard::rh);
}

// The r.r of the last iteration enqueued, when its combine was left to the
// next k_poisson_p (rr_unsummed): formed now by the combine kernels, for the
// host to read (or a later call's first k_poisson_p, which sums the same
// partials again).
int settle_rr(cgx_ctx *c) {
    if (!c->rr_unsummed) return CGX_OK;
    TRY(exchange_scalar(c, S_LRR + ring(c->k), S_RR + ring(c->k)));
    c->rr_unsummed = false;
    return CGX_OK;
}

// The end of a cgx_iterate call (the device's loop count known: c->k): when
// the last iteration run left x's update out (xmode 0), x += alpha_K p_K.
// Gated solves enqueue iterations past the stop that skip themselves, so this
// is decided from c->k, never from what was enqueued.
int poisson_x_finish(cgx_ctx *c) {
    if (!c->fused || c->xd == 1) return CGX_OK;
    const int64_t last = c->k - 1;
    const int64_t jx = last >= c->xd_k0 ? (last - c->xd_k0) % c->xd : c->xd - 1;
    if (jx != c->xd - 1) {  // jx + 1 updates left out: iterations last - jx .. last
        for (auto &s : c->sh) {
            TRY(set_dev(s));
            char *pa = poisson_slab(c, s, last - jx), *pb = jx == 1 ? poisson_slab(c, s, last) : nullptr;
            HIPT(poisson_xflush_f64(reinterpret_cast<const double *>(pa), reinterpret_cast<const double *>(pb),
                                    reinterpret_cast<double *>(s.x), s.nloc / c->m, c->m,
                                    reinterpret_cast<const double *>(slot(s, S_XALPHA)), s.stream));
        }
    }
    c->xd_k0 = c->k;
    c->xalpha_pending = false;
    return CGX_OK;
}

int check_x_complete(const cgx_ctx *c) {
    if (!c->x_incomplete) return CGX_OK;
    if (c->x_deferred)
        return fail(CGX_ERR_STATE, "an earlier cgx_iterate failed with x updates still deferred (Poisson, x every "
                                   "%d-th iteration): x is incomplete until cgx_set_x or the next cgx_solve_begin",
                    c->xd);
    return fail(CGX_ERR_STATE, "an earlier cgx_iterate failed part-way through iteration %lld: x may hold part of it "
                               "and is incomplete until cgx_set_x or the next cgx_solve_begin", (long long)c->k);
}

// One loop iteration k (serialConjugate.c:215-244 / parallel_cg.c:290-323).
// Returns 1 in *stop when sqrt(r.r) < eps ended the loop (before the p update,
// as the reference breaks at :235-238).
// gated: fp64 device-side convergence (the host does not read r.r here; the
// update kernel decides sqrt(r.r) < eps and later kernels skip themselves).
// The two-launch iteration of a small dense fp64 system on one GPU
// (c->fused_p): the matVec with its fused p.Ap, then k_update_xrp_f64, whose
// last block decides the stop and forms p for the next iteration.  The same
// expressions in the same order as the three launches below (bitwise the same
// x), one kernel boundary and one host launch fewer per iteration.
static int do_iteration_fused_p(cgx_ctx *c, double eps, int *stop, bool gated) {
    const int64_t k = c->k;
    *stop = 0;
    Shard &s = c->sh[0];
    const int pg = S_PAP + ring(k), rg = S_RR + ring(k + 1);
    auto D = [](void *q) { return reinterpret_cast<double *>(q); };
    TRY(phase_iter_begin(c));
    TRY(launch_matvec(c, s, s.pfull, true, pg, gated));  // serialConjugate.c:215,219
    HIPT(update_xrp_f64(s.nloc, D(s.x), D(s.r), D(s.pown), D(s.Ap), D(slot(s, S_RR + ring(k))), D(slot(s, pg)),
                        D(slot(s, rg)), s.ws, s.stream, gate_of(s, gated), gated ? eps : -1.0, k,
                        gated ? reinterpret_cast<int64_t *>(slot(s, S_KDONE)) : nullptr,
                        gated ? D(slot(s, S_RRFINAL)) : nullptr, rec_of(c, s, gated), ts_of(c, s, TK_UXP)));  // :221-243
    phase_iter_end(c);
    c->k = k + 1;
    c->total_iters += 1;
    if (!gated && eps >= 0.0) {  // host-checked stop; x is already current
        double rr = 0.0;
        TRY(read_scalar(c, rg, &rr));
        c->last_rr = rr;
        if (std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
            *stop = 1;
        }
    }
    return CGX_OK;
}

// The two-launch iteration with the p update folded into the matVec
// (c->fold_p): k_matvec_fold_f64 forms p_k = r_k + beta p_{k-1} as it
// multiplies it (its row owners store p_k into the other p buffer and fuse
// p_k . A p_k), then k_update_xr_stop_f64 does x, r, r.r and the stopping
// decision on every block -- no single-block pass over p.  Iteration 0 uses
// p_0 = r_0 as the residual left it.  p_k lives in pfull for even k, in
// p_alt for odd k.  The expressions are the three-launch kernels' (bitwise
// the same x, test_two_launch_iteration_bitwise_equals_three).
static int do_iteration_fold_p(cgx_ctx *c, double eps, int *stop, bool gated) {
    const int64_t k = c->k;
    *stop = 0;
    Shard &s = c->sh[0];
    const int pg = S_PAP + ring(k), rg = S_RR + ring(k + 1);
    auto D = [](void *q) { return reinterpret_cast<double *>(q); };
    char *pk = (k & 1) ? s.p_alt : s.pfull, *pkm1 = (k & 1) ? s.pfull : s.p_alt;
    TRY(phase_iter_begin(c));
    if (k == 0) {
        TRY(launch_matvec(c, s, s.pfull, true, pg, gated));  // serialConjugate.c:215,219 with p_0 = r_0
    } else {
        const bool timing = (c->flags & CGX_TIMING) != 0;
        if (timing && s.ev_used >= kEvPairs) TRY(timing_resolve(c));
        if (timing) HIPT(hipEventRecord(s.ev_t[2 * s.ev_used], s.stream));
        // every column up to lda, as the plain matVec runs them (A, r and both p
        // buffers are zero there), so the row sums add in the same order
        HIPT(matvec_fold_f64(s.fold_plan, D(s.A), c->lda, s.nloc, c->lda, D(s.r), D(pkm1), D(pk), D(slot(s, S_RR + ring(k))),
                             D(slot(s, S_RR + ring(k + 3))), D(s.Ap), D(slot(s, pg)), s.ws, s.stream,
                             gate_of(s, gated), ts_of(c, s, TK_MV)));  // :239-243 of k-1, then :215,219
        if (timing) {
            HIPT(hipEventRecord(s.ev_t[2 * s.ev_used + 1], s.stream));
            s.ev_used++;
        }
    }
    HIPT(update_xr_stop_f64(s.nloc, D(s.x), D(s.r), D(pk), D(s.Ap), D(slot(s, S_RR + ring(k))), D(slot(s, pg)),
                            D(slot(s, rg)), s.ws, s.stream, gate_of(s, gated), gated ? eps : -1.0, k,
                            gated ? reinterpret_cast<int64_t *>(slot(s, S_KDONE)) : nullptr,
                            gated ? D(slot(s, S_RRFINAL)) : nullptr, rec_of(c, s, gated), ts_of(c, s, TK_UXP)));
    phase_iter_end(c);
    c->k = k + 1;
    c->total_iters += 1;
    if (!gated && eps >= 0.0) {  // host-checked stop; x is already current
        double rr = 0.0;
        TRY(read_scalar(c, rg, &rr));
        c->last_rr = rr;
        if (std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
            *stop = 1;
        }
    }
    return CGX_OK;
}

// The same for CGX_F32_REF (c->ref_fused): the matVec whose last block runs
// vecVec(p, Ap), then one single-block launch for x += p alpha, r -= Ap alpha,
// r.r, the stopping test and p = r + p (rr/rsold) -- four launches' float
// operations in their order (bitwise the same x and loop count).
static int do_iteration_ref_fused(cgx_ctx *c, double eps, int *stop, bool gated) {
    const int64_t k = c->k;
    *stop = 0;
    Shard &s = c->sh[0];
    const int pg = S_PAP + ring(k), rg = S_RR + ring(k + 1);
    auto F = [](void *q) { return reinterpret_cast<float *>(q); };
    TRY(launch_matvec(c, s, s.pfull, true, pg, gated));  // serialConjugate.c:215,219
    HIPT(update_xrp_dot_ref_f32(s.nloc, F(s.x), F(s.r), F(s.pown), F(s.Ap), F(slot(s, S_RR + ring(k))),
                                F(slot(s, pg)), F(slot(s, rg)), s.stream, gate_of(s, gated), gated ? eps : -1.0, k,
                                gated ? reinterpret_cast<int64_t *>(slot(s, S_KDONE)) : nullptr,
                                gated ? reinterpret_cast<double *>(slot(s, S_RRFINAL)) : nullptr,
                                rec_of(c, s, gated)));  // :220-243
    c->k = k + 1;
    c->total_iters += 1;
    if (!gated && eps >= 0.0) {  // host-checked stop; x is already current
        double rr = 0.0;
        TRY(read_scalar(c, rg, &rr));
        c->last_rr = rr;
        if (std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
            *stop = 1;
        }
    }
    return CGX_OK;
}

int do_iteration(cgx_ctx *c, double eps, int *stop, bool gated) {
    if (c->fused) return do_iteration_poisson(c, eps, stop, gated);
    if (c->fold_p) return do_iteration_fold_p(c, eps, stop, gated);
    if (c->fused_p) return do_iteration_fused_p(c, eps, stop, gated);
    if (c->ref_fused) return do_iteration_ref_fused(c, eps, stop, gated);
    const int64_t k = c->k;
    *stop = 0;
    const int pg = S_PAP + ring(k), pl = S_LPAP + ring(k);
    TRY(phase_iter_begin(c));
    if (c->pool && (gated || eps < 0.0)) {  // each row block's thread enqueues its own work (cgx_local_mt.hip)
        TRY(local_mt_iteration(c, eps, gated));
        phase_iter_end(c);
        c->k = k + 1;
        c->total_iters += 1;
        return CGX_OK;
    }
    if (c->overlap) {
        TRY(overlapped_matvec(c, out_slot(c, pl, pg), gated));  // parallel_cg.c:290-293, overlapped
    } else {
        TRY(exchange_allgather(c, false));  // MPI_Allgather(local_p -> p)  parallel_cg.c:290
        for (auto &s : c->sh) {
            TRY(set_dev(s));
            TRY(launch_matvec(c, s, s.pfull, true, out_slot(c, pl, pg), gated));  // :215 / :292-293
        }
    }
    // MPI_Allreduce(p.Ap)  parallel_cg.c:294 -- multi-shard fp64: summed by
    // k_update_r_f64 itself after the barrier (fuse_combine)
    // (F32_REF, fuse_f32: summed in MPICH order by k_dot_ref_f32_blk<kDotXR>)
    const bool fold = c->fuse_combine || c->fuse_f32;
    if (fold) TRY(local_barrier(c));
    else TRY(exchange_scalar(c, pl, pg));
    const int rg = S_RR + ring(k + 1), rl = S_LRR + ring(k + 1);
    const int ro = out_slot(c, rl, rg);
    // the r.r combine folds into k_update_xp_f64 (F32_REF: k_update_p_ref_f32)
    // unless the host reads r.r first (host-checked convergence)
    const bool fuse_rr = fold && (gated || eps < 0.0);
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        if (f32ref(c)) {
            // x += alpha p; r -= alpha Ap; r.r in one launch  (serialConjugate.c:219-234)
            const PeerSumF32 ps = c->fuse_f32 ? peer_sum_f32(c, s, pl, pg) : PeerSumF32{};
            HIPT(update_xr_dot_ref_f32(s.nloc, reinterpret_cast<float *>(s.x), reinterpret_cast<float *>(s.r),
                                       reinterpret_cast<const float *>(s.pown), reinterpret_cast<const float *>(s.Ap),
                                       reinterpret_cast<const float *>(slot(s, S_RR + ring(k))),
                                       reinterpret_cast<const float *>(slot(s, pg)),
                                       reinterpret_cast<float *>(slot(s, ro)), s.stream, gate_of(s, gated),
                                       c->fuse_f32 ? &ps : nullptr));
        } else {
            // r -= alpha Ap, r.r; x's update is deferred into the p update
            const PeerSum ps = c->fuse_combine ? peer_sum(c, s, pl, pg) : PeerSum{};
            HIPT(update_r_f64(s.nloc, reinterpret_cast<double *>(s.r), reinterpret_cast<const double *>(s.Ap),
                              reinterpret_cast<const double *>(slot(s, S_RR + ring(k))),
                              reinterpret_cast<const double *>(slot(s, pg)), reinterpret_cast<double *>(slot(s, ro)),
                              s.ws, s.stream, gate_of(s, gated), ts_of(c, s, TK_UR), c->fuse_combine ? &ps : nullptr));
        }
    }
    if (fuse_rr) TRY(local_barrier(c));  // MPI_Allreduce(r.r)  parallel_cg.c:313, summed by k_update_xp_f64
    else TRY(exchange_scalar(c, rl, rg));
    c->k = k + 1;
    c->total_iters += 1;
    if (gated) {  // x (+ p unless converged) on the device, stopping rule decided there
        for (auto &s : c->sh) {
            TRY(set_dev(s));
            if (f32ref(c)) {  // x is current; the p update decides the stop first
                const PeerSumF32 ps = fuse_rr ? peer_sum_f32(c, s, rl, rg) : PeerSumF32{};
                HIPT(update_p_ref_f32(s.nloc, reinterpret_cast<float *>(s.pown), reinterpret_cast<const float *>(s.r),
                                      reinterpret_cast<const float *>(slot(s, rg)),
                                      reinterpret_cast<const float *>(slot(s, S_RR + ring(k))), s.stream, eps, k,
                                      reinterpret_cast<int64_t *>(slot(s, S_KDONE)),
                                      reinterpret_cast<double *>(slot(s, S_RRFINAL)), rec_of(c, s, gated),
                                      fuse_rr ? &ps : nullptr));
                continue;
            }
            const PeerSum ps = fuse_rr ? peer_sum(c, s, rl, rg) : PeerSum{};
            HIPT(update_xp_f64(s.nloc, reinterpret_cast<double *>(s.x), reinterpret_cast<double *>(s.pown),
                               reinterpret_cast<const double *>(s.r),
                               reinterpret_cast<const double *>(slot(s, S_RR + ring(k))),
                               reinterpret_cast<const double *>(slot(s, pg)),
                               reinterpret_cast<const double *>(slot(s, rg)), s.stream, eps, k,
                               reinterpret_cast<int64_t *>(slot(s, S_KDONE)),
                               reinterpret_cast<double *>(slot(s, S_RRFINAL)), rec_of(c, s, gated),
                               ts_of(c, s, TK_UXP), fuse_rr ? &ps : nullptr));
        }
        phase_iter_end(c);
        return CGX_OK;
    }
    if (eps >= 0.0) {  // if (sqrt(beta) < EPSILON) break;  serialConjugate.c:235-238
        double rr = 0.0;
        TRY(read_scalar(c, rg, &rr));
        c->last_rr = rr;
        if (std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
            *stop = 1;
            if (!f32ref(c))  // the deferred x += alpha p, without the p update
                for (auto &s : c->sh) {
                    TRY(set_dev(s));
                    HIPT(update_xp_f64(s.nloc, reinterpret_cast<double *>(s.x), reinterpret_cast<double *>(s.pown),
                                       reinterpret_cast<const double *>(s.r),
                                       reinterpret_cast<const double *>(slot(s, S_RR + ring(k))),
                                       reinterpret_cast<const double *>(slot(s, pg)), nullptr, s.stream, -1.0, 0,
                                       nullptr, nullptr, nullptr, ts_of(c, s, TK_UXP)));
                }
            phase_iter_end(c);
            return CGX_OK;
        }
    }
    for (auto &s : c->sh) {  // p = r + (beta/rsold) p    serialConjugate.c:239-243
        TRY(set_dev(s));
        if (f32ref(c)) {
            const PeerSumF32 ps = fuse_rr ? peer_sum_f32(c, s, rl, rg) : PeerSumF32{};
            HIPT(update_p_ref_f32(s.nloc, reinterpret_cast<float *>(s.pown),
                                  reinterpret_cast<const float *>(s.r), reinterpret_cast<const float *>(slot(s, rg)),
                                  reinterpret_cast<const float *>(slot(s, S_RR + ring(k))), s.stream, -1.0, 0,
                                  nullptr, nullptr, nullptr, fuse_rr ? &ps : nullptr));
        } else {  // x += alpha p (deferred from the r update), then p = r + beta p
            const PeerSum ps = fuse_rr ? peer_sum(c, s, rl, rg) : PeerSum{};
            HIPT(update_xp_f64(s.nloc, reinterpret_cast<double *>(s.x), reinterpret_cast<double *>(s.pown),
                               reinterpret_cast<const double *>(s.r),
                               reinterpret_cast<const double *>(slot(s, S_RR + ring(k))),
                               reinterpret_cast<const double *>(slot(s, pg)),
                               reinterpret_cast<const double *>(slot(s, rg)), s.stream, -1.0, 0, nullptr, nullptr,
                               nullptr, ts_of(c, s, TK_UXP), fuse_rr ? &ps : nullptr));
        }
    }
    phase_iter_end(c);
    return CGX_OK;
}

// The first launch of each kernel in a process costs the HIP runtime several
// microseconds more than later launches (rocprofv3 --hip-trace of a fresh
// process's first solve: 9-14 us against 6-7 us per hipLaunchKernel), about
// 20 us over a small system's first solve -- the only solve `cg_hip` runs.
// One GPU, small n: the context pays it at creation.  The solve's start runs
// for real on alloc_shard's zeroed x and b (A x with x = 0, whatever A holds:
// only r, p, Ap and the scalar slots are written), then two gated iterations
// whose kernels all return at once (the record holds -1: converged before
// any iteration, under both gate tests) and one record of each lookahead
// event; the written buffers and the host
// state then go back to what alloc_shard left.  CGX_WARM=0: no warm-up.
constexpr int64_t kWarmMaxN = 16384;
bool warm_eligible(const cgx_ctx *c) {
    if (c->mode != M_SINGLE || c->op != OP_DENSE || c->n > kWarmMaxN) return false;
    if (c->flags & (CGX_TIMING | CGX_PHASES | CGX_HOST_STREAM | CGX_SYMMETRIC)) return false;
    const char *e = std::getenv("CGX_WARM");
    return !(e && *e == '0');
}

int warm_solve_kernels(cgx_ctx *c) {
    Shard &s = c->sh[0];
    TRY(set_dev(s));
    TRY(do_begin(c));
    int64_t *pin = reinterpret_cast<int64_t *>(s.h_pin);
    pin[0] = -1;
    HIPT(hipMemcpyAsync(slot(s, S_KDONE), pin, 8, hipMemcpyHostToDevice, s.stream));
    int stop = 0;
    for (int i = 0; i < 2; ++i) TRY(do_iteration(c, 0.0, &stop, /*gated=*/true));
    for (auto &e : s.ev_look) HIPT(hipEventRecord(e, s.stream));  // the gated loop's events: first records too
    const size_t es = (size_t)c->es;
    HIPT(hipMemsetAsync(s.r, 0, (c->fold_p ? c->lda : s.nloc) * es, s.stream));
    HIPT(hipMemsetAsync(s.Ap, 0, s.nloc * es, s.stream));
    HIPT(hipMemsetAsync(s.pfull, 0, c->lda * es, s.stream));
    if (s.p_alt) HIPT(hipMemsetAsync(s.p_alt, 0, c->lda * es, s.stream));
    HIPT(hipMemsetAsync(s.scal, 0, kScalSlots * 8, s.stream));
    HIPT(hipStreamSynchronize(s.stream));
    s.x_zero = true;
    s.h_rec[0] = s.h_rec[1] = 0;
    c->state = ST_IDLE;
    c->k = c->xd_k0 = c->total_iters = 0;
    c->converged = 0;
    c->last_rr = 0.0;
    c->rr_unsummed = c->x_incomplete = c->x_deferred = c->xalpha_pending = c->iter_failed = false;
    return CGX_OK;
}

}  // namespace cgxh

extern "C" {

int cgx_solve_begin(cgx_ctx *c) {
    const Range range_("cgx_solve_begin");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    return do_begin(c);
}

// Convergence-tested iterations without a host round trip per iteration:
// the update kernel decides sqrt(r.r) < eps on the device and records k+1;
// queued later iterations skip themselves.  The host keeps `look` iterations
// in flight and reads the record of an older iteration (pinned memory,
// event-ordered), so at most `look` no-op iterations are ever enqueued.
static int iterate_gated(cgx_ctx *c, int64_t count, double eps, int64_t *done, int *converged) {
    Shard &s0 = c->sh[0];
    // One GPU: one iteration ahead keeps the device fed (its iteration takes
    // longer than the host's enqueue) and enqueues one no-op iteration fewer
    // after the stop; several row blocks: two (the host's enqueue is the
    // longer one at 8 blocks).  profiles/r06_lookahead_ab.jsonl
    const char *la = std::getenv("CGX_LOOKAHEAD");
    const int look_def = c->mode == M_SINGLE ? 1 : 2;
    const int look = std::max(1, std::min(kLookRing - 1, (la && *la) ? std::atoi(la) : look_def));
    const int64_t k0 = c->k;
    int64_t issued = 0, kd = 0;
    volatile int64_t *rec = s0.h_rec;  // {kdone, r.r bits}, stored by the deciding kernel
    // One process (single GPU or row blocks on several): the record may also
    // be read as soon as it appears, without an event, so a GPU that runs
    // ahead of the host's launches (small N) stops the enqueueing after the
    // deciding iteration.  Never in rank mode, where every rank must enqueue
    // the same iterations (their collectives pair up).
    const bool early = c->mode != M_RCCL;
    for (; issued < count && kd == 0; ++issued) {
        if (early && rec[0] != 0) break;
        int stop = 0;
        TRY(do_iteration(c, eps, &stop, /*gated=*/true));
        TRY(set_dev(s0));
        const int64_t ev = issued;  // an event after every iteration
        HIPT(hipEventRecord(s0.ev_look[ev % kLookRing], s0.stream));
        if (ev >= look) {
            TRY(rank_wait_event(c, s0.ev_look[(ev - look) % kLookRing], "an earlier iteration"));
            const int64_t synced = ev - look;  // the last iteration that event covers
            // Only a record left by an iteration the event covers counts: the
            // host-mapped word may already show a later iteration's decision,
            // and acting on that would make the number of enqueued iterations
            // (and so of collectives) depend on timing, rank by rank.  The
            // record's k is the deciding launch's iteration index (dense: the
            // converged iteration + 1, Poisson: the next iteration), so
            // k <= the synced iteration means that launch is covered.
            const int64_t r = rec[0];
            if (r != 0 && r <= k0 + synced) kd = r;
        }
    }
    TRY(sync_all(c));
    const int64_t kdev = rec[0];
    const int64_t did = kdev ? (kdev - k0) : issued;
    c->total_iters += did - issued;  // do_iteration counted every enqueued one
    if (kdev) {
        const int64_t bits = rec[1];
        double rrf;
        std::memcpy(&rrf, &bits, 8);
        c->last_rr = rrf;
        c->k = kdev;
        c->converged = 1;
        c->state = ST_CONVERGED;
        // fused Poisson: the deciding k_poisson_p (iteration kdev) formed
        // r.r_kdev from the slabs' partials into its slot before it decided,
        // and the launches after it skip themselves: nothing is left unsummed
        c->rr_unsummed = false;
    } else {
        double rr = 0.0;
        TRY(settle_rr(c));
        TRY(read_scalar(c, S_RR + ring(c->k), &rr));
        c->last_rr = rr;
        // The fused Poisson iteration decides a stop one iteration later (at
        // the start of the next k_poisson_p); the last issued iteration's
        // r.r is tested here.  (The dense kernels already tested it.)
        if (c->fused && eps >= 0.0 && std::sqrt(rr) < eps) {
            c->converged = 1;
            c->state = ST_CONVERGED;
        }
    }
    TRY(poisson_x_finish(c));
    if (done) *done = did;
    if (converged) *converged = c->converged;
    return CGX_OK;
}

static int iterate_calls(cgx_ctx *c, int64_t count, double eps, int64_t *done, int *converged);

int cgx_iterate(cgx_ctx *c, int64_t count, double eps, int64_t *done, int *converged) {
    const Range range_("cgx_iterate");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    if (c->state == ST_IDLE) return fail(CGX_ERR_STATE, "cgx_iterate before cgx_solve_begin");
    if (c->iter_failed)
        return fail(CGX_ERR_STATE, "an earlier cgx_iterate failed part-way through iteration %lld: the solve "
                                   "cannot continue (cgx_solve_begin starts a new one)", (long long)c->k);
    TRY(check_x_complete(c));
    const int rc = iterate_calls(c, count, eps, done, converged);
    if (rc != CGX_OK) {
        // Part of an iteration may have run on some row blocks (or all of
        // r's update without x's): repeating it would apply it twice.  And
        // when x updates were left out (poisson_x_finish not reached), say so
        // at the next use of x instead of handing out an x with terms missing.
        c->iter_failed = true;
        c->x_incomplete = true;
        c->x_deferred = c->fused && c->xd > 1 && (c->k > c->xd_k0 || c->xalpha_pending);
    }
    return rc;
}

static int iterate_calls(cgx_ctx *c, int64_t count, double eps, int64_t *done, int *converged) {
    const char *gv = std::getenv("CGX_GATED");
    const bool gate_ok = !(gv && *gv == '0');
    c->xd_k0 = c->k;
    if (c->state == ST_BEGUN && count > 0 && eps >= 0.0 && !(c->flags & CGX_HOST_STREAM) && gate_ok)
        return iterate_gated(c, count, eps, done, converged);
    int64_t did = 0;
    while (did < count && c->state == ST_BEGUN) {
        int stop = 0;
        TRY(do_iteration(c, eps, &stop));
        TRY(progress_mark(c));
        ++did;
        if (stop) break;
    }
    TRY(settle_rr(c));
    TRY(poisson_x_finish(c));
    if (done) *done = did;
    if (converged) *converged = c->converged;
    return CGX_OK;
}

int cgx_solve(cgx_ctx *c, void *x_inout, double eps, int64_t max_iter, cgx_stats *st) {
    const Range range_("cgx_solve");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    if (x_inout) TRY(cgx_set_x(c, x_inout));
    TRY(sync_all(c));
    const auto t0 = std::chrono::steady_clock::now();
    TRY(do_begin(c));
    const int64_t cap = max_iter < 0 ? c->n : max_iter;  // for(k=0; k<ROWS; ++k)
    int64_t done = 0;
    int conv = 0;
    TRY(cgx_iterate(c, cap, eps, &done, &conv));
    TRY(sync_all(c));
    const auto t1 = std::chrono::steady_clock::now();
    c->solve_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (eps < 0.0 && c->k > 0) {
        double rr = 0.0;
        TRY(read_scalar(c, S_RR + ring(c->k), &rr));
        c->last_rr = rr;
    }
    if (x_inout) TRY(cgx_get_x(c, x_inout));
    if (st) TRY(cgx_get_stats(c, st));
    return CGX_OK;
}

int cgx_get_stats(cgx_ctx *c, cgx_stats *st) {
    if (!c || !st) return fail(CGX_ERR_ARG, "NULL argument");
    TRY(sync_all(c));
    TRY(timing_resolve(c));
    st->iterations = c->k;
    st->converged = c->converged;
    // fixed-count iterations read nothing back: the current r.r from its slot
    // (iterate_calls settled a folded Poisson r.r already)
    if (c->state == ST_BEGUN && c->k > 0 && !c->rr_unsummed) TRY(read_scalar(c, S_RR + ring(c->k), &c->last_rr));
    st->rr = c->last_rr;
    st->solve_ms = c->solve_ms;
    st->matvec_ms = c->matvec_ms;
    st->matvec_count = c->matvec_count;
    st->total_iterations = c->total_iters;
    return CGX_OK;
}

int cgx_reset_timing(cgx_ctx *c) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    TRY(sync_all(c));
    c->sh[0].ev_used = 0;
    if (c->sh[0].ts_used > 0) {  // drop the stamps recorded so far (warmup)
        TRY(set_dev(c->sh[0]));
        HIPT(hipMemsetAsync(c->sh[0].ts_dev, 0, (size_t)c->sh[0].ts_used * kTsKern * kTsSlot * 8, c->sh[0].stream));
        c->sh[0].ts_used = 0;
    }
    c->ts_prev_start = c->ts_prev_end = 0;
    for (auto &v : c->ph_samples) v.clear();
    c->matvec_ms = 0.0;
    c->matvec_count = 0;
    return CGX_OK;
}

int cgx_get_phase_times(cgx_ctx *c, cgx_phase_times *out) {
    if (!c || !out) return fail(CGX_ERR_ARG, "NULL argument");
    if (!(c->flags & CGX_PHASES)) return fail(CGX_ERR_STATE, "the context was created without CGX_PHASES");
    TRY(sync_all(c));
    TRY(phase_resolve(c));
    for (int q = 0; q < CGX_PH_COUNT; ++q) {
        std::vector<float> v = c->ph_samples[q];
        out->samples[q] = (int64_t)v.size();
        out->median_us[q] = out->mean_us[q] = 0.0;
        if (v.empty()) continue;
        double sum = 0.0;
        for (float t : v) sum += t;
        out->mean_us[q] = sum / (double)v.size();
        std::sort(v.begin(), v.end());
        const size_t h = v.size() / 2;
        out->median_us[q] = (v.size() & 1) ? v[h] : 0.5 * ((double)v[h - 1] + (double)v[h]);
    }
    return CGX_OK;
}

int cgx_synchronize(cgx_ctx *c) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    return sync_all(c);
}

void *cgx_stream(cgx_ctx *c) { return c ? (void *)c->sh[0].stream : nullptr; }

int cgx_set_matvec_plan(cgx_ctx *c, int rows_per_wave, int chunks_in_flight, int nontemporal, int blocks_per_cu) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    if (f32ref(c) || c->op != OP_DENSE || (c->flags & CGX_SYMMETRIC))
        return fail(CGX_ERR_ARG, "only the fp64 row-major dense matVec has a tunable plan");
    const int R = rows_per_wave, U = chunks_in_flight;
    if (R != 1 && R != 2 && R != 4 && R != 8) return fail(CGX_ERR_ARG, "rows_per_wave must be 1, 2, 4 or 8");
    if (U != 2 && U != 4 && U != 8) return fail(CGX_ERR_ARG, "chunks_in_flight must be 2, 4 or 8");
    if (nontemporal != 0 && nontemporal != 1 && nontemporal != 2 && nontemporal != 8)
        return fail(CGX_ERR_ARG, "load policy must be 0 (plain), 1 (non-temporal), 2 (pipelined) or 8 (pipelined "
                                 "non-temporal)");
    // The folded iteration keeps p_k in pfull / p_alt by the parity of k, and
    // the other forms keep it in pfull: switching forms inside a solve would
    // multiply a stale p.  A plan that turns the fold off waits for the next
    // cgx_solve_begin.
    if (R > 2 && c->fold_p && c->state == ST_BEGUN)
        return fail(CGX_ERR_STATE, "rows_per_wave %d turns the folded iteration off: not inside a solve "
                                   "(set the plan before cgx_solve_begin)", R);
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        MatvecPlan pl = plan_matvec_f64(s.dev, s.nloc, R, U, nontemporal, blocks_per_cu, c->lda);
        s.plan = pl;
        s.fold_plan = pl;  // the folded matVec follows the same rows per wave and grid (same p.Ap order)
    }
    if (R > 2) c->fold_p = false;  // the folded matVec has one or two rows per wave
    return CGX_OK;
}

int cgx_get_matvec_plan(cgx_ctx *c, int *rows_per_wave, int *chunks_in_flight, int *nontemporal, int *blocks) {
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    const MatvecPlan &pl = c->sh[0].plan;
    if (rows_per_wave) *rows_per_wave = pl.R;
    if (chunks_in_flight) *chunks_in_flight = pl.U;
    if (nontemporal) *nontemporal = pl.nt;
    if (blocks) *blocks = pl.blocks;
    return CGX_OK;
}

int cgx_residual_norm(cgx_ctx *c, double *rnorm, double *bnorm) {
    const Range range_("cgx_residual_norm");
    if (!c) return fail(CGX_ERR_ARG, "ctx is NULL");
    TRY(check_x_complete(c));
    // ||b - A x|| with the current x: allgather x, matVec, residual, two dots.
    TRY(settle_halo(c));
    TRY(exchange_allgather(c, /*from_x=*/true));
    const int tro = out_slot(c, S_LTR, S_TR), tbo = out_slot(c, S_LTB, S_TB);
    for (auto &s : c->sh) {
        TRY(set_dev(s));
        TRY(launch_matvec(c, s, s.pfull, false, 0));
        if (f32ref(c)) {
            HIPT(residual_ref_f32(s.nloc, reinterpret_cast<const float *>(s.b), reinterpret_cast<const float *>(s.Ap),
                                  reinterpret_cast<float *>(s.r), nullptr, s.stream));
            HIPT(dot_ref_f32(s.nloc, reinterpret_cast<const float *>(s.r), reinterpret_cast<const float *>(s.r),
                             reinterpret_cast<float *>(slot(s, tro)), s.stream));
            HIPT(dot_ref_f32(s.nloc, reinterpret_cast<const float *>(s.b), reinterpret_cast<const float *>(s.b),
                             reinterpret_cast<float *>(slot(s, tbo)), s.stream));
        } else {
            HIPT(residual_f64(s.nloc, reinterpret_cast<const double *>(s.b), reinterpret_cast<const double *>(s.Ap),
                              reinterpret_cast<double *>(s.r), nullptr, reinterpret_cast<double *>(slot(s, tro)), s.ws,
                              s.stream));
            HIPT(dot_f64(s.nloc, reinterpret_cast<const double *>(s.b), reinterpret_cast<const double *>(s.b),
                         reinterpret_cast<double *>(slot(s, tbo)), s.ws, s.stream));
        }
    }
    TRY(exchange_scalar(c, S_LTR, S_TR));
    TRY(exchange_scalar(c, S_LTB, S_TB));
    double rr = 0.0, bb = 0.0;
    TRY(read_scalar(c, S_TR, &rr));
    TRY(read_scalar(c, S_TB, &bb));
    if (rnorm) *rnorm = std::sqrt(rr);
    if (bnorm) *bnorm = std::sqrt(bb);
    c->state = ST_IDLE;  // r and p were overwritten
    return CGX_OK;
}

}  // extern "C"
