/*
 * cg_hip -- drop-in for the reference's solver programs, host code in C over
 * the libcgx C ABI (include/cgx.h).
 *
 *   serialConjugate.c  : cg_hip matrixA.txt vectorb.txt initialguess.txt
 *   parallel_cg.c      : cg_hip --gpus P matrixA.txt vectorb.txt initialguess.txt
 *   point-to-point_cg.c: cg_hip --gpus P --p2p matrixA.txt vectorb.txt initialguess.txt
 *                        (its exchange: every slice to block 0, then from block 0
 *                        to every block; the scalars summed in rank order)
 *
 * Same positional arguments (serialConjugate.c:48-52, 65-67), same text
 * formats, same stdout lines:
 *   "Computing cg of matrix size : <N*N>"             serialConjugate.c:58
 *   "average clock execution time in seconds: %f"     serialConjugate.c:250
 *   with --gpus > 1 additionally, as parallel_cg.c:123-126 / :334-335:
 *   "collective data distribution time in seconds: %f"  (--p2p: "p2p data
 *    distribution time in seconds: %f", point-to-point_cg.c:133)
 *   "cg method execution time in seconds: %f"
 *   "clock execution time in seconds: %f"
 * Same stopping rule: stop when sqrt(r.r) < EPSILON (1.0e-6,
 * serialConjugate.c:28, :235), at most N iterations (:213).
 *
 * Differences (documented in DESIGN.md s2): N is read at run time (count of
 * values in vectorb, or --dims dimensions.txt, or --n); errors exit non-zero
 * (the reference exits 0, serialConjugate.c:51,56); arithmetic is fp64 unless
 * --fp32-ref, which reproduces serialConjugate.c's float results bit for bit.
 *
 * Extra options: --eps E, --max-iter M, --print-x, --stats, --threads T (text
 * parsing), --spd N [--seed S] (on-device synthetic system instead of files),
 * --symmetric (fp64, one GPU: keep only A's upper-triangle tiles, half the
 * bytes per matVec; CG's A is symmetric by contract, the lower triangle
 * outside the diagonal tiles is not read).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "cgx.h"
#include "cgx_textio.h"

#define EPSILON_DEFAULT 1.0e-6 /* serialConjugate.c:28 */

/* The matrix buffer: anonymous memory 2 MiB-aligned with transparent huge
 * pages requested (CGX_CLI_HUGEPAGES=0: plain malloc).  The parse threads
 * fault it in 512x fewer pages, and releasing it is one short munmap
 * instead of freeing 4-KiB pages one by one (~30 ms for 268 MB). */
typedef struct {
    void *p;     /* aligned start */
    void *base;  /* mapping (or malloc block) */
    size_t len;  /* mapping length; 0 = malloc */
} big_buf;

static int big_alloc(big_buf *bb, size_t bytes) {
    const size_t huge = (size_t)2 << 20;
    const char *e = getenv("CGX_CLI_HUGEPAGES");
    memset(bb, 0, sizeof *bb);
    if (bytes >= huge && !(e && !strcmp(e, "0"))) {
        const size_t len = bytes + huge;
        void *m = mmap(NULL, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m != MAP_FAILED) {
            uintptr_t a = ((uintptr_t)m + huge - 1) & ~(uintptr_t)(huge - 1);
            (void)madvise((void *)a, bytes, MADV_HUGEPAGE);
            bb->p = (void *)a;
            bb->base = m;
            bb->len = len;
            return 0;
        }
    }
    bb->p = bb->base = malloc(bytes ? bytes : 1);
    return bb->p ? 0 : -1;
}

static void big_free(big_buf *bb) {
    if (bb->len) munmap(bb->base, bb->len);
    else free(bb->base);
    memset(bb, 0, sizeof *bb);
}

/* Buffers released on a helper thread, off the critical path: the matrix
 * (or the ring A streamed through) and the mapping of A's text file.  Two
 * munmaps of a GiB or more serialise on the process's mm lock with anything
 * else that maps memory (the b and x0 reads), so this starts after them. */
typedef struct {
    big_buf buf;
    cgx_text *text;
} release_job;

static void *release_buf(void *arg) {
    release_job *r = (release_job *)arg;
    cgx_text_close(r->text);
    big_free(&r->buf);
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void usage(const char *prog) {
    fprintf(stderr,
            "usage: %s [--gpus P [--p2p]] [--fp32-ref | --symmetric] [--eps E] [--max-iter M] [--dims FILE] [--n N]\n"
            "          [--threads T] [--print-x] [--stats] matrixA vectorb initialguess\n"
            "       %s --spd N [--seed S] [--gpus P] [--eps E] [--max-iter M] [--stats]\n",
            prog, prog);
}

static int die_cgx(int rc, const char *what) {
    fprintf(stderr, "%s failed: %s (%s)\n", what, cgx_strerror(rc), cgx_last_error());
    return 1;
}

static int read_file(const char *path, int64_t count, int as_float, void *out, int threads) {
    int rc = cgx_text_read(path, count, as_float, out, threads);
    if (rc == -1) {
        printf("Could not open file\n"); /* serialConjugate.c:103 */
        fprintf(stderr, "%s: cannot open\n", path);
    } else if (rc == -2) {
        fprintf(stderr, "%s: fewer than %lld numbers\n", path, (long long)count);
    } else if (rc != 0) {
        fprintf(stderr, "%s: malformed number\n", path);
    }
    return rc;
}

/* Context creation (HIP runtime start, device buffers) runs on its own thread
 * while the text files are parsed: the two are independent until the H2D. */
typedef struct {
    int64_t n;
    int gpus, flags, rc;
    cgx_ctx *ctx;
    double t_rt, t_done;  /* when the HIP runtime was up / creation finished (now_s) */
} create_job;

static void *create_ctx(void *arg) {
    create_job *j = (create_job *)arg;
    int ndev0 = 0;
    cgx_device_count(&ndev0); /* starts the HIP runtime */
    j->t_rt = now_s();
    if (j->gpus == 1) {
        j->rc = cgx_create(&j->ctx, j->n, 0, j->flags);
    } else {
        int devs[32];
        int ndev = 0;
        cgx_device_count(&ndev);
        for (int g = 0; g < j->gpus; ++g) devs[g] = ndev > 0 ? g % ndev : 0;
        j->rc = cgx_create_multi(&j->ctx, j->n, j->gpus, devs, j->flags);
    }
    j->t_done = now_s();
    return NULL;
}

/* A streamed to the GPU row block by row block (parallel_cg.c's MPI_Scatter,
 * :112-113, one block at a time): the main thread parses block k+1 from the
 * indexed file while a copy thread sends block k with cgx_set_rows, through
 * a ring of block buffers, so host memory holds at most CGX_CLI_RING_MB
 * (default 1024) of A and, once the context is up, the H2D runs under the
 * parse.  The ring is one buffer: when the copy thread finds several parsed
 * blocks waiting (the HIP runtime came up after them) it sends the run of
 * them that is contiguous in the ring with one cgx_set_rows, since pageable
 * H2D copies run at ~5 GB/s per 32 MB call and ~20 GB/s per 256 MB call.
 * Blocks are CGX_CLI_BLOCK_MB (default 128) of A.
 * (CGX_CLI_STREAM=0: parse all of A, then one cgx_set_system.) */
typedef struct {
    cgx_text *text;
    int64_t n, block_rows, nblocks;
    int nslots, as_float, threads;
    size_t es;
    big_buf ring;         /* nslots slots of block_rows * n values (huge pages) */
    size_t slot_bytes;
    int *filled;          /* slot holds block filled[s] - 1 (0 = free) */
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int abort_rc;         /* the copy side failed: the parse stops */
    pthread_t creator;    /* joined by the copy thread */
    int creator_threaded;
    create_job *job;
    int rc;               /* first cgx_set_rows failure */
    double t_last_h2d;
} a_stream;

static void *stream_copy(void *arg) {
    a_stream *st = (a_stream *)arg;
    if (st->creator_threaded) pthread_join(st->creator, NULL);
    int rc = st->job->rc;
    for (int64_t k = 0; k < st->nblocks && rc == CGX_OK;) {
        const int sl = (int)(k % st->nslots);
        pthread_mutex_lock(&st->mu);
        while (st->filled[sl] != k + 1 && !st->abort_rc) pthread_cond_wait(&st->cv, &st->mu);
        int64_t run = 1; /* parsed blocks k, k+1, ... in consecutive slots */
        while (k + run < st->nblocks && sl + run < st->nslots && st->filled[sl + run] == k + run + 1) ++run;
        const int stop = st->abort_rc;
        pthread_mutex_unlock(&st->mu);
        if (stop) break;
        const int64_t row0 = k * st->block_rows, end = (k + run) * st->block_rows < st->n ? (k + run) * st->block_rows : st->n;
        rc = cgx_set_rows(st->job->ctx, row0, end - row0, (char *)st->ring.p + (size_t)sl * st->slot_bytes, st->n,
                          NULL, NULL);
        pthread_mutex_lock(&st->mu);
        for (int64_t q = 0; q < run; ++q) st->filled[sl + q] = 0;
        pthread_cond_broadcast(&st->cv);
        pthread_mutex_unlock(&st->mu);
        k += run;
    }
    st->t_last_h2d = now_s();
    pthread_mutex_lock(&st->mu);
    st->rc = rc;
    if (rc != CGX_OK && !st->abort_rc) st->abort_rc = 1;
    pthread_cond_broadcast(&st->cv);
    pthread_mutex_unlock(&st->mu);
    return NULL;
}

/* The parse side (main thread).  Returns 0, or the text reader's error. */
static int stream_parse(a_stream *st) {
    for (int64_t k = 0; k < st->nblocks; ++k) {
        const int sl = (int)(k % st->nslots);
        pthread_mutex_lock(&st->mu);
        while (st->filled[sl] != 0 && !st->abort_rc) pthread_cond_wait(&st->cv, &st->mu);
        const int stop = st->abort_rc;
        pthread_mutex_unlock(&st->mu);
        if (stop) return 0; /* the copy side reports its own error */
        const int64_t row0 = k * st->block_rows, rows = row0 + st->block_rows <= st->n ? st->block_rows : st->n - row0;
        const int rc = cgx_text_read_range(st->text, row0 * st->n, rows * st->n, st->as_float,
                                           (char *)st->ring.p + (size_t)sl * st->slot_bytes, st->threads);
        pthread_mutex_lock(&st->mu);
        if (rc != 0) st->abort_rc = 1;
        else st->filled[sl] = (int)(k + 1);
        pthread_cond_broadcast(&st->cv);
        pthread_mutex_unlock(&st->mu);
        if (rc != 0) return rc;
    }
    return 0;
}

/* Whole-string numeric option values: "--eps abc" or "--gpus 2x" is an
 * error (exit 2), not a silent 0. */
static int opt_ll(const char *name, const char *v, long long *out) {
    char *end = NULL;
    errno = 0;
    const long long x = strtoll(v, &end, 10);
    if (!*v || *end || errno) { fprintf(stderr, "%s: not an integer: '%s'\n", name, v); return 0; }
    *out = x;
    return 1;
}
static int opt_double(const char *name, const char *v, double *out) {
    char *end = NULL;
    errno = 0;
    const double x = strtod(v, &end);
    if (!*v || *end || errno) { fprintf(stderr, "%s: not a number: '%s'\n", name, v); return 0; }
    *out = x;
    return 1;
}

int main(int argc, char **argv) {
    const double t_prog0 = now_s();
    int gpus = 1, fp32ref = 0, symmetric = 0, print_x = 0, stats = 0, p2p = 0;
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    int threads = (int)(ncpu < 1 ? 1 : (ncpu > 16 ? 16 : ncpu)); /* text parsing threads */
    double eps = EPSILON_DEFAULT;
    long long max_iter = -1, n_opt = -1, spd_n = -1;
    unsigned long long seed = 42;
    const char *dims_path = NULL;
    const char *pos[3];
    int npos = 0;

    long long v = 0;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        int has_val = (i + 1 < argc);
        if (!strcmp(a, "--gpus") && has_val) {
            if (!opt_ll(a, argv[++i], &v)) return 2;
            gpus = (v < 0 || v > 1000) ? -1 : (int)v;
        } else if (!strcmp(a, "--fp32-ref")) fp32ref = 1;
        else if (!strcmp(a, "--symmetric")) symmetric = 1;
        else if (!strcmp(a, "--p2p")) p2p = 1;
        else if (!strcmp(a, "--eps") && has_val) {
            if (!opt_double(a, argv[++i], &eps)) return 2;
        } else if (!strcmp(a, "--max-iter") && has_val) {
            if (!opt_ll(a, argv[++i], &max_iter)) return 2;
        } else if (!strcmp(a, "--dims") && has_val) dims_path = argv[++i];
        else if (!strcmp(a, "--n") && has_val) {
            if (!opt_ll(a, argv[++i], &n_opt)) return 2;
        } else if (!strcmp(a, "--threads") && has_val) {
            if (!opt_ll(a, argv[++i], &v)) return 2;
            threads = v < 1 ? 1 : (v > 256 ? 256 : (int)v);
        } else if (!strcmp(a, "--spd") && has_val) {
            if (!opt_ll(a, argv[++i], &spd_n)) return 2;
        } else if (!strcmp(a, "--seed") && has_val) {
            if (!opt_ll(a, argv[++i], &v)) return 2;
            seed = (unsigned long long)v;
        } else if (!strcmp(a, "--print-x")) print_x = 1;
        else if (!strcmp(a, "--stats")) stats = 1;
        else if (!strcmp(a, "-h") || !strcmp(a, "--help")) { usage(argv[0]); return 0; }
        else if (a[0] == '-' && a[1] == '-') { usage(argv[0]); return 2; }
        else if (npos < 3) pos[npos++] = a;
        else npos = 4;
    }
    if (spd_n < 0 && npos != 3) {
        printf("serialCongugate.c requires four (4) files \n"); /* serialConjugate.c:50 */
        usage(argv[0]);
        return 1;
    }
    if (gpus < 1) { fprintf(stderr, "--gpus must be >= 1\n"); return 2; }
    if (gpus > 32) { fprintf(stderr, "--gpus must be <= 32\n"); return 2; }
    if (p2p && symmetric) {
        fprintf(stderr, "--p2p is an exchange of several row blocks (--symmetric is one GPU)\n");
        return 2;
    }
    if (symmetric && (fp32ref || gpus != 1)) {
        fprintf(stderr, "--symmetric is fp64 on one GPU (no --fp32-ref, --gpus 1)\n");
        return 2;
    }

    /* ---- N ---------------------------------------------------------------- */
    int64_t n = 0;
    if (spd_n > 0) n = spd_n;
    else if (n_opt > 0) n = n_opt;
    else if (dims_path) {
        int64_t d[4];
        if (cgx_text_dims(dims_path, d) != 0) { fprintf(stderr, "%s: cannot read dimensions\n", dims_path); return 1; }
        if (d[0] != d[1]) { printf("%lld and %lld must be same size\n", (long long)d[0], (long long)d[1]); return 1; }
        if (d[2] != d[0] || d[3] != 1) { fprintf(stderr, "%s: b must be %lld x 1\n", dims_path, (long long)d[0]); return 1; }
        n = d[0];
    } else {
        n = cgx_text_count(pos[1]);
        if (n < 0) { printf("Could not open file\n"); fprintf(stderr, "%s: cannot open\n", pos[1]); return 1; }
    }
    if (n < 1) { fprintf(stderr, "empty system\n"); return 1; }
    if (n % gpus != 0) { printf("%lld is not divisible by %d\n", (long long)n, gpus); return 1; } /* parallel_cg.c:88 */

    printf("Computing cg of matrix size : %lld\n", (long long)n * (long long)n); /* serialConjugate.c:58 */
    fflush(stdout);

    const int flags = (fp32ref ? CGX_F32_REF : (CGX_F64 | (symmetric ? CGX_SYMMETRIC : 0))) | (p2p ? CGX_COMM_P2P : 0);
    const size_t es = fp32ref ? 4 : 8;
    void *x = malloc((size_t)n * es);
    void *A = NULL, *b = NULL;
    /* static: the release thread may still read it while an error path
     * returns from main */
    static release_job rel = {{NULL, NULL, 0}, NULL};
    big_buf Abuf = {NULL, NULL, 0};
    pthread_t freer;
    int freeing = 0;
    /* A's buffers are released on a helper thread AFTER the solve.  Two
     * munmaps of a GiB or more hold the process's mm lock, and a solve that
     * enqueues while they run waits on it: with several row blocks (host-bound:
     * one thread enqueues every block's launches, records and waits) `cg_hip
     * --gpus P --fp32-ref` at N = 4096 / 8192 measured 1-24 ms per solve
     * against 0.7-3.9 ms in a process with nothing to release
     * (profiles/r06_published_mpi_sizes_before.json, r06_multi_solve_latency.jsonl);
     * on one GPU 0.23-0.25 against 0.19-0.20 ms at N = 1024 and 0.33-0.36
     * against 0.30-0.31 at 2048, the same at 4096 / 8192
     * (profiles/r06_cli_release_ab.jsonl).  CGX_CLI_RELEASE=during keeps the
     * release beside the solve (it then overlaps the solve instead of the
     * process's exit). */
    const char *re = getenv("CGX_CLI_RELEASE");
    const int defer_release = !(re && !strcmp(re, "during"));
    const char *se = getenv("CGX_CLI_STREAM");
    const int stream_a = spd_n <= 0 && !(se && !strcmp(se, "0"));
    if (!x) { fprintf(stderr, "can't allocate memory for vector\n"); return 1; }
    if (spd_n > 0) {
        memset(x, 0, (size_t)n * es);
    } else if (stream_a) {
        b = malloc((size_t)n * es);
        if (!b) { fprintf(stderr, "can't allocate memory for vector\n"); return 1; }
    } else {
        /* initialize(A), initialize(b), initialize(x0): serialConjugate.c:65-67 */
        if (big_alloc(&Abuf, (size_t)n * (size_t)n * es) != 0) A = NULL;
        else A = Abuf.p;
        b = malloc((size_t)n * es);
        if (!A || !b) { fprintf(stderr, "can't allocate memory for vector\n"); return 1; }
    }
    create_job job = {n, gpus, flags, CGX_OK, NULL, 0.0, 0.0};
    const double t_start = now_s();
    pthread_t creator;
    const int threaded = pthread_create(&creator, NULL, create_ctx, &job) == 0;
    if (!threaded) create_ctx(&job);
    int read_rc = 0, stream_rc = CGX_OK;
    double t_parsed = 0.0, t_h2d = 0.0;
    if (stream_a) {
        /* A: indexed once, then parsed and sent row block by row block */
        a_stream st;
        memset(&st, 0, sizeof st);
        const int orc = cgx_text_open(pos[0], threads, &st.text);
        int stopped = 0;
        const int64_t have = orc == 0 ? cgx_text_available(st.text, &stopped) : -1;
        if (orc != 0) {
            printf("Could not open file\n"); /* serialConjugate.c:103 */
            fprintf(stderr, "%s: cannot open\n", pos[0]);
            read_rc = -1;
        } else if (have < n * n) {
            fprintf(stderr, stopped ? "%s: malformed number\n" : "%s: fewer than %lld numbers\n", pos[0],
                    (long long)(n * n));
            read_rc = stopped ? -3 : -2;
        }
        if (!read_rc) {
            const char *rm = getenv("CGX_CLI_RING_MB"), *bm = getenv("CGX_CLI_BLOCK_MB");
            const double ring_mb = (rm && atof(rm) > 0) ? atof(rm) : 1024.0;
            const size_t row_bytes = (size_t)n * es;
            const size_t block_bytes = (size_t)(((bm && atof(bm) > 0) ? atof(bm) : 128.0) * 1048576.0);
            st.n = n;
            st.es = es;
            st.block_rows = (int64_t)(block_bytes / row_bytes) > 0 ? (int64_t)(block_bytes / row_bytes) : 1;
            if (st.block_rows > n) st.block_rows = n;
            st.nblocks = (n + st.block_rows - 1) / st.block_rows;
            int64_t slots = (int64_t)(ring_mb * 1048576.0 / ((double)st.block_rows * (double)row_bytes));
            if (slots < 2) slots = 2;
            if (slots > st.nblocks) slots = st.nblocks;
            st.nslots = (int)slots;
            st.as_float = fp32ref;
            st.threads = threads;
            st.slot_bytes = (size_t)st.block_rows * row_bytes;
            st.filled = calloc((size_t)st.nslots, sizeof(int));
            if (!st.filled || big_alloc(&st.ring, (size_t)st.nslots * st.slot_bytes) != 0) {
                fprintf(stderr, "can't allocate memory for vector\n");
                return 1;
            }
            pthread_mutex_init(&st.mu, NULL);
            pthread_cond_init(&st.cv, NULL);
            st.creator = creator;
            st.creator_threaded = threaded;
            st.job = &job;
            pthread_t copier;
            const int copy_threaded = pthread_create(&copier, NULL, stream_copy, &st) == 0;
            if (copy_threaded) {
                const int prc = stream_parse(&st);
                if (prc) {
                    fprintf(stderr, prc == -2 ? "%s: fewer than %lld numbers\n" : "%s: malformed number\n", pos[0],
                            (long long)(n * n));
                    read_rc = prc;
                }
                t_parsed = now_s();
                pthread_join(copier, NULL); /* also joined the creator */
                stream_rc = st.rc;
            } else {
                read_rc = -1;
                if (threaded) pthread_join(creator, NULL);
            }
            t_h2d = st.t_last_h2d;
            rel.buf = st.ring;  /* released after the b and x0 reads */
            free(st.filled);
        } else if (threaded) {
            pthread_join(creator, NULL);
        }
        if (!read_rc) read_rc = read_file(pos[1], n, fp32ref, b, threads) || read_file(pos[2], n, fp32ref, x, 1);
        rel.text = st.text;
        if (!defer_release) {
            if (pthread_create(&freer, NULL, release_buf, &rel) == 0) freeing = 1;
            else release_buf(&rel);
        }
    } else {
        read_rc = spd_n > 0 ? 0
                            : (read_file(pos[0], n * n, fp32ref, A, threads) ||
                               read_file(pos[1], n, fp32ref, b, threads) || read_file(pos[2], n, fp32ref, x, 1));
        t_parsed = now_s();
        if (threaded) pthread_join(creator, NULL);  /* before any exit: HIP may be starting up on it */
    }
    const double t_read = now_s();
    if (read_rc) {
        if (job.ctx) cgx_destroy(job.ctx);
        return 1;
    }
    cgx_ctx *ctx = job.ctx;
    int rc = job.rc;
    if (rc != CGX_OK) return die_cgx(rc, "cgx_create");
    if (stream_rc != CGX_OK) return die_cgx(stream_rc, "cgx_set_rows");

    double t_dist0 = stream_a ? t_parsed : now_s(), t_dist1;
    if (spd_n > 0) {
        rc = cgx_generate_spd(ctx, seed);
        t_dist1 = now_s();
        if (rc != CGX_OK) return die_cgx(rc, "cgx_generate_spd");
    } else if (stream_a) {
        /* A is on the device; b and x0 (MPI_Bcast / MPI_Scatter of the vectors) */
        rc = cgx_set_rows(ctx, 0, n, NULL, n, b, x);
        t_dist1 = now_s();
        free(b);
        if (rc != CGX_OK) return die_cgx(rc, "cgx_set_rows");
    } else {
        /* MPI_Bcast(x0) + MPI_Scatter(A, b): parallel_cg.c:109-117 */
        rc = cgx_set_system(ctx, A, b, x);
        t_dist1 = now_s();
        /* A is no longer needed: release it on a helper thread while the
         * solve runs (unmapping 268 MB took 16-30 ms on the critical path) */
        rel.buf = Abuf;
        if (!defer_release) {
            if (pthread_create(&freer, NULL, release_buf, &rel) == 0) freeing = 1;
            else release_buf(&rel);
        }
        free(b);
        if (rc != CGX_OK) return die_cgx(rc, "cgx_set_system");
    }

    const double t_freed = now_s();
    cgx_stats st;
    const double t_solve0 = now_s();
    rc = cgx_solve(ctx, NULL, eps, max_iter, &st);
    const double t_solve1 = now_s();
    if (rc != CGX_OK) return die_cgx(rc, "cgx_solve");
    rc = cgx_get_x(ctx, x);
    if (rc != CGX_OK) return die_cgx(rc, "cgx_get_x");
    const double t_x = now_s();
    if (defer_release) {
        if (pthread_create(&freer, NULL, release_buf, &rel) == 0) freeing = 1;
        else release_buf(&rel);
    }

    if (gpus > 1) {
        printf("cg method execution time in seconds: %f\n", st.solve_ms / 1e3);
        printf("%s data distribution time in seconds: %f\n", p2p ? "p2p" : "collective", t_dist1 - t_dist0);
        printf("clock execution time in seconds: %f\n", now_s() - t_prog0);
    } else {
        printf("average clock execution time in seconds: %f\n", st.solve_ms / 1e3);
    }
    if (stats)
        printf("iterations: %lld converged: %d residual_norm: %.6e\n", (long long)st.iterations, st.converged,
               st.rr >= 0 ? __builtin_sqrt(st.rr) : -1.0);
    if (print_x) {
        for (int64_t i = 0; i < n; ++i) {
            if (fp32ref) printf("%.9g\n", (double)((float *)x)[i]);
            else printf("%.17g\n", ((double *)x)[i]);
        }
    }
    fflush(stdout);
    const double t_printed = now_s();
    const char *fx = getenv("CGX_CLI_FAST_EXIT");
    const int fast_exit = !(fx && !strcmp(fx, "0"));
    if (!fast_exit) {
        if (freeing) pthread_join(freer, NULL);
        free(x);
        cgx_destroy(ctx);
    }
    if (getenv("CGX_CLI_TIMES")) /* phase breakdown, seconds since program start */
        fprintf(stderr,
                "{\"setup_s\": %.6f, \"read_s\": %.6f, \"hip_runtime_s\": %.6f, \"create_s\": %.6f, \"distribute_s\": %.6f, "
                "\"solve_s\": %.6f, \"to_x_s\": %.6f, \"printed_s\": %.6f, \"teardown_s\": %.6f, \"fast_exit\": %d, "
                "\"dist_start_s\": %.6f, \"solve_call_s\": %.6f, \"free_s\": %.6f, \"get_x_s\": %.6f, "
                "\"streamed\": %d, \"a_parsed_s\": %.6f, \"a_on_device_s\": %.6f}\n",
                t_start - t_prog0, t_read - t_start, job.t_rt - t_start, job.t_done - t_start, t_dist1 - t_dist0, st.solve_ms / 1e3,
                t_x - t_prog0, t_printed - t_prog0, now_s() - t_printed, fast_exit, t_dist0 - t_start, t_solve1 - t_solve0, t_freed - t_dist1, t_x - t_solve1,
                stream_a, t_parsed > 0 ? t_parsed - t_start : 0.0, t_h2d > 0 ? t_h2d - t_start : 0.0);
    if (fast_exit) {
        /* Every result is written and flushed.  The process ends here without
         * freeing the device/pinned buffers or running the HIP runtime's exit
         * teardown: the kernel driver reclaims both at process exit.  Flush
         * to exit: 29 ms against 71 ms with the teardown at N=8192
         * (CGX_CLI_FAST_EXIT=0 keeps it). */
        fflush(stderr);
        _exit(0);
    }
    return 0;
}
