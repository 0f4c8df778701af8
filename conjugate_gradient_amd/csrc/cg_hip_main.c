/*
 * cg_hip -- drop-in for the reference's solver programs, host code in C over
 * the libcgx C ABI (include/cgx.h).
 *
 *   serialConjugate.c  : cg_hip matrixA.txt vectorb.txt initialguess.txt
 *   parallel_cg.c      : cg_hip --gpus P matrixA.txt vectorb.txt initialguess.txt
 *
 * Same positional arguments (serialConjugate.c:48-52, 65-67), same text
 * formats, same stdout lines:
 *   "Computing cg of matrix size : <N*N>"             serialConjugate.c:58
 *   "average clock execution time in seconds: %f"     serialConjugate.c:250
 *   with --gpus > 1 additionally, as parallel_cg.c:123-126 / :334-335:
 *   "collective data distribution time in seconds: %f"
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

static void *release_buf(void *arg) {
    big_free((big_buf *)arg);
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void usage(const char *prog) {
    fprintf(stderr,
            "usage: %s [--gpus P] [--fp32-ref | --symmetric] [--eps E] [--max-iter M] [--dims FILE] [--n N]\n"
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
    int gpus = 1, fp32ref = 0, symmetric = 0, print_x = 0, stats = 0;
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

    const int flags = fp32ref ? CGX_F32_REF : (CGX_F64 | (symmetric ? CGX_SYMMETRIC : 0));
    const size_t es = fp32ref ? 4 : 8;
    void *x = malloc((size_t)n * es);
    void *A = NULL, *b = NULL;
    big_buf Abuf = {NULL, NULL, 0};
    pthread_t freer;
    int freeing = 0;
    if (!x) { fprintf(stderr, "can't allocate memory for vector\n"); return 1; }
    if (spd_n > 0) {
        memset(x, 0, (size_t)n * es);
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
    const int read_rc = spd_n > 0 ? 0
                        : (read_file(pos[0], n * n, fp32ref, A, threads) ||
                           read_file(pos[1], n, fp32ref, b, threads) || read_file(pos[2], n, fp32ref, x, 1));
    const double t_read = now_s();
    if (threaded) pthread_join(creator, NULL);  /* before any exit: HIP may be starting up on it */
    if (read_rc) {
        if (job.ctx) cgx_destroy(job.ctx);
        return 1;
    }
    cgx_ctx *ctx = job.ctx;
    int rc = job.rc;
    if (rc != CGX_OK) return die_cgx(rc, "cgx_create");

    double t_dist0 = now_s(), t_dist1;
    if (spd_n > 0) {
        rc = cgx_generate_spd(ctx, seed);
        t_dist1 = now_s();
        if (rc != CGX_OK) return die_cgx(rc, "cgx_generate_spd");
    } else {
        /* MPI_Bcast(x0) + MPI_Scatter(A, b): parallel_cg.c:109-117 */
        rc = cgx_set_system(ctx, A, b, x);
        t_dist1 = now_s();
        /* A is no longer needed: release it on a helper thread while the
         * solve runs (unmapping 268 MB took 16-30 ms on the critical path) */
        if (pthread_create(&freer, NULL, release_buf, &Abuf) == 0) freeing = 1;
        else big_free(&Abuf);
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

    if (gpus > 1) {
        printf("cg method execution time in seconds: %f\n", st.solve_ms / 1e3);
        printf("collective data distribution time in seconds: %f\n", t_dist1 - t_dist0);
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
                "\"dist_start_s\": %.6f, \"solve_call_s\": %.6f, \"free_s\": %.6f, \"get_x_s\": %.6f}\n",
                t_start - t_prog0, t_read - t_start, job.t_rt - t_start, job.t_done - t_start, t_dist1 - t_dist0, st.solve_ms / 1e3,
                t_x - t_prog0, t_printed - t_prog0, now_s() - t_printed, fast_exit, t_dist0 - t_start, t_solve1 - t_solve0, t_freed - t_dist1, t_x - t_solve1);
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
