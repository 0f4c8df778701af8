/* cg_mpi: the drop-in for `mpiexec -np P ./parallel_cg A.txt b.txt x0.txt`
 * (and, with --p2p, for point-to-point_cg), one process per GPU.
 *
 * MPI is the launcher and the bootstrap only: rank 0 makes the RCCL unique
 * id and MPI_Bcast hands it out; every per-iteration
 * exchange is RCCL inside libcgx (cgx_create_rank).  What parallel_cg.c
 * does with MPI and what this does instead:
 *   - rank 0 reads all of A, b, x0 with initialize() (parallel_cg.c:104-107)
 *     -> every rank indexes the text files and parses only its own rows
 *        (cgx_text_read_range), so the parse runs on all ranks at once;
 *   - MPI_Bcast(x0) + MPI_Scatter(A, b) (:109-115) -> cgx_set_rows with the
 *     rank's rows (the full x0 for the first A x0 is allgathered on the GPUs);
 *   - conjugrad's MPI_Allgather / MPI_Allreduce (:283-323) -> cgx_solve.
 * Same output lines from rank 0 (:334, :123-126), the CG time bracketed by
 * barriers on every rank as conjugrad does (:278-279, :328-329); with --p2p
 * point-to-point_cg.c's contract instead: its lines (:493, :133-135, the
 * distribution bracket taking in the reads of A and b as scatterRow's does,
 * :119-127) and its error texts (:101, :226).  With --fp32-ref the x is
 * parallel_cg.c's (point-to-point_cg.c's with --p2p) bit for bit.
 *
 *   mpiexec -np P cg_mpi [--fp32-ref] [--p2p] [--eps E] [--max-iter M]
 *                        [--dims FILE | --n N] [--threads T] [--print-x]
 *                        [--stats] matrixA vectorb initialguess
 * Device: the rank's index among the ranks on its node, modulo the visible
 * GPUs (CGX_DEVICE overrides). */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <mpi.h>

#include "cgx.h"
#include "cgx_textio.h"

#define EPSILON_DEFAULT 1.0e-6 /* parallel_cg.c:19 */

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int opt_ll(const char *v, long long *out) {
    char *end = NULL;
    errno = 0;
    const long long x = strtoll(v, &end, 10);
    if (!*v || *end || errno) return 0;
    *out = x;
    return 1;
}

static int opt_double(const char *v, double *out) {
    char *end = NULL;
    errno = 0;
    const double x = strtod(v, &end);
    if (!*v || *end || errno) return 0;
    *out = x;
    return 1;
}

static void usage(void) {
    fprintf(stderr,
            "usage: mpiexec -np P cg_mpi [--fp32-ref] [--p2p] [--eps E] [--max-iter M] [--dims FILE | --n N]\n"
            "                            [--threads T] [--print-x] [--stats] matrixA vectorb initialguess\n");
}

/* values [first, first + count) of a text file, read as the reference's
 * fscanf("%f%*c") loop reads it; 0 or the reader's error (-1 open, -2 short,
 * -3 malformed) */
static int read_values(const char *path, int64_t first, int64_t count, int as_float, void *out, int threads) {
    cgx_text *t = NULL;
    int rc = cgx_text_open(path, threads, &t);
    if (rc == 0) rc = cgx_text_read_range(t, first, count, as_float, out, threads);
    cgx_text_close(t);
    return rc;
}

/* A read failure on any rank stops every rank (the reference reads on rank
 * 0 only and, on a missing file, prints and goes on with whatever memory
 * holds; here every rank exits non-zero).  Rank 0 prints the reference's
 * message for the first file that failed: initialize()'s "Could not open
 * file" (parallel_cg.c:166, and x0 in point-to-point_cg.c:176), scatterRow's
 * "Could not open %s file. " for A and b in point-to-point_cg.c (:226). */
static int input_failed(int rank, int p2p, const char *const *pos, const int rc[3]) {
    int worst[3] = {0, 0, 0};
    MPI_Allreduce((void *)rc, worst, 3, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    int f = -1;
    for (int q = 0; q < 3 && f < 0; ++q) {
        const int order = q == 0 ? 2 : q - 1; /* x0 is read first, then A, then b */
        if (worst[order] != 0) f = order;
    }
    if (f < 0) return 0;
    if (rc[f] != 0 && rc[f] != -1)
        fprintf(stderr, "rank %d: %s: %s\n", rank, pos[f],
                rc[f] == -2 ? "holds fewer numbers than the system needs"
                            : rc[f] == -4 ? "can't allocate memory" : "malformed number");
    if (rank == 0 && worst[f] == -1) {
        if (p2p && f < 2) printf("Could not open %s file. \n", pos[f]);
        else printf("Could not open file\n");
        fflush(stdout);
    }
    return 1;
}

int main(int argc, char **argv) {
    const double t_prog0 = now_s();
    if (MPI_Init(&argc, &argv) != MPI_SUCCESS) {
        printf("MPI_Init failed.\n"); /* parallel_cg.c:78 */
        return 1;
    }
    int rank = 0, nranks = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nranks);
    MPI_Comm node;
    int local_rank = 0;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    MPI_Comm_rank(node, &local_rank);
    MPI_Comm_free(&node);

    int fp32ref = 0, p2p = 0, print_x = 0, stats = 0, threads = 4, bad = 0;
    double eps = EPSILON_DEFAULT;
    long long max_iter = -1, n_opt = -1, v = 0;
    const char *dims_path = NULL, *pos[3] = {NULL, NULL, NULL};
    int npos = 0;
    for (int i = 1; i < argc && !bad; ++i) {
        const char *a = argv[i];
        const int has = i + 1 < argc;
        if (!strcmp(a, "--fp32-ref")) fp32ref = 1;
        else if (!strcmp(a, "--p2p")) p2p = 1;
        else if (!strcmp(a, "--print-x")) print_x = 1;
        else if (!strcmp(a, "--stats")) stats = 1;
        else if (!strcmp(a, "--eps") && has) bad = !opt_double(argv[++i], &eps);
        else if (!strcmp(a, "--max-iter") && has) bad = !opt_ll(argv[++i], &max_iter);
        else if (!strcmp(a, "--n") && has) bad = !opt_ll(argv[++i], &n_opt);
        else if (!strcmp(a, "--dims") && has) dims_path = argv[++i];
        else if (!strcmp(a, "--threads") && has) {
            bad = !opt_ll(argv[++i], &v);
            threads = v < 1 ? 1 : (v > 64 ? 64 : (int)v);
        } else if (a[0] == '-' && a[1] == '-') bad = 1;
        else if (npos < 3) pos[npos++] = a;
        else bad = 1;
    }
    if (bad || npos != 3) {
        if (rank == 0) usage();
        MPI_Finalize();
        return 2;
    }

    /* N: rank 0 decides (dimensions file, --n, or the count of b's values) */
    long long n = 0;
    if (rank == 0) {
        if (n_opt > 0) n = n_opt;
        else if (dims_path) {
            int64_t d[4];
            if (cgx_text_dims(dims_path, d) != 0) n = -1;
            else if (d[0] != d[1]) {
                printf("%lld and %lld must be same size\n", (long long)d[0], (long long)d[1]); /* :93 */
                n = -1;
            } else n = d[0];
        } else {
            n = cgx_text_count(pos[1]);
            if (n < 0) printf("Could not open file\n");
        }
        if (n == 0) fprintf(stderr, "empty system\n");
        if (n > 0 && n % nranks != 0) {
            if (p2p) printf("%lld must be divisible by %d\n", n, nranks); /* point-to-point_cg.c:101 */
            else printf("%lld is not divisible by %d\n", n, nranks);      /* parallel_cg.c:88 */
            n = -1;
        }
        if (n > 0) printf("Computing cg of matrix size : %lld\n", n * n); /* :101 */
        fflush(stdout);
    }
    MPI_Bcast(&n, 1, MPI_LONG_LONG, 0, MPI_COMM_WORLD);
    if (n <= 0) {
        MPI_Finalize();
        return 1;
    }
    const int64_t nloc = n / nranks, row0 = (int64_t)rank * nloc;
    double t_dist0 = 0.0;
    const size_t es = fp32ref ? 4 : 8;

    /* every rank parses its own rows of A, b and x0: x0 first (rank 0's
     * initialize() before the distribution, both programs), A and b where the
     * program reads them -- before the distribution bracket in parallel_cg.c
     * (:104-106), inside it in point-to-point_cg.c (scatterRow reads the file
     * while it sends, :119-127, :183-235) */
    void *A = malloc((size_t)nloc * (size_t)n * es), *b = malloc((size_t)nloc * es), *x = malloc((size_t)n * es);
    int rc[3] = {0, 0, 0};
    if (!(A && b && x)) rc[0] = rc[1] = rc[2] = -4;
    if (!rc[2]) rc[2] = read_values(pos[2], row0, nloc, fp32ref, (char *)x + (size_t)row0 * es, 1);
    if (!p2p && !rc[0]) rc[0] = read_values(pos[0], row0 * n, nloc * n, fp32ref, A, threads);
    if (!p2p && !rc[1]) rc[1] = read_values(pos[1], row0, nloc, fp32ref, b, threads);
    if (p2p) /* the files are parsed inside the bracket; whether they open is known before the GPU set-up */
        for (int f = 0; f < 2; ++f) {
            cgx_text *t = NULL;
            if (!rc[f]) rc[f] = cgx_text_open(pos[f], 1, &t);
            cgx_text_close(t);
        }
    cgx_ctx *ctx = NULL;
    if (input_failed(rank, p2p, pos, rc)) {
        MPI_Finalize();
        return 1;
    }
    /* RCCL bootstrap over MPI, then the rank's context on its GPU -- before
     * the p2p distribution bracket opens, so that bracket holds only what
     * point-to-point_cg.c:119-127 times (the reads and the distribution) */
    cgx_unique_id id;
    memset(&id, 0, sizeof id);
    int id_rc = CGX_OK;
    if (rank == 0 && (id_rc = cgx_get_unique_id(&id)) != CGX_OK)
        fprintf(stderr, "cgx_get_unique_id: %s (%s)\n", cgx_strerror(id_rc), cgx_last_error());
    MPI_Bcast(&id_rc, 1, MPI_INT, 0, MPI_COMM_WORLD);
    if (id_rc != CGX_OK) {  /* no RCCL id: nobody can join, every rank stops */
        MPI_Finalize();
        return 1;
    }
    MPI_Bcast(&id, sizeof id, MPI_BYTE, 0, MPI_COMM_WORLD);
    int ndev = 0;
    cgx_device_count(&ndev);
    const char *de = getenv("CGX_DEVICE");
    const int dev = de ? atoi(de) : (ndev > 0 ? local_rank % ndev : 0);
    const int flags = (fp32ref ? CGX_F32_REF : CGX_F64) | (p2p ? CGX_COMM_P2P : 0);
    const int crc = cgx_create_rank(&ctx, n, rank, nranks, &id, dev, flags);
    if (crc != CGX_OK) {
        fprintf(stderr, "rank %d: cgx_create_rank: %s (%s)\n", rank, cgx_strerror(crc), cgx_last_error());
        MPI_Abort(MPI_COMM_WORLD, 1); /* as parallel_cg.c stops the job */
    }

    if (p2p) {
        MPI_Barrier(MPI_COMM_WORLD); /* point-to-point_cg.c:119-120: the bracket opens before the reads */
        t_dist0 = MPI_Wtime();
        if (!rc[0]) rc[0] = read_values(pos[0], row0 * n, nloc * n, fp32ref, A, threads);
        if (!rc[1]) rc[1] = read_values(pos[1], row0, nloc, fp32ref, b, threads);
    }
    if (p2p && input_failed(rank, p2p, pos, rc)) {
        cgx_destroy(ctx);
        MPI_Finalize();
        return 1;
    }

    /* the scatter of A and b and the broadcast of x0: parallel_cg.c:109-117
     * (MPI_Bcast + MPI_Scatter between two barriers), point-to-point_cg.c:119-127
     * (BcastVector + scatterRow, the reads above included) */
    if (!p2p) {
        MPI_Barrier(MPI_COMM_WORLD);
        t_dist0 = MPI_Wtime();
    }
    int src = cgx_set_rows(ctx, row0, nloc, A, n, b, (char *)x + (size_t)row0 * es);
    MPI_Barrier(MPI_COMM_WORLD);
    const double t_dist1 = MPI_Wtime();
    free(A);
    free(b);
    cgx_stats st;
    memset(&st, 0, sizeof st);
    /* conjugrad's own bracket: MPI_Barrier + MPI_Wtime on every rank before
     * and after the loop (parallel_cg.c:278-279,328-329; point-to-point_cg.c
     * :435-436,488-489), rank 0 prints the difference */
    MPI_Barrier(MPI_COMM_WORLD);
    const double t_cg0 = MPI_Wtime();
    if (src == CGX_OK) src = cgx_solve(ctx, NULL, eps, max_iter, &st);
    if (src != CGX_OK) {
        fprintf(stderr, "rank %d: %s (%s)\n", rank, cgx_strerror(src), cgx_last_error());
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    const double t_cg1 = MPI_Wtime();
    src = cgx_get_x(ctx, x); /* the full x on every rank, as the reference leaves it */
    if (src != CGX_OK) {
        fprintf(stderr, "rank %d: %s (%s)\n", rank, cgx_strerror(src), cgx_last_error());
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    if (rank == 0) {
        printf("cg method execution time in seconds: %f\n", t_cg1 - t_cg0); /* parallel_cg.c:334, p2p :493 */
        if (p2p) printf("p2p data distribution time in seconds: %f\n", t_dist1 - t_dist0);   /* p2p :133-134 */
        else printf("collective data distribution time in seconds: %f\n", t_dist1 - t_dist0); /* :123-124 */
        printf("clock execution time in seconds: %f\n", now_s() - t_prog0);    /* parallel_cg.c:125, p2p :135 */
        if (stats)
            printf("iterations: %lld converged: %d residual_norm: %.6e\n", (long long)st.iterations, st.converged,
                   st.rr >= 0 ? sqrt(st.rr) : -1.0);
        if (print_x)
            for (int64_t i = 0; i < n; ++i) {
                if (fp32ref) printf("%.9g\n", (double)((float *)x)[i]);
                else printf("%.17g\n", ((double *)x)[i]);
            }
        fflush(stdout);
    }
    cgx_destroy(ctx);
    free(x);
    MPI_Finalize();
    return 0;
}
