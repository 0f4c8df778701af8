/*
 * mpi_harness.c -- runs the UNMODIFIED reference MPI solvers
 *   /root/reference/parallel_cg.c       (MPI_Allgather + MPI_Allreduce)
 *   /root/reference/point-to-point_cg.c (MPI_Send/Recv: allGather, allSum, BcastVector)
 * compiled from where they lie by oracle/Makefile with
 * `-Dmain=cg_reference_main_unused -fno-builtin-sqrt`, and writes the
 * solution vector and loop-iteration count of rank 0.
 *
 * TEST INFRASTRUCTURE: used only to produce tests/golden/ fixtures in this
 * container (MPICH 3.3.2, `mpiexec -np P`).  Nothing here is part of the product.
 *
 * The reference fixes N at compile time (`#define ROWS 8192`,
 * parallel_cg.c:30-31, point-to-point_cg.c:30-31) and splits it into
 * P row blocks of ROWS/P (parallel_cg.c:83).  A system of n rows (n % P == 0)
 * is embedded so that EVERY rank owns n/P of its real rows:
 *     real row i  ->  position  (i / (n/P)) * (ROWS/P) + (i % (n/P))
 * (the same map for columns), all other positions being identity rows with
 * b = x0 = 0.  The map is increasing, so each real row's matVec
 * (parallel_cg.c:176-182) adds the real columns in the order a ROWS=n build
 * does, with exact +0 terms between them; padded r and p stay +0, so each
 * rank's local vecVec partial (:216-219) is the sum over its n/P real rows
 * only, exactly as in a ROWS=n build on P ranks -- and the MPI combine of
 * those partials (:287,294,313 / allSum :339-359) is what the fixture pins.
 * (Embedding all real rows in rank 0's block instead would make every other
 * partial 0 and pin nothing about the combine.)
 *
 * The loop count: conjugrad calls sqrt() once per iteration (:314 / :474);
 * this file provides sqrt() and rank 0 counts its calls.
 *
 * usage: mpiexec -np P <prog> <n> <A.f32> <b.f32> <x0.f32> <x_out.f32>
 *        (raw little-endian float32, A row-major n*n)
 * rank 0 prints "iterations <k+1>" after the reference's own timing lines.
 */
#define _POSIX_C_SOURCE 200809L
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define REF_ROWS 8192

/* parallel_cg.c:248 / point-to-point_cg.c:397 (same signature in both) */
void conjugrad(float *local_matrixA, float *local_vectorB, float *local_vectorX,
               int local_row, int myrank, int procsnum);

static long g_sqrt_calls = 0;
double sqrt(double v) {
    ++g_sqrt_calls;
    return __builtin_sqrt(v);
}

static int read_f32_at(FILE *f, long offset_elems, float *dst, size_t count) {
    if (fseek(f, offset_elems * (long)sizeof(float), SEEK_SET) != 0) return -1;
    return fread(dst, sizeof(float), count, f) == count ? 0 : -1;
}

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, P = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    if (argc != 6) {
        if (rank == 0) fprintf(stderr, "usage: %s n A b x0 x_out\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const long n = strtol(argv[1], NULL, 10);
    if (n < 1 || n > REF_ROWS || n % P != 0 || REF_ROWS % P != 0) {
        if (rank == 0) fprintf(stderr, "need 1 <= n <= %d, n %% P == 0\n", REF_ROWS);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const long N = REF_ROWS, nl = n / P, NL = N / P;
    /* position of real index i in the embedded system */
#define POS(i) (((i) / nl) * NL + ((i) % nl))

    float *A = calloc((size_t)NL * N, sizeof(float));  /* this rank's row block */
    float *b = calloc((size_t)NL, sizeof(float));
    float *x = calloc((size_t)N, sizeof(float));       /* full x0, replicated */
    float *row = malloc((size_t)n * sizeof(float));
    float *xs = malloc((size_t)n * sizeof(float));
    if (!A || !b || !x || !row || !xs) MPI_Abort(MPI_COMM_WORLD, 3);

    FILE *fa = fopen(argv[2], "rb"), *fb = fopen(argv[3], "rb"), *fx = fopen(argv[4], "rb");
    if (!fa || !fb || !fx) MPI_Abort(MPI_COMM_WORLD, 5);
    for (long t = 0; t < NL; ++t) {          /* local row t = global position rank*NL + t */
        if (t < nl) {
            const long i = (long)rank * nl + t;  /* the real row placed here */
            if (read_f32_at(fa, i * n, row, (size_t)n)) MPI_Abort(MPI_COMM_WORLD, 5);
            for (long j = 0; j < n; ++j) A[(size_t)t * N + POS(j)] = row[j];
            if (read_f32_at(fb, i, &b[t], 1)) MPI_Abort(MPI_COMM_WORLD, 5);
        } else {
            A[(size_t)t * N + (size_t)rank * NL + t] = 1.0f;
        }
    }
    if (read_f32_at(fx, 0, xs, (size_t)n)) MPI_Abort(MPI_COMM_WORLD, 5);
    for (long i = 0; i < n; ++i) x[POS(i)] = xs[i];
    fclose(fa); fclose(fb); fclose(fx);

    g_sqrt_calls = 0;
    conjugrad(A, b, x, (int)NL, rank, P);
    fflush(stdout);

    if (rank == 0) {
        for (long i = 0; i < n; ++i) xs[i] = x[POS(i)];
        FILE *f = fopen(argv[5], "wb");
        if (!f || fwrite(xs, sizeof(float), (size_t)n, f) != (size_t)n) MPI_Abort(MPI_COMM_WORLD, 6);
        fclose(f);
        printf("iterations %ld\n", g_sqrt_calls);
        fflush(stdout);
    }
    free(A); free(b); free(x); free(row); free(xs);
    MPI_Finalize();
    return 0;
}
