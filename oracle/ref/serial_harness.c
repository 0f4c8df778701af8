/*
 * serial_harness.c -- runs the UNMODIFIED reference solver
 * /root/reference/serialConjugate.c (compiled from where it lies by
 * oracle/Makefile with `-Dmain=cg_reference_main_unused -fno-builtin-sqrt`)
 * and writes its solution vector and loop-iteration count.
 *
 * TEST INFRASTRUCTURE: used only to produce tests/golden/ fixtures in this
 * container.  Nothing here is part of the product.
 *
 * The reference fixes N at compile time (`#define ROWS 8192`,
 * serialConjugate.c:29-30).  A smaller system (n <= 8192) is embedded as
 *     A' = [[A, 0], [0, I]],  b' = [b; 0],  x0' = [x0; 0]
 * For the padded rows r = p = 0 forever, every padded product is 0*0 and
 * every padded partial sum adds +0, so each float operation on the first n
 * components is the one a ROWS=n build performs; the dot products see only
 * exact zeros from the padding.  The one behavioural difference: the loop
 * bound is 8192 instead of n, which matters only for a system that has not
 * met EPSILON within n iterations (none of the fixtures).
 *
 * The loop count is observed without touching the reference: the loop calls
 * sqrt() exactly once per iteration (serialConjugate.c:235), so this file
 * provides sqrt() and counts calls.
 *
 * usage: serial_ref <n> <A.f32> <b.f32> <x0.f32> <x_out.f32>
 *        (raw little-endian float32, A row-major n*n)
 * prints "iterations <k+1>" on stderr-free stdout line after the reference's
 * own timing line.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define REF_ROWS 8192

void conjugrad(float *matrixA, float *vectorB, float *vectorX); /* serialConjugate.c:180 */
void initialize(float *vector, char *filename, int col_num);     /* serialConjugate.c:85  */
float vecVec(float *vect1, float *vect2);                        /* serialConjugate.c:145 */

static long g_sqrt_calls = 0;
double sqrt(double v) {
    ++g_sqrt_calls;
    return __builtin_sqrt(v);
}

static int read_f32(const char *path, float *dst, size_t count) {
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); return -1; }
    size_t got = fread(dst, sizeof(float), count, f);
    fclose(f);
    if (got != count) { fprintf(stderr, "%s: short read %zu/%zu\n", path, got, count); return -1; }
    return 0;
}


static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* serial_ref --initialize <file> <col_num> <out.f32>: time the reference's own
 * text reader (ROWS * col_num values via fscanf "%f%*c", serialConjugate.c:96).
 * The buffer is pre-filled with a signalling-NaN sentinel (0x7FA5A5A5, a
 * pattern no conversion produces), so the output shows which values the
 * reader assigned: it stops assigning at its first failing conversion or at
 * end of file and leaves the rest as they were (uninitialised memory in the
 * reference's own main). */
static int time_initialize(char *path, int cols, const char *out) {
    float *v = malloc((size_t)REF_ROWS * cols * sizeof(float));
    if (!v) return 3;
    const uint32_t sentinel = 0x7FA5A5A5u;
    for (size_t i = 0; i < (size_t)REF_ROWS * cols; ++i) memcpy(v + i, &sentinel, 4);
    double t0 = now_s();
    initialize(v, path, cols);
    double t1 = now_s();
    FILE *f = fopen(out, "wb");
    if (!f || fwrite(v, sizeof(float), (size_t)REF_ROWS * cols, f) != (size_t)REF_ROWS * cols) return 6;
    fclose(f);
    printf("initialize_seconds %.6f\n", t1 - t0);
    free(v);
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 5 && strcmp(argv[1], "--initialize") == 0)
        return time_initialize(argv[2], atoi(argv[3]), argv[4]);
    if (argc != 6) {
        fprintf(stderr, "usage: %s n A b x0 x_out\n", argv[0]);
        return 2;
    }
    long n = strtol(argv[1], NULL, 10);
    if (n < 1 || n > REF_ROWS) { fprintf(stderr, "n must be in [1, %d]\n", REF_ROWS); return 2; }

    size_t N = REF_ROWS;
    float *A = calloc(N * N, sizeof(float));
    float *b = calloc(N, sizeof(float));
    float *x = calloc(N, sizeof(float));
    float *As = malloc((size_t)n * n * sizeof(float));
    if (!A || !b || !x || !As) { fprintf(stderr, "oom\n"); return 3; }

    /* sanity: the compiled-in ROWS must be REF_ROWS (vecVec of ones == ROWS) */
    for (size_t i = 0; i < N; ++i) b[i] = 1.0f;
    if (vecVec(b, b) != (float)REF_ROWS) { fprintf(stderr, "reference ROWS != %d\n", REF_ROWS); return 4; }
    memset(b, 0, N * sizeof(float));

    if (read_f32(argv[2], As, (size_t)n * n) || read_f32(argv[3], b, n) || read_f32(argv[4], x, n)) return 5;
    for (long i = 0; i < n; ++i) memcpy(A + (size_t)i * N, As + (size_t)i * n, n * sizeof(float));
    for (size_t i = n; i < N; ++i) A[i * N + i] = 1.0f;

    g_sqrt_calls = 0;
    conjugrad(A, b, x);
    fflush(stdout);

    FILE *f = fopen(argv[5], "wb");
    if (!f || fwrite(x, sizeof(float), n, f) != (size_t)n) { fprintf(stderr, "write failed\n"); return 6; }
    fclose(f);
    printf("iterations %ld\n", g_sqrt_calls);
    free(A); free(b); free(x); free(As);
    return 0;
}
