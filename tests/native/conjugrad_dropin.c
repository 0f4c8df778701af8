/* The function-level drop-in, as INTEGRATION.md s4.1 shows it: the
 * reference's serial program (serialConjugate.c:43-73) with its text reads
 * and its `conjugrad(A, b, x);` call (:68) replaced -- the reads by
 * cgx_text_read (initialize(), :85-105), the call by cgx_conjugrad.  Prints
 * the loop count and x (%.9g: a float round-trips exactly).  Test program
 * (tests/test_abi.py builds it; tests/test_gpu_cli.py runs it on a GPU).
 *
 *   conjugrad_dropin N matrixA vectorb initialguess
 */
#include <stdio.h>
#include <stdlib.h>

#include "cgx.h"
#include "cgx_textio.h"

int main(int argc, char **argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s N matrixA vectorb initialguess\n", argv[0]);
        return 2;
    }
    const int64_t n = atoll(argv[1]);
    float *A = malloc((size_t)(n * n) * sizeof(float));
    float *b = malloc((size_t)n * sizeof(float));
    float *x = malloc((size_t)n * sizeof(float));
    if (!A || !b || !x) return 1;
    if (cgx_text_read(argv[2], n * n, 1, A, 4) || cgx_text_read(argv[3], n, 1, b, 1) ||
        cgx_text_read(argv[4], n, 1, x, 1)) {
        printf("Could not open file\n");
        return 1;
    }
    cgx_stats st;
    /* conjugrad(A, b, x);  -- serialConjugate.c:68, EPSILON 1.0e-6 (:28), k < ROWS (:213) */
    const int rc = cgx_conjugrad(A, b, x, n, CGX_F32_REF, 1.0e-6, -1, &st);
    if (rc != CGX_OK) {
        fprintf(stderr, "cgx_conjugrad: %s (%s)\n", cgx_strerror(rc), cgx_last_error());
        return 1;
    }
    printf("iterations: %lld converged: %d\n", (long long)st.iterations, st.converged);
    for (int64_t i = 0; i < n; ++i) printf("%.9g\n", (double)x[i]);
    free(A);
    free(b);
    free(x);
    return 0;
}
