/*
 * cg_oracle.h -- CPU restatement of the reference conjugate-gradient path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or, for cpu_baseline, as the thing timed on the host).  The product path
 * (libcgx.so, cg_hip) never links or calls it.
 *
 * What it restates (reference = /root/reference, mawunyega/conjugate_gradient):
 *   - oracle_cg_f32ref : serialConjugate.c:180-259 (conjugrad) with the helper
 *       loops matVec :109-120, residual :124-131, scalarVec :135-142,
 *       vecVec :145-155, vecAdd :159-166, vecSub :170-177, fp32 throughout,
 *       sequential accumulation, no FMA contraction.  With nparts > 1 the dot
 *       products are formed as per-part (row-block, parallel_cg.c:83) partials
 *       and combined in one of two orders:
 *         ORACLE_COMBINE_RANK  : sequentially in part order, point-to-point_cg.c's
 *                                allSum (:339-359);
 *         ORACLE_COMBINE_MPICH : MPICH 3.3's MPI_Allreduce(MPI_SUM) for a
 *                                1-element message, recursive doubling: the
 *                                first 2*rem parts pairwise ((p0+p1), (p2+p3), ..),
 *                                rem = P - pof2, then a balanced pairwise tree over
 *                                the pof2 values -- parallel_cg.c:287,294,313.
 *   - oracle_cg_f64    : conjgrad.m:1-18 in IEEE double (sequential sums).
 *   - oracle_spd_matlab: generateSPDmatrix.m:1-45 under MATLAB `rng default`
 *       (MT19937 seed 5489, genrand_res53, column-major fill), passed through
 *       the script's "%.4f" text format and parsed back exactly as
 *       serialConjugate.c:96 (fscanf "%f") or strtod would.
 *   - oracle_spd_hash  : the counter-hash synthetic SPD system used for
 *       N >= 16384; restated here independently of the HIP
 *       generator so the two can be checked against each other.
 *
 * Parity status: pinned.  tests/golden/ holds outputs of the UNMODIFIED
 * serialConjugate.c (built by oracle/Makefile into oracle/_ref/) on the
 * reference's own 2x2/4x4 fixtures and on generateSPDmatrix inputs, and of the
 * UNMODIFIED parallel_cg.c / point-to-point_cg.c (mpicc, mpiexec -np 1/2/4/8,
 * oracle/ref/mpi_harness.c) on the same inputs; the not-gpu suite checks this
 * oracle against all of them bit for bit (serial, and nparts = P with the
 * matching combine order).
 */
#ifndef CG_ORACLE_H
#define CG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- generators ------------------------------------------------------- */
/* MATLAB-compatible MT19937 stream: first `count` genrand_res53 draws after
 * init_genrand(seed).  seed 5489 == MATLAB `rng default`. */
void oracle_mt_res53(uint32_t seed, int64_t count, double *out);

/* generateSPDmatrix(n) written with "%.4f" and parsed back.
 * as_float != 0 -> A,b are float (strtof, == fscanf "%f"); else double (strtod).
 * A is n*n row-major (the matrix is symmetric, so MATLAB's column-major
 * linear order and C's row-major read agree).  Returns 0 or -1 on OOM. */
int oracle_spd_matlab(int64_t n, int as_float, void *A, void *b);

/* Counter-hash synthetic SPD system (rows [row0, row0+nrows) of A, and
 * b[row0 .. row0+nrows)).  A_ij = 0.5*(u(i,j)+u(j,i)) + n*[i==j].
 * as_float != 0 -> store (float)value.  Either pointer may be NULL. */
void oracle_spd_hash(int64_t n, int64_t row0, int64_t nrows, uint64_t seed,
                     int as_float, void *A_rows, void *b_rows);
double oracle_hash_u01(uint64_t seed, uint64_t i, uint64_t j);

/* ---- BLAS-1/2 pieces in the reference's operation order ---------------- */
void  oracle_matvec_f32ref(int64_t rows, int64_t cols, const float *A,
                           const float *v, float *out);
float oracle_dot_f32ref(int64_t n, const float *a, const float *b);
void  oracle_matvec_f64(int64_t rows, int64_t cols, const double *A,
                        const double *v, double *out);
double oracle_dot_f64(int64_t n, const double *a, const double *b);

/* ---- whole solves ------------------------------------------------------ */
typedef struct {
    int64_t iterations;  /* loop iterations executed (k+1 at the break)   */
    int     converged;   /* 1 if sqrt(r.r) < eps ended the loop           */
    double  rr;          /* final r.r (as computed, widened to double)    */
    double  t_init_s;    /* wall seconds: initial matVec + residual       */
    double  t_loop_s;    /* wall seconds: the iteration loop              */
} oracle_stats;

/* serialConjugate.c conjugrad restated.  x is x0 on entry, solution on exit.
 * max_iter < 0 -> n (the reference's `k < ROWS`); eps < 0 -> never stop.
 * nparts >= 1: dot products as nparts row-block partials, combined in the
 * `combine` order (ORACLE_COMBINE_*; ignored for nparts == 1). */
enum { ORACLE_COMBINE_RANK = 0, ORACLE_COMBINE_MPICH = 1 };
int oracle_cg_f32ref(int64_t n, const float *A, const float *b, float *x,
                     int64_t max_iter, double eps, int nparts, int combine,
                     oracle_stats *st);
/* The combine alone: `cnt` partials in[0..cnt) in the ORACLE_COMBINE_* order. */
float oracle_combine_f32(const float *in, int cnt, int combine);

/* conjgrad.m restated in double. */
int oracle_cg_f64(int64_t n, const double *A, const double *b, double *x,
                  int64_t max_iter, double eps, oracle_stats *st);
/* The same solve of the counter-hash system (oracle_spd_hash, b included)
 * with A regenerated row by row in every matVec instead of stored: identical
 * values and sums, no n*n memory (the configs' N = 65536 / 131072 systems). */
void oracle_hash_matvec_f64(int64_t n, uint64_t seed, int64_t row0, int64_t nrows, const double *v, double *out);
int oracle_cg_f64_hash(int64_t n, uint64_t seed, double *x, int64_t max_iter, double eps, oracle_stats *st);

/* ---- matrix-free 2D Poisson (configs[4], no reference counterpart) ------ */
/* out = A p for the 5-point Laplacian on an m x m interior grid, Dirichlet
 * zero boundary, natural row-major order: 4 p_ij - p_(i-1)j - p_(i+1)j
 * - p_i(j-1) - p_i(j+1) with p = 0 outside the grid. */
void oracle_poisson_apply(int64_t m, const double *p, double *out);
/* conjgrad.m's loop (oracle_cg_f64) with that operator; n = m*m. */
int oracle_cg_poisson_f64(int64_t m, const double *b, double *x, int64_t max_iter, double eps,
                          oracle_stats *st);

/* v[0..count) as one "%.<decimals>f" value per line, as generateSPDmatrix.m
 * writes its files (fprintf('%.4f\n')).  0 or -1. */
int oracle_write_text(const char *path, int64_t count, const double *v, int decimals);

/* threads used by oracle_cg_f64's matVec (rows are independent, so results
 * do not depend on it).  f32ref is always single-threaded, like the reference. */
void oracle_set_threads(int nthreads);

#ifdef __cplusplus
}
#endif
#endif
