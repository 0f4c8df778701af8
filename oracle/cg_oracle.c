/*
 * cg_oracle.c -- CPU restatement of the reference CG path (TEST INFRASTRUCTURE).
 * See cg_oracle.h for what is restated and where it is pinned.
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off, no fast-math; the
 * fp32-ref solve must round exactly like serialConjugate.c compiled by gcc on
 * x86-64, i.e. every multiply and add rounded to float separately).
 */
#include "cg_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_threads = 1;
void oracle_set_threads(int nthreads) { g_threads = nthreads > 0 ? nthreads : 1; }

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ======================================================================= */
/* MT19937 (Matsumoto & Nishimura 1998) as used by MATLAB's default stream  */
/* ======================================================================= */
typedef struct { uint32_t s[624]; int i; } mt_state;

static void mt_seed(mt_state *m, uint32_t seed) {
    m->s[0] = seed;
    for (int k = 1; k < 624; ++k)
        m->s[k] = 1812433253u * (m->s[k - 1] ^ (m->s[k - 1] >> 30)) + (uint32_t)k;
    m->i = 624;
}

static void mt_twist(mt_state *m) {
    for (int k = 0; k < 624; ++k) {
        uint32_t y = (m->s[k] & 0x80000000u) | (m->s[(k + 1) % 624] & 0x7fffffffu);
        uint32_t v = m->s[(k + 397) % 624] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        m->s[k] = v;
    }
    m->i = 0;
}

static uint32_t mt_u32(mt_state *m) {
    if (m->i >= 624) mt_twist(m);
    uint32_t y = m->s[m->i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* genrand_res53: 53-bit uniform on [0,1) from two draws (27 + 26 bits). */
static double mt_res53(mt_state *m) {
    uint32_t hi = mt_u32(m) >> 5, lo = mt_u32(m) >> 6;
    return ((double)hi * 67108864.0 + (double)lo) * (1.0 / 9007199254740992.0);
}

void oracle_mt_res53(uint32_t seed, int64_t count, double *out) {
    mt_state m;
    mt_seed(&m, seed);
    for (int64_t k = 0; k < count; ++k) out[k] = mt_res53(&m);
}

/* ======================================================================= */
/* generateSPDmatrix.m restated (generateSPDmatrix.m:4-17, 28-43)          */
/* ======================================================================= */
/* One value through fprintf('%.4f\n') and back through the C reader. */
static float text4_f(double v) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.4f", v);
    return strtof(buf, NULL);
}
static double text4_d(double v) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.4f", v);
    return strtod(buf, NULL);
}

int oracle_spd_matlab(int64_t n, int as_float, void *A, void *b) {
    /* R = rand(n,n) fills column-major: R(i,j) is draw number j*n + i. */
    double *R = (double *)malloc((size_t)n * (size_t)n * sizeof(double));
    if (!R) return -1;
    mt_state m;
    mt_seed(&m, 5489u);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) R[(size_t)j * n + i] = mt_res53(&m);
    /* A = 0.5*(R+R') + n*eye(n).  Symmetric, so the row-major reader sees
     * the same values as MATLAB's column-major writer. */
    /* the text round trip dominates (snprintf + strtof per value); rows are
     * independent, so it runs on every host core (same values for any count) */
#ifdef _OPENMP
    const int gen_threads = omp_get_num_procs() < 16 ? omp_get_num_procs() : 16;
#else
    const int gen_threads = 1;
#endif
#pragma omp parallel for schedule(dynamic, 16) num_threads(gen_threads)
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = 0; j < n; ++j) {
            double v = 0.5 * (R[(size_t)j * n + i] + R[(size_t)i * n + j]);
            if (i == j) v = v + (double)n;
            size_t at = (size_t)i * n + j;
            if (as_float) ((float *)A)[at] = text4_f(v);
            else ((double *)A)[at] = text4_d(v);
        }
    }
    /* b = rand(n,1) continues the same stream. */
    for (int64_t i = 0; i < n; ++i) {
        double v = mt_res53(&m);
        if (as_float) ((float *)b)[i] = text4_f(v);
        else ((double *)b)[i] = text4_d(v);
    }
    free(R);
    return 0;
}

/* ======================================================================= */
/* counter-hash synthetic SPD system (SURVEY.md s8(d), N >= 16384)          */
/* ======================================================================= */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double oracle_hash_u01(uint64_t seed, uint64_t i, uint64_t j) {
    uint64_t h = mix64(((i << 32) | (j & 0xffffffffull)) ^ mix64(seed));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

static double hash_b(uint64_t seed, uint64_t i) {
    uint64_t h = mix64(i ^ mix64(seed + 1));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

void oracle_spd_hash(int64_t n, int64_t row0, int64_t nrows, uint64_t seed,
                     int as_float, void *A_rows, void *b_rows) {
    if (A_rows) {
#pragma omp parallel for schedule(static) num_threads(g_threads)
        for (int64_t r = 0; r < nrows; ++r) {
            uint64_t i = (uint64_t)(row0 + r);
            for (int64_t jj = 0; jj < n; ++jj) {
                uint64_t j = (uint64_t)jj;
                double v = 0.5 * (oracle_hash_u01(seed, i, j) + oracle_hash_u01(seed, j, i));
                if (i == j) v = v + (double)n;
                size_t at = (size_t)r * (size_t)n + (size_t)jj;
                if (as_float) ((float *)A_rows)[at] = (float)v;
                else ((double *)A_rows)[at] = v;
            }
        }
    }
    if (b_rows) {
        for (int64_t r = 0; r < nrows; ++r) {
            double v = hash_b(seed, (uint64_t)(row0 + r));
            if (as_float) ((float *)b_rows)[r] = (float)v;
            else ((double *)b_rows)[r] = v;
        }
    }
}

/* ======================================================================= */
/* fp32 pieces in serialConjugate.c order                                   */
/* ======================================================================= */
/* matVec (serialConjugate.c:109-120): out[i] starts at 0 and takes
 * += A[i][j]*v[j] for j ascending; product and sum each rounded to float. */
void oracle_matvec_f32ref(int64_t rows, int64_t cols, const float *A,
                          const float *v, float *out) {
    for (int64_t i = 0; i < rows; ++i) {
        const float *row = A + (size_t)i * (size_t)cols;
        float acc = 0.0f;
        for (int64_t j = 0; j < cols; ++j) {
            float prod = row[j] * v[j];
            acc = acc + prod;
        }
        out[i] = acc;
    }
}

/* vecVec (serialConjugate.c:145-155). */
float oracle_dot_f32ref(int64_t n, const float *a, const float *b) {
    float s = 0.0f;
    for (int64_t i = 0; i < n; ++i) {
        float prod = a[i] * b[i];
        s = s + prod;
    }
    return s;
}

/* MPICH 3.3 MPI_Allreduce, commutative op, short message: recursive doubling
 * (MPIR_Allreduce_intra_recursive_doubling).  With pof2 the largest power of
 * two <= cnt and rem = cnt - pof2, ranks 2q and 2q+1 (q < rem) first combine,
 * leaving pof2 values; then at distance 1, 2, 4, .. every value is combined
 * with its partner's.  fp32 addition is commutative, so both partners hold
 * the same bits after each step: the result is the balanced tree below. */
static float combine_mpich_f32(const float *in, int cnt) {
    int pof2 = 1;
    while (pof2 * 2 <= cnt) pof2 *= 2;
    const int rem = cnt - pof2;
    float v[64];
    if (pof2 > 64) return NAN;
    for (int q = 0; q < pof2; ++q)
        v[q] = q < rem ? in[2 * q] + in[2 * q + 1] : in[q + rem];
    for (int d = 1; d < pof2; d *= 2)
        for (int q = 0; q < pof2; q += 2 * d) v[q] = v[q] + v[q + d];
    return v[0];
}

float oracle_combine_f32(const float *in, int cnt, int combine) {
    if (cnt <= 0) return 0.0f;
    if (combine == ORACLE_COMBINE_MPICH) return combine_mpich_f32(in, cnt);
    float total = in[0];                      /* allSum :346-352 */
    for (int q = 1; q < cnt; ++q) total = total + in[q];
    return total;
}

/* Dot product as `nparts` row-block partials, each sequential (vecVec
 * parallel_cg.c:211-221 over local_row), then combined in `combine` order.
 * nparts == 1 is serialConjugate.c's vecVec. */
static float dot_parts_f32(int64_t n, const float *a, const float *b, int nparts, int combine) {
    if (nparts <= 1) return oracle_dot_f32ref(n, a, b);
    int64_t loc = n / nparts;
    float part[64];
    for (int q = 0; q < nparts; ++q)
        part[q] = oracle_dot_f32ref(loc, a + (size_t)q * loc, b + (size_t)q * loc);
    return oracle_combine_f32(part, nparts, combine);
}

int oracle_cg_f32ref(int64_t n, const float *A, const float *b, float *x,
                     int64_t max_iter, double eps, int nparts, int combine, oracle_stats *st) {
    if (nparts < 1) nparts = 1;
    if (n % nparts != 0 || nparts > 64) return -2;
    if (max_iter < 0) max_iter = n;
    float *Av = (float *)malloc((size_t)n * sizeof(float));
    float *r = (float *)malloc((size_t)n * sizeof(float));
    float *p = (float *)malloc((size_t)n * sizeof(float));
    if (!Av || !r || !p) { free(Av); free(r); free(p); return -1; }

    double t0 = now_s();
    /* serialConjugate.c:209-212: r0 = p0 = b - A x0, rsold = r0.r0 */
    oracle_matvec_f32ref(n, n, A, x, Av);
    for (int64_t i = 0; i < n; ++i) r[i] = b[i] - Av[i];
    for (int64_t i = 0; i < n; ++i) p[i] = b[i] - Av[i];
    float rsold = dot_parts_f32(n, r, r, nparts, combine);
    double t1 = now_s();

    int64_t iters = 0;
    int converged = 0;
    float rr = rsold;
    for (int64_t k = 0; k < max_iter; ++k) {
        oracle_matvec_f32ref(n, n, A, p, Av);                 /* :215      */
        float pAp = dot_parts_f32(n, p, Av, nparts, combine);          /* :219      */
        float alpha = rsold / pAp;                            /* :220      */
        for (int64_t i = 0; i < n; ++i) {                     /* :221,225  */
            float t = p[i] * alpha;
            x[i] = x[i] + t;
        }
        for (int64_t i = 0; i < n; ++i) {                     /* :226,230  */
            float t = Av[i] * alpha;
            r[i] = r[i] - t;
        }
        rr = dot_parts_f32(n, r, r, nparts, combine);                  /* :234      */
        iters = k + 1;
        if (eps >= 0.0 && sqrt((double)rr) < eps) {           /* :235-238  */
            converged = 1;
            break;
        }
        float ratio = rr / rsold;                             /* :239      */
        for (int64_t i = 0; i < n; ++i) {                     /* :239,243  */
            float t = p[i] * ratio;
            p[i] = r[i] + t;
        }
        rsold = rr;                                           /* :244      */
    }
    double t2 = now_s();
    if (st) {
        st->iterations = iters;
        st->converged = converged;
        st->rr = (double)rr;
        st->t_init_s = t1 - t0;
        st->t_loop_s = t2 - t1;
    }
    free(Av); free(r); free(p);
    return 0;
}

/* ======================================================================= */
/* fp64 (conjgrad.m)                                                        */
/* ======================================================================= */
void oracle_matvec_f64(int64_t rows, int64_t cols, const double *A,
                       const double *v, double *out) {
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int64_t i = 0; i < rows; ++i) {
        const double *row = A + (size_t)i * (size_t)cols;
        double acc = 0.0;
        for (int64_t j = 0; j < cols; ++j) acc = acc + row[j] * v[j];
        out[i] = acc;
    }
}

double oracle_dot_f64(int64_t n, const double *a, const double *b) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s = s + a[i] * b[i];
    return s;
}

/* The operator of a conjgrad.m solve: a stored row-major A, or the
 * counter-hash matrix regenerated row by row (no n*n storage). */
typedef struct { const double *A; uint64_t seed; int hash; } f64_op;

/* Rows [row0, row0+nrows) of the counter-hash A times v, each row summed in
 * ascending column order (exactly oracle_matvec_f64 on oracle_spd_hash's A). */
void oracle_hash_matvec_f64(int64_t n, uint64_t seed, int64_t row0, int64_t nrows, const double *v, double *out) {
    const uint64_t ms = mix64(seed);  /* oracle_hash_u01's mix64(seed), hoisted */
#pragma omp parallel for schedule(dynamic, 8) num_threads(g_threads)
    for (int64_t r = 0; r < nrows; ++r) {
        const uint64_t i = (uint64_t)(row0 + r);
        double acc = 0.0;
        for (int64_t jj = 0; jj < n; ++jj) {
            const uint64_t j = (uint64_t)jj;
            const double uij = (double)(mix64(((i << 32) | (j & 0xffffffffull)) ^ ms) >> 11) * (1.0 / 9007199254740992.0);
            const double uji = (double)(mix64(((j << 32) | (i & 0xffffffffull)) ^ ms) >> 11) * (1.0 / 9007199254740992.0);
            double a = 0.5 * (uij + uji);
            if (i == j) a = a + (double)n;
            acc = acc + a * v[jj];
        }
        out[r] = acc;
    }
}

static void op_apply(const f64_op *op, int64_t n, const double *v, double *out) {
    if (op->hash) oracle_hash_matvec_f64(n, op->seed, 0, n, v, out);
    else oracle_matvec_f64(n, n, op->A, v, out);
}

static int cg_f64_op(int64_t n, const f64_op *op, const double *b, double *x,
                     int64_t max_iter, double eps, oracle_stats *st);

int oracle_cg_f64(int64_t n, const double *A, const double *b, double *x,
                  int64_t max_iter, double eps, oracle_stats *st) {
    const f64_op op = {A, 0, 0};
    return cg_f64_op(n, &op, b, x, max_iter, eps, st);
}

int oracle_cg_f64_hash(int64_t n, uint64_t seed, double *x, int64_t max_iter, double eps, oracle_stats *st) {
    double *b = (double *)malloc((size_t)n * sizeof(double));
    if (!b) return -1;
    oracle_spd_hash(n, 0, n, seed, 0, NULL, b);
    const f64_op op = {NULL, seed, 1};
    const int rc = cg_f64_op(n, &op, b, x, max_iter, eps, st);
    free(b);
    return rc;
}

static int cg_f64_op(int64_t n, const f64_op *op, const double *b, double *x,
                     int64_t max_iter, double eps, oracle_stats *st) {
    if (max_iter < 0) max_iter = n;
    double *Av = (double *)malloc((size_t)n * sizeof(double));
    double *r = (double *)malloc((size_t)n * sizeof(double));
    double *p = (double *)malloc((size_t)n * sizeof(double));
    if (!Av || !r || !p) { free(Av); free(r); free(p); return -1; }
    double t0 = now_s();
    op_apply(op, n, x, Av);                            /* conjgrad.m:2  r=b-A*x */
    for (int64_t i = 0; i < n; ++i) { r[i] = b[i] - Av[i]; p[i] = r[i]; } /* :3 */
    double rsold = oracle_dot_f64(n, r, r);            /* :4 */
    double t1 = now_s();
    int64_t iters = 0;
    int converged = 0;
    double rr = rsold;
    for (int64_t k = 0; k < max_iter; ++k) {           /* :6 for i=1:length(b) */
        op_apply(op, n, p, Av);                        /* :7 */
        double alpha = rsold / oracle_dot_f64(n, p, Av); /* :8 */
        for (int64_t i = 0; i < n; ++i) x[i] = x[i] + alpha * p[i];  /* :9  */
        for (int64_t i = 0; i < n; ++i) r[i] = r[i] - alpha * Av[i]; /* :10 */
        rr = oracle_dot_f64(n, r, r);                  /* :11 */
        iters = k + 1;
        if (eps >= 0.0 && sqrt(rr) < eps) { converged = 1; break; } /* :12-14 */
        double beta = rr / rsold;
        for (int64_t i = 0; i < n; ++i) p[i] = r[i] + beta * p[i]; /* :15 */
        rsold = rr;                                    /* :16 */
    }
    double t2 = now_s();
    if (st) {
        st->iterations = iters;
        st->converged = converged;
        st->rr = rr;
        st->t_init_s = t1 - t0;
        st->t_loop_s = t2 - t1;
    }
    free(Av); free(r); free(p);
    return 0;
}

/* ======================================================================= */
/* matrix-free 5-point Poisson (configs[4])                                 */
/* ======================================================================= */
void oracle_poisson_apply(int64_t m, const double *p, double *out) {
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int64_t i = 0; i < m; ++i) {
        for (int64_t j = 0; j < m; ++j) {
            const size_t k = (size_t)i * m + j;
            double v = 4.0 * p[k];
            if (i > 0) v -= p[k - m];
            if (i < m - 1) v -= p[k + m];
            if (j > 0) v -= p[k - 1];
            if (j < m - 1) v -= p[k + 1];
            out[k] = v;
        }
    }
}

int oracle_cg_poisson_f64(int64_t m, const double *b, double *x, int64_t max_iter, double eps,
                          oracle_stats *st) {
    const int64_t n = m * m;
    if (max_iter < 0) max_iter = n;
    double *Av = (double *)malloc((size_t)n * sizeof(double));
    double *r = (double *)malloc((size_t)n * sizeof(double));
    double *p = (double *)malloc((size_t)n * sizeof(double));
    if (!Av || !r || !p) { free(Av); free(r); free(p); return -1; }
    double t0 = now_s();
    oracle_poisson_apply(m, x, Av);
    for (int64_t i = 0; i < n; ++i) { r[i] = b[i] - Av[i]; p[i] = r[i]; }
    double rsold = oracle_dot_f64(n, r, r);
    double t1 = now_s();
    int64_t iters = 0;
    int converged = 0;
    double rr = rsold;
    for (int64_t k = 0; k < max_iter; ++k) {
        oracle_poisson_apply(m, p, Av);
        double alpha = rsold / oracle_dot_f64(n, p, Av);
        for (int64_t i = 0; i < n; ++i) x[i] = x[i] + alpha * p[i];
        for (int64_t i = 0; i < n; ++i) r[i] = r[i] - alpha * Av[i];
        rr = oracle_dot_f64(n, r, r);
        iters = k + 1;
        if (eps >= 0.0 && sqrt(rr) < eps) { converged = 1; break; }
        double beta = rr / rsold;
        for (int64_t i = 0; i < n; ++i) p[i] = r[i] + beta * p[i];
        rsold = rr;
    }
    double t2 = now_s();
    if (st) {
        st->iterations = iters;
        st->converged = converged;
        st->rr = rr;
        st->t_init_s = t1 - t0;
        st->t_loop_s = t2 - t1;
    }
    free(Av); free(r); free(p);
    return 0;
}

/* ======================================================================= */
/* text files in the reference's format (test / measurement helper)        */
/* ======================================================================= */
int oracle_write_text(const char *path, int64_t count, const double *v, int decimals) {
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    static char buf[1 << 20];
    setvbuf(f, buf, _IOFBF, sizeof buf);
    for (int64_t i = 0; i < count; ++i) fprintf(f, "%.*f\n", decimals, v[i]);
    return fclose(f) == 0 ? 0 : -1;
}
