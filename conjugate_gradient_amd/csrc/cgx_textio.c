/*
 * cgx_textio.c -- text reader for dimensions.txt / matrixA.txt / vectorb.txt /
 * initialguess.txt (see cgx_textio.h).  Host C, pthreads.
 *
 * Each number is converted on its own, exactly as strtof (== fscanf "%f",
 * serialConjugate.c:96) or strtod would (an exact fast path below, those
 * functions otherwise), so the result does not depend on how the buffer is
 * split among threads.  Separators are whitespace, ',' ';' and any
 * byte >= 0x80 (so a stray UTF-8 BOM, as in the reference's
 * initialguess1.txt, is skipped rather than mis-parsed).
 */
#define _GNU_SOURCE
#include "cgx_textio.h"

#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Exact fast path (Clinger): a token [+-]digits[.digits][(e|E)[+-]digits]
 * with at most 19 significant digits m < 2^53 and decimal exponent |e| <= 22
 * converts with ONE correctly rounded double operation, m * 10^e or
 * m / 10^-e, both operands exact.  For float, the double is rounded once
 * more; that is the correctly rounded float unless the double sits exactly
 * on a float rounding midpoint, which is detected and sent to strtof.
 * Anything else (long mantissas, big exponents, inf/nan, hex) uses
 * strtof/strtod.  Returns 1 and sets *stop on success, 0 to fall back. */
static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

static int fast_number(const char *p, const char *end, int as_float, void *out, int64_t idx, const char **stop) {
    int neg = 0;
    if (p < end && (*p == '-' || *p == '+')) { neg = (*p == '-'); ++p; }
    uint64_t m = 0;
    int sig = 0, frac = 0, any = 0;
    while (p < end && *p >= '0' && *p <= '9') {
        any = 1;
        if (m == 0 && *p == '0') { ++p; continue; }  /* leading zeros */
        if (++sig > 19) return 0;
        m = m * 10 + (uint64_t)(*p - '0');
        ++p;
    }
    if (p < end && *p == '.') {
        ++p;
        while (p < end && *p >= '0' && *p <= '9') {
            any = 1;
            if (m == 0 && *p == '0') { ++frac; ++p; continue; }
            if (++sig > 19) return 0;
            m = m * 10 + (uint64_t)(*p - '0');
            ++frac;
            ++p;
        }
    }
    if (!any) return 0;
    int e10 = -frac;
    if (p < end && (*p == 'e' || *p == 'E')) {
        ++p;
        int eneg = 0, ev = 0, edig = 0;
        if (p < end && (*p == '-' || *p == '+')) { eneg = (*p == '-'); ++p; }
        while (p < end && *p >= '0' && *p <= '9') {
            if (ev < 10000) ev = ev * 10 + (*p - '0');
            ++edig;
            ++p;
        }
        if (!edig) return 0;
        e10 += eneg ? -ev : ev;
    }
    double d;
    if (m == 0) {
        d = 0.0;
    } else {
        if (m > (1ull << 53) || e10 < -22 || e10 > 22) return 0;
        d = (double)m;
        d = (e10 >= 0) ? d * kPow10[e10] : d / kPow10[-e10];
    }
    if (neg) d = -d;
    if (as_float) {
        const float f = (float)d;
        if ((double)f != d) {
            if (!isfinite(f) || fabs(d) < 1.1754943508222875e-38) return 0; /* overflow / subnormal */
            const float g = nextafterf(f, ((double)f < d) ? INFINITY : -INFINITY);
            if (((double)f + (double)g) * 0.5 == d) return 0;                  /* exact midpoint */
        }
        ((float *)out)[idx] = f;
    } else {
        ((double *)out)[idx] = d;
    }
    *stop = p;
    return 1;
}

static int is_sep(unsigned char ch) {
    return ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t' || ch == '\v' || ch == '\f' ||
           ch == ',' || ch == ';' || ch == '\0' || ch >= 0x80;
}

/* Whole file into a NUL-terminated buffer. */
static char *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return NULL; }
    long sz = ftell(f);
    if (sz < 0) { fclose(f); return NULL; }
    rewind(f);
    char *buf = (char *)malloc((size_t)sz + 1);
    if (!buf) { fclose(f); return NULL; }
    size_t got = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    buf[got] = '\0';
    *len = got;
    return buf;
}

static int64_t count_tokens(const char *p, const char *end) {
    int64_t c = 0;
    while (p < end) {
        while (p < end && is_sep((unsigned char)*p)) ++p;
        if (p >= end) break;
        ++c;
        while (p < end && !is_sep((unsigned char)*p)) ++p;
    }
    return c;
}

int64_t cgx_text_count(const char *path) {
    size_t len = 0;
    char *buf = slurp(path, &len);
    if (!buf) return -1;
    int64_t c = count_tokens(buf, buf + len);
    free(buf);
    return c;
}

typedef struct {
    const char *beg, *end;  /* chunk [beg, end), both at token boundaries */
    int64_t first;          /* index of the chunk's first token            */
    int64_t ntok;           /* tokens in the chunk                         */
    int64_t count;          /* total tokens wanted                         */
    int as_float;
    void *out;
    int status;
} chunk_t;

static void *count_job(void *arg) {
    chunk_t *c = (chunk_t *)arg;
    c->ntok = count_tokens(c->beg, c->end);
    return NULL;
}

static void *parse_job(void *arg) {
    chunk_t *c = (chunk_t *)arg;
    const char *p = c->beg;
    int64_t idx = c->first;
    c->status = 0;
    while (p < c->end && idx < c->count) {
        while (p < c->end && is_sep((unsigned char)*p)) ++p;
        if (p >= c->end) break;
        const char *tok_end = p;
        while (tok_end < c->end && !is_sep((unsigned char)*tok_end)) ++tok_end;
        const char *fstop = NULL;
        if (!fast_number(p, tok_end, c->as_float, c->out, idx, &fstop) || fstop != tok_end) {
            char *stop = NULL;
            if (c->as_float) ((float *)c->out)[idx] = strtof(p, &stop);
            else ((double *)c->out)[idx] = strtod(p, &stop);
            if (stop != tok_end) { c->status = -3; return NULL; }
        }
        ++idx;
        p = tok_end;
    }
    return NULL;
}

int cgx_text_read(const char *path, int64_t count, int as_float, void *out, int threads) {
    size_t len = 0;
    char *buf = slurp(path, &len);
    if (!buf) return -1;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (len < (size_t)threads * 4096) threads = 1;
    chunk_t ch[64];
    /* split at separators so no token straddles two chunks */
    const char *pos = buf, *end = buf + len;
    for (int t = 0; t < threads; ++t) {
        const char *stop = (t == threads - 1) ? end : buf + (len * (size_t)(t + 1)) / (size_t)threads;
        while (stop < end && !is_sep((unsigned char)*stop)) ++stop;
        ch[t].beg = pos;
        ch[t].end = stop;
        ch[t].count = count;
        ch[t].as_float = as_float;
        ch[t].out = out;
        ch[t].status = 0;
        pos = stop;
    }
    pthread_t tid[64];
    for (int t = 1; t < threads; ++t) pthread_create(&tid[t], NULL, count_job, &ch[t]);
    count_job(&ch[0]);
    for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
    int64_t total = 0;
    for (int t = 0; t < threads; ++t) {
        ch[t].first = total;
        total += ch[t].ntok;
    }
    if (total < count) { free(buf); return -2; }
    for (int t = 1; t < threads; ++t) pthread_create(&tid[t], NULL, parse_job, &ch[t]);
    parse_job(&ch[0]);
    for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
    free(buf);
    for (int t = 0; t < threads; ++t)
        if (ch[t].status != 0) return ch[t].status;
    return 0;
}

int cgx_text_dims(const char *path, int64_t dims[4]) {
    double v[4];
    int rc = cgx_text_read(path, 4, 0, v, 1);
    if (rc != 0) return rc;
    for (int i = 0; i < 4; ++i) {
        if (v[i] < 0 || v[i] != (double)(int64_t)v[i]) return -3;
        dims[i] = (int64_t)v[i];
    }
    return 0;
}
