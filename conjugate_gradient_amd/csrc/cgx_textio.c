/*
 * cgx_textio.c -- text reader for dimensions.txt / matrixA.txt / vectorb.txt /
 * initialguess.txt (see cgx_textio.h).  Host C, pthreads.
 *
 * The file is memory-mapped; each thread counts, then parses, one slice cut
 * at a separator.  Each number is converted on its own, exactly as strtof
 * (== fscanf "%f", serialConjugate.c:96) or strtod would (an exact fast path
 * below, those functions otherwise), so the result does not depend on how
 * the file is split among threads.  Separators are whitespace, ',' ';' and any
 * byte >= 0x80 (so a stray UTF-8 BOM, as in the reference's
 * initialguess1.txt, is skipped rather than mis-parsed).
 */
#define _GNU_SOURCE
#include "cgx_textio.h"

#include <fcntl.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

/* Separators: whitespace, ',' ';' NUL and bytes >= 0x80 (a UTF-8 BOM). */
static unsigned char kSep[256];
static pthread_once_t kSepOnce = PTHREAD_ONCE_INIT;
static void init_sep(void) {
    const char *s = " \n\r\t\v\f,;";
    for (const char *q = s; *q; ++q) kSep[(unsigned char)*q] = 1;
    kSep[0] = 1;
    for (int ch = 0x80; ch < 256; ++ch) kSep[ch] = 1;
}
#define IS_SEP(ch) (kSep[(unsigned char)(ch)])

/* Exact fast path (Clinger): a token [+-]digits[.digits][(e|E)[+-]digits]
 * with at most 19 significant digits m < 2^53 and decimal exponent |e| <= 22
 * converts with ONE correctly rounded double operation, m * 10^e or
 * m / 10^-e, both operands exact.  For float, the double is rounded once
 * more; that is the correctly rounded float unless the double sits exactly
 * on a float rounding midpoint (its 29 bits below float precision are
 * 1000...0), which is sent to strtof, as are subnormal / overflowing floats.
 * Anything else (long mantissas, big exponents, inf/nan, hex) uses
 * strtof/strtod.  Parses from p up to the first separator (or end); returns
 * the token end, or NULL to fall back. */
static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

static inline const char *fast_number(const char *p, const char *end, int as_float, void *out, int64_t idx) {
    int neg = 0;
    if (p < end && (*p == '-' || *p == '+')) { neg = (*p == '-'); ++p; }
    uint64_t m = 0;
    int sig = 0, frac = 0, any = 0;
    while (p < end && (unsigned)(*p - '0') < 10u) {
        any = 1;
        if (m == 0 && *p == '0') { ++p; continue; }  /* leading zeros */
        if (++sig > 19) return NULL;
        m = m * 10 + (uint64_t)(*p - '0');
        ++p;
    }
    if (p < end && *p == '.') {
        ++p;
        while (p < end && (unsigned)(*p - '0') < 10u) {
            any = 1;
            if (m == 0 && *p == '0') { ++frac; ++p; continue; }
            if (++sig > 19) return NULL;
            m = m * 10 + (uint64_t)(*p - '0');
            ++frac;
            ++p;
        }
    }
    if (!any) return NULL;
    int e10 = -frac;
    if (p < end && (*p == 'e' || *p == 'E')) {
        ++p;
        int eneg = 0, ev = 0, edig = 0;
        if (p < end && (*p == '-' || *p == '+')) { eneg = (*p == '-'); ++p; }
        while (p < end && (unsigned)(*p - '0') < 10u) {
            if (ev < 10000) ev = ev * 10 + (*p - '0');
            ++edig;
            ++p;
        }
        if (!edig) return NULL;
        e10 += eneg ? -ev : ev;
    }
    if (p < end && !IS_SEP(*p)) return NULL; /* trailing garbage: let strto* decide */
    double d;
    if (m == 0) {
        d = 0.0;
    } else {
        if (m > (1ull << 53) || e10 < -22 || e10 > 22) return NULL;
        d = (double)m;
        d = (e10 >= 0) ? d * kPow10[e10] : d / kPow10[-e10];
    }
    if (neg) d = -d;
    if (as_float) {
        if (d != 0.0) {
            const double ad = fabs(d);
            if (ad < 1.1754943508222875e-38 || ad >= 3.4028234663852886e38) return NULL;
            uint64_t bits;
            memcpy(&bits, &d, 8);
            if ((bits & 0x1FFFFFFFull) == 0x10000000ull) return NULL; /* exact float midpoint */
        }
        ((float *)out)[idx] = (float)d;
    } else {
        ((double *)out)[idx] = d;
    }
    return p;
}

/* strtof / strtod on a NUL-terminated copy of [p, tok_end) (the mapping has
 * no terminator).  Returns 0 or -3 if the token is not a whole number. */
static int slow_number(const char *p, const char *tok_end, int as_float, void *out, int64_t idx) {
    char tmp[128];
    size_t n = (size_t)(tok_end - p);
    char *heap = NULL, *s = tmp;
    if (n + 1 > sizeof tmp) {
        heap = (char *)malloc(n + 1);
        if (!heap) return -3;
        s = heap;
    }
    memcpy(s, p, n);
    s[n] = '\0';
    char *stop = NULL;
    if (as_float) ((float *)out)[idx] = strtof(s, &stop);
    else ((double *)out)[idx] = strtod(s, &stop);
    const int ok = stop == s + n && n > 0;
    free(heap);
    return ok ? 0 : -3;
}

/* The file, memory-mapped read-only (falls back to a malloc'd copy). */
typedef struct {
    const char *data;
    size_t len;
    void *map;   /* munmap this (len bytes) ... */
    char *heap;  /* ... or free this */
} text_buf;

static int open_text(const char *path, text_buf *tb) {
    memset(tb, 0, sizeof *tb);
    pthread_once(&kSepOnce, init_sep);
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); return -1; }
    if (S_ISREG(st.st_mode) && st.st_size > 0) {
        void *m = mmap(NULL, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m != MAP_FAILED) {
            (void)madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
            close(fd);
            tb->map = m;
            tb->data = (const char *)m;
            tb->len = (size_t)st.st_size;
            return 0;
        }
    }
    /* not mappable (empty file, pipe, ...): read it */
    size_t cap = 1 << 16, len = 0;
    char *buf = (char *)malloc(cap);
    if (!buf) { close(fd); return -1; }
    for (;;) {
        if (len == cap) {
            char *nb = (char *)realloc(buf, cap * 2);
            if (!nb) { free(buf); close(fd); return -1; }
            buf = nb;
            cap *= 2;
        }
        ssize_t got = read(fd, buf + len, cap - len);
        if (got < 0) { free(buf); close(fd); return -1; }
        if (got == 0) break;
        len += (size_t)got;
    }
    close(fd);
    tb->heap = buf;
    tb->data = buf;
    tb->len = len;
    return 0;
}

static void close_text(text_buf *tb) {
    if (tb->map) munmap(tb->map, tb->len);
    free(tb->heap);
}

static int64_t count_tokens(const char *p, const char *end) {
    int64_t c = 0;
    int in = 0;
    for (; p < end; ++p) {
        const int sep = IS_SEP(*p);
        c += (!sep) & (!in);
        in = !sep;
    }
    return c;
}

int64_t cgx_text_count(const char *path) {
    text_buf tb;
    if (open_text(path, &tb) != 0) return -1;
    int64_t c = count_tokens(tb.data, tb.data + tb.len);
    close_text(&tb);
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
    const char *p = c->beg, *end = c->end;
    int64_t idx = c->first;
    c->status = 0;
    while (idx < c->count) {
        while (p < end && IS_SEP(*p)) ++p;
        if (p >= end) break;
        const char *q = fast_number(p, end, c->as_float, c->out, idx);
        if (!q) {
            q = p;
            while (q < end && !IS_SEP(*q)) ++q;
            if (slow_number(p, q, c->as_float, c->out, idx) != 0) { c->status = -3; return NULL; }
        }
        ++idx;
        p = q;
    }
    return NULL;
}

int cgx_text_read(const char *path, int64_t count, int as_float, void *out, int threads) {
    text_buf tb;
    if (open_text(path, &tb) != 0) return -1;
    const char *buf = tb.data;
    const size_t len = tb.len;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (len < (size_t)threads * 4096) threads = 1;
    chunk_t ch[64];
    /* split at separators so no token straddles two chunks */
    const char *pos = buf, *end = buf + len;
    for (int t = 0; t < threads; ++t) {
        const char *stop = (t == threads - 1) ? end : buf + (len * (size_t)(t + 1)) / (size_t)threads;
        if (stop < pos) stop = pos;
        while (stop < end && !IS_SEP(*stop)) ++stop;
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
    if (total < count) { close_text(&tb); return -2; }
    for (int t = 1; t < threads; ++t) pthread_create(&tid[t], NULL, parse_job, &ch[t]);
    parse_job(&ch[0]);
    for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
    close_text(&tb);
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
