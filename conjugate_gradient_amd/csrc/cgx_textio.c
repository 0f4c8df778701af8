/*
 * cgx_textio.c -- text reader for dimensions.txt / matrixA.txt / vectorb.txt /
 * initialguess.txt (see cgx_textio.h).  Host C, pthreads.
 *
 * The reference reads with `fscanf(reader, "%f%*c", &v)` once per value
 * (serialConjugate.c:96, parallel_cg.c:159): skip white space, take the
 * longest prefix the %f conversion accepts, then consume exactly ONE more
 * byte whatever it is.  This reader follows that rule byte for byte, so
 * "1.5-2.0" reads as 1.5 and 2.0 (the '-' is the consumed byte), CRLF and a
 * trailing byte-order mark after a number are consumed the same way, and
 * "1.0,,2.0" stops where the reference's conversions start to fail.  Where
 * the reference would go on with uninitialised values (a failed conversion,
 * end of file, a missing file) this reader returns an error instead
 * (INTEGRATION.md lists the divergences; tests/test_abi.py pins both against
 * the reference's own initialize()).
 *
 * The file is memory-mapped and cut into one slice per thread at white space
 * (where %f skips anyway, so the cut changes nothing); each thread counts,
 * then parses, its slice.  Each number is converted on its own, exactly as
 * strtof (what glibc's %f calls on the accepted characters) or strtod would
 * (an exact fast path below, those functions otherwise).
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

/* White space of the C locale (what %f skips): ' ' \t \n \v \f \r. */
static unsigned char kSpace[256];
static pthread_once_t kSpaceOnce = PTHREAD_ONCE_INIT;
static void init_space(void) {
    const char *s = " \t\n\v\f\r";
    for (const char *q = s; *q; ++q) kSpace[(unsigned char)*q] = 1;
}
#define IS_SPACE(ch) (kSpace[(unsigned char)(ch)])

static inline int lower(char ch) { return (ch >= 'A' && ch <= 'Z') ? ch - 'A' + 'a' : ch; }
static inline int is_digit(char ch) { return (unsigned)(ch - '0') < 10u; }
static inline int is_xdigit(char ch) { return is_digit(ch) || ((unsigned)(lower(ch) - 'a') < 6u); }
static inline int match_word(const char *p, const char *end, const char *w) {
    for (; *w; ++w, ++p)
        if (p >= end || lower(*p) != *w) return 0;
    return 1;
}

/* The characters glibc's scanf %f consumes from p (C locale), probed against
 * glibc 2.35 fscanf: a sign, then inf / infinity / nan (a '(' after nan is
 * NOT taken), a hexadecimal float (0x...), or decimal digits with an optional
 * '.' and an optional exponent -- an exponent marker (and its sign) is taken
 * even with no digits after it ("1e+" reads as 1).  Returns the end of what
 * it consumes; *ok = 0 where the conversion fails (a lone sign or '.', "0x"
 * with nothing after, "infinit", ...): the reference's fscanf stops there. */
static const char *scan_number(const char *p, const char *end, int *ok) {
    *ok = 0;
    if (p < end && (*p == '+' || *p == '-')) ++p;
    if (p >= end) return p;
    if (lower(*p) == 'i') {
        if (!match_word(p, end, "inf")) return p + 1;
        p += 3;
        if (p < end && lower(*p) == 'i') {  /* "infinity" or nothing */
            if (!match_word(p, end, "inity")) return p + 1;
            p += 5;
        }
        *ok = 1;
        return p;
    }
    if (lower(*p) == 'n') {
        if (!match_word(p, end, "nan")) return p + 1;
        *ok = 1;
        return p + 3;
    }
    int hex = 0, digits = 0, dot = 0;
    if (*p == '0' && p + 1 < end && lower(p[1]) == 'x') {
        hex = 1;
        p += 2;
    }
    while (p < end && (hex ? is_xdigit(*p) : is_digit(*p))) { ++p; ++digits; }
    if (p < end && *p == '.') {
        ++p;
        dot = 1;
        while (p < end && (hex ? is_xdigit(*p) : is_digit(*p))) { ++p; ++digits; }
    }
    if (!digits) {  /* glibc converts "0x." (to 0) and takes no exponent after it */
        *ok = hex && dot;
        return p;
    }
    if (p < end && lower(*p) == (hex ? 'p' : 'e')) {
        ++p;
        if (p < end && (*p == '+' || *p == '-')) ++p;
        while (p < end && is_digit(*p)) ++p;
    }
    *ok = 1;
    return p;
}

/* Exact fast path (Clinger): a token [+-]digits[.digits][(e|E)[+-]digits]
 * with at most 19 significant digits m < 2^53 and decimal exponent |e| <= 22
 * converts with ONE correctly rounded double operation, m * 10^e or
 * m / 10^-e, both operands exact.  For float, the double is rounded once
 * more; that is the correctly rounded float unless the double sits exactly
 * on a float rounding midpoint (its 29 bits below float precision are
 * 1000...0), which is sent to strtof, as are subnormal / overflowing floats.
 * Anything else (long mantissas, big exponents, inf/nan, hex) uses
 * strtof/strtod.  Converts the number [p, end) (scan_number's span); returns
 * end, or NULL to fall back. */
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
    if (p != end) return NULL; /* hex, inf, nan, ...: strto* */
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
 * no terminator), as glibc's %f does on the characters it took: the value is
 * what strtof makes of them ("1e+" -> 1); -3 if it converts nothing. */
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
    const int ok = stop > s;
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
    pthread_once(&kSpaceOnce, init_space);
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

/* The reference's read loop over [p, end): skip white space, a number, one
 * more byte.  Counts the numbers; *bad = 1 if it stopped at a place where the
 * conversion fails (nothing after that is reachable). */
static int64_t count_tokens(const char *p, const char *end, int *bad) {
    int64_t c = 0;
    *bad = 0;
    for (;;) {
        while (p < end && IS_SPACE(*p)) ++p;
        if (p >= end) return c;
        int ok;
        const char *q = scan_number(p, end, &ok);
        if (!ok) {
            *bad = 1;
            return c;
        }
        ++c;
        p = q < end ? q + 1 : q;  /* %*c */
    }
}

int64_t cgx_text_count(const char *path) {
    cgx_text *t = NULL;
    if (cgx_text_open(path, 1, &t) != 0) return -1;
    const int64_t c = cgx_text_available(t, NULL);
    cgx_text_close(t);
    return c;
}

/* ---- the indexed file: pieces cut at white space, each with its count ---- */
/* A piece is ~256 KiB of text (at least 8 per thread); the count pass fills in
 * how many numbers each holds, so a range of values can be parsed from the
 * pieces that hold it alone (row blocks streamed by cg_hip). */
struct cgx_text {
    text_buf tb;
    int npieces;
    const char **beg, **end; /* piece q = [beg[q], end[q])                         */
    int64_t *first;          /* index of piece q's first number (npieces + 1 entries) */
    int64_t *ntok;
    int *bad;                /* piece q stops at a failing conversion                */
    int64_t avail;           /* numbers reachable: up to the first failing conversion */
    int stopped;             /* avail ends at a failing conversion (else at end of file) */
};

typedef struct {
    cgx_text *t;
    int q0, q1;              /* pieces [q0, q1) of this job                          */
    int64_t lo, hi;          /* values wanted: [lo, hi)                              */
    int as_float;
    void *out;               /* out[i - lo]                                          */
    int status;
} piece_job;

static void *count_job(void *arg) {
    piece_job *j = (piece_job *)arg;
    for (int q = j->q0; q < j->q1; ++q) j->t->ntok[q] = count_tokens(j->t->beg[q], j->t->end[q], &j->t->bad[q]);
    return NULL;
}

static void *parse_job(void *arg) {
    piece_job *j = (piece_job *)arg;
    j->status = 0;
    for (int qq = j->q0; qq < j->q1; ++qq) {
        const char *p = j->t->beg[qq], *end = j->t->end[qq];
        int64_t idx = j->t->first[qq];
        if (idx >= j->hi || j->t->first[qq + 1] <= j->lo) continue;
        while (idx < j->hi) {
            while (p < end && IS_SPACE(*p)) ++p;
            if (p >= end) break;
            int ok;
            const char *q = scan_number(p, end, &ok);
            if (!ok) { j->status = -3; return NULL; }
            if (idx >= j->lo) {
                const int64_t o = idx - j->lo;
                if (!fast_number(p, q, j->as_float, j->out, o) &&
                    slow_number(p, q, j->as_float, j->out, o) != 0) { j->status = -3; return NULL; }
            }
            ++idx;
            p = q < end ? q + 1 : q;  /* %*c */
        }
    }
    return NULL;
}

/* Run `fn` over pieces [q0, q1) on up to `threads` threads, contiguous piece
 * ranges per thread.  Returns the first non-zero job status. */
static int run_jobs(cgx_text *t, int q0, int q1, int threads, void *(*fn)(void *), int64_t lo, int64_t hi,
                    int as_float, void *out) {
    piece_job jobs[64];
    pthread_t tid[64];
    const int nq = q1 - q0;
    if (threads > nq) threads = nq;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    for (int k = 0; k < threads; ++k) {
        jobs[k].t = t;
        jobs[k].q0 = q0 + (int)((int64_t)nq * k / threads);
        jobs[k].q1 = q0 + (int)((int64_t)nq * (k + 1) / threads);
        jobs[k].lo = lo;
        jobs[k].hi = hi;
        jobs[k].as_float = as_float;
        jobs[k].out = out;
        jobs[k].status = 0;
    }
    int started[64] = {0};
    for (int k = 1; k < threads; ++k) started[k] = pthread_create(&tid[k], NULL, fn, &jobs[k]) == 0;
    for (int k = 1; k < threads; ++k)
        if (!started[k]) fn(&jobs[k]);
    fn(&jobs[0]);
    for (int k = 1; k < threads; ++k)
        if (started[k]) pthread_join(tid[k], NULL);
    for (int k = 0; k < threads; ++k)
        if (jobs[k].status) return jobs[k].status;
    return 0;
}

int cgx_text_open(const char *path, int threads, cgx_text **out) {
    if (!out) return -1;
    *out = NULL;
    cgx_text *t = (cgx_text *)calloc(1, sizeof *t);
    if (!t) return -1;
    if (open_text(path, &t->tb) != 0) { free(t); return -1; }
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    const size_t len = t->tb.len;
    size_t want = len / ((size_t)1 << 18) + 1;
    if (want < (size_t)threads * 8) want = (size_t)threads * 8;
    if (want > len / 64 + 1) want = len / 64 + 1; /* small files: few pieces */
    const int np = (int)want;
    t->beg = (const char **)malloc(sizeof(char *) * (size_t)np);
    t->end = (const char **)malloc(sizeof(char *) * (size_t)np);
    t->first = (int64_t *)calloc((size_t)np + 1, sizeof(int64_t));
    t->ntok = (int64_t *)calloc((size_t)np, sizeof(int64_t));
    t->bad = (int *)calloc((size_t)np, sizeof(int));
    if (!t->beg || !t->end || !t->first || !t->ntok || !t->bad) { cgx_text_close(t); return -1; }
    /* cut at white space: %f skips it, so a cut changes nothing */
    const char *buf = t->tb.data, *pos = buf, *end = buf + len;
    for (int q = 0; q < np; ++q) {
        const char *stop = (q == np - 1) ? end : buf + (len * (size_t)(q + 1)) / (size_t)np;
        if (stop < pos) stop = pos;
        while (stop < end && !IS_SPACE(*stop)) ++stop;
        t->beg[q] = pos;
        t->end[q] = stop;
        pos = stop;
    }
    t->npieces = np;
    run_jobs(t, 0, np, threads, count_job, 0, 0, 0, NULL);
    /* numbers reachable in file order: up to the first failing conversion */
    int64_t total = 0;
    for (int q = 0; q < np; ++q) {
        t->first[q] = total;
        if (!t->stopped) total += t->ntok[q];
        t->stopped = t->stopped || t->bad[q];
    }
    t->first[np] = total;
    /* pieces after the failing one hold no reachable numbers */
    for (int q = 0, after = 0; q < np; ++q) {
        if (after) { t->first[q] = total; t->ntok[q] = 0; }
        after = after || t->bad[q];
    }
    t->avail = total;
    *out = t;
    return 0;
}

int64_t cgx_text_available(const cgx_text *t, int *stopped) {
    if (!t) return -1;
    if (stopped) *stopped = t->stopped;
    return t->avail;
}

int cgx_text_read_range(cgx_text *t, int64_t first, int64_t count, int as_float, void *out, int threads) {
    if (!t || first < 0 || count < 0) return -3;
    if (count == 0) return 0;
    if (first + count > t->avail) return t->stopped ? -3 : -2;
    /* the pieces holding [first, first + count): first[q] <= first < first[q+1] ... */
    int q0 = 0, q1 = t->npieces;
    {
        int lo = 0, hi = t->npieces - 1;
        while (lo < hi) {  /* last piece with first[q] <= first */
            const int mid = (lo + hi + 1) / 2;
            if (t->first[mid] <= first) lo = mid; else hi = mid - 1;
        }
        q0 = lo;
        while (q0 > 0 && t->ntok[q0] == 0) --q0;
        lo = q0;
        hi = t->npieces - 1;
        const int64_t last = first + count - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (t->first[mid] <= last) lo = mid; else hi = mid - 1;
        }
        q1 = lo + 1;
    }
    return run_jobs(t, q0, q1, threads, parse_job, first, first + count, as_float, out);
}

void cgx_text_close(cgx_text *t) {
    if (!t) return;
    close_text(&t->tb);
    free(t->beg);
    free((void *)t->end);
    free(t->first);
    free(t->ntok);
    free(t->bad);
    free(t);
}

int cgx_text_read(const char *path, int64_t count, int as_float, void *out, int threads) {
    cgx_text *t = NULL;
    const int rc = cgx_text_open(path, threads, &t);
    if (rc != 0) return rc;
    const int r = cgx_text_read_range(t, 0, count, as_float, out, threads);
    cgx_text_close(t);
    return r;
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
