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
    text_buf tb;
    if (open_text(path, &tb) != 0) return -1;
    int bad;
    int64_t c = count_tokens(tb.data, tb.data + tb.len, &bad);
    close_text(&tb);
    return c;
}

typedef struct {
    const char *beg, *end;  /* chunk [beg, end), both at token boundaries */
    int64_t first;          /* index of the chunk's first token            */
    int64_t ntok;           /* numbers in the chunk                         */
    int bad;                /* the chunk stops at a failing conversion      */
    int64_t count;          /* total tokens wanted                         */
    int as_float;
    void *out;
    int status;
} chunk_t;

static void *count_job(void *arg) {
    chunk_t *c = (chunk_t *)arg;
    c->ntok = count_tokens(c->beg, c->end, &c->bad);
    return NULL;
}

static void *parse_job(void *arg) {
    chunk_t *c = (chunk_t *)arg;
    const char *p = c->beg, *end = c->end;
    int64_t idx = c->first;
    c->status = 0;
    while (idx < c->count) {
        while (p < end && IS_SPACE(*p)) ++p;
        if (p >= end) break;
        int ok;
        const char *q = scan_number(p, end, &ok);
        if (!ok) { c->status = -3; return NULL; }
        if (!fast_number(p, q, c->as_float, c->out, idx) &&
            slow_number(p, q, c->as_float, c->out, idx) != 0) { c->status = -3; return NULL; }
        ++idx;
        p = q < end ? q + 1 : q;  /* %*c */
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
    /* cut at white space: %f skips it, so a cut changes nothing */
    const char *pos = buf, *end = buf + len;
    for (int t = 0; t < threads; ++t) {
        const char *stop = (t == threads - 1) ? end : buf + (len * (size_t)(t + 1)) / (size_t)threads;
        if (stop < pos) stop = pos;
        while (stop < end && !IS_SPACE(*stop)) ++stop;
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
    /* numbers reachable in file order: up to the first failing conversion */
    int64_t total = 0;
    int bad = 0;
    for (int t = 0; t < threads; ++t) {
        ch[t].first = total;
        if (!bad) total += ch[t].ntok;
        bad = bad || ch[t].bad;
    }
    if (total < count) { close_text(&tb); return bad ? -3 : -2; }
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
