/*
 * textio_fuzz.c -- randomized check of cgx_text_read (conjugate_gradient_amd/
 * csrc/cgx_textio.c) under AddressSanitizer / UndefinedBehaviorSanitizer
 * (built by tests/test_textio_fuzz.py on the host; test infrastructure).
 *
 * Each case writes a file of random tokens -- well-formed numbers of every
 * shape the fast path and the strtod/strtof fallback take (long mantissas,
 * big exponents, float midpoints, subnormals, inf/nan, hex), and malformed
 * ones -- separated by random runs of white space, ',' and ';', sometimes by
 * a single other byte ('-', '#', 'x', a byte >= 0x80), sometimes with a
 * UTF-8 BOM in front, sometimes without a trailing separator, sometimes
 * padded so the file ends exactly on a page boundary.  The expected values
 * are what the reference's own loop reads: glibc fscanf(f, "%f%*c") (or
 * "%lf%*c" for double) once per value (serialConjugate.c:96).  The reader
 * must return them bit for bit, for 1 and several threads, when all requested
 * values convert; where fscanf fails first (a failing conversion or end of
 * file, after which the reference leaves its values uninitialised) it must
 * return -3 or -2; cgx_text_count must equal the number of values fscanf
 * converts before its first failure.
 *
 *   textio_fuzz <tmpdir> <cases> <seed>     exit 0 = all cases passed
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "cgx_textio.h"

static uint64_t g_s;
static uint64_t rnd(void) {
    g_s ^= g_s << 13;
    g_s ^= g_s >> 7;
    g_s ^= g_s << 17;
    return g_s;
}
static int rint_(int n) { return (int)(rnd() % (uint64_t)n); }

static int digits(char *o, int n, int nonzero_first) {
    for (int i = 0; i < n; ++i) o[i] = (char)('0' + ((i == 0 && nonzero_first) ? 1 + rint_(9) : rint_(10)));
    return n;
}

/* a random token into o (NUL-terminated); returns its length */
static int token(char *o) {
    static const char *special[] = {"nan", "-inf", "inf", "INF", "0x1p3", "1e", "--1", "1.2.3", ".", "e5", "+",
                                    "1e+", "0.5f", "3.4028235e38", "3.4028236e38", "1.17549435e-38",
                                    "1e-45", "7.006492e-46", "2.5e-324", "1.7976931348623157e308", "1e309",
                                    "0.1", "-0", "-0.0e0", "16777217", "0.3333333432674408"};
    const int kind = rint_(20);
    if (kind == 0) return sprintf(o, "%s", special[rint_((int)(sizeof special / sizeof *special))]);
    int n = 0;
    if (rint_(3) == 0) o[n++] = rint_(2) ? '-' : '+';
    if (kind == 1) { /* a long mantissa */
        n += digits(o + n, 20 + rint_(280), 1);
    } else if (kind == 2) { /* a float rounding midpoint, printed exactly */
        const float f = (float)(rnd() % 1000000) / 1024.0f + 1.0f;
        const double mid = (double)f + (double)(nextafterf(f, 2 * f) - f) / 2.0;
        n += sprintf(o + n, "%.17g", mid);
    } else {
        if (rint_(8)) n += digits(o + n, 1 + rint_(kind == 3 ? 19 : 8), rint_(2));
        if (rint_(2)) {
            o[n++] = '.';
            n += digits(o + n, rint_(kind == 4 ? 25 : 8), 0);
        }
        if (rint_(3) == 0) {
            o[n++] = rint_(2) ? 'e' : 'E';
            if (rint_(2)) o[n++] = rint_(2) ? '-' : '+';
            n += digits(o + n, rint_(4), 0);
        }
        if (n == 0) o[n++] = '7';
    }
    o[n] = '\0';
    return n;
}

static const char kSeps[] = " \n\r\t,;";
static const char kOdd[] = "-#x\xEF+|";

/* The reference's loop: fscanf "%f%*c" (float) / "%lf%*c" (double) per value.
 * Returns how many values it converted before the first failure (<= want),
 * and in *eof whether that failure was end of file. */
static int64_t ref_read(const char *path, int64_t want, int as_float, void *out, int *eof) {
    FILE *f = fopen(path, "rb");
    *eof = 0;
    if (!f) return -1;
    int64_t i = 0;
    for (; i < want; ++i) {
        const int r = as_float ? fscanf(f, "%f%*c", (float *)out + i) : fscanf(f, "%lf%*c", (double *)out + i);
        if (r != 1) {
            *eof = r == EOF;
            break;
        }
    }
    fclose(f);
    return i;
}

int main(int argc, char **argv) {
    if (argc != 4) return 2;
    const char *dir = argv[1];
    const int cases = atoi(argv[2]);
    g_s = 0x9E3779B97F4A7C15ull ^ (uint64_t)atoll(argv[3]);
    char path[4096];
    snprintf(path, sizeof path, "%s/fuzz_%d.txt", dir, (int)getpid());
    enum { kMaxTok = 400 };
    static char tok[320];
    int fails = 0, n_fail = 0, n_short = 0, n_page = 0, n_odd = 0;
    for (int c = 0; c < cases; ++c) {
        const int nt = 1 + rint_(kMaxTok - 1);
        const int clean = rint_(3) != 0; /* mostly files whose tokens are all numbers */
        FILE *f = fopen(path, "wb");
        if (!f) return 2;
        long bytes = 0;
        if (rint_(20) == 0) bytes += fprintf(f, "\xEF\xBB\xBF");
        for (int i = 0; i < nt; ++i) {
            int len;
            for (;;) { /* clean files: only tokens strtod consumes whole */
                len = token(tok);
                if (!clean) break;
                char *stop;
                (void)strtod(tok, &stop);
                if (stop == tok + len) break;
            }
            bytes += fprintf(f, "%s", tok);
            const int last = i == nt - 1;
            if (!last || rint_(4)) { /* separators (none after the last token sometimes) */
                if (rint_(12) == 0) { /* one odd byte: %*c consumes it whatever it is */
                    fputc(kOdd[rint_((int)sizeof kOdd - 1)], f);
                    ++bytes;
                    ++n_odd;
                } else {
                    const int ns = 1 + (rint_(4) == 0 ? rint_(3) : 0);
                    for (int q = 0; q < ns; ++q) {
                        fputc(kSeps[rint_((int)sizeof kSeps - 1)], f);
                        ++bytes;
                    }
                }
            }
        }
        if (rint_(8) == 0) { /* end exactly on a page boundary, last token touching it */
            const long pad = (4096 - (bytes + 1) % 4096) % 4096;
            for (long q = 0; q < pad; ++q) fputc(' ', f);
            ++n_page;
            fputc('5', f);
        }
        fclose(f);
        int eof;
        static double all[4 * kMaxTok];
        const int64_t avail = ref_read(path, 4 * kMaxTok, 0, all, &eof);
        if (cgx_text_count(path) != avail) {
            fprintf(stderr, "case %d: count %lld != fscanf's %lld\n", c, (long long)cgx_text_count(path),
                    (long long)avail);
            ++fails;
            continue;
        }
        if (avail > 0) { /* random ranges through the indexed handle (cg_hip's row-block reads) */
            cgx_text *th = NULL;
            if (cgx_text_open(path, 1 + rint_(6), &th) != 0 || cgx_text_available(th, NULL) != avail) {
                fprintf(stderr, "case %d: cgx_text_open / available\n", c);
                ++fails;
            } else {
                for (int rr = 0; rr < 4; ++rr) {
                    const int64_t f0 = rint_((int)avail), cnt = 1 + rint_((int)(avail - f0));
                    double got[4 * kMaxTok];
                    const int rc = cgx_text_read_range(th, f0, cnt, 0, got, 1 + rint_(4));
                    if (rc != 0 || memcmp(got, all + f0, (size_t)cnt * 8) != 0) {
                        fprintf(stderr, "case %d: range [%lld, +%lld) rc %d or values differ\n", c, (long long)f0,
                                (long long)cnt, rc);
                        ++fails;
                        break;
                    }
                }
                double one;
                if (cgx_text_read_range(th, avail, 1, 0, &one, 1) == 0) {
                    fprintf(stderr, "case %d: a range past the last value read\n", c);
                    ++fails;
                }
            }
            cgx_text_close(th);
        }
        const int64_t want = rint_(5) == 0 ? avail + 1 + rint_(3) : 1 + rint_((int)(avail > 0 ? avail : 1));
        for (int as_float = 0; as_float < 2; ++as_float) {
            void *exp = calloc((size_t)want + 1, 8);
            const int64_t got = ref_read(path, want, as_float, exp, &eof);
            const int ref_ok = got == want;
            if (as_float == 0) {
                n_fail += !ref_ok && !eof;
                n_short += !ref_ok && eof;
            }
            for (int threads = 1; threads <= 5; threads += 4) {
                void *out = calloc((size_t)want + 1, 8);
                const int rc = cgx_text_read(path, want, as_float, out, threads);
                int bad = 0;
                if (ref_ok != (rc == 0) || (!ref_ok && rc != -2 && rc != -3)) bad = 1;
                if (rc == 0 && ref_ok)
                    for (int64_t i = 0; i < want; ++i) {
                        const int same = as_float ? !memcmp((float *)out + i, (float *)exp + i, 4)
                                                  : !memcmp((double *)out + i, (double *)exp + i, 8);
                        if (!same) {
                            fprintf(stderr, "case %d value %lld (%s, %d threads): differs from fscanf's\n", c,
                                    (long long)i, as_float ? "float" : "double", threads);
                            bad = 1;
                            break;
                        }
                    }
                if (bad) {
                    fprintf(stderr, "case %d: rc %d, fscanf converted %lld of %lld (%s, %d threads)\n", c, rc,
                            (long long)got, (long long)want, as_float ? "float" : "double", threads);
                    ++fails;
                }
                free(out);
            }
            free(exp);
        }
    }
    unlink(path);
    printf("cases %d failures %d (fscanf failed first %d, short %d, page-end %d, odd separators %d)\n", cases, fails,
           n_fail, n_short, n_page, n_odd);
    return fails ? 1 : 0;
}
