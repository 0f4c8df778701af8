/*
 * cgx_textio.h -- reader for the reference's text formats (host C).
 *
 * Replaces initialize() (serialConjugate.c:85-105, parallel_cg.c:147-168):
 * one number per line (any single separator after each number is accepted,
 * like fscanf("%f%*c")), A row-major, b and x0 one entry per line, and
 * dimensions.txt ("rows cols" of A then of b).  Differences, by design: a
 * missing file or a short / malformed file is an error instead of silently
 * leaving uninitialised memory (serialConjugate.c:101-104), and N is taken at
 * run time instead of from `#define ROWS`.
 */
#ifndef CGX_TEXTIO_H
#define CGX_TEXTIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Counts the numbers in a text file.  Returns -1 if it cannot be opened. */
int64_t cgx_text_count(const char *path);

/* Reads exactly `count` numbers (the first `count` in the file) into out
 * (float if as_float, else double).  0 on success; -1 cannot open; -2 fewer
 * than `count` numbers; -3 malformed token.  `threads` > 1 parses in
 * parallel chunks (same values: every token is converted independently). */
int cgx_text_read(const char *path, int64_t count, int as_float, void *out, int threads);

/* dimensions.txt: four integers "A_rows A_cols b_rows b_cols".  0 or <0. */
int cgx_text_dims(const char *path, int64_t dims[4]);

#ifdef __cplusplus
}
#endif
#endif
