/*
 * cgx_textio.h -- reader for the reference's text formats (host C).
 *
 * Replaces initialize() (serialConjugate.c:85-105, parallel_cg.c:147-168):
 * reads value after value exactly as the reference's fscanf("%f%*c") loop
 * does (white space skipped, the longest prefix glibc's %f accepts, then one
 * more byte consumed whatever it is): A row-major, b and x0 one entry per
 * line, and dimensions.txt ("rows cols" of A then of b).  Differences, by
 * design: a missing file, a short file, or a requested
 * value at or after a failing conversion is an error instead of silently
 * leaving uninitialised memory (serialConjugate.c:101-104), and N is taken
 * at run time instead of from `#define ROWS`.
 */
#ifndef CGX_TEXTIO_H
#define CGX_TEXTIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Counts the numbers the reference's loop would convert before its first
 * failing conversion or end of file.  Returns -1 if it cannot be opened. */
int64_t cgx_text_count(const char *path);

/* Reads exactly `count` numbers (the first `count` in the file) into out
 * (float if as_float, else double: strtof / strtod of the characters %f
 * takes).  0 on success; -1 cannot open; -2 fewer than `count` numbers; -3 a
 * conversion fails before `count` numbers.  `threads` > 1 parses in parallel
 * slices cut at white space (same values). */
int cgx_text_read(const char *path, int64_t count, int as_float, void *out, int threads);

/* The same reader on an opened, indexed file, for reading it in ranges
 * (cg_hip streams A to the GPU row block by row block this way):
 * cgx_text_open maps the file and counts its numbers in ~1 MiB pieces on
 * `threads` threads (0, or -1 cannot open); cgx_text_available gives how many
 * the reference's loop would convert (*stopped = 1 if a failing conversion
 * ends them, 0 if end of file); cgx_text_read_range parses numbers
 * [first, first + count) into out[0 .. count) from the pieces that hold them
 * (0, -2 / -3 as cgx_text_read).  A handle is read-only once open: ranges
 * may be read from several threads at once. */
typedef struct cgx_text cgx_text;
int cgx_text_open(const char *path, int threads, cgx_text **t);
int64_t cgx_text_available(const cgx_text *t, int *stopped);
int cgx_text_read_range(cgx_text *t, int64_t first, int64_t count, int as_float, void *out, int threads);
void cgx_text_close(cgx_text *t);

/* dimensions.txt: four integers "A_rows A_cols b_rows b_cols".  0 or <0. */
int cgx_text_dims(const char *path, int64_t dims[4]);

#ifdef __cplusplus
}
#endif
#endif
