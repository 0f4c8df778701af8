"""The text reader (cgx_textio.c, the replacement for initialize(),
serialConjugate.c:85-105) on randomized files under AddressSanitizer and
UndefinedBehaviorSanitizer: every value bit for bit equal to what the
reference's own loop reads, glibc fscanf(f, "%f%*c") per value (odd single
separators like '-' or a BOM byte consumed by the %*c included); -3 / -2
where that loop fails first (the reference then reads uninitialised memory);
1 and 5 threads; files whose last token ends exactly at a page boundary of
the mapping.  Host-only (tests/native/textio_fuzz.c); no GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed", [1, 2])
def test_text_reader_fuzz_sanitized(tmp_path, seed):
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path / "textio_fuzz")
    build = subprocess.run(
        [cc, "-O1", "-g", "-std=c11", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
         "-I", os.path.join(ROOT, "include"), "-o", exe, os.path.join(ROOT, "tests", "native", "textio_fuzz.c"),
         os.path.join(ROOT, "conjugate_gradient_amd", "csrc", "cgx_textio.c"), "-lpthread", "-lm"],
        capture_output=True, text=True)
    if build.returncode != 0 and "asan" in build.stderr.lower():
        pytest.skip("sanitizer runtime not available: " + build.stderr[-300:])
    assert build.returncode == 0, build.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), "1500", str(seed)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "failures 0" in r.stdout
