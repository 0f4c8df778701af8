"""Builds the test programs under tests/native/ with plain gcc (host code
over the C ABI, as a maintainer of the reference would compile it)."""
import os
import shutil
import subprocess

import pytest

import conjugate_gradient_amd as cg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_conjugrad_dropin(out_dir) -> str:
    """tests/native/conjugrad_dropin.c: INTEGRATION.md s4.1's stub as a program
    -- the reference's serial main with conjugrad() replaced by
    cgx_conjugrad -- against include/ and libcgx.so."""
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not available")
    lib_dir = os.path.dirname(cg.LIB_PATH)
    exe = os.path.join(str(out_dir), "conjugrad_dropin")
    subprocess.run([cc, "-O1", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", exe,
                    os.path.join(ROOT, "tests", "native", "conjugrad_dropin.c"), "-L", lib_dir, "-lcgx",
                    f"-Wl,-rpath,{lib_dir}"], check=True, capture_output=True, text=True)
    return exe
