"""The C-ABI boundary (include/*.h -> lib/libcgx.so) and the host-side pieces
that need no GPU: symbol exports, error reporting, the text reader, the CLI's
argument / file handling."""
import os
import re
import subprocess

import numpy as np
import pytest

import conjugate_gradient_amd as cg
from _cases import FIX, numbers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("cgx.h", "cgx_textio.h")]


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(cgx_\w+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_exported(built):
    out = subprocess.run(["nm", "-D", "--defined-only", cg.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(cgx_\w+)$", out, flags=re.M))
    declared = [f for h in HEADERS for f in declared_functions(h)]
    assert len(declared) >= 35
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    L = cg.lib()
    for f in declared:
        assert hasattr(L, f)


def test_library_links_hip_loads_rccl_on_demand(built):
    """libcgx links the HIP runtime; RCCL is dlopen'ed by rank mode only
    (cgx_rccl.hip), so single-GPU processes do not pay for loading it."""
    out = subprocess.run(["readelf", "-d", cg.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "libamdhip64.so" in out and "librccl.so" not in out
    undef = subprocess.run(["nm", "-D", "--undefined-only", cg.LIB_PATH], capture_output=True, text=True,
                           check=True).stdout
    assert " nccl" not in undef


def test_rccl_loads_on_first_rank_call(built, monkeypatch):
    """cgx_get_unique_id loads RCCL: with a GPU it returns an id; without one
    (this container) RCCL itself reports the error -- never a load failure."""
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    try:
        assert len(cg.get_unique_id()) == 128
    except cg.CgxError as e:
        assert "RCCL error" in str(e) and "cannot load RCCL" not in str(e), str(e)


def test_rccl_entry_points_resolve(built):
    """cgx_rccl_available: librccl.so.1 loads (no GPU needed) and every entry
    point rank mode calls -- init, the collectives, send/recv, groups, and the
    fail-fast pair ncclCommGetAsyncError / ncclCommAbort -- resolves; a
    missing one fails here, not on the GPU box."""
    rc = cg.lib().cgx_rccl_available()
    assert rc == 0, cg.lib().cgx_last_error().decode()


def test_python_mirror_checks_sizes_before_the_c_call():
    """Short or mis-shaped host arrays raise ValueError in the mirror; they
    never reach cgx_set_rows / cgx_solve (which would read or write n
    elements).  No context is needed to get there, so this runs without a GPU."""
    s = cg.Solver.__new__(cg.Solver)
    s.n, s.dtype, s.flags, s._h = 8, np.dtype(np.float64), cg.CGX_F64, None
    A, b = np.eye(8), np.ones(8)
    with pytest.raises(ValueError, match="x0"):
        s.set_system(A, b, np.zeros(7))
    with pytest.raises(ValueError, match="A has shape"):
        s.set_system(np.eye(7), b)
    with pytest.raises(ValueError, match="b has shape"):
        s.set_system(A, np.ones(9))
    with pytest.raises(ValueError, match="x0 has shape"):
        s.solve(np.zeros(5))
    with pytest.raises(ValueError, match="x has shape"):
        s.set_x(np.zeros(3))
    with pytest.raises(ValueError, match="same 2 rows"):
        s.set_rows(0, np.ones((2, 8)), np.ones(3))
    with pytest.raises(ValueError, match="nrows, >= 8"):
        s.set_rows(0, np.ones((2, 5)))
    with pytest.raises(ValueError, match="outside"):
        s.set_rows(6, None, np.ones(3))
    d = cg.DeviceArray.__new__(cg.DeviceArray)
    d.count, d.dtype, d.ptr = 4, np.dtype(np.float64), None
    with pytest.raises(ValueError, match="matVec A"):
        cg.matVec(d, d, d, rows=4, cols=4)
    with pytest.raises(ValueError, match="vecVec"):
        cg.vecVec(d, d, d, n=5)


def test_gfx950_code_object(built):
    # the HIP kernels are compiled for gfx950 (offload bundle inside the .so)
    data = open(cg.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_matvec_f64" in data and b"k_matvec_ref_f32" in data


def test_errors_and_version(built):
    L = cg.lib()
    assert L.cgx_version() == 101
    assert L.cgx_strerror(0) == b"ok"
    for code in (-1, -2, -3, -4, -5, -6, -7):
        assert L.cgx_strerror(code) not in (b"ok", b"unknown error")
    assert L.cgx_strerror(-99) == b"unknown error"


def test_no_gpu_fails_loudly(built):
    if cg.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(cg.CgxError) as ei:
        cg.Solver(4)
    assert ei.value.code == -7 and "no HIP device" in str(ei.value)


def test_bad_shape_rejected_before_device(built):
    # n % P != 0 (parallel_cg.c:86-90) is a shape error whatever the devices
    with pytest.raises(cg.CgxError) as ei:
        cg.Solver(10, devices=[0, 0, 0])
    assert ei.value.code == -4 and "not divisible" in str(ei.value)


def test_text_reader_reference_fixtures(built):
    A = cg.read_text(os.path.join(FIX, "matrixA1.txt"), 16, np.float32)
    assert np.array_equal(A, numbers("matrixA1.txt", 16))
    assert cg.count_text(os.path.join(FIX, "vectorb.txt")) == 2
    assert cg.read_dims(os.path.join(FIX, "dimensions.txt")) == (2, 2, 2, 1)
    # initialguess1.txt ends in a stray UTF-8 BOM: its first byte is the %*c
    # after 0.0, so the two values read (and a third conversion would fail)
    x = cg.read_text(os.path.join(FIX, "initialguess1.txt"), 2, np.float64)
    assert np.array_equal(x, [1.0, 0.0])
    assert cg.count_text(os.path.join(FIX, "initialguess1.txt")) == 2


_INIT_CASES = {
    # the reference's own fixtures (copied data)
    **{name: None for name in ("matrixA.txt", "vectorb.txt", "initialguess.txt", "initialguess1.txt",
                               "matrixA1.txt", "vectorb1.txt", "X0.txt", "dimensions.txt")},
    # separators and edge cases of fscanf("%f%*c")
    "crlf": b"1.5\r\n-2.25\r\n3e2\r\n",
    "minus_eaten": b"1.5-2.0\n4\n",            # %*c eats the '-': 1.5, 2.0, 4
    "dot_eaten": b"1.2.3\n",                   # 1.2, then '.' eaten, 3
    "bom_front": b"\xef\xbb\xbf1.0\n2.0\n",  # the first conversion fails
    "bom_trailing": b"1.0\n0.0\xef\xbb\xbf\n",  # initialguess1.txt's shape
    "trailing_junk": b"1\n2\njunk\n",
    "short": b"7\n",
    "double_comma": b"1.0,,2.0\n",
    "exp_no_digits": b"1e+\n2\n",              # glibc takes "1e+" as 1
    "nan_paren": b"nan(1)\n5\n",               # "nan", '(' eaten, then "1)" -> 1, ')' eaten
    "tabs_spaces": b"  \t 1.25 \t\n\n -0 \n",
    "no_final_newline": b"4\n5",
    "inf_forms": b"inf\nINFINITY\n-Inf\ninfinit\n",
    "hex": b"0x1p3\n0x.p1\n",
}


@pytest.mark.parametrize("name", sorted(_INIT_CASES))
def test_text_reader_pinned_to_reference_initialize(built, tmp_path, name):
    """cgx_text_read against the reference's own initialize()
    (serialConjugate.c:85-105, fscanf "%f%*c" per value), run through the
    unmodified reference (oracle/_ref/serial_ref --initialize, its buffer
    pre-filled with a sentinel so the values it assigned are known).  The
    values it assigns are read bit for bit; where it stops assigning (a
    failing conversion, end of file) cgx_text_read returns an error instead
    of leaving uninitialised values -- the one deliberate divergence."""
    import oracle
    exe = oracle.ref_binary()
    if not exe:
        pytest.skip("oracle/_ref/serial_ref not built (no /root/reference here)")
    data = _INIT_CASES[name]
    path = os.path.join(FIX, name) if data is None else str(tmp_path / f"{name}.txt")
    if data is not None:
        with open(path, "wb") as f:
            f.write(data)
    out = str(tmp_path / "ref.f32")
    r = subprocess.run([exe, "--initialize", path, "1", out], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    ref = np.fromfile(out, dtype=np.uint32)
    unset = np.flatnonzero(ref == 0x7FA5A5A5)
    k = int(unset[0]) if unset.size else ref.size
    assert (ref[k:] == 0x7FA5A5A5).all()  # the reference assigns a prefix, then nothing
    if k:
        got = cg.read_text(path, k, np.float32)
        assert np.array_equal(got.view(np.uint32), ref[:k]), (got, ref[:k].view(np.float32))
        assert cg.count_text(path) == k
    with pytest.raises(ValueError):
        cg.read_text(path, k + 1, np.float32)


def test_text_reader_errors(built, tmp_path):
    with pytest.raises(FileNotFoundError):
        cg.read_text(str(tmp_path / "missing.txt"), 2)
    p = tmp_path / "short.txt"
    p.write_text("1.0\n2.0\n")
    with pytest.raises(ValueError, match="fewer"):
        cg.read_text(str(p), 3)
    p.write_text("1.0\nabc\n")
    with pytest.raises(ValueError, match="malformed"):
        cg.read_text(str(p), 2)


def test_text_reader_parallel_equals_serial(built, tmp_path):
    rng = np.random.default_rng(1)
    vals = rng.random(50000) * 1e3 - 500
    p = tmp_path / "big.txt"
    p.write_text("\n".join(f"{v:.4f}" for v in vals) + "\n")
    one = cg.read_text(str(p), vals.size, np.float32, threads=1)
    many = cg.read_text(str(p), vals.size, np.float32, threads=7)
    assert np.array_equal(one, many)
    # strtof of the "%.4f" text, as fscanf("%f") does (serialConjugate.c:96)
    assert np.array_equal(one, np.array([np.float32(f"{v:.4f}") for v in vals]))
    d = cg.read_text(str(p), vals.size, np.float64, threads=5)
    assert np.array_equal(d, np.array([float(f"{v:.4f}") for v in vals]))


def run_cli(*args):
    return subprocess.run([cg.CLI_PATH, *args], capture_output=True, text=True, timeout=120)


def _cg_mpi():
    exe = os.path.join(os.path.dirname(cg.CLI_PATH), "cg_mpi")
    if not (os.path.exists("/opt/conda/bin/mpiexec") and os.path.exists(exe)):
        pytest.skip("MPICH mpiexec or bin/cg_mpi absent")
    return exe


def test_cg_mpi_rejects_indivisible_n_and_bad_options(built):
    """cg_mpi's checks before any GPU work, under mpiexec as the reference runs."""
    exe = _cg_mpi()
    paths = [os.path.join(FIX, f) for f in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-np", "3", exe, *paths], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "4 is not divisible by 3" in r.stdout  # parallel_cg.c:88
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-np", "2", exe, "--eps", "x", *paths], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "usage: mpiexec -np P cg_mpi" in r.stderr
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-np", "2", exe, str(FIX) + "/nope.txt", paths[1], paths[2]],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "Could not open file\n" in r.stdout  # initialize(), parallel_cg.c:166


def test_cg_mpi_p2p_keeps_point_to_point_cg_texts(built):
    """--p2p speaks point-to-point_cg.c's error texts, not parallel_cg.c's:
    "%d must be divisible by %d" (:101) and scatterRow's "Could not open %s
    file. " for A and b (:226); x0 goes through initialize() (:177)."""
    exe = _cg_mpi()
    paths = [os.path.join(FIX, f) for f in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    run = lambda np_, *a: subprocess.run(["/opt/conda/bin/mpiexec", "-np", str(np_), exe, "--p2p", *a],
                                         capture_output=True, text=True, timeout=120)
    r = run(3, *paths)
    assert r.returncode != 0 and "4 must be divisible by 3\n" in r.stdout and "is not divisible" not in r.stdout
    nope = str(FIX) + "/nope.txt"
    r = run(2, nope, paths[1], paths[2])
    assert r.returncode != 0 and f"Could not open {nope} file. \n" in r.stdout
    r = run(2, paths[0], paths[1], nope)
    assert r.returncode != 0 and "Could not open file\n" in r.stdout and "nope.txt file" not in r.stdout


def test_cli_argument_count(built):
    r = run_cli()
    assert r.returncode == 1
    assert "serialCongugate.c requires four (4) files" in r.stdout  # serialConjugate.c:50


def test_cli_missing_file(built, tmp_path):
    r = run_cli(str(tmp_path / "nope.txt"), os.path.join(FIX, "vectorb.txt"), os.path.join(FIX, "initialguess.txt"))
    assert r.returncode == 1
    assert "Computing cg of matrix size : 4" in r.stdout
    assert "Could not open file" in r.stdout  # serialConjugate.c:103


def test_cli_not_divisible(built):
    f = [os.path.join(FIX, n) for n in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    r = run_cli("--gpus", "3", *f)
    assert r.returncode == 1 and "4 is not divisible by 3" in r.stdout  # parallel_cg.c:88


@pytest.mark.parametrize("opt,val", [("--eps", "abc"), ("--gpus", "2x"), ("--n", "12.5"), ("--max-iter", ""),
                                     ("--seed", "0x"), ("--threads", "four")])
def test_cli_rejects_non_numeric_options(built, opt, val):
    f = [os.path.join(FIX, n) for n in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    r = run_cli(opt, val, *f)
    assert r.returncode == 2 and opt in r.stderr, r.stdout + r.stderr


def test_cli_dims_file(built, tmp_path):
    d = tmp_path / "dims.txt"
    d.write_text("3\n2\n3\n1\n")
    f = [os.path.join(FIX, n) for n in ("matrixA.txt", "vectorb.txt", "initialguess.txt")]
    r = run_cli("--dims", str(d), *f)
    assert r.returncode == 1 and "3 and 2 must be same size" in r.stdout  # serialConjugate.c:55


def test_text_reader_matches_libc_conversion(built, tmp_path):
    """The exact fast path + fallback reproduces strtof / strtod bit for bit,
    including decimals that sit next to float rounding midpoints."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.strtof.restype = ctypes.c_float
    libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    libc.strtod.restype = ctypes.c_double
    libc.strtod.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    rng = np.random.default_rng(7)
    toks = []
    for _ in range(20000):
        digits = int(rng.integers(1, 20))
        mant = "".join(str(d) for d in rng.integers(0, 10, digits))
        dot = int(rng.integers(0, digits + 1))
        s = mant[:dot] + "." + mant[dot:] if dot < digits else mant
        if rng.random() < 0.3:
            s += f"e{int(rng.integers(-30, 31))}"
        if rng.random() < 0.5:
            s = "-" + s
        toks.append(s)
    # decimals within a few double ulps of float midpoints, 17-19 significant digits
    f = rng.random(3000).astype(np.float32) * np.float32(1000)
    g = np.nextafter(f, np.float32(np.inf))
    for a, b in zip(f.astype(np.float64), g.astype(np.float64)):
        mid = (a + b) / 2
        for nd in (17, 18, 19):
            toks.append(f"{mid:.{nd}g}")
            toks.append(f"{np.nextafter(mid, np.inf):.{nd}g}")
    toks += ["0", "-0.0", "0.0000", "1e22", "1e23", "3.4028235e38", "1e-40", "9007199254740993", "4.9e-324",
             "inf", "-nan", "0x1p3", ".5", "5.", "+7"]
    p = tmp_path / "mix.txt"
    p.write_text("\n".join(toks) + "\n")
    got32 = cg.read_text(str(p), len(toks), np.float32, threads=3)
    got64 = cg.read_text(str(p), len(toks), np.float64, threads=3)
    for i, t in enumerate(toks):
        e32 = np.float32(libc.strtof(t.encode(), None))
        e64 = libc.strtod(t.encode(), None)
        if np.isnan(e32):
            assert np.isnan(got32[i]) and np.isnan(got64[i]), t
            continue
        assert got32[i].view(np.uint32) == e32.view(np.uint32), (t, got32[i], e32)
        assert np.float64(got64[i]).view(np.uint64) == np.float64(e64).view(np.uint64), (t, got64[i], e64)


def test_flag_constants_match_header():
    """The Python mirror's CGX_* flag and error values are the header's."""
    import re
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cgx.h")) as f:
        hdr = dict((m.group(1), int(m.group(2), 0)) for m in re.finditer(r"#define\s+(CGX_[A-Z0-9_]+)\s+(-?0x[0-9a-fA-F]+|-?\d+)", f.read()))
    names = [k for k in dir(cg) if k.startswith("CGX_")]
    assert names
    for k in names:
        assert k in hdr and getattr(cg, k) == hdr[k], k


def test_phase_indices_match_header():
    """cgx_phase_times' index order (CGX_PH_*) is the mirror's PHASE_NAMES order,
    and the mirror's structs have the header's sizes."""
    import ctypes
    with open(os.path.join(ROOT, "include", "cgx.h")) as f:
        src = f.read()
    idx = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define\s+CGX_PH_([A-Z_]+)\s+(\d+)", src)}
    count = idx.pop("count")
    assert count == len(cg.PHASE_NAMES) == len(idx)
    assert [n for n, _ in sorted(idx.items(), key=lambda kv: kv[1])] == list(cg.PHASE_NAMES)
    assert ctypes.sizeof(cg.PhaseTimes) == 8 * 3 * count
    assert ctypes.sizeof(cg.CommInfo) == 4 * 4 + 32


def test_device_queries_without_a_gpu_fail_cleanly(built):
    """cgx_device_link / cgx_device_pci_bus_id return an error code (no
    abort) when the device does not exist."""
    if cg.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(cg.CgxError):
        cg.device_link(0, 1)
    with pytest.raises(cg.CgxError):
        cg.device_pci_bus_id(0)


def test_conjugrad_dropin_builds_and_checks_arguments(built, tmp_path):
    """The one-call drop-in compiles and links as a maintainer would write it;
    without a GPU (or with a NULL array) it returns an error code instead of
    aborting."""
    from _native import build_conjugrad_dropin
    exe = build_conjugrad_dropin(tmp_path)
    assert os.path.exists(exe)
    L = cg.lib()
    assert L.cgx_conjugrad(None, None, None, 4, cg.CGX_F32_REF, 1e-6, -1, None) == -1  # CGX_ERR_ARG
    if cg.device_count() == 0:
        import numpy as np
        A = np.eye(4, dtype=np.float32)
        b = np.ones(4, np.float32)
        x = np.zeros(4, np.float32)
        assert L.cgx_conjugrad(A.ctypes.data, b.ctypes.data, x.ctypes.data, 4, cg.CGX_F32_REF, 1e-6, -1,
                               None) == -7  # CGX_ERR_NODEV
