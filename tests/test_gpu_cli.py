"""The cg_hip program as a drop-in for serialConjugate / parallel_cg: same
argv, same stdout lines, the reference's x with --fp32-ref (bit-exact, via
--print-x), fp64 by default."""
import os
import subprocess

import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle
from _cases import FIX, case, golden_mpi, golden_x, mpi_golden_x

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1


# One device for every cg_hip run here (`--gpus P` puts its row blocks on
# devices g % visible): on a node with several GPUs the distinct-device CLI
# run is tests/test_gpu_multidevice.py's, collected last.
ONE_GPU = dict(os.environ, HIP_VISIBLE_DEVICES="0")


def run(*args, timeout=300):
    r = subprocess.run([cg.CLI_PATH, *args], capture_output=True, text=True, timeout=timeout, env=ONE_GPU)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def printed_x(out, n, dtype):
    lines = out.strip().splitlines()
    return np.array([float(v) for v in lines[-n:]], dtype=dtype)


@pytest.mark.parametrize("name,files", [
    ("kat2", ("matrixA.txt", "vectorb.txt", "initialguess.txt")),
    ("kat2_x0", ("matrixA.txt", "vectorb.txt", "initialguess1.txt")),
    ("kat4", ("matrixA1.txt", "vectorb1.txt", "X0.txt")),
])
def test_cli_fp32ref_reference_fixtures(golden, name, files):
    paths = [os.path.join(FIX, f) for f in files]
    n = golden["cases"][name]["n"]
    out = run("--fp32-ref", "--print-x", "--stats", *paths)
    assert f"Computing cg of matrix size : {n * n}" in out          # serialConjugate.c:58
    assert "average clock execution time in seconds:" in out        # serialConjugate.c:250
    assert f"iterations: {golden['cases'][name]['ref_iterations']} converged: 1" in out
    x = printed_x(out, n, np.float32)   # %.9g round-trips a float exactly
    assert np.array_equal(x.view(np.uint32), golden_x(golden, name).view(np.uint32))


def test_cli_full_teardown_same_output(golden, tmp_path):
    """The default fast exit (no teardown after the output is flushed) and the
    full teardown (CGX_CLI_FAST_EXIT=0), with A in huge pages (default) or
    malloc'd (CGX_CLI_HUGEPAGES=0), print the same x and exit 0; the phase
    line reports which ran.  Stdout to a file checks the flush before
    _exit."""
    paths = [os.path.join(FIX, f) for f in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    outs = {}
    for mode in ("1", "0"):
        dst = tmp_path / f"out{mode}.txt"
        with open(dst, "w") as f:
            r = subprocess.run([cg.CLI_PATH, "--fp32-ref", "--print-x", "--stats", *paths], stdout=f,
                               stderr=subprocess.PIPE, text=True, timeout=300,
                               env=dict(ONE_GPU, CGX_CLI_FAST_EXIT=mode, CGX_CLI_HUGEPAGES=mode, CGX_CLI_TIMES="1"))
        assert r.returncode == 0, r.stderr
        assert f'"fast_exit": {mode}' in r.stderr
        outs[mode] = dst.read_text().splitlines()
    assert len(outs["1"]) == len(outs["0"]) and outs["1"][-4:] == outs["0"][-4:]
    assert np.array_equal(printed_x("\n".join(outs["1"]), 4, np.float32).view(np.uint32),
                          golden_x(golden, "kat4").view(np.uint32))


def test_cli_dims_file_and_fp64(golden):
    paths = [os.path.join(FIX, f) for f in ("matrixA.txt", "vectorb.txt", "initialguess.txt")]
    out = run("--dims", os.path.join(FIX, "dimensions.txt"), "--eps", "1e-12", "--print-x", *paths)
    x = printed_x(out, 2, np.float64)
    assert np.allclose(x, [2 / 3, 1 / 3], rtol=0, atol=1e-12)


def test_cli_generated_text_files_multi_gpu(golden, tmp_path):
    """generateSPDmatrix(512) written as the MATLAB script writes it; the
    parallel_cg.c-style run (--gpus 2: two row blocks) prints its lines."""
    n = 512
    A, b = oracle.spd_matlab(n, np.float64)
    for name, arr, dec in (("A.txt", A, 4), ("b.txt", b, 4), ("x0.txt", np.zeros(n), 1)):
        oracle.write_text(str(tmp_path / name), arr, dec)
    paths = [str(tmp_path / f) for f in ("A.txt", "b.txt", "x0.txt")]
    out = run("--fp32-ref", "--print-x", *paths)
    x = printed_x(out, n, np.float32)
    assert np.array_equal(x.view(np.uint32), golden_x(golden, "spd512").view(np.uint32))
    out2 = run("--gpus", "2", "--stats", "--eps", "1e-10", "--print-x", *paths)
    for line in ("cg method execution time in seconds:", "collective data distribution time in seconds:",
                 "clock execution time in seconds:"):
        assert line in out2                                        # parallel_cg.c:123-126, :334
    x2 = printed_x(out2, n, np.float64)
    A64, b64, x064 = case("spd512", np.float64)
    xo, _ = oracle.cg_f64(A64, b64, x064, eps=1e-10)
    assert np.linalg.norm(x2 - xo) <= 1e-10 * np.linalg.norm(xo)
    # --symmetric: the same files, only the upper-triangle tiles kept
    out3 = run("--symmetric", "--stats", "--eps", "1e-10", "--print-x", *paths)
    x3 = printed_x(out3, n, np.float64)
    assert np.linalg.norm(x3 - xo) <= 1e-10 * np.linalg.norm(xo)
    r = subprocess.run([cg.CLI_PATH, "--symmetric", "--fp32-ref", *paths], capture_output=True, text=True, env=ONE_GPU)
    assert r.returncode == 2


def test_cli_synthetic_spd():
    out = run("--spd", "4096", "--stats", "--eps", "1e-10")
    assert "Computing cg of matrix size : 16777216" in out
    it = int(out.split("iterations:")[1].split()[0])
    assert 3 <= it <= 20 and "converged: 1" in out


def _spd512_files(tmp_path):
    n = 512
    A, b = oracle.spd_matlab(n, np.float64)
    for name, arr, dec in (("A.txt", A, 4), ("b.txt", b, 4), ("x0.txt", np.zeros(n), 1)):
        oracle.write_text(str(tmp_path / name), arr, dec)
    return n, [str(tmp_path / f) for f in ("A.txt", "b.txt", "x0.txt")]


@pytest.mark.parametrize("args", [("--fp32-ref",), ("--gpus", "2", "--fp32-ref"), ("--eps", "1e-10"),
                                  ("--gpus", "2", "--eps", "1e-10"), ("--symmetric", "--eps", "1e-10")])
def test_cli_streamed_a_equals_materialized(golden, tmp_path, args):
    """A streamed to the device in ragged row blocks (25 rows of 512: 21
    blocks, the last 12 rows) through a ring of 3 slots, so the parse wraps
    the ring, waits for free slots and the copy side merges runs of parsed
    blocks: the same x, bit for bit, as A parsed whole and sent in one copy
    (CGX_CLI_STREAM=0), and the reference's x for --fp32-ref
    (serialConjugate.c's on one GPU, parallel_cg.c's at np=2 on two)."""
    n, paths = _spd512_files(tmp_path)
    es = 4 if "--fp32-ref" in args else 8
    block_mb = 25 * n * es / 1048576
    outs = {}
    for mode, extra in (("stream", {"CGX_CLI_BLOCK_MB": repr(block_mb), "CGX_CLI_RING_MB": repr(3 * block_mb)}),
                        ("whole", {"CGX_CLI_STREAM": "0"})):
        r = subprocess.run([cg.CLI_PATH, *args, "--print-x", "--stats", *paths], capture_output=True, text=True,
                           timeout=300, env=dict(ONE_GPU, CGX_CLI_TIMES="1", **extra))
        assert r.returncode == 0, r.stdout + r.stderr
        assert f'"streamed": {int(mode == "stream")}' in r.stderr
        outs[mode] = r.stdout
    dt = np.float32 if es == 4 else np.float64
    xs, xw = printed_x(outs["stream"], n, dt), printed_x(outs["whole"], n, dt)
    assert np.array_equal(xs, xw)
    if es == 4:
        ref = golden_x(golden, "spd512") if "--gpus" not in args else mpi_golden_x("parallel_spd512_np2")
        assert np.array_equal(xs.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("cut", ["short", "bad"])
def test_cli_streamed_a_bad_file_fails(tmp_path, cut):
    """A truncated A, or one whose last block holds a value fscanf("%f")
    cannot read, stops the streamed run with the reader's message and exit 1
    (the index pass over the file finds it before any block is parsed)."""
    n, paths = _spd512_files(tmp_path)
    lines = open(paths[0]).read().splitlines()
    lines = lines[:-7] if cut == "short" else lines[:-7] + ["abc"] + lines[-6:]
    with open(paths[0], "w") as f:
        f.write("\n".join(lines) + "\n")
    r = subprocess.run([cg.CLI_PATH, "--fp32-ref", *paths], capture_output=True, text=True, timeout=300,
                       env=dict(ONE_GPU, CGX_CLI_BLOCK_MB=repr(25 * n * 4 / 1048576)))
    assert r.returncode == 1
    assert ("fewer than" if cut == "short" else "malformed number") in r.stderr


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("program", ["parallel", "p2p"])
def test_cli_gpus_equals_mpi_programs(tmp_path, program, P):
    """`cg_hip --gpus P [--p2p] --fp32-ref` in one process == `mpiexec -np P`
    of the unmodified parallel_cg.c / point-to-point_cg.c on the same files:
    x bit for bit, the loop count, and each program's lines in its order (cg
    time, then its distribution time, then the clock time)."""
    n, paths = _spd512_files(tmp_path)
    key = f"{program}_spd512_np{P}"
    out = run("--gpus", str(P), *(["--p2p"] if program == "p2p" else []), "--fp32-ref", "--print-x", "--stats", *paths)
    dist = "p2p" if program == "p2p" else "collective"  # point-to-point_cg.c:133 / parallel_cg.c:123
    lines = [ln.split(":")[0] for ln in out.splitlines() if "time in seconds:" in ln]
    assert lines == ["cg method execution time in seconds", f"{dist} data distribution time in seconds",
                     "clock execution time in seconds"], lines
    assert f"iterations: {golden_mpi()['runs'][key]['ref_iterations']} converged: 1" in out
    x = printed_x(out, n, np.float32)
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


@pytest.mark.parametrize("name,files", [
    ("kat2", ("matrixA.txt", "vectorb.txt", "initialguess.txt")),
    ("kat4", ("matrixA1.txt", "vectorb1.txt", "X0.txt")),
])
def test_conjugrad_dropin_program(golden, tmp_path, name, files):
    """The function-level drop-in: the reference's serial
    main with `conjugrad(A, b, x)` replaced by one cgx_conjugrad call gives
    serialConjugate.c's x bit for bit and its loop count."""
    from _native import build_conjugrad_dropin
    exe = build_conjugrad_dropin(tmp_path)
    n = golden["cases"][name]["n"]
    r = subprocess.run([exe, str(n), *[os.path.join(FIX, f) for f in files]], capture_output=True, text=True,
                       timeout=120, env=ONE_GPU)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"iterations: {golden['cases'][name]['ref_iterations']} converged: 1" in r.stdout
    x = printed_x(r.stdout, n, np.float32)
    assert np.array_equal(x.view(np.uint32), golden_x(golden, name).view(np.uint32))


def test_conjugrad_dropin_generated_spd512(golden, tmp_path):
    """The same program on generateSPDmatrix(512) written as the MATLAB script
    writes it."""
    from _native import build_conjugrad_dropin
    exe = build_conjugrad_dropin(tmp_path)
    n, paths = _spd512_files(tmp_path)
    r = subprocess.run([exe, str(n), *paths], capture_output=True, text=True, timeout=120, env=ONE_GPU)
    assert r.returncode == 0, r.stdout + r.stderr
    x = printed_x(r.stdout, n, np.float32)
    assert np.array_equal(x.view(np.uint32), golden_x(golden, "spd512").view(np.uint32))
