"""cg_mpi, the one-process-per-GPU drop-in for `mpiexec -np P ./parallel_cg`
(and `./point-to-point_cg` with --p2p), launched by MPICH's mpiexec as the
reference is.  All ranks share the box's one GPU: each gets its own
NCCL_HOSTID (MPMD blocks of mpiexec), so RCCL carries the exchange over its
socket transport.  With --fp32-ref the printed x must equal the unmodified
MPI programs' x from `mpiexec -np P` on the same files bit for bit
(tests/golden/mpi/)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle
from _cases import FIX, case, golden_mpi, mpi_golden_x

pytestmark = pytest.mark.gpu

MPIEXEC = "/opt/conda/bin/mpiexec"
CG_MPI = os.path.join(os.path.dirname(cg.CLI_PATH), "cg_mpi")


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1
    if not (os.path.exists(MPIEXEC) and os.path.exists(CG_MPI)):
        pytest.skip("MPICH mpiexec or bin/cg_mpi absent")


def run_mpi(nranks, *args, timeout=240):
    cmd = [MPIEXEC]
    for r in range(nranks):
        if r:
            cmd.append(":")
        # every rank on device 0 (CGX_DEVICE), also on a node with several GPUs: the one-rank-per-GPU
        # cg_mpi run is tests/test_gpu_multidevice.py's, collected last
        cmd += ["-np", "1", "-env", "NCCL_HOSTID", f"cgx-mpi-host-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                "-env", "NCCL_IB_DISABLE", "1", "-env", "CGX_RCCL_TIMEOUT_S", "120", "-env", "CGX_DEVICE", "0",
                CG_MPI, *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def printed_x(out, n, dtype):
    return np.array([float(v) for v in out.strip().splitlines()[-n:]], dtype=dtype)


@pytest.fixture(scope="module")
def spd512_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("spd512")
    A, b = oracle.spd_matlab(512, np.float64)
    for name, arr, dec in (("A.txt", A, 4), ("b.txt", b, 4), ("x0.txt", np.zeros(512), 1)):
        oracle.write_text(str(d / name), arr, dec)
    return [str(d / f) for f in ("A.txt", "b.txt", "x0.txt")]


@pytest.mark.parametrize("program", ["parallel", "p2p"])
@pytest.mark.parametrize("nranks", [2, 4])
def test_cg_mpi_fp32ref_equals_mpi_programs(spd512_files, program, nranks):
    """generateSPDmatrix(512) files: parallel_cg.c's x (MPICH's MPI_Allreduce
    order) and point-to-point_cg.c's (--p2p, allSum's rank order), with the
    loop count."""
    key = f"{program}_spd512_np{nranks}"
    args = ["--fp32-ref", "--print-x", "--stats"] + (["--p2p"] if program == "p2p" else []) + spd512_files
    out = run_mpi(nranks, *args)
    assert "Computing cg of matrix size : 262144" in out      # parallel_cg.c:101, point-to-point_cg.c:116
    # each program's own lines, in its order: cg time (printed by conjugrad),
    # then the distribution time, then the clock time
    dist = "p2p" if program == "p2p" else "collective"  # point-to-point_cg.c:133 / parallel_cg.c:123
    lines = [ln for ln in out.splitlines() if "time in seconds:" in ln]
    assert [ln.split(":")[0] for ln in lines] == ["cg method execution time in seconds",
                                                 f"{dist} data distribution time in seconds",
                                                 "clock execution time in seconds"], lines
    assert ("collective" if program == "p2p" else "p2p") + " data distribution" not in out
    assert all(float(ln.split(":")[1]) >= 0 for ln in lines)
    assert f"iterations: {golden_mpi()['runs'][key]['ref_iterations']} converged: 1" in out
    x = printed_x(out, 512, np.float32)
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


def test_cg_mpi_reference_fixture_kat4_np2():
    """The reference's own 4x4 fixture (matrixA1.txt, vectorb1.txt, X0.txt) at np=2."""
    paths = [os.path.join(FIX, f) for f in ("matrixA1.txt", "vectorb1.txt", "X0.txt")]
    out = run_mpi(2, "--fp32-ref", "--print-x", *paths)
    x = printed_x(out, 4, np.float32)
    assert np.array_equal(x.view(np.uint32), mpi_golden_x("parallel_kat4_np2").view(np.uint32))


def test_cg_mpi_fp64_np2_against_oracle(spd512_files):
    out = run_mpi(2, "--eps", "1e-10", "--print-x", "--stats", *spd512_files)
    x = printed_x(out, 512, np.float64)
    A, b, x0 = case("spd512", np.float64)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert f"iterations: {so.iterations} converged: 1" in out
    assert np.linalg.norm(x - xo) <= 1e-10 * np.linalg.norm(xo)
