"""Row blocks on distinct GPUs: the paths a one-GPU box cannot execute.

Everything else in the suite puts every row block (or rank) on device 0.
These tests run where two or more GPUs are visible -- the driver's 8-GPU
node -- and are skipped with the reason otherwise:

  * cgx_create_multi over devices 0..G-1 (G = min(8, visible)): the pull
    kernels read the other devices' p slices and scalar partials over xGMI
    with system-scope loads after the producers' events; the threaded
    enqueue (CGX_LOCAL_THREADS=1, one host thread per device); the folded
    and separate scalar combines; the per-pair peer copies.  Each must give
    x bit for bit equal to the same partition on one device ([0] * G),
    overlapped and plain, gated and fixed-count.
  * the rank path with one process per GPU (parallel_cg.c's one MPI rank per
    process, :109-117 and :288-324): RCCL over xGMI between distinct devices,
    x within 1e-10 of the fp64 oracle with conjgrad.m's loop count.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-10


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def gpus() -> int:
    return min(8, cg.device_count())


def visible() -> int:
    try:
        return cg.device_count()
    except cg.CgxError:
        return 0


needs_two = pytest.mark.skipif("visible() < 2",
                               reason="fewer than 2 GPUs visible: distinct-device row blocks need >= 2 GPUs "
                                      "(the 8-GPU node)")


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1, "no GPU visible: the HIP path must run"


def solve_multi(monkeypatch, n, devices, form, overlap):
    monkeypatch.setenv("CGX_LOCAL_XCHG", "copy" if form == "copy" else "kernel")
    monkeypatch.setenv("CGX_LOCAL_FUSE", "0" if form == "nofuse" else "1")
    monkeypatch.setenv("CGX_LOCAL_THREADS", "1" if form == "threads" else "0")
    monkeypatch.setenv("CGX_OVERLAP", "1" if overlap else "0")
    x0 = np.full(n, 0.125)
    with cg.Solver(n, devices=devices) as s:
        flags = s.info.flags
        s.generate_spd(42)
        xg, st = s.solve(None, eps=1e-10)
        xf, _ = s.solve(x0, eps=-1.0, max_iter=12)
        rn, bn = s.residual_norm()
    return flags, xg, st.iterations, xf, rn / bn


@needs_two
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("form", ["kernel", "threads", "nofuse", "copy"])
def test_distinct_devices_bitwise_equal_one_device(monkeypatch, form, overlap):
    G = gpus()
    n = 1024 * G  # 1024-row blocks: aligned, so both exchange forms apply
    ref = solve_multi(monkeypatch, n, [0] * G, "kernel", overlap)
    got = solve_multi(monkeypatch, n, list(range(G)), form, overlap)
    assert got[0] & cg.CGX_PEER_ACTIVE and bool(got[0] & cg.CGX_OVERLAP_ACTIVE) == overlap
    assert got[2] == ref[2], (got[2], ref[2])
    assert np.array_equal(got[1], ref[1]) and np.array_equal(got[3], ref[3])
    assert got[4] == ref[4] and got[4] <= TOL


@needs_two
def test_distinct_devices_measured_choice_matches_oracle():
    """The default (measured) exchange form across distinct devices, against
    the fp64 oracle on a MATLAB-generated system."""
    G = gpus()
    n = 1024 * G
    A, b = oracle.spd_matlab(n, np.float64)
    x = np.zeros(n)
    st = cg.conjugrad(A, b, x, eps=1e-10, shards=list(range(G)))
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert st.iterations == so.iterations and rel(x, xo) <= TOL


@needs_two
@pytest.mark.timeout(300)
def test_rank_path_one_process_per_gpu(tmp_path):
    """torchrun's placement: world = min(8, visible) rank processes, rank r on
    device r, RCCL over xGMI (no NCCL_HOSTID: RCCL sees one host)."""
    G = gpus()
    n = 1024 * G
    uidfile, out = str(tmp_path / "uid.bin"), str(tmp_path / "sized")
    procs = []
    for r in range(G):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CGX_TEST_RANK_DEVICE="rank")
        env.pop("NCCL_HOSTID", None)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_worker.py"), "sized", str(n), str(G),
                                       str(r), uidfile, out], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    res = [json.load(open(out + f"_r{r}.json")) for r in range(G)]
    xs = [np.load(out + f"_x{r}.npy") for r in range(G)]
    assert sorted(r["comm"]["rccl_device"] for r in res) == list(range(G))
    for r in range(1, G):
        assert np.array_equal(xs[r], xs[0]) and res[r]["iterations"] == res[0]["iterations"]
    assert res[0]["overlap_info"]["decided_by"] == "measured"
    A, b = oracle.spd_matlab(n, np.float64)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert res[0]["iterations"] == so.iterations
    assert rel(xs[0], xo) <= TOL and res[0]["relres"] <= TOL
