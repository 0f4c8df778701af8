"""Row blocks on distinct GPUs: the paths a one-GPU box cannot execute.

Everything else in the suite puts every row block (or rank) on device 0.
These tests run where two or more GPUs are visible -- the driver's 8-GPU
node -- and are skipped with the reason otherwise.  tests/conftest.py
collects this file last, so under `pytest -x` a failure on a topology no
earlier round has run cannot keep the full-size configuration tests of the
other files from running.

  * cgx_create_multi over devices 0..G-1 (G = min(8, visible)): the pull
    kernels read the other devices' p slices and scalar partials over xGMI
    with system-scope loads after the producers' events; the threaded
    enqueue (CGX_LOCAL_THREADS=1, one host thread per device); the folded
    and separate scalar combines; the per-pair peer copies.  Each must give
    x bit for bit equal to the same partition on one device ([0] * G),
    overlapped and plain, gated and fixed-count.
  * configs[2] at its stated size (N = 65536) over G distinct GPUs, in one
    process and with one process per GPU: within 1e-10 of the fp64 oracle
    with conjgrad.m's loop count.
  * CGX_F32_REF over distinct devices, collective and p2p: bit for bit the
    unmodified parallel_cg.c / point-to-point_cg.c under mpiexec -np G
    (tests/golden/mpi/; parallel_cg.c:288-324, point-to-point_cg.c:444-473).
  * Poisson slabs over distinct devices (the halo pull and the folded
    PeerSum combines over xGMI): bitwise against [0] * G and against the
    oracle; and a Poisson rank run with one process per GPU.
  * the rank path with one process per GPU (parallel_cg.c's one MPI rank per
    process, :109-117 and :288-324): RCCL over xGMI between distinct devices.
  * bench.py --gpus G without a launcher, the one-process line a SCALE run
    would print.
  * the drop-in programs: `cg_hip --gpus G` over devices 0..G-1 and
    `mpiexec -np G cg_mpi` with one rank per GPU, x bit for bit the
    unmodified MPI programs' (the other files pin their CLI runs to device 0).

Rehearsal (CGX_TEST_MULTIDEVICE_REHEARSAL=1, one GPU): the same tests with
8 "devices" that are all device 0 -- row blocks [0] * G, rank processes
with their own NCCL_HOSTID (RCCL's socket transport), bench.py --devices
0,...,0 -- and the assertions about distinct devices and peer access
skipped.  It runs the tests' own code paths before the first node with
several GPUs does (tools/multidevice_rehearsal.sh).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import conjugate_gradient_amd as cg
import oracle
from _cases import case, golden_mpi, hash_oracle, mpi_golden_x

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-10
REHEARSAL = os.environ.get("CGX_TEST_MULTIDEVICE_REHEARSAL") == "1"


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def visible() -> int:
    if REHEARSAL:
        return 8
    try:
        return cg.device_count()
    except cg.CgxError:
        return 0


def devs(G: int) -> list:
    """Devices 0..G-1 (the rehearsal: device 0, G times)."""
    return [0] * G if REHEARSAL else list(range(G))


def distinct(flags: int) -> bool:
    """The context spans distinct devices with peer access (trivially true
    in the rehearsal, where there is one device)."""
    return REHEARSAL or bool(flags & cg.CGX_PEER_ACTIVE)


def gpus() -> int:
    return min(8, visible())


def gpus_pow2() -> int:
    """The largest of 2 / 4 / 8 that the visible GPUs allow: the MPI goldens
    exist for np = 2, 4, 8, and N = 65536 splits evenly over them."""
    g = gpus()
    return 8 if g >= 8 else 4 if g >= 4 else 2


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


def run_ranks_per_gpu(tmp_path, mode, n, G, timeout=240):
    """torchrun's placement: G rank processes, rank r on device r, RCCL over
    xGMI (no NCCL_HOSTID: RCCL sees one host).  Returns (x of rank 0, every
    rank's result dict); every rank must end with the same x."""
    uidfile, out = str(tmp_path / "uid.bin"), str(tmp_path / mode)
    procs = []
    for r in range(G):
        if REHEARSAL:  # every rank on device 0: RCCL needs a host id per rank (socket transport)
            env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", NCCL_HOSTID=f"cgx-rehearsal-{r}",
                       NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
            env.pop("CGX_TEST_RANK_DEVICE", None)
        else:
            env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CGX_TEST_RANK_DEVICE="rank")
            env.pop("NCCL_HOSTID", None)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_worker.py"), mode, str(n), str(G),
                                       str(r), uidfile, out], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    res = [json.load(open(out + f"_r{r}.json")) for r in range(G)]
    xs = [np.load(out + f"_x{r}.npy") for r in range(G)]
    assert sorted(r["comm"]["device"] for r in res) == devs(G)
    for r in range(1, G):
        assert np.array_equal(xs[r], xs[0]) and res[r]["iterations"] == res[0]["iterations"]
    return xs[0], res


# ---- one process, dense ----------------------------------------------------------
@needs_two
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("form", ["kernel", "threads", "nofuse", "copy"])
def test_distinct_devices_bitwise_equal_one_device(monkeypatch, form, overlap):
    G = gpus()
    n = 1024 * G  # 1024-row blocks: aligned, so both exchange forms apply
    ref = solve_multi(monkeypatch, n, [0] * G, "kernel", overlap)
    got = solve_multi(monkeypatch, n, devs(G), form, overlap)
    assert distinct(got[0]) and bool(got[0] & cg.CGX_OVERLAP_ACTIVE) == overlap
    assert bool(got[0] & cg.CGX_THREADS_ACTIVE) == (form == "threads")
    assert bool(got[0] & cg.CGX_PULL_ACTIVE) == (form != "copy")
    assert got[2] == ref[2], (got[2], ref[2])
    assert np.array_equal(got[1], ref[1]) and np.array_equal(got[3], ref[3])
    assert got[4] == ref[4] and got[4] <= TOL


@needs_two
def test_create_multi_distinct_devices_peer_access():
    """cgx_create_multi over devices 0 and 1 enables peer access after
    hipDeviceCanAccessPeer and leaves no HIP error pending; without peer
    access it is refused by name, never a silent host-staged copy."""
    if REHEARSAL:
        pytest.skip("rehearsal: one device, nothing to enable")
    L = cg.lib()
    link = cg.device_link(0, 1)
    if link["peer_access"]:
        with cg.Solver(1024, devices=[0, 1]) as s:
            assert L.cgx_hip_last_error() == 0 and s.info.flags & cg.CGX_PEER_ACTIVE
    else:
        with pytest.raises(cg.CgxError, match="cannot access"):
            cg.Solver(1024, devices=[0, 1])


@needs_two
def test_distinct_devices_measured_choice_matches_oracle():
    """The default (measured) exchange form across distinct devices, against
    the fp64 oracle on a MATLAB-generated system; the decision follows the
    rule on the two forms timed end to end."""
    G = gpus()
    n = 1024 * G
    A, b = oracle.spd_matlab(n, np.float64)
    with cg.Solver(n, devices=devs(G)) as s:
        info = s.overlap_info()
        assert info["decided_by"] == "measured" and info["on"] == cg.overlap_rule(info)
        s.set_system(A, b)
        x, st = s.solve(None, eps=1e-10)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert st.iterations == so.iterations and rel(x, xo) <= TOL


@needs_two
@pytest.mark.timeout(900)
def test_headline_n65536_distinct_devices_one_process():
    """configs[2] at its stated size over G distinct GPUs from one process
    (cgx_create_multi: 65536/G rows x 65536 of A per GPU, p gathered by pull
    kernels over xGMI in the measured form), generated on the devices,
    converged at eps 1e-10: loop count == conjgrad.m's, x within 1e-10 of the
    fp64 oracle, true residual <= 1e-10 ||b||."""
    n, G = 65536, gpus_pow2()
    with cg.Solver(n, devices=devs(G)) as s:
        assert distinct(s.info.flags) and s.overlap_info()["decided_by"] == "measured"
        s.generate_spd(42)
        x, st = s.solve(None, eps=1e-10)
        rn, bn = s.residual_norm()
    xo, so = hash_oracle(n)
    assert st.converged and st.iterations == so.iterations
    assert rel(x, xo) <= TOL and rn <= TOL * bn


@needs_two
@pytest.mark.parametrize("program", ["parallel", "p2p"])
def test_f32ref_distinct_devices_bitwise_vs_mpi_reference(program):
    """CGX_F32_REF over G distinct GPUs in one process == the unmodified
    parallel_cg.c (MPICH's MPI_Allreduce order) / point-to-point_cg.c (allSum,
    rank order) under mpiexec -np G on spd8192, bit for bit, same loop count."""
    G = gpus_pow2()
    key = f"{program}_spd8192_np{G}"
    r = golden_mpi()["runs"][key]
    A, b, x0 = case(r["case"])
    flags = cg.CGX_F32_REF | (cg.CGX_COMM_P2P if program == "p2p" else 0)
    with cg.Solver(b.size, flags=flags, devices=devs(G)) as s:
        assert distinct(s.info.flags)
        s.set_system(A, b, x0)
        x, st = s.solve(None, eps=1e-6)
    assert st.iterations == r["ref_iterations"] and st.converged == 1
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


# ---- one process, Poisson slabs ----------------------------------------------------
@needs_two
@pytest.mark.parametrize("form", ["pull", "nofuse", "copy"])
def test_poisson_distinct_devices_bitwise_equal_one_device(monkeypatch, form):
    """Poisson slabs on G distinct GPUs: k_poisson_p reads the neighbours'
    halo rows of r in place over xGMI (halo pull), the r.r and p.Ap partials
    are summed in rank order by the consuming kernels (PeerSum) -- or, nofuse,
    by combine kernels, or, copy, round 4's peer copies.  x bit for bit the
    same partition's on one device, gated and fixed-count; against the oracle
    at m = 128 (1e-10 converged, 1e-9 after 40 fixed iterations)."""
    G = gpus_pow2()
    m = 128
    monkeypatch.setenv("CGX_LOCAL_XCHG", "copy" if form == "copy" else "kernel")
    monkeypatch.setenv("CGX_LOCAL_FUSE", "0" if form == "nofuse" else "1")

    def run(devices):
        with cg.Solver(None, poisson_m=m, devices=devices) as s:
            flags = s.info.flags
            s.fill(1.0, 0.0)
            xg, st = s.solve(None, eps=1e-8)
            s.fill(1.0, 0.0)
            xf, _ = s.solve(None, eps=-1.0, max_iter=40)
        return flags, xg, st.iterations, xf

    ref = run([0] * G)
    got = run(devs(G))
    assert distinct(got[0])
    assert bool(got[0] & cg.CGX_HALO_PULL_ACTIVE) == (form != "copy")
    assert bool(got[0] & cg.CGX_FOLDED_ACTIVE) == (form == "pull")
    assert got[2] == ref[2] and np.array_equal(got[1], ref[1]) and np.array_equal(got[3], ref[3])
    n = m * m
    xo, so = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=1e-8)
    assert got[2] == so.iterations and rel(got[1], xo) <= TOL
    xo, _ = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), eps=-1.0, max_iter=40)
    assert rel(got[3], xo) <= 1e-9


# ---- one process per GPU (RCCL over xGMI) ------------------------------------------
@needs_two
@pytest.mark.timeout(300)
def test_rank_path_one_process_per_gpu(tmp_path):
    G = gpus()
    n = 1024 * G
    x, res = run_ranks_per_gpu(tmp_path, "sized", n, G)
    assert sorted(r["comm"]["rccl_device"] for r in res) == devs(G)
    info = res[0]["overlap_info"]
    assert info["decided_by"] == "measured" and info["on"] == cg.overlap_rule(info)
    A, b = oracle.spd_matlab(n, np.float64)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL


@needs_two
@pytest.mark.timeout(900)
def test_headline_n65536_one_process_per_gpu(tmp_path):
    """configs[2] in the driver's placement on real GPUs: N = 65536 over G
    rank processes, rank r on device r, RCCL allgather / allreduce over xGMI,
    generated on the devices, converged at eps 1e-10 -- conjgrad.m's loop
    count, x within 1e-10 of the fp64 oracle."""
    n, G = 65536, gpus_pow2()
    x, res = run_ranks_per_gpu(tmp_path, "headline", n, G, timeout=780)
    assert res[0]["nrows"] == n // G and res[0]["overlap_info"]["decided_by"] == "measured"
    xo, so = hash_oracle(n)
    assert res[0]["converged"] and res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL


@needs_two
@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["f32ref", "p2p_f32ref"])
def test_rank_f32ref_one_process_per_gpu_bitwise_vs_mpi_reference(tmp_path, mode):
    """G RCCL ranks on G GPUs == parallel_cg.c / point-to-point_cg.c on G MPI
    ranks (spd8192), bit for bit, same loop count."""
    n, G = 8192, gpus_pow2()
    x, res = run_ranks_per_gpu(tmp_path, mode, n, G)
    key = ("p2p" if mode.startswith("p2p") else "parallel") + f"_spd{n}_np{G}"
    assert res[0]["iterations"] == golden_mpi()["runs"][key]["ref_iterations"]
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


@needs_two
@pytest.mark.timeout(300)
def test_poisson_rank_one_process_per_gpu(tmp_path):
    """Poisson slabs, one rank process per GPU: r's halo rows by
    ncclSend/Recv over xGMI, both scalars by allreduce; against the oracle."""
    m, G = 128, gpus_pow2()
    x, res = run_ranks_per_gpu(tmp_path, "poisson_eps", m, G)
    xo, so = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), eps=1e-8, max_iter=-1)
    assert res[0]["iterations"] == so.iterations and rel(x, xo) <= TOL


# ---- the bench line without a launcher ---------------------------------------------
@needs_two
@pytest.mark.timeout(300)
@pytest.mark.parametrize("workload", ["dense", "poisson"])
def test_bench_without_launcher_distinct_devices(workload):
    """`bench.py --gpus G` without torchrun (cgx_create_multi over devices
    0..G-1): one JSON line whose multi_device lists G distinct devices with
    peer access, whose exchange text follows the context's flags, which
    carries the measured overlap choice (dense) and the host's enqueue time
    per iteration."""
    import bench
    G = gpus()
    args = (["--devices", ",".join(map(str, devs(G)))] if REHEARSAL else ["--gpus", str(G)])
    args += ["--steps", "5", "--warmup", "1", "--settle", "0", "--no-cpu"]
    args += ["--size", str(8192 * G)] if workload == "dense" else ["--workload", "poisson", "--grid", str(512 * G)]
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "bench.py")] + args,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    md = out["multi_device"]
    assert md["devices"] == devs(G) and out["config"]["row_blocks"] == G
    if not REHEARSAL:
        assert out["n_gpus"] == G and md["distinct_devices"] == G
        assert md["peer_active"] and len(set(md["pci_bus_ids"])) == G
        assert all(lk["link"] != "same device" for lk in md["links_from_block0"])
    assert out["host_enqueue_us_per_iteration"] > 0
    assert out["config"]["exchange"] == bench.exchange_text(G, md["flags"], devices=md["devices"],
                                                            poisson=workload == "poisson")
    if workload == "dense":
        ov = out["overlap"]
        assert ov["decided_by"] == "measured" and ov["on"] == cg.overlap_rule(ov)
        assert out["check"]["relres"] < 1e-6
    else:
        assert "halo pull" in out["config"]["exchange"]


# ---- the two drop-in programs over distinct devices --------------------------------
@pytest.fixture(scope="module")
def spd512_files(tmp_path_factory):
    """generateSPDmatrix(512) written as the MATLAB script writes it."""
    d = tmp_path_factory.mktemp("spd512")
    A, b = oracle.spd_matlab(512, np.float64)
    for name, arr, dec in (("A.txt", A, 4), ("b.txt", b, 4), ("x0.txt", np.zeros(512), 1)):
        oracle.write_text(str(d / name), arr, dec)
    return [str(d / f) for f in ("A.txt", "b.txt", "x0.txt")]


def printed_x(out, n, dtype):
    return np.array([float(v) for v in out.strip().splitlines()[-n:]], dtype=dtype)


@needs_two
@pytest.mark.timeout(300)
@pytest.mark.parametrize("program", ["parallel", "p2p"])
def test_cg_hip_gpus_distinct_devices_bitwise_vs_mpi_reference(spd512_files, program):
    """`cg_hip --gpus G [--p2p]` (one process, row blocks on devices 0..G-1)
    on the text files == `mpiexec -np G` of the unmodified parallel_cg.c /
    point-to-point_cg.c, bit for bit, with the loop count."""
    G = gpus_pow2()
    key = f"{program}_spd512_np{G}"
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0") if REHEARSAL else dict(os.environ)
    args = ["--gpus", str(G), "--fp32-ref", "--print-x", "--stats"] + (["--p2p"] if program == "p2p" else [])
    r = subprocess.run([cg.CLI_PATH, *args, *spd512_files], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert f"iterations: {golden_mpi()['runs'][key]['ref_iterations']} converged: 1" in r.stdout
    x = printed_x(r.stdout, 512, np.float32)
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


@needs_two
@pytest.mark.timeout(300)
@pytest.mark.parametrize("program", ["parallel", "p2p"])
def test_cg_mpi_one_rank_per_gpu_bitwise_vs_mpi_reference(spd512_files, program):
    """`mpiexec -np G cg_mpi` as parallel_cg.c is launched: one rank per
    GPU (the node-local rank picks the device), RCCL over xGMI (no per-rank
    host id), x bit for bit the unmodified program's under mpiexec -np G."""
    mpiexec = "/opt/conda/bin/mpiexec"
    cg_mpi = os.path.join(os.path.dirname(cg.CLI_PATH), "cg_mpi")
    if not (os.path.exists(mpiexec) and os.path.exists(cg_mpi)):
        pytest.skip("MPICH mpiexec or bin/cg_mpi absent")
    G = gpus_pow2()
    key = f"{program}_spd512_np{G}"
    args = ["--fp32-ref", "--print-x", "--stats"] + (["--p2p"] if program == "p2p" else []) + spd512_files
    cmd = [mpiexec]
    for r in range(G):
        if r:
            cmd.append(":")
        cmd += ["-np", "1", "-env", "CGX_RCCL_TIMEOUT_S", "120"]
        if REHEARSAL:  # every rank on device 0: a host id per rank (RCCL's socket transport)
            cmd += ["-env", "NCCL_HOSTID", f"cgx-rehearsal-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                    "-env", "NCCL_IB_DISABLE", "1", "-env", "CGX_DEVICE", "0"]
        cmd += [cg_mpi, *args]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("NCCL_HOSTID", None)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"iterations: {golden_mpi()['runs'][key]['ref_iterations']} converged: 1" in p.stdout
    x = printed_x(p.stdout, 512, np.float32)
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))
