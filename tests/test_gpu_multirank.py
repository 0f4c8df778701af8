"""Rank mode (one process per rank, RCCL) at world size 2, 4 and 8 on one GPU.

The driver's N = 2/4/8 bench runs use one process per GPU over RCCL.  One
GPU box cannot run that placement (RCCL refuses two ranks on one device of
one host), so each rank here gets its own NCCL_HOSTID: RCCL then sees P hosts
and moves the data over its socket transport on the loopback interface.  The
transport differs from xGMI; libcgx's rank-mode logic is what is checked:
row-block offsets, the in-place allgather slots, the overlapped exchange on
the comm stream, the scalar combines, the p2p pattern, the Poisson halo
exchange and the final x allgather (tests/_rank_worker.py).

Pins: fp64 x vs the fp64 oracle (conjgrad.m order) to 1e-10 with its loop
count; CGX_DETERMINISTIC bitwise equal to the multi-shard run with the same
partition; CGX_F32_REF bitwise equal to the unmodified parallel_cg.c
(collective) / point-to-point_cg.c (p2p) run under mpiexec -np P
(tests/golden/mpi/); every rank ends with the same x.
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


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.fixture(scope="module", autouse=True)
def _gpu(built):
    assert cg.device_count() >= 1, "no GPU visible: the HIP path must run"


def run_ranks(tmp_path, mode, n, P, timeout=150):
    uidfile = str(tmp_path / "uid.bin")
    out = str(tmp_path / mode)
    procs = []
    for r in range(P):
        env = dict(os.environ, NCCL_HOSTID=f"cgx-test-host-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_worker.py"), mode, str(n), str(P),
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
    xs = [np.load(out + f"_x{r}.npy") for r in range(P)]
    res = []
    for r in range(P):
        with open(out + f"_r{r}.json") as f:
            res.append(json.load(f))
    for r in range(1, P):  # every rank holds the same allgathered x
        assert np.array_equal(xs[r], xs[0])
        assert res[r]["iterations"] == res[0]["iterations"]
    return xs[0], res


@pytest.mark.timeout(200)
@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("mode", ["collective", "overlap_on", "nooverlap", "p2p", "deterministic", "det_overlap"])
def test_rank_mode_f64(tmp_path, mode, P):
    """Row blocks of 1024/P rows (multiples of 128): the exchange form is
    chosen at creation from the measured allgather and split cost (the same
    on every rank), or forced (CGX_OVERLAP=1, CGX_NO_OVERLAP); p2p has no
    choice.  Both forms give the same bits: the rank-ordered combine equals
    the multi-shard solve, overlapped or not."""
    n = 1024
    x, res = run_ranks(tmp_path, mode, n, P)
    assert res[0]["nrows"] == n // P
    info = res[0]["overlap_info"]
    same = lambda o: {k: v for k, v in o.items() if k != "forms_ms"}  # noqa: E731  (forms_ms: each rank's own clock)
    for r in res:  # every rank decided alike, from the same (max over ranks) numbers
        assert same(r["overlap_info"]) == same(info) and r["overlap"] == res[0]["overlap"]
        assert (r["overlap_info"]["forms_ms"] or 0) > 0 or info["decided_by"] == "n/a"
    if mode in ("collective", "deterministic"):
        assert info["decided_by"] == "measured" and info["allgather_us"] > 0 and info["one_launch_us"] > 0
        assert info["overlap_form_us"] > 0 and info["plain_form_us"] > 0
        assert res[0]["overlap"] == cg.overlap_rule(info)
    elif mode in ("overlap_on", "det_overlap"):
        assert res[0]["overlap"] and info["decided_by"] == "forced_on"
    elif mode == "nooverlap":
        assert not res[0]["overlap"] and info["decided_by"] == "off"
    else:
        assert not res[0]["overlap"] and info["decided_by"] == "n/a"
    A, b, x0 = case(f"spd{n}", np.float64)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL
    if mode in ("deterministic", "det_overlap"):  # rank-ordered scalar combine == the multi-shard bits
        xs = x0.copy()
        cg.conjugrad(A, b, xs, eps=1e-10, shards=[0] * P)
        assert np.array_equal(x, xs)
    if mode == "collective":
        assert res[0]["fixed_iterations"] == 5 and res[0]["fixed_relres"] < 1.0


@pytest.mark.timeout(200)
@pytest.mark.parametrize("n,P", [(1000, 2), (2000, 4), (4096, 4)])
def test_rank_mode_f64_sizes(tmp_path, n, P):
    """Row blocks that are not multiples of 128 rows (no overlap, ragged
    chunks) and a larger system, collective exchange."""
    x, res = run_ranks(tmp_path, "sized", n, P)
    assert res[0]["nrows"] == n // P
    aligned = (n // P) % 128 == 0  # the form is chosen (measured) only for aligned row blocks
    assert res[0]["overlap_info"]["decided_by"] == ("measured" if aligned else "n/a")
    assert aligned or not res[0]["overlap"]
    A, b = oracle.spd_matlab(n, np.float64)
    xo, so = oracle.cg_f64(A, b, np.zeros(n), eps=1e-10)
    assert res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL


@pytest.mark.timeout(200)
@pytest.mark.parametrize("mode", ["f32ref", "p2p_f32ref"])
def test_rank_mode_f32ref_bitwise(tmp_path, mode):
    """4 RCCL ranks == parallel_cg.c / point-to-point_cg.c on 4 MPI ranks."""
    n, P = 2048, 4
    x, res = run_ranks(tmp_path, mode, n, P)
    _check_mpi_golden(x, res, ("p2p" if mode.startswith("p2p") else "parallel") + f"_spd{n}_np{P}")


def _check_mpi_golden(x, res, key):
    r = golden_mpi()["runs"][key]
    assert res[0]["iterations"] == r["ref_iterations"]
    assert np.array_equal(x.view(np.uint32), mpi_golden_x(key).view(np.uint32))


@pytest.mark.timeout(200)
@pytest.mark.parametrize("mode", ["poisson", "poisson_eps"])
def test_rank_mode_poisson_halo(tmp_path, mode):
    m, P = 128, 4
    x, res = run_ranks(tmp_path, mode, m, P)
    eps = 1e-8 if mode == "poisson_eps" else -1.0
    xo, so = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), eps=eps,
                                   max_iter=-1 if eps > 0 else 120)
    assert res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= (TOL if eps > 0 else 1e-9)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("mode", ["collective", "p2p", "deterministic", "f32ref", "p2p_f32ref", "poisson_eps"])
def test_rank_mode_world8(tmp_path, mode):
    """The driver's largest placement, 8 ranks (here on one GPU): 8 row
    blocks of 128 / 256 rows, the p2p pattern's 7 sends per exchange, 8
    gathered partials, 8 Poisson slabs of 16 rows."""
    P = 8
    if mode == "poisson_eps":
        m = 128
        x, res = run_ranks(tmp_path, mode, m, P, timeout=200)
        xo, so = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), eps=1e-8, max_iter=-1)
        assert res[0]["iterations"] == so.iterations and rel(x, xo) <= TOL
        return
    n = 2048 if "f32ref" in mode else 1024
    x, res = run_ranks(tmp_path, mode, n, P, timeout=200)
    assert res[0]["nrows"] == n // P
    if "f32ref" in mode:  # == mpiexec -np 8 of the unmodified program
        _check_mpi_golden(x, res, ("p2p" if mode.startswith("p2p") else "parallel") + f"_spd{n}_np{P}")
        return
    A, b, x0 = case(f"spd{n}", np.float64)
    xo, so = oracle.cg_f64(A, b, x0, eps=1e-10)
    assert res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL
    if mode == "deterministic":
        xs = x0.copy()
        cg.conjugrad(A, b, xs, eps=1e-10, shards=[0] * P)
        assert np.array_equal(x, xs)


@pytest.mark.timeout(600)
def test_rank_mode_headline_n65536_world2(tmp_path):
    """BASELINE configs[2] through the rank path at full size: N=65536 on 2
    RCCL ranks (17.2 GB of A each, the allgather in the measured form, the scalar
    allreduces), generated on the device; x within 1e-10 of the fp64 oracle
    with conjgrad.m's loop count, true residual <= 1e-10 ||b||."""
    n, P = 65536, 2
    x, res = run_ranks(tmp_path, "headline", n, P, timeout=500)
    assert res[0]["nrows"] == n // P and res[0]["overlap_info"]["decided_by"] == "measured"
    xo, so = hash_oracle(n)
    assert res[0]["converged"] and res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["headline", "headline_det"])
def test_rank_mode_headline_n65536_world8(tmp_path, mode):
    """configs[2] in the driver's placement: N=65536 over 8 RCCL rank
    processes (parallel_cg.c:83's row blocks: 8192 rows x 65536 = 4.3 GB of A
    each; the loop :283-323 with the allgather in the measured form and the two scalar
    exchanges), generated on the device, converged at eps 1e-10.  Every rank
    ends with the same x; the loop count is conjgrad.m's; x within 1e-10 of
    the fp64 oracle; true residual <= 1e-10 ||b||.  CGX_DETERMINISTIC
    (headline_det) must also equal, bit for bit, the 8-shard multi-shard
    solve of the same system in one process."""
    n, P = 65536, 8
    x, res = run_ranks(tmp_path, mode, n, P, timeout=780)
    assert res[0]["nrows"] == n // P and res[0]["overlap_info"]["decided_by"] == "measured"
    xo, so = hash_oracle(n)
    assert res[0]["converged"] and res[0]["iterations"] == so.iterations
    assert rel(x, xo) <= TOL and res[0]["relres"] <= TOL
    if mode == "headline_det":  # the rank-ordered combine == the LOCAL mode's combine of the same partition
        with cg.Solver(n, devices=[0] * P) as s:
            s.generate_spd(42)
            xs, st = s.solve(None, eps=1e-10)
        assert st.iterations == res[0]["iterations"]
        assert np.array_equal(x, xs)


@pytest.mark.timeout(150)
@pytest.mark.parametrize("mode", ["peer_dies", "peer_absent", "poisson_peer_dies"])
def test_rank_mode_fails_fast_when_a_peer_is_gone(tmp_path, mode):
    """A dead or absent rank must not hang the others (the reference's
    fail-stop is MPI_Abort, parallel_cg.c:79,89,94,143): with
    CGX_RCCL_TIMEOUT_S=20, rank 0 gets CGX_ERR_RCCL (-3) naming what it waited
    for -- from the solve when rank 1 died after cgx_create_rank, from
    cgx_create_rank when rank 1 never joined -- and exits on its own."""
    n, P, limit = (64 if mode.startswith("poisson") else 1024), 2, 20
    uidfile, out = str(tmp_path / "uid.bin"), str(tmp_path / mode)
    procs, logs = [], [str(tmp_path / f"rank{r}.log") for r in range(P)]
    for r in range(P):
        env = dict(os.environ, NCCL_HOSTID=f"cgx-test-host-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0", CGX_RCCL_TIMEOUT_S=str(limit), CGX_DEBUG="1")
        with open(logs[r], "w") as lf:
            procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_rank_worker.py"), mode, str(n),
                                           str(P), str(r), uidfile, out], env=env, stdout=lf,
                                          stderr=subprocess.STDOUT))
    hung = False
    try:
        for p in procs:
            p.wait(timeout=120)
    except subprocess.TimeoutExpired:
        hung = True
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    tail = "\n".join(f"--- rank {r}:\n" + open(logs[r]).read()[-4000:] for r in range(P))
    assert not hung and procs[0].returncode == 0, tail
    with open(out + "_r0.json") as f:
        res = json.load(f)
    assert res["error"] is not None and res["code"] == -3, (res, tail)
    assert res["elapsed_s"] <= limit + 30, res
    if mode == "peer_absent":
        assert "cgx_create" in res["error"] and "created_s" not in res, res
    elif mode == "poisson_peer_dies":  # x updates were deferred when the iterate failed: x is refused
        assert res["xdefer"] and res["get_x_code"] == -6 and "incomplete" in res["get_x"], res
    else:
        assert "created_s" in res and "aborted" not in res["error"], res
        if res["failed_in"] == "cgx_iterate":  # part of an iteration may have run: x is refused, not handed out
            assert res["get_x_code"] == -6 and "part-way" in res["get_x"], res


@pytest.mark.timeout(240)
@pytest.mark.parametrize("workload", ["dense", "poisson"])
def test_bench_under_torchrun_world2(workload):
    """The driver's N>1 command shape (torch.distributed.run, one process per
    rank, RCCL inside libcgx, gloo control plane), at world size 2 on this GPU."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    steps = 30 if workload == "dense" else 4
    args = ["--gpus", "2", "--steps", str(steps), "--warmup", "1", "--no-cpu"]
    args += ["--size", "4096"] if workload == "dense" else ["--workload", "poisson", "--grid", "512"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(HERE, "_bench_rank_wrapper.py")] + args
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == steps and out["value"] > 0
    assert out["config"]["rows_per_gpu"] == (2048 if workload == "dense" else 512 * 512 // 2)
    # what RCCL ran on: 2 ranks; here both on this box's one GPU (per-rank host ids)
    rc = out["rccl"]
    assert rc["nranks"] == 2 and len(rc["pci_bus_ids"]) == 2 and rc["distinct_devices"] == 1
    assert [r["rccl_rank"] for r in rc["ranks"]] == [0, 1] and rc["links_from_rank0"][0]["link"] == "same device"
    if workload == "dense":
        assert "allgather" in out["config"]["exchange"]
        assert out["check"]["relres"] < 1e-6
        # the per-phase breakdown: every rank, every phase, and the phases tile the iteration
        ph = out["phases_us"]
        assert ph["iterations_sampled"] == steps - 1 and len(ph["per_rank"]) == 2
        # the exchange form the context measured and chose at creation, named in the line
        ov = out["overlap"]
        assert ov["decided_by"] == "measured" and ov["on"] == cg.overlap_rule(ov), ov
        for r in ph["per_rank"]:
            assert set(r) == set(cg.PHASE_NAMES)
            assert (r["matvec_own"] > 0) == ov["on"] and r["matvec"] > 0 and r["combine_pap"] > 0
            assert r["iteration"] > 0 and r["matvec_busy"] >= r["matvec"]
        # the phases never add up to more than the step; here (two ranks sharing one GPU over RCCL's socket
        # transport) a stall outside the sampled iterations -- the first timed one, or between the host's
        # barrier and the first launch -- lands in ms_per_step alone (one run in many: 0.63), so the lower
        # bound only catches a phase missing from the tiling
        assert 0.5 <= ph["tiling_mean_sum_over_ms_per_step"] <= 1.05, ph
        # the matVec roofline uses the two kernels' own spans (slowest rank), not the event bracket around
        # the allgather wait, which matvec_ms keeps
        assert "CGX_TIMING" in out["matvec_ms_source"] and out["matvec_kernel_ms"] <= out["matvec_ms"] * 1.01
        assert out["roofline"]["achieved"] == pytest.approx(out["matvec_kernel_gbps"])
        assert 0.5 <= ph["tiling_sum_over_ms_per_step"] <= 1.25, ph  # medians of a noisy socket transport (above)
    else:  # 1 warmup + 4 timed iterations from x0 = 0: the oracle's true residual after 5
        m = 512
        xo, _ = oracle.cg_poisson_f64(m, np.ones(m * m), np.zeros(m * m), max_iter=5, eps=-1.0)
        ro = np.linalg.norm(np.ones(m * m) - oracle.poisson_apply(m, xo)) / m
        assert abs(out["check"]["relres"] - ro) <= 1e-9 * ro


@pytest.mark.timeout(200)
def test_bench_multi_gpu_without_launcher():
    """`bench.py --gpus 2` without torchrun drives two row blocks from one
    process (cgx_create_multi) -- or, with fewer than 2 GPUs visible, exits
    non-zero saying so; never a 1-GPU line for a 2-GPU request (the run on
    distinct GPUs: tests/test_gpu_multidevice.py).  --devices 0,0 runs the
    same flow with both blocks on this GPU and reports that."""
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    base = [sys.executable, bench, "--size", "4096", "--steps", "30", "--warmup", "2", "--settle", "0", "--no-cpu"]
    if cg.device_count() < 2:
        p = subprocess.run(base + ["--gpus", "2"], capture_output=True, text=True, timeout=150)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert p.returncode != 0 and not lines and "device(s) are visible" in p.stderr, p.stderr[-2000:]
    p = subprocess.run(base + ["--devices", "0,0"], capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["row_blocks"] == 2 and out["config"]["rows_per_gpu"] == 2048
    assert "2 row blocks on 1 GPU" in out["config"]["workload"] and "pull kernel" in out["config"]["exchange"]
    assert "folded combines" in out["config"]["exchange"] and out["host_enqueue_us_per_iteration"] > 0
    md = out["multi_device"]
    assert md["devices"] == [0, 0] and md["distinct_devices"] == 1 and md["links_from_block0"][0]["link"] == "same device"
    # the form measured at creation (on one GPU the pull gather is short: usually the plain form)
    ov = out["overlap"]
    assert ov["decided_by"] == "measured" and ov["on"] == cg.overlap_rule(ov)
    assert out["check"]["relres"] < 1e-6 and (out["phases_us"]["per_rank"][0]["matvec_own"] > 0) == ov["on"]


@pytest.mark.timeout(200)
def test_bench_single_gpu_line():
    """The driver's N=1 command shape at a small size: one JSON line with the
    contract's keys, the roofline and the per-phase breakdown whose tiling
    phases add up to ms_per_step."""
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--size", "8192", "--steps", "40",
           "--warmup", "2", "--settle", "0", "--no-cpu"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in out, key
    assert out["n_gpus"] == 1 and out["steps"] == 40 and out["dtype"] == "f64" and out["value"] > 0
    rf = out["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"])
    ph = out["phases_us"]
    assert ph["iterations_sampled"] == 39 and ph["per_rank"][0]["matvec"] > 0
    # (a host stall before the first sampled iteration lands in ms_per_step alone)
    assert abs(ph["tiling_mean_sum_over_ms_per_step"] - 1) <= 0.10, ph
    assert out["check"]["relres"] < 1e-10
