"""bench.py's multi-process control plane on CPU (gloo, world size 2):
rendezvous on 127.0.0.1, broadcast of the 128-byte RCCL id (which contains
NULs), max-over-ranks of the timings, and the row-block arithmetic each rank
derives (parallel_cg.c:83 local_row = ROWS / procsnum)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    try:
        assert bench.launched_by_torchrun()
        r, lr, w = bench.dist_env()
        dist = bench.dist_init()
        payload = bytes(range(128)) if r == 0 else None  # byte 0 is NUL
        got = bench.bcast_bytes(dist, payload)
        mx = bench.max_over_ranks(dist, float(r + 1) * 1.5)
        sm = bench.sum_over_ranks(dist, 1.0)
        n = 65536
        nloc = n // w
        objs = bench.gather_objects(dist, {"rank": r, "pci_bus_id": f"0000:{r:02x}:00.0"})
        assert [o["rank"] for o in objs] == list(range(w)), objs  # every rank's, in rank order
        q.put((r, got == bytes(range(128)), mx, sm, bench.matvec_bytes(n, nloc)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(120)
def test_gloo_world2_control_plane():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert len(r) == 5, r
        rank, ok, mx, sm, mvb = r
        assert ok and mx == 3.0 and sm == 2.0
        assert mvb == 8 * 32768 * 65536 + 8 * 65536 + 8 * 32768


def test_matvec_bytes_formula():
    # 34.36 GB on 1 GPU, 4.295 GB per GPU on 8 at N = 65536
    assert abs(bench.matvec_bytes(65536, 65536) / 1e9 - 34.36) < 0.01
    assert abs(bench.matvec_bytes(65536, 8192) / 1e9 - 4.295) < 0.001


def test_traffic_lookup_names_its_source():
    """roofline.traffic is the committed PMC figure for the same workload
    (rocprofv3 cannot run inside the bench process): the bench reports where
    it came from, and null where no pass exists (e.g. N=4096)."""
    t, src = bench.pmc_traffic("n65536_g1")
    assert t is not None and 1.0 <= t / bench.matvec_bytes(65536, 65536) < 1.01
    assert "pmc_summary.json[n65536_g1]" in src and "FETCH_SIZE" in src
    for g in (2, 4, 8):
        t, src = bench.pmc_traffic(f"n65536_g{g}")
        assert t is not None and 1.0 <= t / bench.matvec_bytes(65536, 65536 // g) < 1.01, g
    assert bench.pmc_traffic("n4096_g1") == (None, None)
    # configs[4]: the xr kernels' bytes per launch over the x cycle, against the line's algorithmic figure
    t, src = bench.pmc_traffic("poisson_m8192_g1")
    m = 8192
    assert t is not None and 1.0 <= t / (104.0 / 3 * m * m + 16 * m) < 1.06 and "poisson_m8192_g1" in src


def _phases(scale):
    import conjugate_gradient_amd as cg
    base = dict(zip(cg.PHASE_NAMES, (80.0, 2.0, 550.0, 15.0, 4.5, 15.0, 4.5, 3.0, 674.0)))
    return {k: {"median_us": v * scale, "mean_us": v * scale, "samples": 19} for k, v in base.items()}


def test_phase_summary_tiles_the_step():
    """The N>1 line's breakdown: per-rank medians, the max over ranks, and the
    tiling phases (all but `iteration`) added up against ms_per_step."""
    out = bench.phase_summary([_phases(1.0), _phases(1.02)], ms_per_step=0.6885)
    assert out["iterations_sampled"] == 19 and len(out["per_rank"]) == 2
    assert out["max_over_ranks"]["matvec"] == 561.0
    tiles = (80 + 2 + 550 + 15 + 4.5 + 15 + 4.5 + 3) * 1.02
    assert abs(out["tiling_sum_ms_per_rank"][1] - tiles / 1e3) < 1e-4
    assert abs(out["tiling_sum_over_ms_per_step"] - tiles / 1e3 / 0.6885) < 1e-9
    assert abs(out["tiling_mean_sum_over_ms_per_step"] - tiles / 1e3 / 0.6885) < 1e-9


def test_rccl_summary_counts_devices():
    """`rccl`: the ranks' own view, distinct devices by PCI bus id; a device
    rank 0 cannot see is named as such (no GPU here: none visible)."""
    ranks = [{"rccl_nranks": 2, "rccl_device": d, "rccl_rank": r, "device": d, "pci_bus_id": f"0000:{0x11 + d:02x}:00.0"}
             for r, d in ((0, 0), (1, 1))]
    out = bench.rccl_summary(ranks, solver_device=0)
    assert out["nranks"] == 2 and out["distinct_devices"] == 2 and len(out["pci_bus_ids"]) == 2
    assert out["links_from_rank0"][0]["to_rank"] == 1 and "link" in out["links_from_rank0"][0]


@pytest.mark.timeout(120)
def test_bench_gpus_without_launcher_fails_loudly_when_devices_are_missing():
    """`bench.py --gpus 2` outside torchrun drives devices 0 and 1 from one
    process; with fewer GPUs visible (none here) it exits non-zero and says
    so, and prints no JSON line -- never a 1-GPU line for a 2-GPU request."""
    import subprocess
    import sys

    import conjugate_gradient_amd as cg
    if cg.device_count() >= 2:
        pytest.skip("two GPUs are visible: the run would proceed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--no-cpu"],
                       capture_output=True, text=True, timeout=100)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "--gpus 2" in p.stderr and "device(s) are visible" in p.stderr
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--devices", "0,0",
                        "--no-cpu"], capture_output=True, text=True, timeout=100)
    assert p.returncode != 0 and "--devices lists 2" in p.stderr
