#!/usr/bin/env python3
"""bench.py -- CG iterations/s and matVec HBM GB/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 65536] [--no-cpu]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one CG iteration (serialConjugate.c:213-245 / parallel_cg.c:288-324):
allgather p, A.p matVec with the fused p.Ap dot, allreduce, x/r update with the
r.r dot, allreduce, p update.  The workload is configs[2] of BASELINE.json:
N = 65536 dense SPD fp64 (generateSPDmatrix.m-style, generated on device),
row-block partitioned over the N GPUs -- the 1-GPU point fits one GPU's HBM
(34.4 GB), so the 1/2/4/8 series is strong scaling of one fixed system.
Iterations run in fixed-count mode (no early stop) so every step does the full
work; the true residual ||b - A x|| / ||b|| is checked after the timed region.

Under torchrun each process drives one GPU (cgx_create_rank): RCCL carries the
per-iteration exchange inside libcgx; torch.distributed (gloo, CPU) is only the
control plane (RCCL id broadcast, barriers, max-over-ranks of the timings).
Run without torchrun, N=1 uses a single-GPU context and no torch; N>1 drives
devices 0..N-1 from this one process (cgx_create_multi: row blocks on N GPUs,
p gathered and the scalars combined by pull kernels over peer access), and
exits non-zero when fewer than N devices are visible -- never a 1-GPU line
for an N-GPU request.  --devices lists them explicitly (repeats allowed: row
blocks sharing a GPU, reported as such).

Output: ONE JSON line on rank 0 (see the keys below).  `roofline.achieved`
is ALGORITHMIC matVec bytes per launch (8*N_loc*N + 8*N + 8*N_loc, SURVEY.md
s8(d)) / the average matVec kernel duration measured with HIP events on the
stream the kernel runs on, over the timed region.  `roofline.traffic` is the
HBM bytes per launch from rocprofv3 PMC counters (profiles/pmc_summary.json,
FETCH_SIZE doubled per the gfx950 correction) when a summary for this
workload exists, else null.  `cpu_baseline` times the oracle's fp32-ref
restatement of serialConjugate.c (bit-identical to it, tests/test_oracle.py)
on one host core, on a bounded sample: 5 iterations of the same system (~10 s);
`cpu_baseline_reference` runs serialConjugate.c itself (oracle/_ref, built
from the reference's sources) at its compiled N=8192 in the same run.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

# before torch (and its libgomp) loads: the oracle's OpenMP loops in the CPU
# legs need passive waiting to scale (see oracle/__init__.py)
os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CG iterations/sec + matVec HBM GB/s, N×N dense SPD fp64, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, Chip-level parameters)
H2D_PEAK_GBS = 63.0    # PCIe Gen5 x16 host link per GPU (same table, spec)
SEED = 42


# ----------------------------------------------------------------------------
# control plane (torch.distributed gloo) -- also exercised by tests/test_dist.py
# ----------------------------------------------------------------------------
def launched_by_torchrun() -> bool:
    return "TORCHELASTIC_RUN_ID" in os.environ or "LOCAL_RANK" in os.environ


def dist_env() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def dist_init():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one node (every rank local): RCCL's bootstrap over loopback, whatever
        # interfaces the box has; the data path is xGMI either way
        if os.environ.get("LOCAL_WORLD_SIZE", "1") == os.environ.get("WORLD_SIZE", "1"):
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo")
    return dist


def bcast_bytes(dist, payload: bytes | None, src: int = 0) -> bytes:
    obj = [payload]
    dist.broadcast_object_list(obj, src=src)
    return obj[0]


def max_over_ranks(dist, value: float) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(dist, obj) -> list:
    """Every rank's `obj` on every rank (gloo, CPU), in rank order."""
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def sum_over_ranks(dist, value: float) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


# ----------------------------------------------------------------------------
def matvec_bytes(n: int, nloc: int) -> int:
    """Algorithmic bytes of one matVec launch on one GPU."""
    return 8 * nloc * n + 8 * n + 8 * nloc


def pmc_traffic(key: str) -> tuple[float | None, str | None]:
    """HBM bytes per launch of the roofline's kernel from the committed PMC
    passes (rocprofv3 cannot run inside this process), and where that figure
    came from.  Keys: "n<N>_g<G>[_symmetric]" (the dense matVec),
    "poisson_m<M>_g<G>" (the Poisson xr kernels, averaged over their x-update
    cycle)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            s = json.load(f)
        if key not in s:
            return None, None
        e = s[key]
        src = (f"profiles/pmc_summary.json[{key}]: 2*FETCH_SIZE + WRITE_SIZE from separate rocprofv3 --pmc passes "
               f"of this workload (tag {e.get('tag', '?')}), not counted in this run")
        return float(e.get("hbm_bytes_per_launch", e.get("hbm_bytes_per_matvec"))), src
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


def exchange_text(world: int, flags: int, *, devices=None, poisson: bool = False, comm: str = "collective") -> str:
    """What the per-iteration exchange ran as, from the context's reported
    flags (cgx_info.flags: CGX_OVERLAP_ACTIVE, CGX_PULL_ACTIVE,
    CGX_FOLDED_ACTIVE, CGX_HALO_PULL_ACTIVE, CGX_THREADS_ACTIVE,
    CGX_HALO_OVERLAP_ACTIVE), not from what the defaults are meant to be."""
    import conjugate_gradient_amd as cg
    if world == 1:
        return "none (single GPU)"
    overlap = bool(flags & cg.CGX_OVERLAP_ACTIVE)
    pull, folded = bool(flags & cg.CGX_PULL_ACTIVE), bool(flags & cg.CGX_FOLDED_ACTIVE)
    if devices:
        where = "one process, row blocks on devices " + ",".join(map(str, devices))
        if poisson:
            halo = ("r's halo rows read in place from the neighbouring slabs by k_poisson_p (halo pull)"
                    if flags & cg.CGX_HALO_PULL_ACTIVE else
                    "halo rows by peer copies" + (" beside k_poisson_p's interior"
                                                  if flags & cg.CGX_HALO_OVERLAP_ACTIVE else ""))
            scal = ("r.r and p.Ap summed in rank order inside k_poisson_p / k_poisson_xr (folded combines)" if folded
                    else "scalars combined in rank order by a pull kernel per slab" if pull else
                    "scalars by peer copies + a combine kernel per slab")
            text = f"{where}: {halo} + {scal}"
        elif comm == "p2p":
            text = f"{where}: point-to-point_cg.c pattern, device copies through block 0"
        else:
            gather = ("p gathered by a pull kernel per block over peer access" if pull else
                      "p gathered by a peer copy per block pair")
            gather += " (overlapped with the own-block matVec)" if overlap else ""
            scal = ("p.Ap and r.r summed in rank order inside k_update_r / k_update_xp (folded combines)" if folded
                    else "scalars combined in rank order by a pull kernel per block" if pull else
                    "scalars by peer copies + a combine kernel per block")
            text = f"{where}: {gather} + {scal}"
        return text + ("; one enqueuing host thread per block" if flags & cg.CGX_THREADS_ACTIVE else "")
    if poisson:
        return ("RCCL halo ncclSend/Recv" + (" beside k_poisson_p's interior" if flags & cg.CGX_HALO_OVERLAP_ACTIVE
                                               else "") + " + 2x allreduce")
    if comm == "p2p":
        return "point-to-point_cg.c pattern: ncclSend/Recv via rank 0"
    if comm == "deterministic":
        return ("RCCL allgather(p)" + (" overlapped" if overlap else "")
                + " + rank-ordered scalar combine (allgather of partials)")
    return ("RCCL allgather(p) overlapped with own-block matVec + 2x allreduce" if overlap else
            "RCCL allgather(p) + 2x allreduce")


def cpu_baseline(n: int, iters: int = 5, threads_gen: int = 16) -> dict:
    """Oracle fp32-ref restatement of serialConjugate.c, 1 host core, `iters` iterations."""
    import numpy as np

    import oracle
    oracle.set_threads(threads_gen)  # generation only; the timed solve is single-threaded
    A, b = oracle.spd_hash(n, seed=SEED, dtype=np.float32)
    _, st = oracle.cg_f32ref(A, b, np.zeros(n, np.float32), max_iter=iters, eps=-1.0)
    del A
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": iters / st.t_loop_s,
        "unit": "iterations/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{iters} CG iterations (matVec + 2 dots + 3 vector updates each) of the same N={n} system in fp32, "
                   f"oracle/cg_oracle.c restatement of serialConjugate.c (bit-identical to it), single thread; "
                   f"initial residual matVec excluded; loop {st.t_loop_s:.2f} s, init {st.t_init_s:.2f} s; "
                   f"host CPU: {cpu}, {os.cpu_count()} logical CPUs visible"),
        "matvec_gbps_est": iters * 4.0 * n * n / st.t_loop_s / 1e9,
    }


def cpu_baseline_mt(n: int, iters: int = 3, threads: int = 16) -> dict:
    """SURVEY.md s8(d)'s optional non-reference leg: the fp64 oracle (conjgrad.m
    order, row-parallel matVec) on `threads` host cores, same system."""
    import numpy as np

    import oracle
    oracle.set_threads(threads)
    A, b = oracle.spd_hash(n, seed=SEED, dtype=np.float64)
    _, st = oracle.cg_f64(A, b, np.zeros(n), max_iter=iters, eps=-1.0)
    del A
    return {
        "value": iters / st.t_loop_s,
        "unit": "iterations/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{iters} CG iterations of the same N={n} system in fp64 (oracle_cg_f64, matVec rows split over "
                   f"{threads} threads; not the reference's algorithm order), loop {st.t_loop_s:.2f} s"),
        "matvec_gbps_est": iters * 8.0 * n * n / st.t_loop_s / 1e9,
    }


def cpu_baseline_reference(n_ref: int = 8192, n_bench: int = 65536) -> dict | None:
    """serialConjugate.c itself (unmodified, compiled by oracle/Makefile into
    oracle/_ref/serial_ref), timed in the same run on this host: its
    conjugrad() at its compiled size ROWS=8192 (serialConjugate.c:29) on the
    same generator's fp32 system, to convergence (EPSILON 1e-6), timed by its
    own clock() line (serialConjugate.c:208,249-251; the initial residual
    matVec included).  None when the reference build is absent."""
    import re
    import subprocess
    import tempfile

    import numpy as np

    import oracle
    exe = oracle.ref_binary()
    if not exe:
        return None
    oracle.set_threads(16)
    A, b = oracle.spd_hash(n_ref, seed=SEED, dtype=np.float32)
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        paths = [os.path.join(td, k) for k in ("A.f32", "b.f32", "x0.f32", "x.f32")]
        A.tofile(paths[0])
        b.tofile(paths[1])
        np.zeros(n_ref, np.float32).tofile(paths[2])
        del A
        out = subprocess.run([exe, str(n_ref), *paths], check=True, capture_output=True, text=True,
                             timeout=300).stdout
    t = float(re.search(r"average clock execution time in seconds: ([0-9.eE+-]+)", out).group(1))
    k = int(re.search(r"iterations (\d+)", out).group(1))
    value = k / t
    return {
        "value": value,
        "unit": "iterations/s",
        "cores": 1,
        "kind": "reference",
        "n": n_ref,
        "sample": (f"serialConjugate.c unmodified (oracle/_ref/serial_ref) at its compiled N={n_ref}, fp32, the same "
                   f"generator's system: {k} loop iterations plus the initial residual matVec in {t:.3f} s by its own "
                   f"clock() line, single thread"),
        "matvec_gbps_est": (k + 1) * 4.0 * n_ref * n_ref / t / 1e9,
        # per-iteration work is the N^2 matVec: the same core at the bench's N
        "scaled_to_bench_n": value * (n_ref / n_bench) ** 2,
    }


def cpu_baseline_poisson(m: int, iters: int = 3) -> dict:
    """Oracle matrix-free Poisson CG (fp64 restatement), 1 host core."""
    import numpy as np

    import oracle
    oracle.set_threads(1)
    n = m * m
    _, st = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), max_iter=iters, eps=-1.0)
    return {
        "value": iters / st.t_loop_s,
        "unit": "iterations/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{iters} iterations of the same m={m} Poisson CG (fp64, oracle/cg_oracle.c "
                   f"oracle_cg_poisson_f64; no reference counterpart exists), single thread; loop {st.t_loop_s:.2f} s"),
    }


def check_summary(rnorm: float, bnorm: float, rr_rec: float) -> dict:
    """The true residual ||b - A x|| / ||b|| after the run, next to the CG
    recurrence's sqrt(r.r) / ||b||: while the residual is well above
    rounding the two agree (x and r updated consistently, at full size);
    near convergence the recurrence goes on falling and they part."""
    import math
    rel_true = rnorm / bnorm
    rel_rec = math.sqrt(max(rr_rec, 0.0)) / bnorm
    out = {"relres": rel_true, "recurrence_relres": rel_rec}
    if rel_true > 1e-8:
        gap = abs(rel_true - rel_rec) / rel_true
        out.update(recurrence_gap=gap, recurrence_agrees=gap <= 1e-6)
    return out


def poisson_oracle_check(m: int, iters: int, x_gpu) -> dict:
    """configs[4] at full size against the oracle: the same fixed iteration
    count of the fp64 matrix-free CG (oracle_cg_poisson_f64, the restatement
    the tests pin) from x0 = 0, b = 1, on the host's cores (not timed, not a
    baseline); x within 1e-9 (the Poisson tests' tolerance)."""
    import numpy as np

    import oracle
    oracle.set_threads(16)
    n = m * m
    xo, _ = oracle.cg_poisson_f64(m, np.ones(n), np.zeros(n), max_iter=iters, eps=-1.0)
    rel = float(np.linalg.norm(x_gpu - xo) / np.linalg.norm(xo))
    return {"oracle_iterations": iters, "x_vs_oracle": rel, "x_vs_oracle_tol": 1e-9, "oracle_agrees": rel <= 1e-9}


# The phases that tile an iteration on the compute stream (cgx.h CGX_PH_*):
# their medians add up to about the iteration time.
TILING_PHASES = ("matvec_own", "gather_exposed", "matvec", "combine_pap", "update_r", "combine_rr", "update_xp", "gap")


def phase_summary(all_ph: list, ms_per_step: float) -> dict:
    """Per-rank medians (us) of each phase over the timed iterations, the max
    over ranks, and how the tiling phases add up against ms_per_step."""
    per_rank = [{k: round(v["median_us"], 2) for k, v in ph.items()} for ph in all_ph]
    sums = [sum(r[k] for k in TILING_PHASES) for r in per_rank]
    # means tile exactly (the phases are consecutive intervals), medians nearly
    mean_sums = [sum(ph[k]["mean_us"] for k in TILING_PHASES) for ph in all_ph]
    return {
        "what": "median over the timed iterations, per rank, of each phase of the rank's compute stream, from "
                "start / end stamps its kernels take on the device clock (CGX_PHASES: nothing inserted between "
                "kernels): a kernel's own span, or the span between two consecutive kernels (the exchange "
                "enqueued there, or a launch gap); matvec_own + gather_exposed + matvec + combine_pap + update_r "
                "+ combine_rr + update_xp + gap tile an iteration (parallel_cg.c:288-323)",
        "iterations_sampled": int(all_ph[0]["iteration"]["samples"]),
        "per_rank": per_rank,
        "max_over_ranks": {k: max(r[k] for r in per_rank) for k in per_rank[0]},
        "tiling_sum_ms_per_rank": [round(x / 1e3, 4) for x in sums],
        "tiling_sum_over_ms_per_step": max(sums) / 1e3 / ms_per_step,
        "tiling_mean_sum_over_ms_per_step": max(mean_sums) / 1e3 / ms_per_step,
    }


def rccl_summary(all_comm: list, solver_device: int) -> dict:
    """Did RCCL see N ranks on N devices, and what links join them: every
    rank's communicator view and PCI bus id, and the HIP link type / hops /
    peer access from rank 0's device to each other rank's device."""
    import conjugate_gradient_amd as cg
    visible = {}
    for d in range(cg.device_count()):
        try:
            visible[cg.device_pci_bus_id(d).lower()] = d
        except cg.CgxError:
            pass
    links = []
    for r, ci in enumerate(all_comm[1:], start=1):
        d = visible.get(ci["pci_bus_id"].lower())
        if d is None:
            links.append({"to_rank": r, "link": "device not visible to rank 0"})
        elif d == solver_device:
            links.append({"to_rank": r, "link": "same device"})
        else:
            links.append({"to_rank": r, **cg.device_link(solver_device, d)})
    return {
        "nranks": all_comm[0]["rccl_nranks"],
        "distinct_devices": len({ci["pci_bus_id"].lower() for ci in all_comm}),
        "pci_bus_ids": [ci["pci_bus_id"] for ci in all_comm],
        "ranks": all_comm,
        "links_from_rank0": links,
        "nccl_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith(("NCCL_", "RCCL_"))},
    }


def local_summary(devices: list, peer_active: bool, flags: int = 0) -> dict:
    """The single-process multi-GPU run (cgx_create_multi): which devices hold
    the row blocks, their PCI bus ids, the link / peer access from the first
    block's device to each other device, and the context's reported flags
    (cgx_info.flags: what the exchange ran as)."""
    import conjugate_gradient_amd as cg
    d0 = devices[0]
    return {
        "mode": "one process, cgx_create_multi",
        "devices": devices,
        "distinct_devices": len(set(devices)),
        "pci_bus_ids": [cg.device_pci_bus_id(d) for d in devices],
        "peer_active": peer_active,
        "flags": flags,
        "links_from_block0": [{"to_block": q, "link": "same device"} if d == d0 else
                              {"to_block": q, **cg.device_link(d0, d)} for q, d in enumerate(devices) if q],
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle", type=float, default=3.0,
                    help="seconds to idle after setting up the system, before the warmup steps")
    ap.add_argument("--workload", choices=["dense", "symmetric", "stream", "stream_symmetric", "poisson"],
                    default="dense",
                    help="dense: configs[2], A resident in HBM (default); "
                         "symmetric: configs[2]'s system with A kept as its upper triangle (CGX_SYMMETRIC, "
                         "one GPU, half the matVec bytes); "
                         "stream: configs[3], A kept in pinned host memory and streamed every matVec; "
                         "stream_symmetric: configs[3] with only the upper-triangle tiles streamed; "
                         "poisson: configs[4], matrix-free 5-point Poisson on an m x m grid (b=1, x0=0)")
    # --size / --grid: aliases that torch.distributed.run's own parser does not
    # mistake for abbreviations of its options (--n, --m are ambiguous there)
    ap.add_argument("--m", "--grid", dest="m", type=int, default=8192, help="Poisson grid width (n = m*m)")
    ap.add_argument("--comm", choices=["collective", "p2p", "nooverlap", "deterministic"], default="collective",
                    help="exchange: RCCL collectives, the p allgather overlapped with the own-block matVec "
                         "when the context measured that faster at creation (default; the same bits either "
                         "way), point-to-point_cg.c's gather-to-root + send-to-all (p2p), collectives "
                         "without overlap, or the scalars combined in rank order (deterministic)")
    ap.add_argument("--n", "--size", dest="n", type=int, default=None,
                    help="system size (default 65536 dense, 131072 stream)")
    ap.add_argument("--resident-gb", type=float, default=0.0,
                    help="stream workload: keep this many GB of each GPU's rows of A in HBM and stream only the "
                         "rest (CGX_STREAM_RESIDENT_MB; an out-of-core matrix keeps what fits). Default 0: all "
                         "of A streams every matVec, as configs[3] states")
    ap.add_argument("--phases", choices=["auto", "on", "off"], default="auto",
                    help="the iteration's kernels stamp their start / end on the device clock (CGX_PHASES; "
                         "nothing is inserted between kernels, overhead within run-to-run noise, "
                         "profiles/r03_phases_ab.jsonl) and the line reports per-phase medians per rank; "
                         "auto: on for the dense resident workloads")
    ap.add_argument("--devices", default=None,
                    help="without a launcher: the devices of the row blocks, comma-separated (default 0..N-1 for "
                         "--gpus N); repeats put several row blocks on one GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-n", type=int, default=None, help="N for the CPU baseline (default: --n)")
    args = ap.parse_args(argv)

    rank, local_rank, world = dist_env()
    use_dist = launched_by_torchrun()
    dist = dist_init() if use_dist else None
    if use_dist and world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    import conjugate_gradient_amd as cg
    # Without a launcher, --gpus N > 1 (or --devices) runs the N row blocks from
    # this process (cgx_create_multi); world is then the number of row blocks.
    devices = None
    if not use_dist and (args.gpus > 1 or args.devices):
        devices = ([int(v) for v in args.devices.split(",")] if args.devices else list(range(args.gpus)))
        if args.devices and args.gpus not in (1, len(devices)):
            raise SystemExit(f"bench.py: --gpus {args.gpus} but --devices lists {len(devices)} row blocks")
        ndev = cg.device_count()
        missing = sorted({d for d in devices if not 0 <= d < ndev})
        if missing:
            raise SystemExit(f"bench.py: --gpus {len(devices)} asks for device(s) {missing}, but {ndev} "
                             f"device(s) are visible; run on a node with {len(devices)} GPUs, or under "
                             f"torch.distributed.run with one process per GPU")
        world = len(devices)
    n_gpus = len(set(devices)) if devices else world
    span = f"{world} GPU(s)" if n_gpus == world else f"{world} row blocks on {n_gpus} GPU(s)"
    stream = args.workload in ("stream", "stream_symmetric")
    poisson = args.workload == "poisson"
    symmetric = args.workload in ("symmetric", "stream_symmetric")
    if symmetric and world > 1:
        raise SystemExit(f"--workload {args.workload} runs on one GPU")
    m = args.m if poisson else None
    n = m * m if poisson else (args.n or (131072 if stream else 65536))
    if (m if poisson else n) % world:
        raise SystemExit(f"{m if poisson else n} is not divisible by {world}")
    flags = cg.CGX_F64 | cg.CGX_TIMING | (cg.CGX_HOST_STREAM if stream else 0) | (cg.CGX_SYMMETRIC if symmetric else 0)
    flags |= {"collective": 0, "p2p": cg.CGX_COMM_P2P, "nooverlap": cg.CGX_NO_OVERLAP,
              "deterministic": cg.CGX_DETERMINISTIC}[args.comm]
    phases = args.phases != "off" and not (poisson or stream or symmetric)
    if phases:
        flags |= cg.CGX_PHASES
    if stream and args.resident_gb > 0:
        os.environ["CGX_STREAM_RESIDENT_MB"] = str(int(args.resident_gb * 1024))
    if use_dist:
        uid = bcast_bytes(dist, cg.get_unique_id() if rank == 0 else None)
        # one GPU per process: LOCAL_RANK indexes the visible devices; if the
        # launcher already narrowed the visibility per rank (one device seen),
        # that device is the rank's
        ndev = max(1, cg.device_count())
        solver = cg.Solver(n, rank=rank, nranks=world, unique_id=uid, device=local_rank % ndev, flags=flags,
                           poisson_m=m)
    elif devices is not None:
        solver = cg.Solver(n, devices=devices, flags=flags, poisson_m=m)
    else:
        solver = cg.Solver(n, device=0, flags=flags, poisson_m=m)
    nloc = solver.info.nrows // len(devices or [0])
    ctx_flags = solver.info.flags
    overlap = solver.overlap_info() if world > 1 and not (poisson or stream or symmetric) else None
    fused = bool(solver.info.flags & cg.CGX_FUSED_ACTIVE)
    # fused Poisson: x every other (or third) iteration
    xperiod = (3 if solver.info.flags & cg.CGX_XDEFER3_ACTIVE else 2) if solver.info.flags & cg.CGX_XDEFER_ACTIVE else 1
    plan = None if (poisson or symmetric) else solver.matvec_plan()

    if poisson:
        solver.fill(1.0, 0.0)
    else:
        solver.generate_spd(SEED)
    solver.synchronize()
    # Settle before the warmup: a process that starts right after another
    # one freed tens of GB measured its matVec 2-5 % slower (the release of
    # that memory shares HBM with it); with a few seconds of gap every run
    # read the same rate (profiles/r01_bench_variance.json).  Setup only: no
    # step is skipped or added.
    if args.settle > 0:
        time.sleep(args.settle)
    solver.begin()
    if args.warmup:
        solver.iterate(args.warmup, eps=-1.0)
    solver.synchronize()
    cg.lib().cgx_dev_synchronize()
    solver.reset_timing()

    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    done, _ = solver.iterate(args.steps, eps=-1.0)
    t_enq = time.perf_counter()  # fixed-count cgx_iterate returns once everything is enqueued
    solver.synchronize()
    cg.lib().cgx_dev_synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    assert done == args.steps
    elapsed = t1 - t0
    enqueue_s = t_enq - t0
    st = solver.stats()
    mv_ms = st.matvec_ms / max(1, st.matvec_count)
    if dist:
        elapsed = max_over_ranks(dist, elapsed)
        enqueue_s = max_over_ranks(dist, enqueue_s)
        mv_ms_max = max_over_ranks(dist, mv_ms)
    else:
        mv_ms_max = mv_ms

    # after the timed region: what each phase of an iteration cost (the
    # events recorded inside it are resolved only now), and what RCCL ran on
    ph = solver.phase_times() if phases else None
    comm = solver.comm_info() if (use_dist and world > 1) else None
    peer_flag = bool(solver.info.flags & cg.CGX_PEER_ACTIVE) if devices else False
    all_ph = gather_objects(dist, ph) if (dist and phases) else ([ph] if phases else None)
    all_comm = gather_objects(dist, comm) if comm is not None else None

    # correctness after the timed region (not timed): the true residual of x,
    # and the CG recurrence's r.r, which must agree with it while the
    # residual is above rounding (x and r updated consistently at full size)
    rr_rec = st.rr
    rnorm, bnorm = solver.residual_norm()
    x_gpu = solver.get_x() if (poisson and world == 1 and not args.no_cpu and rank == 0) else None
    solver.close()

    if rank != 0:
        if dist:
            dist.barrier()
        return 0

    # stencil: read the slab once (+2 halo rows), write Ap; dense: SURVEY.md s8(d)
    # fused Poisson: the timed kernel is k_poisson_xr_f64 (reads p_k with its two
    # halo rows, x and r; writes x and r); unfused: the stencil (p -> Ap).
    # dense: SURVEY.md s8(d)
    # With x updated every other iteration the xr launches alternate between
    # 24 B/point (p_k, r -> r) and 48 (p_{k-1}, p_k, x, r -> x, r): 36 on average;
    # every third: 24, 24, 56 (p_{k-2} too): 34.67.
    xr_bpp = {1: 40.0, 2: 36.0, 3: 104.0 / 3}[xperiod]
    if poisson:
        bytes_launch = (xr_bpp * nloc + 16 * m) if fused else (16 * nloc + 16 * m)
    elif symmetric:  # the stored tiles + p + y (the per-tile partials are extra traffic, not algorithmic)
        lda = (n + 127) // 128 * 128
        bytes_launch = 8 * (lda // 128) * (lda // 128 + 1) // 2 * 128 * 128 + 8 * n + 8 * n
    else:
        bytes_launch = matvec_bytes(n, nloc)
    lda = (n + 127) // 128 * 128
    res_rows = res_bytes = 0  # the rows (symmetric: 128x128 tiles) kept in HBM, setup's rounding
    if stream and args.resident_gb > 0:
        unit = 128 * 128 * 8 if symmetric else lda * 8
        units = (lda // 128) * (lda // 128 + 1) // 2 if symmetric else nloc
        res_rows = min(units, int(args.resident_gb * 1024) * (1 << 20) // unit)
        res_bytes = res_rows * unit if symmetric else 8 * res_rows * n
    # a streamed workload's roofline is the host link: the bytes that cross it
    link_bytes = bytes_launch - res_bytes if stream else bytes_launch
    # ... unless so much of A is resident that HBM, not the link, bounds the matVec
    link_bound = stream and link_bytes / H2D_PEAK_GBS >= bytes_launch / HBM_PEAK_GBS
    # Several row blocks: the matVec is one rotated launch after p's
    # allgather, or (overlap chosen) the own-column-block launch beside the
    # allgather and the rest launch after it, both on the compute stream; the
    # CGX_TIMING events bracket all of it, the wait for the allgather
    # included.  The kernels' own spans come from the CGX_PHASES stamps
    # (device clock, first block's start to last block's end): the union of
    # their spans (matvec_busy) is the matVec's duration on rank 0's GPU.
    # The roofline takes the slowest rank's kernel spans (max over ranks);
    # matvec_ms stays the CGX_TIMING event figure of earlier rounds.
    mv_kernel_ms = None
    if all_ph is not None and world > 1 and all_ph[0]["matvec_busy"]["samples"] > 0:
        # the union of the matVec kernels' spans (one launch, or the overlap's own-block and rest
        # launches): the matVec's duration without the wait for p
        mv_kernel_ms = max(ph["matvec_busy"]["median_us"] for ph in all_ph) / 1e3
    achieved = (link_bytes if link_bound else bytes_launch) / ((mv_kernel_ms or mv_ms) * 1e-3) / 1e9
    traffic, traffic_src = (None, None) if stream else pmc_traffic(
        f"poisson_m{m}_g{world}" if poisson else f"n{n}_g{world}" + ("_symmetric" if symmetric else ""))
    peak = H2D_PEAK_GBS if link_bound else HBM_PEAK_GBS
    iters_per_s = args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": iters_per_s,
        "unit": "iterations/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_s": args.settle,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: 5-point Laplacian, b = 1, x0 = 0" if poisson else
                 f"synthetic: generateSPDmatrix.m-style dense SPD (0.5(R+R')+nI, counter hash, seed {SEED}) "
                 f"generated on device; x0 = 0"),
        "config": {
            "workload": (f"configs[3]: N={n} dense SPD fp64 CG, A streamed from pinned host memory every matVec"
                         + (" as its upper-triangle tiles (CGX_SYMMETRIC)" if symmetric else "")
                         + (f" except the first {res_rows} {'tiles' if symmetric else 'rows per GPU'}, kept in HBM "
                            f"({args.resident_gb:g} GB budget)" if res_rows else "")
                         + f", row-block over {span}, fixed-count iterations") if stream else
                        (f"configs[4]: matrix-free 5-point Poisson CG, m={m} (N={n}), b=1, x0=0, slabs over {span}, "
                         f"halo exchange, fixed-count iterations") if poisson else
                        (f"configs[{1 if n == 16384 else 2}] system, A stored as its upper triangle (128x128 tiles, "
                         f"CGX_SYMMETRIC), N={n} dense SPD fp64 CG on 1 GPU, fixed-count iterations") if symmetric else
                        (f"configs[{1 if n == 16384 else 2}]: N={n} dense SPD fp64 CG, row-block over {span}, "
                         f"fixed-count iterations"),
            "n": n,
            "rows_per_gpu": nloc,
            "parallelism": f"rowblock{world}",
            "exchange": exchange_text(world, ctx_flags, devices=devices, poisson=poisson, comm=args.comm),
        },
        # the host's side: time inside the fixed-count cgx_iterate call (it returns once the K
        # iterations are enqueued; a full hardware queue makes it wait, so a value near ms_per_step
        # means the device ran behind, one above it means the host bounds the loop); max over ranks
        "host_enqueue_us_per_iteration": enqueue_s / args.steps * 1e6,
        "matvec_gbps": bytes_launch / (mv_ms * 1e-3) / 1e9,
        "matvec_ms": mv_ms,
        "matvec_ms_source": ("HIP events around the matVec launch(es) on rank 0's / block 0's stream (CGX_TIMING); "
                             "with several row blocks and the overlap they bracket both launches and the wait for "
                             "p's allgather between them"),
        "matvec_ms_max_rank": mv_ms_max,
        # the kernels alone: the union of the matVec kernels' spans on the device clock, the slowest rank's
        # (roofline.achieved)
        "matvec_kernel_ms": mv_kernel_ms,
        "matvec_kernel_gbps": bytes_launch / (mv_kernel_ms * 1e-3) / 1e9 if mv_kernel_ms else None,
        "roofline": {
            "bound": "h2d" if link_bound else "hbm",
            "achieved": achieved,
            "peak": peak,
            "unit": "GB/s",
            "frac": achieved / peak,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": (("k_poisson_xr_f64" if fused else "k_stencil5_f64") if poisson else
                       "H2D copies + k_symv_f64 per chunk + k_symv_reduce_f64" if (symmetric and stream) else
                       "k_symv_f64 + k_symv_reduce_f64" if symmetric else "k_matvec_f64"),
            "plan": plan,
            "algorithmic_bytes_per_launch": bytes_launch,
            "link_bytes_per_launch": link_bytes if stream else None,
        },
        "check": check_summary(rnorm, bnorm, rr_rec),
        # algorithmic bytes of a whole iteration: 64 B/point fused (r, p_{k-1} -> p_k;
        # p_k, x, r -> x, r), 60 with x updated every other iteration (58.67 every
        # third), 80 B/point for the stencil / r / x,p split
        "iteration_gbps": (((24.0 + xr_bpp) if fused else 80.0) * n / (elapsed / args.steps) / 1e9)
        if poisson else None,
    }
    if overlap is not None:
        out["overlap"] = overlap
    if all_ph is not None:
        out["phases_us"] = phase_summary(all_ph, elapsed / args.steps * 1e3)
    if all_comm is not None:
        out["rccl"] = rccl_summary(all_comm, solver_device=local_rank % max(1, cg.device_count()))
    if devices:
        out["config"]["row_blocks"] = len(devices)
        out["multi_device"] = local_summary(devices, peer_flag, ctx_flags)
    if world == 1 and not args.no_cpu and poisson:
        out["cpu_baseline"] = cpu_baseline_poisson(m)
        out["check"].update(poisson_oracle_check(m, args.warmup + args.steps, x_gpu))
        del x_gpu
    elif world == 1 and not args.no_cpu and not stream and not symmetric:
        out["cpu_baseline"] = cpu_baseline(args.cpu_n or n)
        out["cpu_baseline_mt"] = cpu_baseline_mt(args.cpu_n or n)
        ref = cpu_baseline_reference(n_bench=n)
        if ref:
            out["cpu_baseline_reference"] = ref
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
    return 0


def run() -> int:
    """main(), failing fast: a libcgx error (in rank mode e.g. CGX_ERR_RCCL when
    a peer died or ranks diverged, after CGX_RCCL_TIMEOUT_S at most) ends this
    rank with a non-zero status and the message on stderr, so the launcher
    stops the job instead of the other ranks waiting in a barrier."""
    import conjugate_gradient_amd as cg
    try:
        return main()
    except cg.CgxError as e:
        rank = os.environ.get("RANK", "0")
        print(f"bench.py rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)  # skip interpreter / process-group teardown that could wait on dead peers


if __name__ == "__main__":
    sys.exit(run())
