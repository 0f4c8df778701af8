"""Per-iteration cost of the single-process multi-shard path (cgx_create_multi,
`cg_hip --gpus P`) at S = 1/2/4/8 row blocks, every shard on device 0
(devices=[0]*S): fixed-count iterations (dense fp64, the overlapped exchange),
timed four ways:
  enqueue_us  host time inside cgx_iterate per iteration (it returns without
              a sync for eps < 0, so this is the host's enqueue cost alone);
  wall_us     host time from the call to the end of cgx_synchronize;
  enqueue_10_us  the same for 10 (enqueue_16_us: 16) iterations right after a sync (empty queues:
              the host's cost alone even when the device is the slower side);
  phases      the CGX_PHASES device-clock medians on shard 0.
On one GPU the shards' kernels share the device, so wall_us is the sum of all
shards' work; the host side (enqueue_us) is what a distinct-device run pays
too.  Exchange forms (read at context creation), interleaved: "kernel" (the
default: one pull kernel per consuming shard for p's gather, the two scalar
combines folded into the update kernels, one enqueuing thread per block),
"onethread" (the same, all enqueued by the calling thread), "nofuse" (CGX_LOCAL_FUSE=0: a
combine kernel per shard and scalar) and "copy" (CGX_LOCAL_XCHG=copy: round
3's hipMemcpyPeerAsync per pair).  (Round 4's "graph" form, a hipGraph replay
with every block on one device, was removed in round 6: no deployment puts
every row block on one GPU.)
With --poisson the sizes are grid widths m and the operator is the fused
Poisson iteration (no CGX_PHASES): forms "pull" (round 5's default: r's halo
rows read in place by k_poisson_p, both scalar combines folded into the
kernels), "nofuse" (the pull with a combine kernel per slab and scalar) and
"copy" (round 4's default: per-neighbour hipMemcpyPeerAsync of the halo rows
behind k_poisson_p's interior runs, combine kernels).
Usage:  python tools/multishard_floor.py [--poisson] [rounds] [n or m,...] [S,...] [forms]
  > profiles/rNN_multishard_floor.jsonl"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402


def run(n, shards, steps=200, warm=32, phases=True):
    flags = cg.CGX_PHASES if phases else 0
    with cg.Solver(n, flags=flags, devices=[0] * shards) as s:
        s.generate_spd(42)
        info = s.info
        s.begin()
        s.iterate(warm, eps=-1.0)
        s.synchronize()
        s.reset_timing()
        t0 = time.perf_counter()
        s.iterate(steps, eps=-1.0)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        ph = s.phase_times() if phases else {}
        # the enqueue alone, with the queues empty: 10 iterations (200 can fill
        # the hardware queues on one GPU and then time the device instead)
        t3 = time.perf_counter()
        s.iterate(10, eps=-1.0)
        t4 = time.perf_counter()
        s.synchronize()
        t5 = time.perf_counter()
        s.iterate(16, eps=-1.0)
        t6 = time.perf_counter()
        s.synchronize()
        rn, bn = s.residual_norm()
    return {"n": n, "shards": shards, "steps": steps, "exchange": ("copy" if os.environ.get("CGX_LOCAL_XCHG") == "copy" else
                                             "nofuse" if os.environ.get("CGX_LOCAL_FUSE") == "0" else
                                             "onethread" if os.environ.get("CGX_LOCAL_THREADS") == "0" else "kernel"),
            "flags": int(info.flags),
            "enqueue_us": round((t1 - t0) / steps * 1e6, 2), "wall_us": round((t2 - t0) / steps * 1e6, 2),
            "enqueue_10_us": round((t4 - t3) / 10 * 1e6, 2),
            "enqueue_16_us": round((t6 - t5) / 16 * 1e6, 2),
            "relres": rn / bn,
            "phases_median_us": {k: round(v["median_us"], 2) for k, v in ph.items() if v["samples"]}}


def run_poisson(m, shards, steps=200, warm=30):
    with cg.Solver(None, poisson_m=m, devices=[0] * shards) as s:
        s.fill(1.0, 0.0)
        info = s.info
        s.begin()
        s.iterate(warm, eps=-1.0)
        s.synchronize()
        t0 = time.perf_counter()
        s.iterate(steps, eps=-1.0)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        s.iterate(9, eps=-1.0)  # the enqueue alone, queues empty (a multiple of the x period 3)
        t3 = time.perf_counter()
        s.synchronize()
    return {"m": m, "shards": shards, "steps": steps,
            "exchange": ("copy" if os.environ.get("CGX_LOCAL_XCHG") == "copy" else
                         "nofuse" if os.environ.get("CGX_LOCAL_FUSE") == "0" else "pull"),
            "flags": int(info.flags), "enqueue_us": round((t1 - t0) / steps * 1e6, 2),
            "wall_us": round((t2 - t0) / steps * 1e6, 2), "enqueue_9_us": round((t3 - t2) / 9 * 1e6, 2)}


def main_poisson(argv):
    rounds = int(argv[0]) if len(argv) > 0 else 2
    sizes = tuple(int(v) for v in argv[1].split(",")) if len(argv) > 1 else (1024, 2048, 4096, 8192)
    counts = tuple(int(v) for v in argv[2].split(",")) if len(argv) > 2 else (8,)
    forms = tuple(argv[3].split(",")) if len(argv) > 3 else ("pull", "nofuse", "copy")
    for r in range(rounds):
        for m in sizes:
            for S in counts:
                for form in forms:
                    os.environ["CGX_LOCAL_XCHG"] = "copy" if form == "copy" else "kernel"
                    os.environ["CGX_LOCAL_FUSE"] = "0" if form == "nofuse" else "1"
                    out = run_poisson(m, S)
                    out["round"] = r
                    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--poisson":
        return main_poisson(sys.argv[2:])
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else (4096,)
    counts = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else (1, 2, 4, 8)
    forms = tuple(sys.argv[4].split(",")) if len(sys.argv) > 4 else ("kernel", "onethread", "nofuse", "copy")
    for r in range(rounds):
        for n in sizes:
            for S in counts:
                for form in forms if S > 1 else forms[:1]:
                    os.environ["CGX_LOCAL_XCHG"] = "copy" if form == "copy" else "kernel"
                    os.environ["CGX_LOCAL_FUSE"] = "0" if form == "nofuse" else "1"
                    os.environ["CGX_LOCAL_THREADS"] = "0" if form in ("onethread", "nofuse", "copy") else "1"
                    out = run(n, S)
                    out["round"] = r
                    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
