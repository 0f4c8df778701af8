#!/usr/bin/env python3
"""Measured inputs of the scale model's one-process (LOCAL) prediction, on
one GPU: configs[2] (N = 65536) as S = 2 / 4 / 8 row blocks on device 0
(cgx_create_multi, devices=[0]*S), per S and enqueue form:

  overlap_info    what the context measured at creation: the pull-kernel
                  gather alone (allgather_us: S gathers at once on one device,
                  events included, no xGMI), the two whole forms end to end;
  enqueue_us      host time inside a fixed-count cgx_iterate per iteration,
                  10 iterations right after a sync (empty queues: the host's
                  cost alone);
  wall_us         the same 10 iterations to the end of the sync (on one GPU:
                  every block's kernels together).

Forms: "onethread" (the default: the calling thread enqueues every block's
work) and "threads" (CGX_LOCAL_THREADS=1: one host thread per block; on one
GPU the runtime serialises their launches).

  python tools/local_inputs.py [rounds] [--blocks 2,4,8] [--forms onethread,threads] [--iters 10]
      > profiles/rNN_local_inputs.jsonl
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

N = 65536


def run(S, form, iters=10, n=N):
    os.environ["CGX_LOCAL_THREADS"] = "1" if form == "threads" else "0"
    with cg.Solver(n, devices=[0] * S) as s:
        info = s.overlap_info()
        flags = s.info.flags
        s.generate_spd(42)
        s.begin()
        s.iterate(3, eps=-1.0)
        s.synchronize()
        t0 = time.perf_counter()
        s.iterate(iters, eps=-1.0)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
    return {"n": n, "blocks": S, "form": form, "flags": int(flags),
            "threads_active": bool(flags & cg.CGX_THREADS_ACTIVE), "overlap_info": info,
            "enqueue_us": round((t1 - t0) / iters * 1e6, 2), "wall_us": round((t2 - t0) / iters * 1e6, 2)}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("rounds", type=int, nargs="?", default=2)
    ap.add_argument("--blocks", default="2,4,8")
    ap.add_argument("--forms", default="onethread,threads")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--n", type=int, default=N,
                    help="system size; at N = 65536 the shared GPU runs behind the host, whose launches then "
                         "wait for queue space, so the host's own cost is read at a small N (4096)")
    a = ap.parse_args()
    for r in range(a.rounds):
        for S in (int(v) for v in a.blocks.split(",")):
            for form in a.forms.split(","):
                out = run(S, form, a.iters, a.n)
                out["round"] = r
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
