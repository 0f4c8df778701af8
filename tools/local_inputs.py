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

  python tools/local_inputs.py [rounds] > profiles/rNN_local_inputs.jsonl
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

N = 65536


def run(S, form, iters=10):
    os.environ["CGX_LOCAL_THREADS"] = "1" if form == "threads" else "0"
    with cg.Solver(N, devices=[0] * S) as s:
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
    return {"n": N, "blocks": S, "form": form, "flags": int(flags),
            "threads_active": bool(flags & cg.CGX_THREADS_ACTIVE), "overlap_info": info,
            "enqueue_us": round((t1 - t0) / iters * 1e6, 2), "wall_us": round((t2 - t0) / iters * 1e6, 2)}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for r in range(rounds):
        for S in (2, 4, 8):
            for form in ("onethread", "threads"):
                out = run(S, form)
                out["round"] = r
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
