"""The 1 -> 2/4/8 GPU prediction for configs[2] (N=65536, row blocks), made
from what one GPU can measure, so that a SCALE line's per-phase breakdown
(bench.py `phases_us`) can be read against it phase by phase.

Measured inputs (committed under profiles/):
  - the 1-GPU iteration: bench.py ms_per_step (BENCH_r03 / the round's line);
  - one rank's kernels of an overlapped iteration at G ranks, without the
    collectives (tools/microbench/rank_iteration, its wall time per iteration
    and a rocprofv3 kernel trace: own-block matVec, rest matVec, update_r,
    update_xp, the idle gaps between them);
  - the one-process mode's host enqueue per iteration at S row blocks
    (tools/r04_multishard_floor.py).
Stated assumptions (not measurable on a one-GPU box, where RCCL runs over
loopback sockets): the latency of RCCL's 8-byte allreduce and of the p
allgather over xGMI, as a low / mid / high range.

  python tools/r04_scale_model.py > profiles/r04_scale_model.json
  python tools/r04_scale_model.py --compare LINE.json [...]
      (bench.py lines of an N>1 run, e.g. from the driver's SCALE record:
      each phase's max over ranks against the model's mid prediction, and
      the phase that is furthest above it)
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.environ.get("R04_PROF_DIR", os.path.join(ROOT, "profiles"))
N = 65536

# RCCL small-message collectives over xGMI on one 8-GPU MI300-class node (LL
# protocol): an 8-byte allreduce in the tens of microseconds at most; the
# allgather of 8*N/G bytes per rank adds its transfer at ~100 GB/s effective
# per peer link (MI355X: 7 xGMI links per GPU, ~153 GB/s each, per the project
# brief).  These are
# assumptions, labelled as such in the output.
ALLREDUCE_US = {"low": 6.0, "mid": 12.0, "high": 25.0}
GATHER_LAT_US = {"low": 6.0, "mid": 12.0, "high": 25.0}
GATHER_GBPS_PER_LINK = 100.0


def kernel_spans(trace_csv):
    """Per-kernel durations (us) of the timed iterations, grouped by role."""
    rows = list(csv.DictReader(open(trace_csv)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    it = [k for k in ks if "k_matvec_f64" in k[2] or "k_update_r_f64" in k[2] or "k_update_xp_f64" in k[2]]
    roles = {"matvec_own": [], "matvec": [], "update_r": [], "update_xp": []}
    gaps = []
    # iterations are 4 launches: matVec (own), matVec (rest), update_r, update_xp
    for q in range(0, len(it) - 3, 4):
        grp = it[q:q + 4]
        if not ("k_matvec" in grp[0][2] and "k_matvec" in grp[1][2] and "update_r" in grp[2][2]):
            continue
        for name, k in zip(("matvec_own", "matvec", "update_r", "update_xp"), grp):
            roles[name].append((k[1] - k[0]) / 1e3)
        gaps.append(sum(max(0, grp[j + 1][0] - grp[j][1]) for j in range(3)) / 1e3)
    med = {k: statistics.median(v) for k, v in roles.items() if v}
    med["gap"] = statistics.median(gaps) if gaps else 0.0
    med["iterations_traced"] = len(gaps)
    return med


def main():
    one_gpu = json.load(open(os.path.join(PROF, "r04_scale_inputs.json")))
    ms1 = one_gpu["one_gpu_ms_per_step"]
    walls = {}
    for line in open(os.path.join(PROF, "r04_rank_iteration.jsonl")):
        d = json.loads(line)
        walls[d["ranks"]] = d["us_per_iteration_without_collectives"]
    floor = {}
    fpath = os.path.join(PROF, "r04_multishard_floor.jsonl")
    if os.path.exists(fpath):
        for line in open(fpath):
            d = json.loads(line)
            if d["n"] == 4096 and d["exchange"] == "kernel":
                floor.setdefault(d["shards"], []).append(d.get("enqueue_10_us", d["enqueue_us"]))
    out = {
        "what": "configs[2] (N=65536 dense fp64, row blocks) at G GPUs: one rank's measured kernels plus assumed "
                "collective latencies -> predicted iteration, it/s and speed-up over the measured 1-GPU step; "
                "the phase keys are bench.py phases_us's",
        "one_gpu": {"ms_per_step": ms1, "it_per_s": 1e3 / ms1, "source": one_gpu["source"]},
        "assumptions": {
            "allreduce_8B_us": ALLREDUCE_US,
            "allgather_latency_us": GATHER_LAT_US,
            "allgather_GBps_per_peer_link": GATHER_GBPS_PER_LINK,
            "source": "not measurable on a one-GPU box (RCCL runs over loopback sockets there); RCCL's LL-protocol "
                      "small-message latency on one xGMI-connected node is assumed in the 5-25 us range (not from a "
                      "document available here); the MI355X has 7 xGMI links per GPU at ~153 GB/s each (the "
                      "project brief), taken at 100 GB/s effective per peer",
        },
        "per_G": {},
    }
    for G in (2, 4, 8):
        tr = os.path.join(PROF, f"r04_rank_kernel_trace_g{G}.csv")
        if G not in walls or not os.path.exists(tr):
            continue
        k = kernel_spans(tr)
        slice_bytes = 8 * N // G
        entry = {"rows_per_rank": N // G, "measured": {
            "us_per_iteration_without_collectives": walls[G],
            "kernel_medians_us": {x: round(k[x], 2) for x in ("matvec_own", "matvec", "update_r", "update_xp")},
            "gaps_between_kernels_us": round(k["gap"], 2), "iterations_traced": k["iterations_traced"],
            "matvec_TBps": round((8 * (N // G) * N + 8 * N + 8 * (N // G)) / ((k["matvec_own"] + k["matvec"]) * 1e-6)
                                 / 1e12, 3)}}
        pred = {}
        for case in ("low", "mid", "high"):
            gather = GATHER_LAT_US[case] + slice_bytes / (GATHER_GBPS_PER_LINK * 1e3)  # per peer, peers in parallel
            exposed = max(0.0, gather - k["matvec_own"])
            ar = ALLREDUCE_US[case]
            it_us = walls[G] + exposed + 2 * ar
            pred[case] = {
                "phases_us": {"matvec_own": round(k["matvec_own"], 2), "gather_exposed": round(exposed, 2),
                              "matvec": round(k["matvec"], 2), "combine_pap": ar, "update_r": round(k["update_r"], 2),
                              "combine_rr": ar, "update_xp": round(k["update_xp"], 2),
                              "gap": round(max(0.0, walls[G] - k["matvec_own"] - k["matvec"] - k["update_r"]
                                               - k["update_xp"]), 2)},
                "iteration_us": round(it_us, 1), "it_per_s": round(1e6 / it_us, 1),
                "speedup_vs_1gpu": round(ms1 * 1e3 / it_us, 2),
                "efficiency": round(ms1 * 1e3 / it_us / G, 3)}
        entry["predicted"] = pred
        if G in floor:
            enq = statistics.median(floor[G])
            entry["one_process_mode"] = {
                "host_enqueue_us_per_iteration": enq,
                "host_bound": enq > pred["mid"]["iteration_us"],
                "note": "cg_hip --gpus G / bench.py --gpus G without a launcher: the host enqueues every block's "
                        "launches from one thread; the iteration is the larger of this and the device's",
            }
        out["per_G"][str(G)] = entry
    json.dump(out, sys.stdout, indent=1)
    print()


def compare(paths):
    model = json.load(open(os.path.join(PROF, "r04_scale_model.json")))
    for path in paths:
        text = open(path).read()
        line = json.loads([ln for ln in text.splitlines() if ln.strip().startswith("{")][-1])
        G = str(line["n_gpus"])
        pred = model["per_G"].get(G, {}).get("predicted", {}).get("mid")
        meas = line.get("phases_us", {}).get("max_over_ranks")
        if not pred or not meas:
            print(json.dumps({"file": path, "n_gpus": G, "error": "no model entry or no phases_us"}))
            continue
        delta = {k: round(meas.get(k, 0.0) - v, 2) for k, v in pred["phases_us"].items()}
        culprit = max(delta, key=delta.get)
        print(json.dumps({"file": path, "n_gpus": G, "it_per_s": line["value"],
                          "predicted_it_per_s": pred["it_per_s"], "measured_phases_us": meas,
                          "predicted_phases_us": pred["phases_us"], "delta_us": delta,
                          "furthest_above_model": culprit}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--compare":
        compare(sys.argv[2:])
    else:
        main()
