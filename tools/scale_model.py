"""The 1 -> 2/4/8 GPU prediction for configs[2] (N=65536, row blocks), made
from what one GPU can measure, so that a SCALE line's per-phase breakdown
(bench.py `phases_us`) can be read against it phase by phase.

Measured inputs (committed under profiles/):
  - the 1-GPU iteration: the driver's latest N=1 bench line (the highest
    BENCH_rNN.json at the repo root: ms_per_step), or
    profiles/<tag>_scale_inputs.json;
  - one rank's kernels at G ranks without the collectives, in both forms the
    context chooses between at creation (cgx_exchange.hip choose_overlap):
    split (own-column-block launch beside the allgather, then the rest) and
    one (the allgather, then one launch of the same bits) -- the wall time per
    iteration from tools/microbench/rank_iteration (profiles/r05_rank_iteration.jsonl)
    and, where present, a rocprofv3 kernel trace of it
    (profiles/r05_rank_kernel_trace_g{G}.csv) for the per-kernel medians.
Stated assumptions (not measurable on a one-GPU box, where RCCL runs over
loopback sockets): the latency of RCCL's 8-byte allreduce and of the p
allgather over xGMI, as a low / mid / high range.

Per G and case the model predicts both forms and the one the library would
pick (overlap only when that form is the faster one end to end), which is
the form a SCALE line reports in its "overlap" key.

Two deployments, two predictions per G:
  "rccl"  -- one process per GPU (torchrun, the driver's N>1 launch): the
             RCCL allgather and two 8-byte allreduces per iteration;
  "local" -- `bench.py --gpus G` without a launcher (cgx_create_multi over
             devices 0..G-1): p gathered by a pull kernel per device over
             xGMI, both scalars summed by the update kernels themselves
             (folded combines, no collective), every launch enqueued by one
             host thread.  Measured inputs (profiles/r06_local_inputs.jsonl,
             tools/local_inputs.py: the configs[2] blocks all on one GPU):
             the host's enqueue per iteration at S blocks, and the pull
             gather as the context times it at creation (S gathers at once
             on one device: per device, its S-th share).  Assumed: the xGMI
             latency of a peer read.  The iteration is the slower of the
             device's work and the host's enqueue, and the model says which.

  python tools/scale_model.py > profiles/r06_scale_model.json
  python tools/scale_model.py --compare LINE.json [...]
      (bench.py lines of an N>1 run, e.g. from the driver's SCALE record:
      the deployment (the line's `rccl` or `multi_device` key), the form that
      ran, each phase's max over ranks against that deployment's mid
      prediction for that form, and the phase furthest above it)
"""
import collections
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.environ.get("SCALE_PROF_DIR", os.path.join(ROOT, "profiles"))
TAG = os.environ.get("SCALE_TAG", "r05")          # the rank-iteration inputs
LOCAL_TAG = os.environ.get("SCALE_LOCAL_TAG", "r06")  # the one-process inputs
MODEL_TAG = os.environ.get("SCALE_MODEL_TAG", "r06")  # the committed model --compare reads
N = 65536

# RCCL small-message collectives over xGMI on one 8-GPU MI300-class node (LL
# protocol): an 8-byte allreduce in the tens of microseconds at most; the
# allgather of 8*N/G bytes per rank adds its transfer at ~100 GB/s effective
# per peer link (MI355X: 7 xGMI links per GPU, ~153 GB/s each, per the project
# brief).  These are assumptions, labelled as such in the output.
ALLREDUCE_US = {"low": 6.0, "mid": 12.0, "high": 25.0}
GATHER_LAT_US = {"low": 6.0, "mid": 12.0, "high": 25.0}
GATHER_GBPS_PER_LINK = 100.0
# one process: a system-scope load of a peer device's memory over xGMI (the
# pull gather's first bytes, each folded combine's partials)
PEER_LOAD_US = {"low": 2.0, "mid": 4.0, "high": 8.0}


def one_gpu_anchor():
    recs = sorted((int(m.group(1)), f) for f in os.listdir(ROOT) if (m := re.fullmatch(r"BENCH_r(\d+)\.json", f)))
    for num, f in reversed(recs):
        d = json.load(open(os.path.join(ROOT, f))).get("parsed") or {}
        if d.get("ms_per_step"):
            return d["ms_per_step"], f"{f}: the driver's round-{num} N=1 bench line ({d['value']:.2f} it/s)"
    d = json.load(open(os.path.join(PROF, f"{TAG}_scale_inputs.json")))
    return d["one_gpu_ms_per_step"], d["source"]


def local_inputs():
    """Per block count S: the medians over rounds of the default enqueue form
    (one host thread) and of the creation-time pull-gather figure.  The
    host's cost is read at N = 4096 (<tag>_local_inputs_n4096.jsonl), where
    the shared GPU keeps up with the host; at N = 65536 the one GPU runs
    every block's kernels, falls behind, and the host's launches wait for
    queue space, so that figure (kept as host_enqueue_n65536_*) overstates
    what the host pays when every block has a GPU of its own."""
    path = os.path.join(PROF, f"{LOCAL_TAG}_local_inputs.jsonl")
    if not os.path.exists(path):
        return None

    def rows_of(p):
        rows = collections.defaultdict(lambda: {"enqueue_us": [], "gather_us": []})
        if os.path.exists(p):
            for line in open(p):
                d = json.loads(line)
                if d["form"] == "onethread":
                    rows[d["blocks"]]["enqueue_us"].append(d["enqueue_us"])
                    rows[d["blocks"]]["gather_us"].append(d["overlap_info"]["allgather_us"])
        return rows
    big, small = rows_of(path), rows_of(os.path.join(PROF, f"{LOCAL_TAG}_local_inputs_n4096.jsonl"))
    out = {}
    for S, v in big.items():
        host = small[S]["enqueue_us"] if S in small else v["enqueue_us"]
        out[S] = {"host_enqueue_us": statistics.median(host), "host_enqueue_range_us": [min(host), max(host)],
                  "host_enqueue_source": "N = 4096" if S in small else "N = 65536",
                  "host_enqueue_n65536_us": statistics.median(v["enqueue_us"]),
                  "host_enqueue_n65536_range_us": [min(v["enqueue_us"]), max(v["enqueue_us"])],
                  "gather_one_gpu_us": statistics.median(v["gather_us"]), "rounds": len(host)}
    return out


def kernel_spans(trace_csv):
    """Per-kernel medians (us) of rank_iteration's traced iterations, by form:
    split = [matVec own, matVec rest, update_r, update_xp], one = [matVec
    (rotated, ROT), update_r, update_xp], natural = [matVec, update_r, update_xp]."""
    rows = list(csv.DictReader(open(trace_csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ks = [k for k in ks if any(x in k[2] for x in ("k_matvec_f64<", "k_matvec_add_f64<", "k_update_r_f64", "k_update_xp_f64"))]
    dur = lambda k: (k[1] - k[0]) / 1e3  # noqa: E731
    rot = lambda k: "k_matvec_f64<" in k[2] and re.search(r"k_matvec_f64<[^>]*true, true>", k[2]) is not None  # noqa: E731
    mv = lambda k: "k_matvec_f64<" in k[2]  # noqa: E731
    out = {"split": {"matvec_own": [], "matvec": [], "update_r": [], "update_xp": []},
           "conc": {"matvec_own": [], "matvec_rest": [], "add": [], "update_r": [], "update_xp": []},
           "one": {"matvec": [], "update_r": [], "update_xp": []},
           "natural": {"matvec": [], "update_r": [], "update_xp": []}}
    i = 0
    while i < len(ks) - 2:
        a, b, c = ks[i], ks[i + 1], ks[i + 2]
        if mv(a) and not rot(a) and mv(b) and i + 4 < len(ks) and "k_matvec_add_f64" in c[2]:
            # the conc form (measured, not adopted): own and rest on two streams (whichever started first), the add
            own, rest = (a, b) if a[1] - a[0] < b[1] - b[0] else (b, a)
            for key, k in zip(("matvec_own", "matvec_rest", "add", "update_r", "update_xp"),
                              (own, rest, c, ks[i + 3], ks[i + 4])):
                out["conc"][key].append(dur(k))
            i += 5
        elif mv(a) and not rot(a) and mv(b) and i + 3 < len(ks) and "update_r" in c[2]:
            for key, k in zip(("matvec_own", "matvec", "update_r", "update_xp"), ks[i:i + 4]):
                out["split"][key].append(dur(k))
            i += 4
        elif mv(a) and "update_r" in b[2] and "update_xp" in c[2]:
            form = "one" if rot(a) else "natural"
            for key, k in zip(("matvec", "update_r", "update_xp"), (a, b, c)):
                out[form][key].append(dur(k))
            i += 3
        else:
            i += 1
    return {f: {k: round(statistics.median(v), 2) for k, v in d.items() if v} for f, d in out.items()}


def local_prediction(G, split, one, own, ms1, li):
    """bench.py --gpus G without a launcher: the pull gather on each device
    (its share of the one-GPU figure + the peer-read latency + the slice
    transfer), the two folded combines (a peer read each, inside the update
    kernels), against the host enqueueing every block's launches."""
    slice_bytes = 8 * N // G
    pred = {}
    for case in ("low", "mid", "high"):
        lat = PEER_LOAD_US[case]
        gather = li["gather_one_gpu_us"] / G + lat + slice_bytes / (GATHER_GBPS_PER_LINK * 1e3)
        forms = {"overlap": split + max(0.0, gather - own) + 2 * lat, "plain": one + gather + 2 * lat}
        chosen = min(forms, key=forms.get)
        device_us = forms[chosen]
        host_us = li["host_enqueue_us"]
        it_us = max(device_us, host_us)
        pred[case] = {
            "allgather_us": round(gather, 2),
            "device_iteration_us": {f: round(v, 1) for f, v in forms.items()},
            "chosen": chosen,
            "host_enqueue_us": host_us,
            "bound": "host" if host_us > device_us else "device",
            "iteration_us": round(it_us, 1),
            "phases_us": ({"matvec_own": round(own, 2), "gather_exposed": round(max(0.0, gather - own), 2)}
                          if chosen == "overlap" else {"matvec_own": 0.0, "gather_exposed": round(gather, 2)}),
            "it_per_s": round(1e6 / it_us, 1),
            "speedup_vs_1gpu": round(ms1 * 1e3 / it_us, 2),
            "efficiency": round(ms1 * 1e3 / it_us / G, 3)}
    return {"inputs": li | {"source": f"profiles/{LOCAL_TAG}_local_inputs.jsonl and "
                                      f"{LOCAL_TAG}_local_inputs_n4096.jsonl (tools/local_inputs.py)"},
            "predicted": pred}


def main():
    ms1, src1 = one_gpu_anchor()
    loc = local_inputs()
    walls = {}
    for line in open(os.path.join(PROF, f"{TAG}_rank_iteration.jsonl")):
        d = json.loads(line)
        w = d["us_per_iteration_without_collectives"]
        # a middle rank (its rest wraps), no emulated gather (the model adds the exchange itself)
        if d.get("rank", d["ranks"] // 2) == d["ranks"] // 2 and not d.get("gather_us"):
            walls.setdefault(d["ranks"], []).append(w)
    out = {
        "what": "configs[2] (N=65536 dense fp64, row blocks) at G GPUs: one rank's measured kernels in both "
                "exchange forms plus assumed collective latencies -> predicted iteration, it/s and speed-up over "
                "the measured 1-GPU step, and the form the library picks (the faster one end to end, as the "
                "library times both at creation); the phase keys are bench.py phases_us's; 'local' = the "
                "one-process deployment (host enqueue against device work)",
        "one_gpu": {"ms_per_step": ms1, "it_per_s": 1e3 / ms1, "source": src1},
        "assumptions": {
            "allreduce_8B_us": ALLREDUCE_US,
            "allgather_latency_us": GATHER_LAT_US,
            "allgather_GBps_per_peer_link": GATHER_GBPS_PER_LINK,
            "peer_load_latency_us": PEER_LOAD_US,
            "source": "not measurable on a one-GPU box (RCCL runs over loopback sockets there); RCCL's LL-protocol "
                      "small-message latency on one xGMI-connected node is assumed in the 5-25 us range (not from a "
                      "document available here); the MI355X has 7 xGMI links per GPU at ~153 GB/s each (the "
                      "project brief), taken at 100 GB/s effective per peer; a peer read's latency over xGMI "
                      "(one process) assumed 2-8 us",
        },
        "per_G": {},
    }
    for G in (2, 4, 8):
        if G not in walls:
            continue
        split = statistics.median(w["split"] for w in walls[G])
        one = statistics.median(w["one"] for w in walls[G])
        tr = os.path.join(PROF, f"{TAG}_rank_kernel_trace_g{G}.csv")
        k = kernel_spans(tr) if os.path.exists(tr) else None
        own = (k["split"]["matvec_own"] if k else split * 0.13)
        slice_bytes = 8 * N // G
        entry = {"rows_per_rank": N // G, "measured": {
            "us_per_iteration_without_collectives": {"split": round(split, 2), "one": round(one, 2),
                                                     "rounds": len(walls[G])},
            "split_cost_us": round(split - one, 2),
            "kernel_medians_us": k,
            "matvec_TBps_one_launch": round((8 * (N // G) * N + 8 * N + 8 * (N // G))
                                            / (k["one"]["matvec"] * 1e-6) / 1e12, 3) if k else None}}
        pred = {}
        for case in ("low", "mid", "high"):
            gather = GATHER_LAT_US[case] + slice_bytes / (GATHER_GBPS_PER_LINK * 1e3)  # per peer, peers in parallel
            ar = ALLREDUCE_US[case]
            forms = {"overlap": split + max(0.0, gather - own) + 2 * ar, "plain": one + gather + 2 * ar}
            chosen = min(forms, key=forms.get)  # the library times both forms end to end and runs the faster
            it_us = forms[chosen]
            pred[case] = {
                "allgather_us": round(gather, 2),
                "iteration_us": {f: round(v, 1) for f, v in forms.items()},
                "chosen": chosen,
                "phases_us": ({"matvec_own": round(own, 2), "gather_exposed": round(max(0.0, gather - own), 2)}
                              if chosen == "overlap" else {"matvec_own": 0.0, "gather_exposed": round(gather, 2)})
                | {"combine_pap": ar, "combine_rr": ar},
                "it_per_s": round(1e6 / it_us, 1),
                "speedup_vs_1gpu": round(ms1 * 1e3 / it_us, 2),
                "efficiency": round(ms1 * 1e3 / it_us / G, 3)}
        entry["predicted"] = pred
        li = (loc or {}).get(G)
        if li:
            entry["local"] = local_prediction(G, split, one, own, ms1, li)
        out["per_G"][str(G)] = entry
    json.dump(out, sys.stdout, indent=1)
    print()


def bench_lines(path):
    """The bench.py lines in a file: a driver record (BENCH_/SCALE_rNN.json: the
    lines sit inside it, e.g. under "parsed", one per N), or a captured
    stdout (the last JSON line)."""
    text = open(path).read()
    try:
        doc = json.loads(text)
    except ValueError:
        return [json.loads([ln for ln in text.splitlines() if ln.strip().startswith("{")][-1])]
    found = []

    def walk(o):
        if isinstance(o, dict):
            if "n_gpus" in o and "value" in o:
                found.append(o)
                return
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)
    walk(doc)
    return found


def compare(paths):
    model = json.load(open(os.path.join(PROF, f"{MODEL_TAG}_scale_model.json")))
    for path, line in ((p, ln) for p in paths for ln in bench_lines(p)):
        local = "multi_device" in line and "rccl" not in line
        # one process: the row blocks (a rehearsal puts several on one GPU; n_gpus counts devices)
        G = str(line.get("config", {}).get("row_blocks") or line["n_gpus"]) if local else str(line["n_gpus"])
        entry = model["per_G"].get(G, {})
        pred = (entry.get("local") or {}).get("predicted", {}).get("mid") if local else \
            entry.get("predicted", {}).get("mid")
        meas = line.get("phases_us", {}).get("max_over_ranks")
        if not pred or not meas:
            print(json.dumps({"file": path, "n_gpus": G, "deployment": "local" if local else "rccl",
                              "error": "no model entry or no phases_us"}))
            continue
        ran = "overlap" if line.get("overlap", {}).get("on") else "plain"
        delta = {ph: round(meas.get(ph, 0.0) - v, 2) for ph, v in pred["phases_us"].items()}
        out = {"file": path, "n_gpus": G, "deployment": "local" if local else "rccl", "it_per_s": line["value"],
               "form_ran": ran, "form_model_picks": pred["chosen"], "overlap_measured": line.get("overlap"),
               "measured_iteration_us": meas.get("iteration"), "measured_phases_us": meas,
               "predicted_phases_us": pred["phases_us"], "delta_us": delta,
               "furthest_above_model": max(delta, key=delta.get)}
        if local:  # the slower of the device's work and the host's enqueue
            host = line.get("host_enqueue_us_per_iteration")
            out.update(predicted_iteration_us=pred["iteration_us"], predicted_bound=pred["bound"],
                       predicted_host_enqueue_us=pred["host_enqueue_us"], measured_host_enqueue_us=host,
                       measured_bound=None if host is None or meas.get("iteration") is None else
                       "host" if host >= 0.95 * meas["iteration"] else "device")
        else:
            out["predicted_iteration_us"] = pred["iteration_us"][ran]
        print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--compare":
        compare(sys.argv[2:])
    else:
        main()
