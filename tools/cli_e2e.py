#!/usr/bin/env python3
"""End to end on the reference's own input format (configs[0]-style plumbing,
larger): generateSPDmatrix(n) written as the MATLAB script writes it
("%.4f", one value per line), then
  - the reference: its own initialize() on the three files
    (oracle/_ref/serial_ref --initialize, the unmodified serialConjugate.c
    reader) and its conjugrad() on the parsed system (serial_ref solve mode),
    single thread, timed separately;
  - cg_hip --fp32-ref --print-x on the same three files, wall time of the
    whole program (parse + H2D + GPU solve + print), in three modes: the
    default (A parsed and sent to the GPU row block by row block through a
    ring of up to 1 GiB), A parsed whole and sent in one copy
    (CGX_CLI_STREAM=0, round 1's path), the stream through a 64 MiB
    ring (CGX_CLI_RING_MB=64: host memory for A bounded) and the stream in
    32 MiB blocks (CGX_CLI_BLOCK_MB=32; the default is 128).
The x vectors of every mode must be identical bit for bit (to the
reference's when it runs).  oracle/_ref is the reference
compiled here from its sources (it travels with the repo snapshot; the
reference sources do not).

  python tools/cli_e2e.py [--n 8192] [--threads 16] [--out profiles/r01_cli_e2e_n8192.json]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402


def run_reference(exe, n, td, paths, res):
    """The reference: initialize() on the three files, then conjugrad()."""
    t_init = 0.0
    raw = {}
    for k, cols in (("A", n), ("b", 1), ("x0", 1)):
        raw[k] = os.path.join(td, k + ".f32")
        out = subprocess.run([exe, "--initialize", paths[k], str(cols), raw[k]], check=True,
                             capture_output=True, text=True).stdout
        t_init += float(out.split()[-1])
    xref = os.path.join(td, "xref.f32")
    t0 = time.perf_counter()
    out = subprocess.run([exe, str(n), raw["A"], raw["b"], raw["x0"], xref], check=True,
                         capture_output=True, text=True).stdout
    t_solve = time.perf_counter() - t0
    ref_iters = int(out.split("iterations")[-1].split()[0])
    res.update({"reference_initialize_s": t_init, "reference_conjugrad_process_s": t_solve,
                "reference_total_s": t_init + t_solve, "reference_iterations": ref_iters,
                "reference_stdout": out.strip().splitlines()[0]})
    return t_init, t_solve, xref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-reference", action="store_true",
                    help="skip the reference program (it is compiled for n <= 8192)")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    exe = None if a.no_reference else oracle.ref_binary()
    if not exe and not a.no_reference:
        raise SystemExit("oracle/_ref/serial_ref is not built")
    res = {"n": n}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        A, b = oracle.spd_matlab(n, np.float64)
        paths = {k: os.path.join(td, k + ".txt") for k in ("A", "b", "x0")}
        for k, arr, dec in (("A", A, 4), ("b", b, 4), ("x0", np.zeros(n), 1)):
            oracle.write_text(paths[k], arr, dec)
        del A
        # reference: initialize() on each file (ROWS = 8192 values per column)
        t_init, t_solve, xref = 0.0, 0.0, None
        if exe:
            t_init, t_solve, xref = run_reference(exe, n, td, paths, res)
        # cg_hip: the whole program, alternating the modes
        modes = {"fast": {}, "materialize": {"CGX_CLI_STREAM": "0"}, "ring64": {"CGX_CLI_RING_MB": "64"},
                 "block32": {"CGX_CLI_BLOCK_MB": "32"}}
        runs = {k: [] for k in modes}
        phases = {}
        xs = {}
        for rep in range(a.reps):
            for mode, extra in modes.items():
                env = dict(os.environ, CGX_CLI_TIMES="1", **extra)
                t0 = time.perf_counter()
                proc = subprocess.run([cg.CLI_PATH, "--fp32-ref", "--print-x", "--stats", "--threads", str(a.threads),
                                       paths["A"], paths["b"], paths["x0"]], check=True, capture_output=True,
                                      text=True, env=env)
                runs[mode].append(time.perf_counter() - t0)
                ph = [ln for ln in proc.stderr.splitlines() if ln.startswith("{")]
                if ph:
                    rec = json.loads(ph[-1])
                    rec["process_s"] = runs[mode][-1]
                    rec["after_output_s"] = rec["process_s"] - rec["printed_s"]  # teardown + exit, as seen outside
                    phases.setdefault(mode, []).append(rec)
                lines = proc.stdout.strip().splitlines()
                xs.setdefault(mode, []).append(np.array([float(v) for v in lines[-n:]], dtype=np.float32))
                if mode == "fast":
                    head = lines[:4]
        med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
        res["cg_hip_phases_s"] = phases.get("fast", [])
        res["cg_hip_phases_materialize_s"] = phases.get("materialize", [])
        res["cg_hip_phases_ring64_s"] = phases.get("ring64", [])
        res["cg_hip_phases_block32_s"] = phases.get("block32", [])
        for mode in modes:
            recs = phases.get(mode, [])
            for r in recs:  # the critical path once HIP is up: context, distribution, solve, x back
                r["after_hip_up_to_x_s"] = r["to_x_s"] - r["hip_runtime_s"]
            for key in ("after_output_s", "distribute_s", "read_s", "free_s", "get_x_s", "after_hip_up_to_x_s",
                        "hip_runtime_s", "a_parsed_s", "a_on_device_s", "to_x_s"):
                v = sorted(r[key] for r in recs if key in r)
                if v:
                    res[f"cg_hip_{key[:-2]}_med_s_{mode}"] = v[len(v) // 2]
        xr = np.fromfile(xref, dtype=np.float32) if xref else xs["fast"][0]
        same = all(np.array_equal(x.view(np.uint32), xr.view(np.uint32)) for v in xs.values() for x in v)
        t_cli = med["fast"]
        res.update({"cg_hip_total_s": t_cli, "cg_hip_total_runs_s": runs["fast"],
                    "cg_hip_total_materialize_s": med["materialize"], "cg_hip_total_materialize_runs_s": runs["materialize"],
                    "cg_hip_total_ring64_s": med["ring64"], "cg_hip_total_ring64_runs_s": runs["ring64"],
                    "cg_hip_total_block32_s": med["block32"], "cg_hip_total_block32_runs_s": runs["block32"],
                    "cg_hip_stdout_head": head,
                    "x_bit_identical": bool(same),
                    "speedup_total": (t_init + t_solve) / t_cli if exe else None, "threads": a.threads,
                    "note": "reference_conjugrad_process_s includes the harness reading raw float files "
                            "and embedding the system (n <= 8192); the reference itself is single-threaded; "
                            f"cg_hip times are medians of {a.reps} alternating runs per mode"})
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
