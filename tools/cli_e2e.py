#!/usr/bin/env python3
"""End to end on the reference's own input format (configs[0]-style plumbing,
larger): generateSPDmatrix(n) written as the MATLAB script writes it
("%.4f", one value per line), then
  - the reference: its own initialize() on the three files
    (oracle/_ref/serial_ref --initialize, the unmodified serialConjugate.c
    reader) and its conjugrad() on the parsed system (serial_ref solve mode),
    single thread, timed separately;
  - cg_hip --fp32-ref --print-x on the same three files, wall time of the
    whole program (parse + H2D + GPU solve + print), with its default fast
    exit and A in huge pages, with A malloc'd (CGX_CLI_HUGEPAGES=0), and
    with the full teardown (CGX_CLI_FAST_EXIT=0).
The x vectors must be identical bit for bit.  oracle/_ref is the reference
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = a.n
    exe = oracle.ref_binary()
    if not exe:
        raise SystemExit("oracle/_ref/serial_ref is not built")
    res = {"n": n}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        A, b = oracle.spd_matlab(n, np.float64)
        paths = {k: os.path.join(td, k + ".txt") for k in ("A", "b", "x0")}
        for k, arr, fmt in (("A", A.ravel(), "%.4f"), ("b", b, "%.4f"), ("x0", np.zeros(n), "%.1f")):
            arr.tofile(paths[k], sep="\n", format=fmt)
            with open(paths[k], "a") as f:
                f.write("\n")
        del A
        # reference: initialize() on each file (ROWS = 8192 values per column)
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
        # cg_hip: the whole program, alternating: the defaults (A in huge pages,
        # fast exit after the output is flushed), A malloc'd
        # (CGX_CLI_HUGEPAGES=0), and the full teardown (CGX_CLI_FAST_EXIT=0)
        modes = {"fast": {}, "no_hugepages": {"CGX_CLI_HUGEPAGES": "0"}, "teardown": {"CGX_CLI_FAST_EXIT": "0"}}
        runs = {k: [] for k in modes}
        phases = {}
        out = ""
        for rep in range(5):
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
                if mode == "fast":
                    out = proc.stdout
        med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
        res["cg_hip_phases_s"] = phases.get("fast", [])
        res["cg_hip_phases_no_hugepages_s"] = phases.get("no_hugepages", [])
        res["cg_hip_phases_full_teardown_s"] = phases.get("teardown", [])
        for mode in modes:
            recs = phases.get(mode, [])
            for r in recs:  # the critical path once HIP is up: context, distribution, solve, x back
                r["after_hip_up_to_x_s"] = r["to_x_s"] - r["hip_runtime_s"]
            for key in ("after_output_s", "distribute_s", "read_s", "free_s", "get_x_s", "after_hip_up_to_x_s"):
                v = sorted(r[key] for r in recs)
                if v:
                    res[f"cg_hip_{key[:-2]}_med_s_{mode}"] = v[len(v) // 2]
        lines = out.strip().splitlines()
        x = np.array([float(v) for v in lines[-n:]], dtype=np.float32)
        xr = np.fromfile(xref, dtype=np.float32)
        t_cli = med["fast"]
        res.update({"cg_hip_total_s": t_cli, "cg_hip_total_runs_s": runs["fast"],
                    "cg_hip_total_no_hugepages_s": med["no_hugepages"], "cg_hip_total_full_teardown_s": med["teardown"],
                    "cg_hip_total_full_teardown_runs_s": runs["teardown"], "cg_hip_stdout_head": lines[:4],
                    "x_bit_identical": bool(np.array_equal(x.view(np.uint32), xr.view(np.uint32))),
                    "speedup_total": (t_init + t_solve) / t_cli, "threads": a.threads,
                    "note": "reference_conjugrad_process_s includes the harness reading raw float files "
                            "and embedding the system (n <= 8192); the reference itself is single-threaded; "
                            "cg_hip times are medians of 5 alternating runs per mode"})
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
