"""Per-iteration time of small dense fp64 systems on one GPU, the launch forms
interleaved in one process: three launches (CGX_FUSE_P=0), two launches with
the single-block p pass (k_update_xrp_f64), two launches with the p update
folded into the matVec (CGX_FOLD_P=1); "_l2p": the same with round 2's
matVec (p read through L2, CGX_MV_SMALL=0) instead of k_matvec_small_f64.  Fixed-count iterations, timed by
the host around a synchronize, with the CGX_PHASES stamps alongside.
  python tools/floor_small_n.py [rounds] > profiles/r03_iteration_floor.jsonl"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

KNOBS = ("CGX_FUSE_P", "CGX_FOLD_P", "CGX_MV_PLAN", "CGX_MV_SMALL", "CGX_SMALL_PLAN")
# form -> the knobs it sets (the rest: the library's default)
FORMS = {"three": {"CGX_FUSE_P": "0", "CGX_FOLD_P": "0"}, "two": {"CGX_FUSE_P": "1", "CGX_FOLD_P": "0"},
         "fold": {"CGX_FUSE_P": "1", "CGX_FOLD_P": "1"}, "default": {},
         # round 2's kernels: k_matvec_f64 reading p through L2 (no LDS staging)
         "two_l2p": {"CGX_FUSE_P": "1", "CGX_FOLD_P": "0", "CGX_MV_SMALL": "0"},
         "fold_l2p": {"CGX_FUSE_P": "1", "CGX_FOLD_P": "1", "CGX_MV_SMALL": "0"}}
if os.environ.get("SMALL_VARIANTS"):  # k_matvec_small_f64's block size and chunks per step
    for nt in ("512", "1024"):
        for u in ("4", "8"):
            FORMS[f"fold_nt{nt}u{u}"] = {"CGX_FUSE_P": "1", "CGX_FOLD_P": "1", "CGX_SMALL_PLAN": f"threads={nt},U={u}"}


def run(n, form, steps=400, warm=50):
    for k in KNOBS:
        os.environ[k] = FORMS[form].get(k, "")
    with cg.Solver(n, flags=cg.CGX_PHASES) as s:
        s.generate_spd(42)
        s.begin()
        s.iterate(warm, eps=-1.0)
        s.synchronize()
        s.reset_timing()
        t0 = time.perf_counter()
        s.iterate(steps, eps=-1.0)
        s.synchronize()
        t1 = time.perf_counter()
        ph = s.phase_times()
    return {"n": n, "form": form, "us_per_iter": (t1 - t0) / steps * 1e6,
            "phases_median_us": {k: round(v["median_us"], 2) for k, v in ph.items() if v["samples"]}}


SIZES = (512, 1024, 2048, 4096, 8192)


def main():
    global SIZES
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    if len(sys.argv) > 2:
        SIZES = tuple(int(v) for v in sys.argv[2].split(","))
    for r in range(rounds):
        for n in SIZES:
            for form in FORMS:
                out = run(n, form)
                out["round"] = r
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
