"""Per-iteration time of small dense fp64 systems on one GPU, the launch forms
interleaved in one process: three launches (CGX_FUSE_P=0), two launches with
the single-block p pass (k_update_xrp_f64), two launches with the p update
folded into the matVec (CGX_FOLD_P=1).  Fixed-count iterations, timed by
the host around a synchronize, with the CGX_PHASES stamps alongside.
  python tools/r03_floor.py [rounds] > profiles/r03_iteration_floor.jsonl"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

# (CGX_FUSE_P, CGX_FOLD_P, CGX_MV_R, CGX_MV_U); "" = the library's default
FORMS = {"three": ("0", "0", "", ""), "two": ("1", "0", "", ""), "fold": ("1", "1", "", ""), "default": ("", "", "", "")}
if os.environ.get("R03_FOLD_VARIANTS"):  # the plans tried for the fold (CGX_MV_* also sets the k = 0 matVec's)
    FORMS.update({"fold_r2u4": ("1", "1", "2", "4"), "fold_r2u8": ("1", "1", "2", "8")})


def run(n, form, steps=400, warm=50):
    os.environ["CGX_FUSE_P"], os.environ["CGX_FOLD_P"], os.environ["CGX_MV_R"], os.environ["CGX_MV_U"] = FORMS[form]
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
