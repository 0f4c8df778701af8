"""tools/scale_model.py on the committed round-5 inputs (CPU only): the
prediction a SCALE line is read against, and --compare on a
bench line of the shape bench.py prints at N > 1."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "scale_model.py")


def run(*args, env=None):
    p = subprocess.run([sys.executable, TOOL, *args], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout


def test_model_per_g_picks_the_faster_form():
    m = json.loads(run())
    assert m["one_gpu"]["ms_per_step"] > 0 and "BENCH_r04" in m["one_gpu"]["source"]
    assert set(m["per_G"]) == {"2", "4", "8"}
    for G, e in m["per_G"].items():
        meas = e["measured"]
        us = meas["us_per_iteration_without_collectives"]
        assert us["split"] > us["one"] > 0 and meas["split_cost_us"] == round(us["split"] - us["one"], 2)
        for case, p in e["predicted"].items():
            # the library's rule: overlap only when the allgather is longer than the split costs
            assert p["chosen"] == ("overlap" if p["allgather_us"] > meas["split_cost_us"] else "plain"), (G, case)
            assert 0 < p["speedup_vs_1gpu"] <= int(G) and p["phases_us"]["combine_pap"] > 0
    k = m["per_G"]["8"]["measured"]["kernel_medians_us"]
    # the G = 8 trace holds both forms' matVec launches (the name parse sees through "(anonymous namespace)")
    assert k["one"]["matvec"] > k["split"]["matvec"] > k["split"]["matvec_own"] > 0
    assert 6.5 < m["per_G"]["8"]["measured"]["matvec_TBps_one_launch"] < 8.0


def test_compare_reads_a_scale_line(tmp_path):
    model = json.loads(run())
    (tmp_path / "r05_scale_model.json").write_text(json.dumps(model))
    pred = model["per_G"]["8"]["predicted"]["mid"]
    phases = dict(pred["phases_us"], iteration=pred["iteration_us"][pred["chosen"]] + 7.0, matvec=600.0)
    phases["gather_exposed"] += 7.0
    line = {"n_gpus": 8, "value": 1500.0, "overlap": {"on": pred["chosen"] == "overlap", "decided_by": "measured"},
            "phases_us": {"max_over_ranks": phases}}
    path = tmp_path / "scale_g8.json"
    path.write_text("rank noise\n" + json.dumps(line) + "\n")
    # the committed prediction, read back from tmp_path (SCALE_PROF_DIR)
    out = json.loads(run("--compare", str(path), env={"SCALE_PROF_DIR": str(tmp_path)}).strip().splitlines()[-1])
    assert out["n_gpus"] == "8" and out["form_ran"] == out["form_model_picks"] == pred["chosen"]
    assert out["furthest_above_model"] == "gather_exposed" and out["delta_us"]["gather_exposed"] == 7.0
