"""tools/scale_model.py on the committed inputs (CPU only): the prediction a
SCALE line is read against, for both deployments (RCCL rank
processes, and one process over distinct devices), and --compare on bench
lines of the shapes bench.py prints at N > 1."""
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
    # anchored to the driver's latest N=1 line
    latest = max(int(f[7:-5]) for f in os.listdir(ROOT) if f.startswith("BENCH_r") and f.endswith(".json"))
    assert m["one_gpu"]["ms_per_step"] > 0 and f"BENCH_r{latest:02d}" in m["one_gpu"]["source"]
    assert set(m["per_G"]) == {"2", "4", "8"}
    for G, e in m["per_G"].items():
        meas = e["measured"]
        us = meas["us_per_iteration_without_collectives"]
        assert us["split"] > us["one"] > 0 and meas["split_cost_us"] == round(us["split"] - us["one"], 2)
        for case, p in e["predicted"].items():
            # the library's rule: the form that is faster end to end
            assert p["chosen"] == min(p["iteration_us"], key=p["iteration_us"].get), (G, case)
            assert 0 < p["speedup_vs_1gpu"] <= int(G) and p["phases_us"]["combine_pap"] > 0
        loc = e["local"]
        assert loc["inputs"]["rounds"] >= 2 and loc["inputs"]["host_enqueue_us"] > 0
        for case, p in loc["predicted"].items():
            dev = p["device_iteration_us"]
            assert p["chosen"] == min(dev, key=dev.get), (G, case)
            assert p["iteration_us"] == round(max(dev[p["chosen"]], p["host_enqueue_us"]), 1)
            assert p["bound"] == ("host" if p["host_enqueue_us"] > dev[p["chosen"]] else "device")
            assert 0 < p["speedup_vs_1gpu"] <= int(G)
    k = m["per_G"]["8"]["measured"]["kernel_medians_us"]
    # the G = 8 trace holds both forms' matVec launches (the name parse sees through "(anonymous namespace)")
    assert k["one"]["matvec"] > k["split"]["matvec"] > k["split"]["matvec_own"] > 0
    assert 6.5 < m["per_G"]["8"]["measured"]["matvec_TBps_one_launch"] < 8.0


def test_compare_reads_a_scale_line(tmp_path):
    model = json.loads(run())
    (tmp_path / "r06_scale_model.json").write_text(json.dumps(model))
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
    assert out["deployment"] == "rccl"
    assert out["furthest_above_model"] == "gather_exposed" and out["delta_us"]["gather_exposed"] == 7.0


def test_compare_reads_a_local_line(tmp_path):
    """A `bench.py --gpus 8` line without a launcher (its `multi_device` key):
    read against the one-process prediction, with the host's enqueue."""
    model = json.loads(run())
    (tmp_path / "r06_scale_model.json").write_text(json.dumps(model))
    pred = model["per_G"]["8"]["local"]["predicted"]["mid"]
    phases = dict(pred["phases_us"], iteration=700.0, matvec=600.0, combine_pap=3.0)
    line = {"n_gpus": 8, "value": 1400.0, "overlap": {"on": pred["chosen"] == "overlap", "decided_by": "measured"},
            "multi_device": {"devices": list(range(8)), "distinct_devices": 8},
            "host_enqueue_us_per_iteration": 690.0, "phases_us": {"max_over_ranks": phases}}
    path = tmp_path / "local_g8.json"
    path.write_text(json.dumps(line) + "\n")
    out = json.loads(run("--compare", str(path), env={"SCALE_PROF_DIR": str(tmp_path)}).strip().splitlines()[-1])
    assert out["deployment"] == "local" and out["form_ran"] == pred["chosen"]
    assert out["predicted_iteration_us"] == pred["iteration_us"] and out["predicted_bound"] == pred["bound"]
    assert out["measured_host_enqueue_us"] == 690.0 and out["measured_bound"] == "host"


def test_compare_reads_a_driver_record(tmp_path):
    """A driver record (the bench lines inside a JSON document, e.g. under
    "parsed", one per N) is read line by line."""
    model = json.loads(run())
    (tmp_path / "r06_scale_model.json").write_text(json.dumps(model))
    pred = model["per_G"]["4"]["predicted"]["mid"]
    line4 = {"n_gpus": 4, "value": 800.0, "overlap": {"on": pred["chosen"] == "overlap"},
             "rccl": {"nranks": 4}, "phases_us": {"max_over_ranks": dict(pred["phases_us"], iteration=1250.0)}}
    rec = {"runs": [{"n": 1, "parsed": {"n_gpus": 1, "value": 210.0}}, {"n": 4, "parsed": line4}]}
    path = tmp_path / "SCALE_rXX.json"
    path.write_text(json.dumps(rec, indent=1))
    outs = [json.loads(ln) for ln in run("--compare", str(path), env={"SCALE_PROF_DIR": str(tmp_path)}).splitlines()]
    assert [o["n_gpus"] for o in outs] == ["1", "4"]
    assert "error" in outs[0] and outs[1]["deployment"] == "rccl" and outs[1]["measured_iteration_us"] == 1250.0
