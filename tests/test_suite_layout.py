"""CPU checks of the suite's own layout and of what the bench line says.

  * the distinct-device tests collect last (tests/conftest.py), so a failure
    on a node no round has run cannot stop the full-size config tests;
  * every CGX_* environment variable the library reads is documented in
    INTEGRATION.md;
  * bench.py's exchange text follows the context's reported flags, and its
    check block compares the true residual with the recurrence's.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_multidevice_tests_collect_last():
    p = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu", "tests"], cwd=ROOT,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    ids = [ln for ln in p.stdout.splitlines() if "::" in ln]
    files = [ln.split("::")[0] for ln in ids]
    assert "tests/test_gpu_multidevice.py" in files and "tests/test_gpu_solver.py" in files
    first = files.index("tests/test_gpu_multidevice.py")
    assert all(f == "tests/test_gpu_multidevice.py" for f in files[first:]), files[first:]
    assert len(files[first:]) >= 15


def test_every_env_variable_is_documented():
    csrc = os.path.join(ROOT, "conjugate_gradient_amd", "csrc")
    read = set()
    for name in os.listdir(csrc):
        if name.endswith((".hip", ".h", ".c")):
            with open(os.path.join(csrc, name)) as f:
                read |= set(re.findall(r'getenv\("(CGX_\w+)"\)', f.read()))
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    assert read, "no getenv found"
    missing = sorted(v for v in read if f"`{v}`" not in doc)
    assert not missing, missing


def test_exchange_text_follows_flags():
    import bench
    import conjugate_gradient_amd as cg
    dev = [0, 1, 2, 3]
    assert bench.exchange_text(1, 0) == "none (single GPU)"
    t = bench.exchange_text(4, cg.CGX_PULL_ACTIVE | cg.CGX_FOLDED_ACTIVE | cg.CGX_OVERLAP_ACTIVE, devices=dev)
    assert "pull kernel" in t and "overlapped" in t and "folded combines" in t and "0,1,2,3" in t
    t = bench.exchange_text(4, cg.CGX_PULL_ACTIVE, devices=dev)
    assert "pull kernel" in t and "overlapped" not in t and "by a pull kernel per block" in t
    t = bench.exchange_text(4, 0, devices=dev)
    assert "peer copy per block pair" in t and "combine kernel" in t
    t = bench.exchange_text(4, cg.CGX_PULL_ACTIVE | cg.CGX_FOLDED_ACTIVE | cg.CGX_THREADS_ACTIVE, devices=dev)
    assert t.endswith("one enqueuing host thread per block")
    t = bench.exchange_text(4, cg.CGX_PULL_ACTIVE | cg.CGX_FOLDED_ACTIVE | cg.CGX_HALO_PULL_ACTIVE, devices=dev,
                            poisson=True)
    assert "halo pull" in t and "inside k_poisson_p / k_poisson_xr" in t and "peer copies" not in t
    t = bench.exchange_text(4, cg.CGX_HALO_OVERLAP_ACTIVE, devices=dev, poisson=True)
    assert "halo rows by peer copies beside k_poisson_p's interior" in t
    assert bench.exchange_text(8, cg.CGX_OVERLAP_ACTIVE) == \
        "RCCL allgather(p) overlapped with own-block matVec + 2x allreduce"
    assert bench.exchange_text(8, 0) == "RCCL allgather(p) + 2x allreduce"
    assert "via rank 0" in bench.exchange_text(8, 0, comm="p2p")
    assert "rank-ordered" in bench.exchange_text(8, 0, comm="deterministic")
    assert bench.exchange_text(8, cg.CGX_HALO_OVERLAP_ACTIVE, poisson=True) == \
        "RCCL halo ncclSend/Recv beside k_poisson_p's interior + 2x allreduce"


def test_check_summary():
    import bench
    c = bench.check_summary(54.3, 1.0, 54.3 ** 2 * (1 + 2e-9))
    assert c["recurrence_agrees"] and c["recurrence_gap"] < 1e-8
    c = bench.check_summary(2.0, 1.0, 1.0)
    assert not c["recurrence_agrees"]
    c = bench.check_summary(1e-15, 1.0, 1e-40)  # at rounding the two part: not compared
    assert "recurrence_agrees" not in c and c["relres"] == 1e-15


def test_overlap_rule():
    import conjugate_gradient_amd as cg
    assert cg.overlap_rule({"overlap_form_us": 600.0, "plain_form_us": 620.0, "margin": 0.01})
    assert not cg.overlap_rule({"overlap_form_us": 615.0, "plain_form_us": 620.0, "margin": 0.01})
