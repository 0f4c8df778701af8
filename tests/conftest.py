"""Test configuration.

Markers:
  gpu  -- needs a visible MI355X (run with `-m gpu` on the GPU box).  Everything
          else runs on the CPU in a few minutes (`-m "not gpu"`).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# Collected after every other test: the paths only a node with several GPUs
# executes (distinct devices, xGMI).  A failure there under `pytest -x` must
# not keep the full-size configuration tests of the other files from running.
LAST_MODULES = ("test_gpu_multidevice.py",)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (libcgx kernels run)")


def pytest_collection_modifyitems(config, items):
    last = [it for it in items if os.path.basename(str(it.fspath)) in LAST_MODULES]
    if last:
        keep = [it for it in items if os.path.basename(str(it.fspath)) not in LAST_MODULES]
        items[:] = keep + last


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def built():
    """libcgx.so + cg_hip + liboracle.so built in-tree (hipcc cross-compiles here)."""
    import conjugate_gradient_amd as cg
    import oracle
    if not os.path.exists(cg.LIB_PATH) or not os.path.exists(cg.CLI_PATH):
        cg.build()
    oracle.lib()
    return True
