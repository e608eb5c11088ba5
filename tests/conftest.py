import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _build_all():
    # product library (in-tree, only if stale) and the oracle (test infrastructure)
    spec = importlib.util.spec_from_file_location("_dp_build", os.path.join(ROOT, "densepoints_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "programs", "densify")], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")
    _build_all()


def pytest_sessionstart(session):
    # on a GPU box, torch's bundled HIP runtime initialises the device before
    # libdensepoints' contexts (tests that put views into torch tensors need
    # it; bench.py uses the same order); a no-op without a GPU
    try:
        import torch

        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:
        pass


@pytest.fixture(scope="session")
def orc():
    from oracle import pyoracle

    return pyoracle
