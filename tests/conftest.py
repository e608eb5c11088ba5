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


@pytest.fixture(scope="session")
def orc():
    from oracle import pyoracle

    return pyoracle
