import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "0g-ec-gpu_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950); runs via gpurun")
    # The CPU oracle is test infrastructure; build it if the .so is missing.
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gpu_programs():
    import ecgpu

    devs = ecgpu.Device.all()
    if not devs:
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X (the HIP path has no CPU fallback)")
    return [ecgpu.program(devs[0])], devs[:1]
