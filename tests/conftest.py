import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))

NEEDED = [
    REPO / "orb_slam_fusion_amd" / "lib" / "liborbgpu.so",
    REPO / "orb_slam_fusion_amd" / "lib" / "liborbsynth.so",
    REPO / "oracle" / "_build" / "liborboracle.so",
]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    if any(not p.exists() for p in NEEDED):
        subprocess.run(["make", "-s", "-j8"], cwd=REPO, check=True)


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


@pytest.fixture(autouse=True)
def _uniform_branch_guard(request):
    """Under the checked build (make checkuniform; ORBGPU_LIB pointing at
    liborbgpu_checkuniform.so) every wave-uniform branch verifies that all
    active lanes agree (csrc/uniform_dev.h): a GPU test that raised a
    violation fails here."""
    yield
    if request.node.get_closest_marker("gpu") is None or "checkuniform" not in os.environ.get("ORBGPU_LIB", ""):
        return
    from orb_slam_fusion_amd._lib import lib

    so = lib()
    if not hasattr(so, "orbgpu_debug_uniform_violations"):
        pytest.fail("ORBGPU_LIB names a checkuniform build without orbgpu_debug_uniform_violations")
    import ctypes

    fn = so.orbgpu_debug_uniform_violations
    fn.restype = ctypes.c_uint
    n = fn()
    assert n == 0, f"{n} wave-uniform branch violations (csrc/uniform_dev.h)"
