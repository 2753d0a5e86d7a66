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
