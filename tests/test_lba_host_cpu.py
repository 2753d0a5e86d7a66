"""The LocalBundleAdjustment host path without a GPU: lba_api.cpp built
against no-op HIP / launcher stubs (tools/lba_host_bench.cpp) under
AddressSanitizer (host code only), run on a C4-like window in the caller's
point-major order and shuffled.  Covers the layout walks (free-pose indices,
pose pairs, point ranges, slot records), the upload image and the one-rank
results path (the stub publishes the call number the device would)."""
import json
import os
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not Path(HIPCC).exists() or shutil.which("ld") is None:
        pytest.skip("no hipcc")
    exe = tmp_path_factory.mktemp("lba_host") / "lba_host_asan"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-fsanitize=address", "-fno-gpu-sanitize", "-o", str(exe),
           str(REPO / "tools" / "lba_host_bench.cpp"), "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return exe


@pytest.mark.parametrize("shuffle,lia", [(False, False), (True, False), (False, True)])
def test_lba_host_path_under_asan(harness, shuffle, lia):
    """lia: then the LocalInertialBA layout on the same graph (link records,
    zero iterations: the explicit results launch)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    if shuffle:
        env["SHUFFLE"] = "1"
    if lia:
        env["LIA"] = "1"
    r = subprocess.run([str(harness), "3"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert lines[0]["edges"] == 18000
    if lia:
        assert lines[1]["lia_status"] == 0
