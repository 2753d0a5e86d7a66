"""Generated data the kernels and the oracle share, pinned against its source
(VERDICT r5 item 6): a drift there would be common-mode and invisible to every
parity test.

* csrc/pattern31.inc (read by k_describe and oracle/orb_oracle.cc) against
  kBitPattern31 (orb_extractor.cc:148-405) re-parsed from the reference when
  it is present, and always against the SHA-256 of its 1024 values as int8
  (the same table OpenCV ships as bit_pattern_31_; first pairs spot-checked);
* csrc/inertial_gj.inc against a fresh run of tools/gen_inertial_gj.py.
"""
import hashlib
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))

import gen_pattern31  # noqa: E402

INC = REPO / "orb_slam_fusion_amd" / "csrc"
REF_SRC = Path("/root/reference/src/cam/orb_feature/orb_extractor.cc")
# SHA-256 of kBitPattern31's 1024 integers as int8, in table order
PATTERN31_SHA256 = "2164181aea6ff9ac426ca512d5130d15e1f6e3cd47b1cbdd568bbe1e55d49023"


def _pattern_inc():
    return gen_pattern31.parse_include((INC / "pattern31.inc").read_text())


def test_pattern31_hash_and_shape():
    vals = _pattern_inc()
    assert len(vals) == 1024
    assert all(-13 <= v <= 12 for v in vals)  # a 31x31 patch: offsets within [-13, 12]
    assert vals[:8] == [8, -3, 9, 5, 4, 2, 7, -12]
    assert vals[-4:] == [-1, -6, 0, -11]
    assert hashlib.sha256(np.array(vals, np.int8).tobytes()).hexdigest() == PATTERN31_SHA256


@pytest.mark.skipif(not REF_SRC.exists(), reason="reference source not present")
def test_pattern31_equals_reference_table():
    assert _pattern_inc() == gen_pattern31.parse_reference(REF_SRC.read_text())


def test_inertial_gj_regenerates_identically():
    r = subprocess.run([sys.executable, str(REPO / "tools" / "gen_inertial_gj.py")],
                       capture_output=True, text=True, timeout=120, check=True)
    assert r.stdout == (INC / "inertial_gj.inc").read_text()
