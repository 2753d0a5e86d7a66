"""Diagnose spec vs re-linearised LocalInertialBA runs: which key frames /
fields differ, and whether two spec runs on fresh contexts agree."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam_fusion_amd import LocalBundleAdjuster, synth  # noqa: E402

pb = synth.lia_problem()
a = LocalBundleAdjuster().optimize_inertial(pb)
b = LocalBundleAdjuster().optimize_inertial(pb)
os.environ["ORBGPU_LBA_RELINEARIZE"] = "1"
c = LocalBundleAdjuster().optimize_inertial(pb)
d = LocalBundleAdjuster().optimize_inertial(pb)
for name, x, y in (("spec/spec", a, b), ("relin/relin", c, d), ("spec/relin", a, c)):
    diff = np.abs(x["kfs21"] - y["kfs21"])
    kf, f = np.nonzero(diff)
    print(name, "stats equal", np.array_equal(x["stats"], y["stats"]), "pts equal", np.array_equal(x["pts"], y["pts"]),
          "max kfs21 diff", float(diff.max()), "kfs", sorted(set(kf.tolist()))[:20], "fields", sorted(set(f.tolist())))
print("fixed", np.nonzero(pb.fixed)[0].tolist())
