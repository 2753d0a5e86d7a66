"""Writes tests/golden/*.json from the CPU oracle on seeded synthetic inputs.

The reference ships no golden vectors or known-answer tests for this path
(SURVEY.md §4, §8c), so these fixtures pin the oracle itself against
regressions; they are NOT an independent pin of the OpenCV boundary.
Run: python tools/make_golden.py  (after `make`).
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))

import binding as oracle  # noqa: E402
from orb_slam_fusion_amd import synth  # noqa: E402

OUT = REPO / "tests" / "golden"


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def extractor_cases():
    cases = []
    for frame in range(5):
        left, right = synth.stereo_frame(frame)
        for side, img in (("L", left), ("R", right)):
            cases.append(dict(name=f"stereo{frame}{side}", gen=["stereo", frame, side, 752, 480],
                              params=[1000, 1.2, 8, 20, 7], lapping=[0, 0], img=img))
    left, _ = synth.stereo_frame(10)
    cases.append(dict(name="euroc10L", gen=["stereo", 10, "L", 752, 480],
                      params=[1200, 1.2, 8, 20, 7], lapping=[0, 0], img=left))
    cases.append(dict(name="lapping3L", gen=["stereo", 3, "L", 752, 480],
                      params=[1000, 1.2, 8, 20, 7], lapping=[200, 500], img=synth.stereo_frame(3)[0]))
    cases.append(dict(name="noise99", gen=["noise", 99, 320, 256], params=[500, 1.2, 4, 20, 7],
                      lapping=[0, 0], img=synth.noise_image(99, 320, 256)))
    return cases


def main() -> int:
    OUT.mkdir(parents=True, exist_ok=True)
    ext = []
    for c in extractor_cases():
        ex = oracle.OracleExtractor(*c["params"])
        mono, k, d = ex.extract(c["img"], c["lapping"])
        pyr = [sha(ex.level(l)) for l in range(c["params"][2])]
        ext.append(dict(
            name=c["name"], gen=c["gen"], params=c["params"], lapping=c["lapping"],
            image_sha256=sha(c["img"]), n=int(len(k)), mono=int(mono),
            keypoints_sha256=sha(k), descriptors_sha256=sha(d), pyramid_sha256=pyr,
            first_keypoints=[[float(v) for v in k[i].tolist()] for i in range(min(3, len(k)))],
            first_descriptors_hex=[d[i].tobytes().hex() for i in range(min(3, len(k)))],
        ))
    (OUT / "extractor_golden.json").write_text(json.dumps(ext, indent=1) + "\n")

    pose = []
    for seed, n, pct in [(7, 600, 10), (8, 600, 10), (9, 600, 10), (11, 50, 30), (12, 1200, 10)]:
        cam, pin, pt, obs = synth.pose_problem(seed, n, pct)
        inl, pout, out, pd = oracle.pose_opt(cam, pin, obs)
        pose.append(dict(seed=seed, n=n, outlier_pct=pct, obs_sha256=sha(obs), inliers=int(inl),
                         outlier_sha256=sha(out), pose=[float(v) for v in pout],
                         pose_f64=[float(v) for v in pd]))
    (OUT / "pose_golden.json").write_text(json.dumps(pose, indent=1) + "\n")
    print(f"wrote {len(ext)} extractor and {len(pose)} pose fixtures to {OUT}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
