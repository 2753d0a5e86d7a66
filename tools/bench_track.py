"""Tracking chain (config C3's path on synthetic data: extract + ORBmatcher
Hamming + PoseOptimization) resident on the GPU: for B pairs of consecutive
752x480 stereo frames (synth.track_pair, camera moving 6 px per frame) the
current frames go through

    extract (2B images) -> ComputeStereoMatches -> SearchByProjection(
    CurrentFrame, LastFrame) (th 7, rotation check) -> PoseOptimization's
    observation list -> PoseOptimization (from the motion-model pose)

with nothing leaving HBM, as Tracking::TrackWithMotionModel runs them
(tracking.cc:2163-2216).  The LastFrame map points are the last frames'
stereo keypoints (Frame::UnprojectStereo, identity pose), built once.
Timed with HIP events over the whole chain per batch; beside it the CPU
oracle running the same chain per frame (extraction on two threads), and a
parity check of the chain's outputs against the oracle's on a few frames
(keypoints, descriptors, stereo, matches bit-exact; pose within 1e-5).

    python tools/bench_track.py [--frames 64] [--calls 10]
"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

from bench_match import BASE, DISP, FX, SHIFT, last_frame_points  # noqa: E402

PARAMS = (1000, 1.2, 8, 20, 7)
TH = 7.0


class Chain:
    """The device-resident chain for B frame pairs."""

    def __init__(self, B: int):
        import torch

        from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, synth
        from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, PROJ_POINT_DTYPE
        from orb_slam_fusion_amd.matcher import ORBmatcher, frame_geom

        self.B = B
        dev = self.dev = torch.device("cuda", 0)
        self.quads = [synth.track_pair(i, SHIFT) for i in range(B)]
        self.last = torch.from_numpy(np.stack([im for q in self.quads for im in q[:2]])).to(dev)
        self.cur = torch.from_numpy(np.stack([im for q in self.quads for im in q[2:]])).to(dev)
        self.ex = ex = OrbExtractor(*PARAMS, max_images=2 * B)
        cap = self.cap = ex.max_keypoints(752, 480)
        self.bf = np.float32(FX * BASE)
        self.mb = np.float32(self.bf / np.float32(FX))
        self.cam = np.array([FX, FX, 376.0, 240.0, self.bf], np.float32)
        self.geom = frame_geom(752, 480, ex.GetScaleFactors())
        self.inv_sigma2 = ex.GetInverseScaleSigmaSquares()
        z = np.float32(self.bf) / np.float32(DISP)
        self.Tcw = np.tile(np.array([0, 0, 0, 1, SHIFT * z / FX, 0, 0], np.float32), (B, 1))
        self.Tlw = np.tile(np.array([0, 0, 0, 1, 0, 0, 0], np.float32), (B, 1))
        Z = lambda *s, dt=torch.int32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self.kps, self.desc = Z(2 * B, cap, 7), Z(2 * B, cap, 32, dt=torch.uint8)
        self.n, self.mono = Z(2 * B), Z(2 * B)
        self.ur, self.dep = Z(B, cap, dt=torch.float32), Z(B, cap, dt=torch.float32)
        # LastFrame map points (setup, once)
        ex.extract_batch(self.last, self.kps, self.desc, self.n, self.mono)
        ex.stereo_match_batch(self.last, self.kps, self.desc, self.n, self.bf, self.mb, self.ur,
                              self.dep)
        lk = self.kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(2 * B, cap)
        ld, ln, ldep = self.desc.cpu().numpy(), self.n.cpu().numpy(), self.dep.cpu().numpy()
        self.pts = [last_frame_points(lk[2 * f, :ln[2 * f]], ld[2 * f, :ln[2 * f]],
                                      ldep[f, :ln[2 * f]], self.cam) for f in range(B)]
        P = max(1, max(len(p) for p in self.pts))
        pa = np.zeros((B, P), PROJ_POINT_DTYPE)
        for f, p in enumerate(self.pts):
            pa[f, :len(p)] = p
        self.d_pts = torch.from_numpy(pa.view(np.uint8).reshape(B, P, 56).copy()).to(dev)
        self.d_npts = torch.tensor([len(p) for p in self.pts], dtype=torch.int32, device=dev)
        self.d_tcw = torch.from_numpy(self.Tcw).to(dev)
        self.d_tlw = torch.from_numpy(self.Tlw).to(dev)
        self.matcher = ORBmatcher(0.9, True, max_keypoints=cap, max_points=P)
        self.match, self.nm = Z(B, cap), Z(B)
        self.obs = Z(B, cap, 7, dt=torch.float32)
        self.nobs = Z(B)
        self.obs_index = Z(B, cap)
        self.opt = PoseOptimizer(max_problems=B, max_obs=cap)
        self.pose_out = Z(B, 7, dt=torch.float32)
        self.outlier = Z(B, cap, dt=torch.uint8)
        self.inliers = Z(B)
        # the current frames' left rows (views into the batch outputs)
        self.lk, self.ld, self.lnn = self.kps[0::2], self.desc[0::2], self.n[0::2]

    def run(self):
        s = None  # torch's current stream (ordered by launch_stream)
        self.ex.extract_batch(self.cur, self.kps, self.desc, self.n, self.mono, stream=s)
        self.ex.stereo_match_batch(self.cur, self.kps, self.desc, self.n, self.bf, self.mb,
                                   self.ur, self.dep, stream=s)
        lk, ld, lnn = self.lk.contiguous(), self.ld.contiguous(), self.lnn.contiguous()
        self.matcher.search_last_batch(self.geom, self.cam, self.mb, self.d_tcw, self.d_tlw, lk,
                                       ld, self.ur, None, lnn, self.d_pts, self.d_npts, TH, False,
                                       self.match, self.nm, stream=s)
        self.matcher.matches_to_pose_obs_batch(lk, self.ur, self.match, lnn, self.d_pts,
                                               self.inv_sigma2, self.obs, self.nobs,
                                               self.obs_index, stream=s)
        self.opt.batch(self.cam, self.d_tcw, self.obs, self.nobs, self.pose_out, self.outlier,
                       self.inliers, stream=s)


def oracle_chain(oracle, c: "Chain", f: int):
    """The same chain on the CPU oracle for frame pair f: returns the
    intermediate and final results."""
    from orb_slam_fusion_amd._lib import POSE_OBS_DTYPE

    _, _, cl, cr = c.quads[f]
    ol, orr = oracle.OracleExtractor(*PARAMS), oracle.OracleExtractor(*PARAMS)
    res = {}
    th = threading.Thread(target=lambda: res.__setitem__("r", orr.extract(cr)))
    th.start()
    _, kl, dl = ol.extract(cl)
    th.join()
    _, kr, dr = res["r"]
    p = ol.params()
    ur, _, _ = oracle.stereo_match(kl, dl, kr, dr, [ol.level(l) for l in range(8)],
                                   [orr.level(l) for l in range(8)], p["scale"], p["inv_scale"],
                                   c.bf, c.mb)
    nm, match = oracle.search_last(c.geom, c.cam, c.mb, c.Tcw[f], c.Tlw[f], kl, dl, ur, None,
                                   c.pts[f], TH, False, True)
    sel = np.nonzero(match >= 0)[0]
    obs = np.zeros(len(sel), POSE_OBS_DTYPE)
    obs["Xw"] = c.pts[f]["Xw"][match[sel]]
    obs["u"], obs["v"], obs["ur"] = kl["x"][sel], kl["y"][sel], ur[sel]
    obs["inv_sigma2"] = p["inv_sigma2"][kl["octave"][sel]]
    inl, pose, out, _ = oracle.pose_opt(c.cam, c.Tcw[f], obs)
    return dict(kps=kl, desc=dl, ur=ur, nm=nm, match=match, obs=obs, inliers=inl, pose=pose,
                outlier=out)


def measure(frames: int = 64, calls: int = 10, cpu_frames: int = 4) -> dict:
    import torch

    with torch.cuda.stream(torch.cuda.Stream()):
        return _measure(frames, calls, cpu_frames)


def _measure(frames, calls, cpu_frames):
    import torch

    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE

    c = Chain(frames)
    for _ in range(3):
        c.run()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(calls):
        c.run()
    e1.record(s)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / calls
    nm, inl = c.nm.cpu().numpy(), c.inliers.cpu().numpy()
    out = {"workload": f"tracking chain per frame pair (extract L+R, ComputeStereoMatches, "
                       f"SearchByProjection(CurrentFrame, LastFrame) th 7, PoseOptimization); {frames} "
                       f"synthetic 752x480 pairs per batch, camera moving {SHIFT} px per frame, all "
                       "intermediates resident in HBM",
           "gpu_ms_per_batch": round(gpu_ms, 4), "gpu_fps": round(frames / gpu_ms * 1e3, 1),
           "matches_per_frame": round(float(nm.mean()), 1),
           "pose_inliers_per_frame": round(float(inl.mean()), 1)}
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline / checker leg only

        lk = c.lk.cpu().numpy().view(KEYPOINT_DTYPE).reshape(frames, c.cap)
        ld, lnn = c.ld.cpu().numpy(), c.lnn.cpu().numpy()
        ur, match = c.ur.cpu().numpy(), c.match.cpu().numpy()
        pose, outl = c.pose_out.cpu().numpy(), c.outlier.cpu().numpy()
        exact, dpose = True, 0.0
        t0 = time.perf_counter()
        for f in range(min(cpu_frames, frames)):
            o = oracle_chain(oracle, c, f)
            k = int(lnn[f])
            exact &= (lk[f, :k].tobytes() == o["kps"].tobytes() and
                      ld[f, :k].tobytes() == o["desc"].tobytes() and
                      ur[f, :k].tobytes() == o["ur"].tobytes() and
                      int(nm[f]) == o["nm"] and np.array_equal(match[f, :k], o["match"]) and
                      int(inl[f]) == o["inliers"] and
                      np.array_equal(outl[f, :len(o["obs"])], o["outlier"]))
            dpose = max(dpose, float(np.max(np.abs(pose[f] - o["pose"]))))
        el = time.perf_counter() - t0
        out["cpu_oracle_ms_per_frame"] = round(el / min(cpu_frames, frames) * 1e3, 2)
        out["cpu_cores"] = 2
        out["exact_vs_oracle"] = bool(exact)
        out["max_pose_diff_vs_oracle"] = dpose
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, a.calls)))
