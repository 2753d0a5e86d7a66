"""Config C5 on synthetic data: S stereo sequences per GPU (default 1, the
reference's one-sequence-per-process layout, `tests/slam_euroc_si.cc`), one
process per GPU, each carrying the device-resident tracking chain frame to
frame for its own sequences, as Tracking::TrackWithMotionModel runs it
(tracking.cc:2163-2216):

    extract L+R -> ComputeStereoMatches -> SearchByProjection(CurrentFrame,
    LastFrame) at the motion-model pose (th 7, rotation check) -> the
    observation list -> PoseOptimization -> Frame::UnprojectStereo of the
    frame's stereo keypoints at the optimised pose (the next frame's
    LastFrame points, orbgpu_unproject_stereo_batch)

The motion model (mVelocity = Tcw * Tlw^-1, tracking.cc:1777-1786) runs on the
host from the optimised pose, as the reference's tracking thread does; that
is the chain's one host round trip per frame.  The S sequences of a rank are
batched through every stage (B = S).  Sequences are synthetic (synth.sequence:
a camera translating 6 px per frame over a textured plane at depth bf/24, no
EuRoC data here), so the trajectory error against the known motion (ATE, m)
is reported beside the rate.

    python tools/c5_runner.py [--frames 200] [--warmup 10] [--seqs-per-gpu 1]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P tools/c5_runner.py ...

Rank 0 prints one JSON line: node frames/s = all ranks' timed frames / the
slowest rank's time (barrier + device sync around the timed region).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

PARAMS = (1000, 1.2, 8, 20, 7)
SHIFT, DISP, FX, BASE = 6, 24, 435.2, 0.11
TH = 7.0


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def quat_rot(q, v):
    x, y, z, w = q
    u = np.array([x, y, z])
    t = 2 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def se3_mul(A, B):  # (qx, qy, qz, qw, tx, ty, tz), A * B
    q = quat_mul(A[:4], B[:4])
    q /= np.linalg.norm(q)
    return np.concatenate([q, quat_rot(A[:4], B[4:]) + A[4:]])


def se3_inv(A):
    qi = np.array([-A[0], -A[1], -A[2], A[3]])
    return np.concatenate([qi, -quat_rot(qi, A[4:])])


class SequenceChain:
    def __init__(self, rank: int, S: int, n_frames: int, device: int):
        import torch

        from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, synth
        from orb_slam_fusion_amd.matcher import ORBmatcher, frame_geom

        self.S, self.N = S, n_frames
        dev = self.dev = torch.device("cuda", device)
        seqs = [synth.sequence(rank * S + s, n_frames, SHIFT) for s in range(S)]
        h, w = seqs[0][0].shape[1:]
        imgs = np.zeros((n_frames, 2 * S, h, w), np.uint8)
        for s, (lft, rgt) in enumerate(seqs):
            imgs[:, 2 * s], imgs[:, 2 * s + 1] = lft, rgt
        self.imgs = torch.from_numpy(imgs).to(dev)  # inputs resident in HBM
        self.ex = ex = OrbExtractor(*PARAMS, max_images=2 * S, device=device)
        cap = self.cap = ex.max_keypoints(w, h)
        self.bf = np.float32(FX * BASE)
        self.mb = np.float32(self.bf / np.float32(FX))
        self.cam = np.array([FX, FX, w / 2.0, h / 2.0, self.bf], np.float32)
        self.geom = frame_geom(w, h, ex.GetScaleFactors())
        self.inv_sigma2 = ex.GetInverseScaleSigmaSquares()
        Z = lambda *s_, dt=torch.int32: torch.zeros(s_, dtype=dt, device=dev)  # noqa: E731
        self.kps, self.desc = Z(2 * S, cap, 7), Z(2 * S, cap, 32, dt=torch.uint8)
        self.n, self.mono = Z(2 * S), Z(2 * S)
        self.ur, self.dep = Z(S, cap, dt=torch.float32), Z(S, cap, dt=torch.float32)
        self.pts, self.npts = Z(S, cap, 56, dt=torch.uint8), Z(S)
        self.matcher = ORBmatcher(0.9, True, device=device, max_keypoints=cap, max_points=cap)
        self.match, self.nm = Z(S, cap), Z(S)
        self.obs, self.nobs = Z(S, cap, 7, dt=torch.float32), Z(S)
        self.opt = PoseOptimizer(device=device, max_problems=S, max_obs=cap)
        self.pose_out = Z(S, 7, dt=torch.float32)
        self.outlier, self.inliers = Z(S, cap, dt=torch.uint8), Z(S)
        self.lk, self.ld, self.lnn = self.kps[0::2], self.desc[0::2], self.n[0::2]
        self.d_last, self.d_pred = Z(S, 7, dt=torch.float32), Z(S, 7, dt=torch.float32)

    def reset(self):
        self.T = np.tile(np.array([0, 0, 0, 1, 0, 0, 0], np.float64), (self.S, 1))
        self.V = None
        self.traj = [self.T.copy()]
        self.matches, self.inl = [], []

    def frame(self, t: int):
        import torch

        ex, m = self.ex, self.matcher
        ex.extract_batch(self.imgs[t], self.kps, self.desc, self.n, self.mono)
        ex.stereo_match_batch(self.imgs[t], self.kps, self.desc, self.n, self.bf, self.mb, self.ur,
                              self.dep)
        lk, ld, lnn = self.lk.contiguous(), self.ld.contiguous(), self.lnn.contiguous()
        if t > 0:
            # TrackWithMotionModel: predicted pose, projection search, PoseOptimization
            pred = self.T if self.V is None else np.stack([se3_mul(self.V[s], self.T[s])
                                                           for s in range(self.S)])
            self.d_pred.copy_(torch.from_numpy(pred.astype(np.float32)))
            self.d_last.copy_(torch.from_numpy(self.T.astype(np.float32)))
            m.search_last_batch(self.geom, self.cam, self.mb, self.d_pred, self.d_last, lk, ld,
                                self.ur, None, lnn, self.pts, self.npts, TH, False, self.match,
                                self.nm)
            m.matches_to_pose_obs_batch(lk, self.ur, self.match, lnn, self.pts, self.inv_sigma2,
                                        self.obs, self.nobs)
            self.opt.batch(self.cam, self.d_pred, self.obs, self.nobs, self.pose_out,
                           self.outlier, self.inliers)
            new = self.pose_out.cpu().numpy().astype(np.float64)  # the host's one round trip
            self.V = np.stack([se3_mul(new[s], se3_inv(self.T[s])) for s in range(self.S)])
            self.T = new
            self.traj.append(self.T.copy())
        else:
            self.d_last.copy_(torch.from_numpy(self.T.astype(np.float32)))
        # this frame's stereo points at its pose: the next frame's LastFrame
        src = self.d_last if t == 0 else self.pose_out
        m.unproject_stereo_batch(self.cam, src, lk, ld, self.dep, lnn, self.pts, self.npts)

    def stats(self):
        nm, inl = self.nm.cpu().numpy(), self.inliers.cpu().numpy()
        return float(nm.mean()), float(inl.mean())

    def ate(self) -> float:
        """RMS camera-centre error against the synthetic motion (frame 0 =
        identity in both): Tcw_k = (I, (k * shift * z / fx, 0, 0)), z = bf / disparity."""
        z = float(self.bf) / DISP
        err = []
        for k, T in enumerate(self.traj):
            for s in range(self.S):
                c_est = se3_inv(T[s])[4:]
                c_true = np.array([-k * SHIFT * z / FX, 0.0, 0.0])
                err.append(np.sum((c_est - c_true) ** 2))
        return float(np.sqrt(np.mean(err)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--seqs-per-gpu", type=int, default=1)
    args = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch

    from orb_slam_fusion_amd import dist

    dist.init(world, rank)
    torch.cuda.set_device(local)
    c = SequenceChain(rank, args.seqs_per_gpu, args.frames + args.warmup, local)
    c.reset()
    for t in range(args.warmup):
        c.frame(t)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.frames):
        c.frame(t)
    torch.cuda.synchronize()
    dist.barrier()
    el = dist.job_time(time.perf_counter() - t0)
    nm, inl = c.stats()
    ate = c.ate()
    if world > 1:
        import torch.distributed as tdist

        a = torch.tensor([ate], dtype=torch.float64)
        tdist.all_reduce(a, op=tdist.ReduceOp.MAX)
        ate = float(a.item())
    if rank == 0:
        frames = world * args.seqs_per_gpu * args.frames
        print(json.dumps({
            "metric": "C5 (synthetic): node frames/s, one tracking chain per sequence, frame to frame",
            "value": round(frames / el, 1), "unit": "frames/s", "n_gpus": world,
            "seqs_per_gpu": args.seqs_per_gpu, "frames_per_seq": args.frames,
            "warmup": args.warmup, "ms_per_frame_per_seq": round(el / args.frames * 1e3, 4),
            "scaling": "weak", "data": "synthetic stereo sequences (synth.sequence, 6 px/frame)",
            "matches_per_frame": round(nm, 1), "pose_inliers_per_frame": round(inl, 1),
            "ate_m_max_over_ranks": ate}))
    dist.finalize()


if __name__ == "__main__":
    main()
