"""ORBmatcher::SearchByProjection(CurrentFrame, LastFrame) timing -- the
motion-model search of Tracking::TrackWithMotionModel (tracking.cc:2163-2216)
-- on a realistic synthetic tracking workload: B pairs of consecutive
752x480 stereo frames (camera translating 6 px per frame over the canvas
plane, synth.track_pair).  The last frames go through the GPU extractor and
stereo matcher; their stereo keypoints become the LastFrame map points
(Frame::UnprojectStereo, identity pose).  The current frames' keypoints,
descriptors and mvuRight stay resident in HBM, and
orbgpu_search_by_projection_last_batch runs over the B frames (th = 7, the
stereo setting; rotation check on), timed with HIP events on the launch
stream.  Beside it: the CPU oracle per frame on one core, and a bit-exact
check of the GPU result against it on those frames.

    python tools/bench_match.py [--frames 64] [--calls 20]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

FX, BASE, SHIFT, DISP = 435.2, 0.11, 6, 24


def last_frame_points(kps, desc, depth, cam):
    """LastFrame map points from its stereo keypoints (Frame::UnprojectStereo,
    frame.cc; identity pose so Xw = Xc), PROJ_POINT rows in index order."""
    from orb_slam_fusion_amd._lib import PROJ_POINT_DTYPE

    fx, fy, cx, cy = (np.float32(c) for c in cam[:4])
    invfx, invfy = np.float32(1) / fx, np.float32(1) / fy
    sel = np.nonzero(depth > 0)[0]
    pts = np.zeros(len(sel), PROJ_POINT_DTYPE)
    z = depth[sel].astype(np.float32)
    pts["Xw"][:, 0] = (kps["x"][sel] - cx) * z * invfx
    pts["Xw"][:, 1] = (kps["y"][sel] - cy) * z * invfy
    pts["Xw"][:, 2] = z
    pts["octave"] = kps["octave"][sel]
    pts["angle"] = kps["angle"][sel]
    pts["has_obs"] = 1
    pts["desc"] = desc[sel]
    return pts


def measure(frames: int = 64, calls: int = 20, cpu_frames: int = 4) -> dict:
    import torch

    # every allocation, copy and launch on one non-default stream
    with torch.cuda.stream(torch.cuda.Stream()):
        return _measure(frames, calls, cpu_frames)


def _measure(frames: int, calls: int, cpu_frames: int) -> dict:
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, PROJ_POINT_DTYPE
    from orb_slam_fusion_amd.matcher import ORBmatcher, frame_geom

    B = frames
    dev = torch.device("cuda", 0)
    quads = [synth.track_pair(i, SHIFT) for i in range(B)]
    last = torch.from_numpy(np.stack([im for q in quads for im in q[:2]])).to(dev)
    cur = torch.from_numpy(np.stack([im for q in quads for im in q[2:]])).to(dev)
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = ex.max_keypoints(752, 480)
    bf = np.float32(FX * BASE)
    mb = np.float32(bf / np.float32(FX))
    cam = np.array([FX, FX, 376.0, 240.0, bf], np.float32)
    s = torch.cuda.current_stream()

    def run(imgs):
        kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device=dev)
        desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device=dev)
        n = torch.zeros(2 * B, dtype=torch.int32, device=dev)
        mono = torch.zeros(2 * B, dtype=torch.int32, device=dev)
        ur = torch.zeros((B, cap), dtype=torch.float32, device=dev)
        dep = torch.zeros((B, cap), dtype=torch.float32, device=dev)
        ex.extract_batch(imgs, kps, desc, n, mono, stream=s)
        ex.stereo_match_batch(imgs, kps, desc, n, bf, mb, ur, dep, stream=s)
        return kps, desc, n, ur, dep

    lk, ld, ln, lur, ldep = run(last)
    lk_h = lk.cpu().numpy().view(KEYPOINT_DTYPE).reshape(2 * B, cap)
    ld_h, ln_h, ldep_h = ld.cpu().numpy(), ln.cpu().numpy(), ldep.cpu().numpy()
    P = 0
    pts_list = []
    for f in range(B):
        nl = int(ln_h[2 * f])
        pts = last_frame_points(lk_h[2 * f, :nl], ld_h[2 * f, :nl], ldep_h[f, :nl], cam)
        pts_list.append(pts)
        P = max(P, len(pts))
    pts_all = np.zeros((B, max(P, 1)), PROJ_POINT_DTYPE)
    for f, p in enumerate(pts_list):
        pts_all[f, :len(p)] = p
    d_pts = torch.from_numpy(pts_all.view(np.uint8).reshape(B, -1, 56).copy()).to(dev)
    d_npts = torch.tensor([len(p) for p in pts_list], dtype=torch.int32, device=dev)

    ck, cd, cn, cur_ur, _ = run(cur)
    # current frames: the left images' rows (every other image of the batch)
    d_kps, d_desc, d_n = ck[0::2].contiguous(), cd[0::2].contiguous(), cn[0::2].contiguous()
    z = np.float32(bf) / np.float32(DISP)
    Tcw = np.tile(np.array([0, 0, 0, 1, SHIFT * z / FX, 0, 0], np.float32), (B, 1))
    Tlw = np.tile(np.array([0, 0, 0, 1, 0, 0, 0], np.float32), (B, 1))
    d_tcw, d_tlw = torch.from_numpy(Tcw).to(dev), torch.from_numpy(Tlw).to(dev)
    d_match = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(B, dtype=torch.int32, device=dev)
    geom = frame_geom(752, 480, ex.GetScaleFactors())
    m = ORBmatcher(0.9, True, max_keypoints=cap, max_points=max(P, 1))
    th = 7.0

    def search():
        m.search_last_batch(geom, cam, mb, d_tcw, d_tlw, d_kps, d_desc, cur_ur, None, d_n, d_pts,
                            d_npts, th, False, d_match, d_nm, stream=s)

    for _ in range(3):
        search()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(calls):
        search()
    e1.record(s)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / calls
    nm = d_nm.cpu().numpy()
    out = {"workload": f"SearchByProjection(CurrentFrame, LastFrame), th 7, rotation check; {B} "
                       f"synthetic 752x480 stereo frame pairs per batch (camera moving {SHIFT} px "
                       "per frame), current-frame extractor + stereo outputs resident in HBM",
           "gpu_ms_per_batch": round(gpu_ms, 4), "gpu_us_per_frame": round(gpu_ms / B * 1e3, 3),
           "points_per_frame": round(float(np.mean([len(p) for p in pts_list])), 1),
           "matches_per_frame": round(float(nm.mean()), 1)}
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline / checker leg only

        ck_h = d_kps.cpu().numpy().view(KEYPOINT_DTYPE).reshape(B, cap)
        cd_h, cn_h, cur_h = d_desc.cpu().numpy(), d_n.cpu().numpy(), cur_ur.cpu().numpy()
        match_h = d_match.cpu().numpy()
        work, exact = [], True
        for f in range(min(cpu_frames, B)):
            k = int(cn_h[f])
            args = (geom, cam, mb, Tcw[f], Tlw[f], ck_h[f, :k], cd_h[f, :k], cur_h[f, :k], None,
                    pts_list[f], th, False, True)
            nm_o, m_o = oracle.search_last(*args)
            exact &= nm_o == int(nm[f]) and np.array_equal(m_o, match_h[f, :k])
            work.append(args)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            for a in work:
                oracle.search_last(*a)
        out["cpu_oracle_us_per_frame"] = round((time.perf_counter() - t0) / (reps * len(work)) * 1e6, 1)
        out["cpu_cores"] = 1
        out["bit_exact_vs_oracle"] = bool(exact)
    m.close()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, a.calls)))
