"""k_mt_resolve work counters (ORB_STAMPS build) on the stereo-inertial
latency workload's SearchLocalPoints calls (tools/bench_latency_inertial.py):
per call the 64-query chunks, resolve rounds, top-K list re-searches.

    ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/mt_stats.py
"""
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))


def main(frames: int = 8):
    from bench_latency_inertial import NN_LOCAL, PARAMS, TH_LOCAL, _local_map
    from bench_track import Chain

    from orb_slam_fusion_amd import OrbExtractor, compute_stereo_matches
    from orb_slam_fusion_amd._lib import lib
    from orb_slam_fusion_amd.matcher import MatchFrame, ORBmatcher

    c = Chain(frames)
    scale = c.ex.GetScaleFactors()
    maps = [_local_map(c, f, scale) for f in range(frames)]
    exl, exr = OrbExtractor(*PARAMS), OrbExtractor(*PARAMS)
    local = ORBmatcher(NN_LOCAL, True, max_keypoints=c.cap, max_points=max(len(m) for m in maps))
    fn = lib().orbgpu_debug_mt_stats
    fn.restype = ctypes.c_int
    buf = (ctypes.c_ulonglong * 6)()
    rows = []
    for f in range(frames):
        _, _, cl, cr = c.quads[f]
        (_, kl, dl), _ = exl.extract_stereo(exr, cl, cr)
        ur, _ = compute_stereo_matches(exl, exr, len(kl), c.bf, c.mb)
        F = MatchFrame(geom=c.geom, cam=c.cam, mb=c.mb, kps=kl, desc=dl, uright=ur, claimed=None, pose=c.Tcw[f])
        fn(buf)
        nm, _, _ = local.search_local_points(F, maps[f], 0.5, TH_LOCAL)
        assert fn(buf) == 0
        rows.append({"keypoints": len(kl), "points": len(maps[f]), "matches": int(nm), "chunks": buf[0],
                     "rounds": buf[1], "re_searches": buf[2],
                     "loop_ticks": buf[4], "re_search_ticks": buf[5]})
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
