"""Host-path extraction latency probe: one image on one thread, a stereo pair
on two threads (frame.cc:179-182) and back to back.

    python tools/lat_probe.py
"""
import sys, time, threading
sys.path.insert(0, '.')
import numpy as np
from orb_slam_fusion_amd import OrbExtractor, synth
l, r = synth.stereo_frame(3)
ex1 = OrbExtractor(1000, 1.2, 8, 20, 7); ex2 = OrbExtractor(1000, 1.2, 8, 20, 7)
for _ in range(5): ex1(l); ex2(r)
ts = []
for _ in range(50):
    t0 = time.perf_counter(); ex1(l); ts.append(time.perf_counter() - t0)
print("single-thread one image: median ms", round(np.median(ts) * 1e3, 3), "min", round(min(ts) * 1e3, 3))
ts = []
for _ in range(50):
    t0 = time.perf_counter()
    th = threading.Thread(target=ex2, args=(r,)); th.start(); ex1(l); th.join()
    ts.append(time.perf_counter() - t0)
print("two threads stereo: median ms", round(np.median(ts) * 1e3, 3), "min", round(min(ts) * 1e3, 3))
ts = []
for _ in range(50):
    t0 = time.perf_counter(); ex1(l); ex2(r); ts.append(time.perf_counter() - t0)
print("sequential stereo: median ms", round(np.median(ts) * 1e3, 3))
