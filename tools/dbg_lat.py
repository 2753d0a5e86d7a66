import sys, os, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tools')
import torch
torch.zeros(1, device='cuda'); torch.cuda.synchronize()
which = sys.argv[1]
if which == 'track':
    from bench_track import measure as m; m(frames=64, calls=2, cpu_frames=0)
elif which == 'inertial':
    from bench_inertial import measure as m; m(problems=64, calls=2, mode=0, cpu_problems=0)
elif which == 'bow':
    from bench_bow import measure as m; m(frames=64, calls=2, cpu_frames=0)
elif which == 'match':
    from bench_match import measure as m; m(frames=64, calls=2, cpu_frames=0)
elif which == 'stereo':
    from bench_stereo import measure as m; m(frames=64, calls=2, cpu_frames=0)
from bench_latency import measure
try:
    r = measure(frames=20, cpu_frames=0, cpp_host=False)
    print(which, 'OK', r['gpu_extract_ms'])
except Exception as e:
    print(which, 'FAIL', e)
