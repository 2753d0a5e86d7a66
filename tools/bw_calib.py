"""Device-copy bandwidth calibration (torch copy_, same process/device as the
kernels) for sizes around the extractor's working sets."""
import json
import torch

res = {}
for mb in (32, 143, 286, 1024):
    n = mb * (1 << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device="cuda").uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    e0.record()
    for _ in range(it):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    res[f"copy_{mb}MB_GBps"] = round(2 * mb * (1 << 20) / (ms * 1e-3) / 1e9, 1)
    res[f"copy_{mb}MB_us"] = round(ms * 1e3, 1)
print(json.dumps(res))
