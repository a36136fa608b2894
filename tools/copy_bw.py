# Calibration: device-to-device copy bandwidth (read + write bytes / time) of torch's copy kernel
# and hipMemcpy on this GPU, for the emit-stage roofline discussion.  usage (GPU box): python tools/copy_bw.py
import json
import time
import torch

res = {}
for mib in (256, 1024):
    n = mib << 20
    a = torch.empty(n, dtype=torch.uint8, device="cuda").random_(0, 255)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        b.copy_(a)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 20
    res[f"copy_{mib}MiB"] = {"ms": round(ms, 4), "rw_TBps": round(2 * n / ms / 1e9, 3)}
    # one read, two writes (the emit's pattern: wire + cache slot)
    c = torch.empty_like(a)
    ev0.record()
    for _ in range(20):
        b.copy_(a)
        c.copy_(a)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 20
    res[f"copy2_{mib}MiB"] = {"ms": round(ms, 4), "rw_TBps": round(4 * n / ms / 1e9, 3)}
    del a, b, c
print(json.dumps(res))
