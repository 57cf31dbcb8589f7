"""Calibration: what a plain streaming kernel achieves on this GPU for the step kernel's traffic
(~53 MB read + ~59 MB written per launch): torch copy_ / fill_ timed with HIP events."""
import torch, json
dev = torch.device("cuda", 0)
res = {}
for mb in (16, 56, 112, 512):
    n = mb * 1024 * 1024
    a = torch.empty(n, dtype=torch.uint8, device=dev); b = torch.empty_like(a)
    for name, fn, traffic in (("copy", lambda: b.copy_(a), 2 * n), ("fill", lambda: a.fill_(7), n)):
        for _ in range(5): fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps): fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[f"{name}_{mb}MB"] = {"us": round(us, 2), "GBps": round(traffic / us / 1e3, 1)}
print(json.dumps(res))
