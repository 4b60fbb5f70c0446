"""Page-locked host -> device copy bandwidth on one MI355X: one stream vs the copy split over
2 / 4 streams (the e2e leg's H2D of 358 MB per 384-pair step), and D2H alongside."""
import json
import time

import torch

torch.cuda.init()
MB = 358
h = torch.empty(MB << 20, dtype=torch.uint8).pin_memory()
d = torch.empty(MB << 20, dtype=torch.uint8, device="cuda")
hd = torch.empty(106 << 20, dtype=torch.uint8).pin_memory()
dd = torch.empty(106 << 20, dtype=torch.uint8, device="cuda")
res = {}
for ns in (1, 2, 3, 4):
    ss = [torch.cuda.Stream() for _ in range(ns)]
    part = (MB << 20) // ns
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(5):
            for i, s in enumerate(ss):
                with torch.cuda.stream(s):
                    d[i * part:(i + 1) * part].copy_(h[i * part:(i + 1) * part], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    res[f"h2d_{ns}streams_GBs"] = round(5 * (MB << 20) / dt / 1e9, 2)
# H2D and D2H together
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
t = time.perf_counter()
for k in range(5):
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2):
        hd.copy_(dd, non_blocking=True)
torch.cuda.synchronize()
dt = time.perf_counter() - t
res["h2d_with_d2h_GBs"] = round(5 * (MB << 20) / dt / 1e9, 2)
print(json.dumps(res))
