#!/usr/bin/env python3
"""Times the batched XXH32 kernel on 4096 device-resident 4 MiB blocks (HIP events) and
checks a few digests against the host implementation."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
import torch
import lz4mi
lz4mi.init(0)
n, B = 4096, 4 << 20
s = torch.cuda.Stream(); torch.cuda.set_stream(s); sp = s.cuda_stream
raw = torch.empty(n * B, dtype=torch.uint8, device="cuda")
lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 1, B, n, sp)
off = torch.arange(n, dtype=torch.int64, device="cuda") * B
ln = torch.full((n,), B, dtype=torch.int32, device="cuda")
h = torch.zeros(n, dtype=torch.int32, device="cuda")
ts = []
for _ in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    lz4mi.xxh32_blocks_dev(raw.data_ptr(), off.data_ptr(), ln.data_ptr(), h.data_ptr(), n, 0, sp)
    e1.record(s); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
ok = all((int(h[b]) & 0xFFFFFFFF) == lz4mi.xxh32(raw[b * B:(b + 1) * B].cpu().numpy(), 0) for b in (0, 1, 777, n - 1))
t = sorted(ts)[len(ts) // 2]
print(json.dumps({"xxh32_ms": round(t, 3), "GBps": round(n * B / t / 1e6, 1), "host_match": ok}))
