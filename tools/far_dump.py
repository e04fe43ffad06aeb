#!/usr/bin/env python3
"""Dump the GPU-compressed bytes and the raw bytes of the `far` blocks that differ from the
oracle (tools/far_check.py) for a host-side diff."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
BLOCK = 4 << 20


def main():
    import numpy as np
    import torch
    import lz4mi
    from microbench import make_raw
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    lz4mi.init(0)
    s = torch.cuda.current_stream().cuda_stream
    n = 16
    raw = make_raw(torch, lz4mi, "far", n, s)
    slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
    comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
    roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
    rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
    coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(), coff.data_ptr(),
                              clen.data_ptr(), n, s)
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    ch = comp.cpu().numpy()
    cl = clen.cpu().numpy()
    for b in (1, 3):
        host[b * BLOCK:(b + 1) * BLOCK].tofile(os.path.join(out, f"far_raw_{b}.bin"))
        ch[b * slot:b * slot + cl[b]].tofile(os.path.join(out, f"far_gpu_{b}.bin"))
    print("dumped", cl[1], cl[3])


if __name__ == "__main__":
    main()
