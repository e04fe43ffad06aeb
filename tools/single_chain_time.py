#!/usr/bin/env python3
"""Latency of one compress chain alone on the GPU: the caller's-table kernel
(lz4mi_compress_block_table, the dependent-block path) vs the batch kernel with
one block, on one 4 MiB block of each generator (host buffers, so the times
include the 4 MiB H2D + output D2H)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import lz4mi
import oracle as O

lz4mi.init(0)
for gen in sys.argv[1].split(","):
    src = O.generate(gen, 1, 4 << 20)
    out = np.zeros(lz4mi.compress_bound(src.size) + 64, dtype=np.uint8)
    for name, fn in (("table", lambda: lz4mi.compress_raw(src, out, 0, src.size, np.zeros(16384, np.int32), 0)),
                     ("batch1", lambda: lz4mi.compress_blocks([src]))):
        fn()
        t0 = time.perf_counter(); reps = 3
        for _ in range(reps): fn()
        dt = (time.perf_counter() - t0) / reps
        print(gen, name, "%.1f ms/block = %.3f GB/s" % (dt * 1e3, src.size / dt / 1e9), flush=True)
