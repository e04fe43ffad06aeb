#!/usr/bin/env python3
"""Dependent-block chain A/B: lz4mi_compress_chain with LZ4MI_CHAIN unset (batched chain) and =v1
(one sequence per step), 4 x 4 MiB of each generator, host buffers; both checked against the
per-block table calls (lz4mi_compress_block_table, the reference's compressBlock semantics)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "divortio-lz4_amd"), os.path.join(ROOT, "oracle")]
import lz4mi
import oracle as O
lz4mi.init(0)
BS = 4 << 20
for gen in (sys.argv[1] if len(sys.argv) > 1 else "tiles216,text,random").split(","):
    data = np.concatenate([O.generate(gen, 7 + k, BS) for k in range(4)])
    t2 = np.zeros(16384, dtype=np.int32)
    out = np.zeros(lz4mi.compress_bound(BS), dtype=np.uint8)
    ref = []
    for b in range(4):
        w = lz4mi.compress_raw(data, out, b * BS, BS, t2, 0)
        ref.append(out[:w].copy())
    for v in ("", "v1"):
        os.environ["LZ4MI_CHAIN"] = v
        t = np.zeros(16384, dtype=np.int32)
        lz4mi.compress_chain(data[:1 << 20], 0, 1 << 20, BS, t)       # warm-up
        t = np.zeros(16384, dtype=np.int32)
        t0 = time.perf_counter()
        got = lz4mi.compress_chain(data, 0, data.size, BS, t)
        tc = time.perf_counter() - t0
        ok = all(np.array_equal(a, b) for a, b in zip(got, ref)) and np.array_equal(t, t2)
        print(f"{gen} chain{'-' + v if v else ''}: {data.size / tc / 1e9:.3f} GB/s ({tc * 1e3 / 4:.1f} ms/block), "
              f"identical to per-block calls: {ok}", flush=True)
