#!/usr/bin/env python3
"""Per-phase wall clock of the dependent-block chain (one wave): build
tools/build_variant.sh cprof 's/^#define LZ4MI_CPROFILE 0 /#define LZ4MI_CPROFILE 1 /' with FILE=lz4mi_compress.hip.
Prints microseconds per probe / per hit in each phase of compress_block_wave."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "divortio-lz4_amd"), os.path.join(ROOT, "oracle")]
import lz4mi
import oracle as O
lz4mi.init(0)
L = ctypes.CDLL(os.path.join(ROOT, "tools/variants/liblz4mi_cprof.so"))
L.lz4mi_compress_chain.argtypes = lz4mi.lib().lz4mi_compress_chain.argtypes
L.lz4mi_compress_chain.restype = ctypes.c_int32
L.lz4mi_compress_block_table.argtypes = lz4mi.lib().lz4mi_compress_block_table.argtypes
L.lz4mi_compress_block_table.restype = ctypes.c_int64
assert L.lz4mi_init(0) == 0
buf = (ctypes.c_ulonglong * 16)()
BS = 4 << 20
names = ["head probe", "reads+emit", "batch", "extend", "tail", "", "ring"]
for gen in (sys.argv[1] if len(sys.argv) > 1 else "tiles216,random").split(","):
    data = O.generate(gen, 7, BS)
    for mode in ("chain", "table"):
        t = np.zeros(16384, dtype=np.int32)
        out = np.zeros(lz4mi.compress_bound(BS) + 64, dtype=np.uint8)
        L.lz4mi_debug_cprof(buf)
        t0 = time.perf_counter()
        if mode == "chain":
            off = np.zeros(1, dtype=np.uint64); cl = np.zeros(1, dtype=np.uint32)
            r = L.lz4mi_compress_chain(data.ctypes.data, data.size, 0, BS, BS, t.ctypes.data, out.ctypes.data,
                                       off.ctypes.data, cl.ctypes.data, 0, None)
        else:
            r = L.lz4mi_compress_block_table(data.ctypes.data, data.size, 0, BS, t.ctypes.data, out.ctypes.data,
                                             out.size, 0, 0, None)
        el = time.perf_counter() - t0
        L.lz4mi_debug_cprof(buf)
        v = list(buf)
        probes, hits = max(1, v[8]), max(1, v[9])
        tot = sum(v[:5]) / 100.0
        print(f"{gen} {mode}: {el*1e3:.1f} ms wall, wave time {tot/1e3:.1f} ms, probes {v[8]}, hits {v[9]}; us/probe "
              + ", ".join(f"{names[k]} {v[k] / 100.0 / probes:.3f}" for k in range(5))
              + f"; us/hit extend {v[3] / 100.0 / hits:.3f} emit {v[4] / 100.0 / hits:.3f}", flush=True)
