"""Host-pointer decode latency (tool): lz4mi_decompress_blocks on host buffers (the N-API route's
C-ABI call: pageable H2D, decode, D2H) against the host codec on one thread, for 4 MiB tiles216
blocks; output arrays pre-faulted (`warm`) or fresh (`cold`: page faults inside the call)."""
import argparse, json, os, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..")); sys.path.insert(0, os.path.join(HERE, "..", "divortio-lz4_amd"))
from oracle import oracle as O  # noqa: E402
import lz4mi  # noqa: E402
from lz4mi import lib, _p  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--counts", default="1,2,4,7,16")
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
L = lib()
blk = 4 << 20
srcs = [O.generate("tiles216", 900 + k, blk) for k in range(16)]
comps = [O.compress_block_bytes(s) for s in srcs]
res = {}
for n in [int(x) for x in args.counts.split(",")]:
    arrs = comps[:n]
    in_len = np.array([a.size for a in arrs], dtype=np.uint32)
    in_off = np.zeros(n, dtype=np.uint64); in_off[1:] = np.cumsum(in_len[:-1].astype(np.uint64))
    src = np.concatenate(arrs)
    cap = np.full(n, blk, dtype=np.uint32)
    out_off = (np.arange(n, dtype=np.uint64) * blk)
    out_len = np.zeros(n, dtype=np.uint32); st = np.zeros(n, dtype=np.int32)
    row = {}
    for mode in ("warm", "cold"):
        ts = []
        out = np.zeros(n * blk, dtype=np.uint8)
        for r in range(args.reps + 1):
            if mode == "cold":
                out = np.empty(n * blk, dtype=np.uint8)   # fresh pages: faulted inside the call
            t0 = time.perf_counter()
            rc = L.lz4mi_decompress_blocks(_p(src), _p(in_off), _p(in_len), _p(out), _p(out_off), _p(cap), None, 0,
                                           _p(out_len), _p(st), n, 0, None)
            t1 = time.perf_counter()
            assert rc == 0 and (st == 0).all()
            if r: ts.append((t1 - t0) * 1e3)
        ok = all(np.array_equal(out[k * blk:(k + 1) * blk], srcs[k]) for k in range(n))
        row["gpu_" + mode + "_ms"] = round(float(np.median(ts)), 3)
        row["ok"] = bool(ok)
    ts = []
    for r in range(args.reps + 1):
        out = np.zeros(n * blk, dtype=np.uint8)
        t0 = time.perf_counter()
        for k in range(n):
            w = L.lz4mi_host_decompress_block(_p(arrs[k]), arrs[k].size, 0, arrs[k].size, _p(out), out.size, k * blk,
                                              None, 0, 0)
            assert w == blk
        t1 = time.perf_counter()
        if r: ts.append((t1 - t0) * 1e3)
    row["host_1thread_warm_ms"] = round(float(np.median(ts)), 3)
    res[n] = row
    print(n, row, flush=True)
print(json.dumps(res))
