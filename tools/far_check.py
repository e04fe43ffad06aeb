#!/usr/bin/env python3
"""Isolate a round-trip failure on the microbench's `far` generator (8-48 KiB copies from the
previous 64 KiB): GPU compressed bytes vs the oracle's, GPU decode of the oracle's bytes, and
the decode with each variant library given (--so), block by block (16 distinct blocks)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
BLOCK = 4 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", nargs="*", default=[])
    ap.add_argument("--n", type=int, default=64)
    args = ap.parse_args()
    import numpy as np
    import torch
    import lz4mi
    import oracle as O
    from microbench import make_raw
    lz4mi.init(0)
    s = torch.cuda.current_stream().cuda_stream
    n = args.n
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
    for b in range(min(n, 16)):
        ref = np.frombuffer(bytes(O.compress_block_bytes(host[b * BLOCK:(b + 1) * BLOCK])), dtype=np.uint8)
        got = ch[b * slot:b * slot + cl[b]]
        same = ref.size == got.size and np.array_equal(ref, got)
        st, dec = O.decompress_block(got, BLOCK)[:2] if False else (None, None)
        print(f"block {b}: gpu comp {cl[b]} oracle {ref.size} identical={same}", flush=True)
    libs = [("default", lz4mi.lib())]
    for p in args.so:
        L = ctypes.CDLL(os.path.abspath(p))
        L.lz4mi_decompress_blocks.restype = ctypes.c_int32
        L.lz4mi_decompress_blocks.argtypes = lz4mi.lib().lz4mi_decompress_blocks.argtypes
        L.lz4mi_init.restype = ctypes.c_int32
        assert L.lz4mi_init(0) == 0
        libs.append((os.path.basename(p), L))
    for name, L in libs:
        for nb in (n, 1):
            dec = torch.zeros(n * BLOCK, dtype=torch.uint8, device="cuda")
            dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
            st = torch.zeros(n, dtype=torch.int32, device="cuda")
            if nb == n:
                r = L.lz4mi_decompress_blocks(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                              roff.data_ptr(), rlen.data_ptr(), None, 0, dlen.data_ptr(),
                                              st.data_ptr(), n, 1, s)
            else:   # one block per call (no batch order, no pacing partner)
                for b in range(n):
                    r = L.lz4mi_decompress_blocks(comp.data_ptr(), coff[b:].data_ptr(), clen[b:].data_ptr(),
                                                  dec.data_ptr(), roff[b:].data_ptr(), rlen[b:].data_ptr(), None, 0,
                                                  dlen[b:].data_ptr(), st[b:].data_ptr(), 1, 1, s)
            torch.cuda.synchronize()
            d = dec.cpu().numpy()
            bad = [b for b in range(n) if not np.array_equal(d[b * BLOCK:(b + 1) * BLOCK], host[b * BLOCK:(b + 1) * BLOCK])]
            stl = st.cpu().tolist()
            first = None
            if bad:
                b = bad[0]
                diff = np.nonzero(d[b * BLOCK:(b + 1) * BLOCK] != host[b * BLOCK:(b + 1) * BLOCK])[0]
                first = (b, int(diff[0]), int(diff.size), stl[b])
            print(f"{name} nblocks={nb}: bad blocks {len(bad)} {bad[:8]} first (block, byte, count, status) {first}",
                  flush=True)


if __name__ == "__main__":
    main()
