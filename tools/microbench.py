#!/usr/bin/env python3
"""Microbenchmark harness for kernel iteration (not the driver bench).

Times lz4mi_decompress_blocks / compress / xxh32 on device-resident batches of
4 MiB blocks for each generator; optionally loads alternative builds of the
library (--so a.so b.so ...) and interleaves them in one process for A/B
comparisons (cdna guide §5.4 rule 24).

  python tools/microbench.py --gens tiles216,random,repetitive --blocks 4096 --reps 5
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20


def make_raw(torch, lz4mi, gen, n, sp):
    """n x 4 MiB raw blocks on the device: device generators (tiles216, random,
    repetitive), bench.py's "mix", or host-made blocks (copy, runs, text from the
    oracle's generators; per:<P> = P random bytes repeated; far = copies of 8-48 KiB
    windows from the previous 64 KiB, non-overlapping), 16 distinct blocks tiled."""
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    if gen in ("mix", "mixc"):   # bench.py's 50/50 random/tiles216 mix (same shuffle), or clustered
        sys.path.insert(0, ROOT)
        from bench import mix_order
        from lz4mi import shard
        tmp = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
        kinds = mix_order(n) if gen == "mix" else shard.clustered_mix_kinds(n)
        for b, kind in enumerate(kinds):
            lz4mi.generate_blocks_dev(tmp.data_ptr(), kind, 1 + b, BLOCK, 1, sp)
            raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
    elif gen in lz4mi.GENERATORS:
        lz4mi.generate_blocks_dev(raw.data_ptr(), gen, 1, BLOCK, n, sp)
    else:   # host-made: oracle generators (copy, runs, text) or per:<P> (P random bytes
        #     repeated), 16 distinct blocks tiled over the batch
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        rng = np.random.default_rng(5)
        host = []
        for k in range(16):
            if gen == "far":
                b = np.empty(BLOCK, dtype=np.uint8)
                b[:65536] = rng.integers(0, 256, 65536, dtype=np.uint8)
                pos = 65536
                while pos < BLOCK:
                    ln = min(int(rng.integers(8192, 49152)), BLOCK - pos)
                    src = pos - int(rng.integers(ln, 65536))
                    b[pos:pos + ln] = b[src:src + ln]
                    pos += ln
                host.append(b)
            elif gen.startswith("per:"):
                P = int(gen[4:])
                host.append(np.resize(rng.integers(0, 256, P, dtype=np.uint8), BLOCK))
            else:
                host.append(O.generate(gen, 1 + k, BLOCK))
        hb = torch.from_numpy(np.concatenate(host)).cuda()
        for b in range(0, n, 16):
            m = min(16, n - b)
            raw[b * BLOCK:(b + m) * BLOCK].copy_(hb[:m * BLOCK])
    return raw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", default="tiles216,random,repetitive")
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--so", nargs="*", default=[])
    ap.add_argument("--what", default="decompress")
    ap.add_argument("--skip-default", action="store_true", help="time only the --so libraries")
    ap.add_argument("--flags", type=lambda x: int(x, 0), default=0, help="extra decode flags (0x8 = LZ4MI_JS_EXACT)")
    args = ap.parse_args()
    import torch
    import lz4mi
    lz4mi.init(0)
    libs = [] if args.skip_default else [("default", lz4mi.lib())]
    for p in args.so:
        L = ctypes.CDLL(os.path.abspath(p))
        L.lz4mi_decompress_blocks.restype = ctypes.c_int32
        L.lz4mi_decompress_blocks.argtypes = lz4mi.lib().lz4mi_decompress_blocks.argtypes
        L.lz4mi_compress_blocks.restype = ctypes.c_int32
        L.lz4mi_compress_blocks.argtypes = lz4mi.lib().lz4mi_compress_blocks.argtypes
        L.lz4mi_init.restype = ctypes.c_int32
        assert L.lz4mi_init(0) == 0
        libs.append((os.path.basename(p), L))
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    n = args.blocks
    res = {}
    for gen in args.gens.split(","):
        raw = make_raw(torch, lz4mi, gen, n, sp)
        slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
        comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
        roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
        rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
        coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
        clen = torch.zeros(n, dtype=torch.int32, device="cuda")
        lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                                  coff.data_ptr(), clen.data_ptr(), n, sp)
        dec = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
        dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        cbytes = int(clen.sum())
        ref = (comp.clone(), clen.clone()) if args.what != "decompress" else None
        for name, L in libs:
            def run():
                if args.what == "decompress":
                    r = L.lz4mi_decompress_blocks(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                                  roff.data_ptr(), rlen.data_ptr(), None, 0, dlen.data_ptr(),
                                                  st.data_ptr(), n, 1 | args.flags, sp)
                else:
                    r = L.lz4mi_compress_blocks(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                                                coff.data_ptr(), clen.data_ptr(), n, 1, sp)
                assert r == 0
            dec.zero_()      # (so "ok" is this build's output, not a leftover of the previous one)
            comp.zero_() if args.what != "decompress" else None
            torch.cuda.synchronize()
            run()
            torch.cuda.synchronize()
            times = []
            for _ in range(args.reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run()
                e1.record(s)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 1e3)
            ok = True
            if args.what == "decompress":
                ok = bool(torch.equal(dec, raw)) and bool((st == 0).all())
            else:   # byte-identical to the first build's output (the bytes past each block's
                #     length are the same leftovers in both buffers)
                ok = bool(torch.equal(clen, ref[1])) and bool(torch.equal(comp, ref[0]))
            t = sorted(times)[len(times) // 2]
            res[f"{gen}/{name}"] = {"ms": round(t * 1e3, 3), "GBps": round(n * BLOCK / t / 1e9, 1),
                                    "hbm_frac": round((n * BLOCK + cbytes) / t / 8e12, 4), "ok": ok,
                                    "ratio": round(n * BLOCK / cbytes, 3)}
            print(gen, name, json.dumps(res[f"{gen}/{name}"]), flush=True)
        del raw, comp, dec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
