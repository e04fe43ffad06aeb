#!/usr/bin/env python3
"""Per-block decode timeline (why is the 50/50 mix slower than all-tiles216?).

Loads a decoder build compiled with -DLZ4MI_TIMELINE=1 (every block records its start and
end time, s_memrealtime at 100 MHz, and its HW_ID / XCC_ID), decodes one 4096-block batch per
generator on a device-resident batch (bench.py's layouts), and summarises when the blocks of
each kind run, per CU and over time. Raw arrays go to <out>/timeline_<gen>.npz.

  tools/build_variant.sh tl 's/^$//' -DLZ4MI_TIMELINE=1
  python tools/timeline.py --so tools/variants/liblz4mi_tl.so --gens mix,mixc,tiles216 --out gpurun_out/tl
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20


def cu_key(hw, xcc):
    """(XCD, SE, SH, CU) of a wave from HW_ID (gfx9 layout: CU 11:8, SH 12, SE 15:13)."""
    return (int(xcc) & 0xF, (int(hw) >> 13) & 0x7, (int(hw) >> 12) & 1, (int(hw) >> 8) & 0xF)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", required=True)
    ap.add_argument("--gens", default="mix,mixc,tiles216")
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--out", default="gpurun_out/tl")
    ap.add_argument("--what", default="decompress", help="decompress, or compress (a -DLZ4MI_CTIMELINE=1 build)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import lz4mi
    import bench
    os.makedirs(args.out, exist_ok=True)
    lz4mi.init(0)
    L = ctypes.CDLL(os.path.abspath(args.so))
    L.lz4mi_decompress_blocks.restype = ctypes.c_int32
    L.lz4mi_decompress_blocks.argtypes = lz4mi.lib().lz4mi_decompress_blocks.argtypes
    L.lz4mi_init.restype = ctypes.c_int32
    assert L.lz4mi_init(0) == 0
    dbg = L.lz4mi_debug_ctimeline if args.what == "compress" else L.lz4mi_debug_timeline
    dbg.restype = ctypes.c_int
    dbg.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    L.lz4mi_compress_blocks.restype = ctypes.c_int32
    L.lz4mi_compress_blocks.argtypes = lz4mi.lib().lz4mi_compress_blocks.argtypes
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    n = args.blocks
    summary = {}
    for gen in args.gens.split(","):
        B = bench.Batch(torch, lz4mi, n, gen, 1, sp)
        B.compress(lz4mi, sp)
        torch.cuda.synchronize()

        def run():
            if args.what == "compress":
                r = L.lz4mi_compress_blocks(B.raw.data_ptr(), B.raw_off.data_ptr(), B.raw_len.data_ptr(),
                                            B.comp.data_ptr(), B.comp_off.data_ptr(), B.comp_len.data_ptr(), n, 1, sp)
            else:
                r = L.lz4mi_decompress_blocks(B.comp.data_ptr(), B.comp_off.data_ptr(), B.comp_len.data_ptr(),
                                              B.dec.data_ptr(), B.raw_off.data_ptr(), B.raw_len.data_ptr(), None, 0,
                                              B.dec_len.data_ptr(), B.status.data_ptr(), n, 1, sp)
            assert r == 0
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        run()
        e1.record(s)
        torch.cuda.synchronize()
        kms = e0.elapsed_time(e1)
        if args.what == "compress":
            B.decompress(lz4mi, sp)
            torch.cuda.synchronize()
        ok = bool(torch.equal(B.dec, B.raw)) and bool((B.status == 0).all())
        t = np.zeros(2 * n, dtype=np.uint64)
        ids = np.zeros(2 * n, dtype=np.uint32)
        assert dbg(t.ctypes.data, ids.ctypes.data, n) == 0
        clen = B.comp_len.cpu().numpy().astype(np.int64)
        t0 = t[0::2].astype(np.int64)
        t1 = t[1::2].astype(np.int64)
        base = t0.min()
        start = (t0 - base) / 1e5      # ms (100 MHz ticks)
        end = (t1 - base) / 1e5
        dur = end - start
        rnd = clen > BLOCK * 0.9
        keys = [cu_key(ids[2 * b], ids[2 * b + 1]) for b in range(n)]
        cus = sorted(set(keys))
        cu_of = np.array([cus.index(k) for k in keys])
        wave = ids[0::2] & 15
        res_slot = [round(float(dur[wave == x].mean()), 3) if (wave == x).any() else None for x in range(4)]
        np.savez(os.path.join(args.out, f"timeline_{args.what}_{gen}.npz"), start=start, end=end, clen=clen, cu=cu_of,
                 hw=ids[0::2], xcc=ids[1::2])

        def st(x):
            if len(x) == 0:
                return None
            q = np.percentile(x, [0, 10, 50, 90, 100])
            return {"n": int(len(x)), "mean": round(float(x.mean()), 3),
                    "min/p10/p50/p90/max": [round(float(v), 3) for v in q]}
        res = {"kernel_ms": round(kms, 3), "ok": ok, "span_ms": round(float(end.max()), 3), "cus": len(cus),
               "dur_by_wave_slot_ms": res_slot,
               "blocks_per_cu": st(np.bincount(cu_of).astype(float)),
               "start_ms": st(start), "tiles_dur_ms": st(dur[~rnd]), "random_dur_ms": st(dur[rnd]),
               "tiles_end_ms": st(end[~rnd]), "random_end_ms": st(end[rnd])}
        if rnd.any() and (~rnd).any():
            # tiles216 duration by how many random blocks share the CU
            nr = np.bincount(cu_of, weights=rnd.astype(float), minlength=len(cus))
            by = {}
            for b in np.where(~rnd)[0]:
                by.setdefault(int(nr[cu_of[b]]), []).append(dur[b])
            res["tiles_dur_by_random_on_cu"] = {k: [len(v), round(float(np.mean(v)), 3)] for k, v in sorted(by.items())}
            # blocks of each kind running, in 20 time bins
            edges = np.linspace(0, end.max(), 21)
            mid = (edges[:-1] + edges[1:]) / 2
            res["running_random"] = [int(((start <= m) & (end > m) & rnd).sum()) for m in mid]
            res["running_tiles"] = [int(((start <= m) & (end > m) & ~rnd).sum()) for m in mid]
            res["bin_ms"] = round(float(edges[1]), 3)
        summary[f"{args.what}/{gen}"] = res
        print(gen, json.dumps(res), flush=True)
        del B
        torch.cuda.empty_cache()
    with open(os.path.join(args.out, f"timeline_summary_{args.what}.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
