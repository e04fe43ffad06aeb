#!/usr/bin/env python3
"""A/B of the batch encoders on device-resident 4 MiB blocks (not the driver bench).

Compresses the same batch with LZ4MI_ENCODER unset (global-table encoder) and with
each encoder named on the command line, checks that every variant's compressed
bytes equal the default's, and prints kernel times from HIP events.

  python tools/compress_ab.py --gens tiles216,random --blocks 4096 --enc pf
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", default="tiles216,random")
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--enc", default="pf")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import lz4mi
    lz4mi.init(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    n = args.blocks
    slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
    for gen in args.gens.split(","):
        raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
        lz4mi.generate_blocks_dev(raw.data_ptr(), gen, 1, BLOCK, n, sp)
        roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
        rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
        coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
        ref = None
        for enc in [""] + args.enc.split(","):
            os.environ["LZ4MI_ENCODER"] = enc
            comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
            clen = torch.zeros(n, dtype=torch.int32, device="cuda")
            times = []
            for _ in range(args.reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                                          coff.data_ptr(), clen.data_ptr(), n, sp)
                e1.record(s)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 1e3)
            t = min(times)
            same = None
            if ref is None:
                ref = (comp, clen)
            else:
                same = bool(torch.equal(comp, ref[0])) and bool(torch.equal(clen, ref[1]))
            print(gen, enc or "default", json.dumps({"ms": round(t * 1e3, 3), "GBps": round(n * BLOCK / t / 1e9, 2),
                                                     "identical_to_default": same}), flush=True)
            if ref[0] is not comp:
                del comp
        os.environ.pop("LZ4MI_ENCODER", None)
        del raw, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
