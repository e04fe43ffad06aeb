#!/usr/bin/env python3
"""Device-resident decode latency of small batches (1..16 blocks of 4 MiB), HIP events on the
launch stream, median of --reps: the small-batch path (csrc/lz4mi_expand.hip) or, with
LZ4MI_SMALL_BLOCKS=0 in the environment, the one-wave-per-block batch kernel."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
BLOCK = 4 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", default="tiles216,text,repetitive")
    ap.add_argument("--counts", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--js-exact", action="store_true", help="reference mode (LZ4MI_JS_EXACT)")
    args = ap.parse_args()
    import torch
    import lz4mi
    from microbench import make_raw
    lz4mi.init(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    n = max(int(x) for x in args.counts.split(","))
    flags = 1 | (8 if args.js_exact else 0)   # LZ4MI_DEVICE_PTRS | LZ4MI_JS_EXACT
    res = {"small_blocks_env": os.environ.get("LZ4MI_SMALL_BLOCKS", "default"), "js_exact": args.js_exact}
    for gen in args.gens.split(","):
        raw = make_raw(torch, lz4mi, gen, n, sp)
        slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
        comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
        roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
        rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
        coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
        clen = torch.zeros(n, dtype=torch.int32, device="cuda")
        lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(), coff.data_ptr(),
                                  clen.data_ptr(), n, sp)
        dec = torch.zeros(n * BLOCK, dtype=torch.uint8, device="cuda")
        dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        row = {}
        for b in (int(x) for x in args.counts.split(",")):
            def run():
                r = lz4mi.lib().lz4mi_decompress_blocks(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                                        roff.data_ptr(), rlen.data_ptr(), None, 0, dlen.data_ptr(),
                                                        st.data_ptr(), b, flags, sp)
                assert r == 0
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run()
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ok = bool(torch.equal(dec[:b * BLOCK], raw[:b * BLOCK])) and bool((st[:b] == 0).all())
            row[b] = {"ms": round(sorted(ts)[len(ts) // 2], 3), "ok": ok}
        res[gen] = row
        print(gen, json.dumps(row), flush=True)
        del raw, comp, dec
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
