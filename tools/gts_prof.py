#!/usr/bin/env python3
"""Per-phase wall-clock profile of the speculative hit-chain encoder (compress_block_gts).
Build: FILE=lz4mi_compress.hip tools/build_variant.sh cprof 's/^#define LZ4MI_CPROFILE 0 /#define LZ4MI_CPROFILE 1 /'"""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20
NAMES = ["hit: seq+hash", "hit: table+emit", "hit: windows", "hit: validate+insert", "hit: end", "miss: seq+dedupe", "miss: table+verify", "miss: extend"]

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=os.path.join(ROOT, "tools/variants/liblz4mi_cprof.so"))
    ap.add_argument("--gens", default="tiles216,random")
    ap.add_argument("--blocks", default="4096")
    a = ap.parse_args()
    import torch, lz4mi
    lz4mi.init(0)
    L = ctypes.CDLL(a.so)
    L.lz4mi_compress_blocks.argtypes = lz4mi.lib().lz4mi_compress_blocks.argtypes
    L.lz4mi_compress_blocks.restype = ctypes.c_int32
    assert L.lz4mi_init(0) == 0
    s = torch.cuda.Stream(); torch.cuda.set_stream(s); sp = s.cuda_stream
    buf = (ctypes.c_ulonglong * 16)()
    for gen in a.gens.split(","):
        from microbench import make_raw
        for n in map(int, a.blocks.split(",")):
            raw = make_raw(torch, lz4mi, gen, n, sp)   # device generators, or host-made (text, copy, ...)
            slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
            comp = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
            roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
            rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
            coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
            clen = torch.zeros(n, dtype=torch.int32, device="cuda")
            run = lambda: L.lz4mi_compress_blocks(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                                                  coff.data_ptr(), clen.data_ptr(), n, 1, sp)
            run(); torch.cuda.synchronize(); L.lz4mi_debug_cprof(buf)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s); run(); e1.record(s); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            L.lz4mi_debug_cprof(buf)
            v = list(buf)
            nb, hits, miss, mhit = v[8], v[9], v[10], v[11]
            print(f"{gen} blocks={n} kernel_ms={ms:.1f} hit batches/block={nb / n:.0f} hits/hit batch={hits / max(1, nb):.2f} "
                  f"miss batches/block={miss / n:.0f} (with a hit: {mhit / n:.0f})")
            print("   us per block:", {NAMES[i]: round(v[i] / 100.0 / n, 1) for i in range(8)},
                  "wave ms:", round(sum(v[:8]) / 100.0 / n / 1000, 1), flush=True)

if __name__ == "__main__":
    main()
