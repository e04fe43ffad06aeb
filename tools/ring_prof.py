#!/usr/bin/env python3
"""Per-phase time of the two-pass ring decoder (timing-only variant build).

  FILE=lz4mi_decompress_ring.hip tools/build_variant.sh ringprof \
      's/^#define LZ4MI_RING_PROFILE 0/#define LZ4MI_RING_PROFILE 1/'
  python tools/ring_prof.py --so tools/variants/liblz4mi_ringprof.so --gen tiles216 --blocks 4096

Phases (wall-clock ticks summed over blocks, shown per chunk-step in ns of one
wave's life): 0 stage write, 1 bitmap check/rebuild, 2 sequence table,
3 owner map, 4 output units, 5 direct sequences;
counters: 14 unit re-passes, 15 chunk steps.
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20
NAMES = ["stage", "bitmap", "table", "owner", "units", "direct", "-", "-"]
COUNTS = {12: "slow units", 13: "deferred units", 14: "re-passes"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", required=True)
    ap.add_argument("--gen", default="tiles216")
    ap.add_argument("--blocks", type=int, default=4096)
    args = ap.parse_args()
    os.environ["LZ4MI_RING_STATS"] = "1"
    import torch
    import lz4mi
    lz4mi.init(0)
    L = ctypes.CDLL(os.path.abspath(args.so))
    L.lz4mi_decompress_blocks.restype = ctypes.c_int32
    L.lz4mi_decompress_blocks.argtypes = lz4mi.lib().lz4mi_decompress_blocks.argtypes
    assert L.lz4mi_init(0) == 0
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sp = s.cuda_stream
    n = args.blocks
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(raw.data_ptr(), args.gen, 1, BLOCK, n, sp)
    slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
    comp = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
    roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
    rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
    coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                              coff.data_ptr(), clen.data_ptr(), n, sp)
    dec = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")

    def run(lib):
        lib.lz4mi_decompress_blocks(ctypes.c_void_p(comp.data_ptr()), ctypes.c_void_p(coff.data_ptr()),
                                    ctypes.c_void_p(clen.data_ptr()), ctypes.c_void_p(dec.data_ptr()),
                                    ctypes.c_void_p(roff.data_ptr()), ctypes.c_void_p(rlen.data_ptr()), None, 0,
                                    ctypes.c_void_p(dlen.data_ptr()), ctypes.c_void_p(st.data_ptr()), n,
                                    lz4mi.DEVICE_PTRS, ctypes.c_void_p(sp))
    run(L)
    torch.cuda.synchronize()
    prof = (ctypes.c_ulonglong * 16)()
    L.lz4mi_debug_ring_prof(prof)
    stats = (ctypes.c_uint32 * 6)()
    L.lz4mi_debug_ring_stats(stats)
    t0 = time.perf_counter()
    run(L)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L.lz4mi_debug_ring_prof(prof)
    L.lz4mi_debug_ring_stats(stats)
    ok = bool(torch.equal(dec, raw)) and bool((st == 0).all().item())
    steps = max(1, prof[15])
    tot = sum(prof[i] for i in range(8))
    print(f"{args.gen}: {n} blocks, {el * 1e3:.1f} ms wall (profiled build), ok={ok}, "
          f"chunk steps {prof[15]} ({prof[15] / n:.0f}/block), re-passes/step {prof[14] / steps:.3f}, "
          f"rebuilt {stats[0]}, direct {stats[1]}, handed back {stats[2]} (why {list(stats)[3:]})")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:9s} {prof[i] * 10 / steps:9.1f} ns/step  {100 * prof[i] / max(1, tot):5.1f}%")
    print(f"  total     {tot * 10 / steps:9.1f} ns/step; per block {tot * 10 / n / 1e6:.2f} ms of wave life")
    print("  per step: " + ", ".join(f"{nm} {prof[i] / steps:.2f}" for i, nm in COUNTS.items()))


if __name__ == "__main__":
    main()
