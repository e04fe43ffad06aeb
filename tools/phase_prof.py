#!/usr/bin/env python3
"""Per-phase wall-clock profile of the decoder (build: tools/build_variant.sh prof
's/^#define LZ4MI_PROFILE 0 /#define LZ4MI_PROFILE 1 /'). Prints, per block
count, the average microseconds a wave spends in each phase per chunk."""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
BLOCK = 4 << 20
NAMES = ["stage", "next", "walk", "table", "cutparse", "round1", "rounds", "cutout", "chunkend"]

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=os.path.join(ROOT, "tools/variants/liblz4mi_prof.so"))
    ap.add_argument("--gens", default="tiles216")
    ap.add_argument("--blocks", default="256,1024,4096")
    a = ap.parse_args()
    import torch, lz4mi
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from microbench import make_raw
    lz4mi.init(0)
    L = ctypes.CDLL(a.so)
    L.lz4mi_decompress_blocks.argtypes = lz4mi.lib().lz4mi_decompress_blocks.argtypes
    L.lz4mi_decompress_blocks.restype = ctypes.c_int32
    assert L.lz4mi_init(0) == 0
    s = torch.cuda.Stream(); torch.cuda.set_stream(s); sp = s.cuda_stream
    buf = (ctypes.c_ulonglong * 24)()
    for gen in a.gens.split(","):
        for n in map(int, a.blocks.split(",")):
            raw = make_raw(torch, lz4mi, gen, n, sp)
            slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
            comp = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
            roff = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
            rlen = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
            coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
            clen = torch.zeros(n, dtype=torch.int32, device="cuda")
            lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(),
                                      coff.data_ptr(), clen.data_ptr(), n, sp)
            dec = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
            dlen = torch.zeros(n, dtype=torch.int32, device="cuda"); st = torch.zeros(n, dtype=torch.int32, device="cuda")
            run = lambda: L.lz4mi_decompress_blocks(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                                    roff.data_ptr(), rlen.data_ptr(), None, 0, dlen.data_ptr(),
                                                    st.data_ptr(), n, 1, sp)
            run(); torch.cuda.synchronize(); L.lz4mi_debug_prof(buf)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s); run(); e1.record(s); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            L.lz4mi_debug_prof(buf)
            v = list(buf)
            chunks = v[10] / n
            per = {NAMES[i]: round(v[i] / 100.0 / n / max(1, chunks), 3) for i in range(9)}
            tot = sum(v[:9]) / 100.0 / n / 1000.0
            ok = bool(torch.equal(dec, raw))
            print(f"{gen} blocks={n} kernel_ms={ms:.2f} wave_ms={tot:.2f} chunks/block={chunks:.0f} "
                  f"rounds/chunk={v[11] / n / max(1, chunks):.2f} cuts/block={v[12] / n:.1f} ok={ok}")
            print("   us/chunk:", per, flush=True)
            extra = {nm: round(v[i] / 100.0 / n / max(1, chunks), 3) for i, nm in
                     ((21, "r1_wait"), (22, "r1_map"), (23, "r1_litruns"), (16, "r1_remap"), (17, "r1_split_lits"),
                      (18, "r1_slow+long"), (19, "r1_pipe"), (20, "rN_compact+wait"))}
            print("   round-1 split:", extra)
            print(f"   cert iterations/chunk={v[13] / n / max(1, chunks):.2f} initially-bad lanes/chunk="
                  f"{v[14] / n / max(1, chunks):.2f} warm-up steps/lane/chunk={v[15] / n / max(1, chunks):.2f}")
            del raw, comp, dec
            torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
