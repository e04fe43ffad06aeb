"""GPU parity of the two-pass ring decoder (lz4mi_decompress_ring.hip).

The default spec-mode batch decode runs pass 1 (token bitmaps) + pass 2 (LDS
ring) and hands any block outside its fast path to the single-pass kernel.
These tests decode batches that exercise every branch of pass 2 — bitmap
rebuilds, direct (multi-byte length) sequences, ring wrap-around, at-risk
sources near the 64 KiB window edge, block tails — and compare bit-exactly with
the source bytes and the CPU oracle's decode of the same compressed blocks.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _ring_for_every_block():
    """Route every block through the ring decoder (the default is the single-pass kernel)."""
    import lz4mi
    lz4mi.init(0)
    lz4mi.lib().lz4mi_debug_set_decoder(1, 0)
    yield
    lz4mi.lib().lz4mi_debug_set_decoder(-1, 0)


def _lz4mi():
    import lz4mi
    lz4mi.init(0)
    return lz4mi


def _stats(lz4mi):
    out = (ctypes.c_uint32 * 6)()
    lz4mi.lib().lz4mi_debug_ring_stats(out)
    return list(out)


def _blocks():
    srcs = []
    sizes = [0, 1, 5, 13, 16, 17, 64, 1000, 1024, 1025, 4096, 65535, 65536, 65537, 200003, 1 << 20]
    for i, n in enumerate(sizes):
        for g in ("tiles216", "text", "copy", "runs", "random", "repetitive"):
            srcs.append(O.generate(g, 7 + i, n))
    # long literal runs inside compressible data, and long matches after a window's worth of output
    rng = np.random.default_rng(5)
    a = O.generate("tiles216", 3, 300000)
    a[100000:101500] = rng.integers(0, 256, 1500, dtype=np.uint8)
    a[200000:230000] = a[130000:160000]
    srcs.append(a)
    b = O.generate("text", 4, 400000)
    b[250000:330000] = 7
    srcs.append(b)
    return srcs


def test_ring_decoder_matches_source_and_oracle():
    lz4mi = _lz4mi()
    srcs = _blocks()
    comps = [O.compress_block_bytes(s) for s in srcs]
    _stats(lz4mi)
    st, outs, lens = lz4mi.decompress_blocks(comps, [s.size for s in srcs])
    assert (st == 0).all(), st
    for s, c, o, n in zip(srcs, comps, outs, lens):
        assert n == s.size
        assert np.array_equal(o, s)
        est, ew, eo = O.decompress_block(c, s.size)
        assert est == 0 and ew == s.size and np.array_equal(eo, s)
    stats = _stats(lz4mi)
    print("ring stats (rebuilt chunks, direct sequences, handed back):", stats)
    assert stats[2] == 0      # every valid block stays on the two-pass path


def test_ring_decoder_device_pointers_full_blocks():
    torch = pytest.importorskip("torch")
    lz4mi = _lz4mi()
    n, blk = 48, 4 << 20
    kinds = ["tiles216", "text", "copy", "random", "repetitive", "runs"]
    srcs = [O.generate(kinds[i % len(kinds)], 100 + i, blk) for i in range(n)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    slot = (max(c.size for c in comps) + 255) & ~255
    comp = torch.zeros(n * slot, dtype=torch.uint8)
    for i, c in enumerate(comps):
        comp[i * slot:i * slot + c.size] = torch.from_numpy(c)
    comp = comp.cuda()
    in_off = (torch.arange(n, dtype=torch.int64) * slot).cuda()
    in_len = torch.tensor([c.size for c in comps], dtype=torch.int32).cuda()
    out = torch.zeros(n * blk, dtype=torch.uint8, device="cuda")
    out_off = (torch.arange(n, dtype=torch.int64) * blk).cuda()
    cap = torch.full((n,), blk, dtype=torch.int32, device="cuda")
    out_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    status = torch.full((n,), 77, dtype=torch.int32, device="cuda")
    lz4mi.decompress_blocks_dev(comp.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), out.data_ptr(),
                                out_off.data_ptr(), cap.data_ptr(), out_len.data_ptr(), status.data_ptr(), n)
    torch.cuda.synchronize()
    assert (status.cpu() == 0).all()
    assert (out_len.cpu() == blk).all()
    o = out.cpu().numpy()
    for i, s in enumerate(srcs):
        assert np.array_equal(o[i * blk:(i + 1) * blk], s), (i, kinds[i % len(kinds)])


def test_ring_decoder_hands_back_bad_blocks():
    """Corrupted / truncated / undersized blocks get exactly the single-pass kernel's result."""
    lz4mi = _lz4mi()
    rng = np.random.default_rng(11)
    srcs = [O.generate(g, 40 + i, 70000) for i, g in enumerate(["tiles216", "text", "copy", "runs"] * 3)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    bad, caps = [], []
    for i, c in enumerate(comps):
        c = c.copy()
        if i % 3 == 0:
            c = c[: c.size // 2]                    # truncated
        elif i % 3 == 1:
            pos = rng.integers(0, c.size, 8)
            c[pos] = rng.integers(0, 256, 8, dtype=np.uint8)   # corrupted
        caps.append(srcs[i].size if i % 3 != 2 else srcs[i].size - 100)   # undersized output
        bad.append(c)
    st, outs, lens = lz4mi.decompress_blocks(bad, caps)
    for t, (c, k) in enumerate(zip(bad, caps)):
        est, ew, eo = O.decompress_block(c, k)
        if st[t] == lz4mi.ERR_CROSS_BLOCK:             # batched: reaches before its own block
            assert est == lz4mi.ERR_DICT_OOB, t
            continue
        assert st[t] == est, t
        if est == 0:
            assert lens[t] == ew, t
            assert np.array_equal(outs[t], eo[:min(ew, k)]), t
