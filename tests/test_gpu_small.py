"""Small-batch decode (<= LZ4MI_SMALL_BLOCKS blocks, spec mode): the batch kernel parses and
exports the sequence tables, the output is computed by pointer jumping over the whole GPU
(csrc/lz4mi_expand.hip). Bit-exact against the oracle decoder (oracle/lz4_oracle.c, the
reference's decompressBlock, blockDecompress.js:55-272): bytes, lengths and statuses, on every
generator (incl. long offset-1 runs, far copies), history before the output offset and
dictionaries, corrupted streams, and a batch mixing exported blocks with one past the export
limit (decoded by the same launch as usual)."""
import os

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

lz4mi = pytest.importorskip("lz4mi")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    lz4mi.init(0)


def _far(rng, n):
    b = np.empty(n, dtype=np.uint8)
    b[:65536] = rng.integers(0, 256, 65536, dtype=np.uint8)
    pos = 65536
    while pos < n:
        ln = min(int(rng.integers(8192, 49152)), n - pos)
        src = pos - int(rng.integers(ln, 65536))
        b[pos:pos + ln] = b[src:src + ln]
        pos += ln
    return b


def _blocks(rng):
    out = []
    for kind in ("tiles216", "random", "repetitive", "text", "copy", "runs"):
        out.append(O.generate(kind, int(rng.integers(1, 1000)), int(rng.choice([1 << 20, 4 << 20, 777777]))))
    out.append(np.zeros(4 << 20, dtype=np.uint8))                                  # one offset-1 run
    out.append(np.resize(rng.integers(0, 256, 3, dtype=np.uint8), 3 << 20))       # period 3
    out.append(_far(rng, 2 << 20))
    # long periodic runs (periods 1..300, one overlapping match each) between random runs: a low
    # ratio, so the block takes the pointer path and its runs the period remap (ratio >= 32 blocks,
    # like the two above, are decoded by one wave)
    parts = []
    for k in range(24):
        parts.append(rng.integers(0, 256, 65536, dtype=np.uint8))
        per = int(rng.integers(1, 301))
        parts.append(np.resize(rng.integers(0, 256, per, dtype=np.uint8), 65536 + int(rng.integers(0, 999))))
    out.append(np.concatenate(parts))
    out.append(O.generate("tiles216", 5, 100))
    out.append(np.zeros(0, dtype=np.uint8))
    out.append(O.generate("text", 9, 13))
    return out


def test_small_batches_match_oracle():
    rng = np.random.default_rng(314)
    srcs = _blocks(rng)
    comps = [O.compress_block_bytes(s) for s in srcs]
    for k in (1, 2, 5, len(srcs)):                       # batches of k blocks
        for start in range(0, len(srcs), k):
            sel = list(range(start, min(start + k, len(srcs))))
            st, outs, lens = lz4mi.decompress_blocks([comps[i] for i in sel], [srcs[i].size for i in sel])
            for j, i in enumerate(sel):
                est, ew, eo = O.decompress_block(comps[i], srcs[i].size)
                assert st[j] == est and lens[j] == ew, (k, i, st[j], est)
                assert np.array_equal(outs[j], srcs[i]), (k, i)


def test_small_batch_device_api_one_to_sixteen():
    torch = pytest.importorskip("torch")
    bs, n = 4 << 20, 16
    s = torch.cuda.current_stream().cuda_stream
    raw = torch.empty(n * bs, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 3, bs, n, s)
    slot = (lz4mi.compress_bound(bs) + 255) & ~255
    comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
    roff = torch.arange(n, dtype=torch.int64, device="cuda") * bs
    rlen = torch.full((n,), bs, dtype=torch.int32, device="cuda")
    coff = torch.arange(n, dtype=torch.int64, device="cuda") * slot
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(), coff.data_ptr(),
                              clen.data_ptr(), n, s)
    for k in (1, 3, 16):
        dec = torch.zeros(n * bs, dtype=torch.uint8, device="cuda")
        dlen = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
        lz4mi.decompress_blocks_dev(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(), roff.data_ptr(),
                                    rlen.data_ptr(), dlen.data_ptr(), st.data_ptr(), k, s)
        torch.cuda.synchronize()
        assert bool((st[:k] == 0).all()) and bool((dlen[:k] == bs).all()), k
        assert torch.equal(dec[:k * bs], raw[:k * bs]), k
        assert not bool(dec[k * bs:].any()), k                       # nothing written past the batch


def test_small_batch_history_and_dictionary():
    """A block whose matches reach bytes before its output offset (dependent blocks) or into
    a dictionary: the pointers into history resolve to the caller's bytes / the dictionary."""
    data = np.concatenate([O.generate("text", 3, 200000), O.generate("tiles216", 4, 300000)])
    table = np.zeros(16384, dtype=np.int32)
    cut = 150000
    O.compress_block(data, 0, cut, table)
    w, out, _ = O.compress_block(data, cut, data.size - cut, table)
    blk = out[:w].copy()
    # history: the output array already holds the first block
    outp = np.zeros(data.size, dtype=np.uint8)
    outp[:cut] = data[:cut]
    got = lz4mi.decompress_raw(blk, 0, blk.size, outp, cut)
    assert got == data.size - cut and np.array_equal(outp, data)
    # dictionary: the same block against a dictionary holding the history, output at 0
    d = data[cut - 65536:cut].copy()
    table = np.zeros(16384, dtype=np.int32)
    src = np.concatenate([d, data[cut:]])
    O.compress_block(src, 0, d.size, table)
    w, out, _ = O.compress_block(src, d.size, src.size - d.size, table)
    blk = out[:w].copy()
    outp = np.zeros(src.size - d.size, dtype=np.uint8)
    got = lz4mi.decompress_raw(blk, 0, blk.size, outp, 0, dictionary=d)
    est, ew, eo = O.decompress_block(blk, outp.size, dictionary=d)
    assert est == 0 and got == ew and np.array_equal(outp, eo[:ew]) and np.array_equal(outp, data[cut:])


def test_small_batch_corrupted_streams_match_oracle():
    rng = np.random.default_rng(99)
    srcs = [O.generate(k, 50 + t, int(rng.choice([5000, 65536, 300000])))
            for t, k in enumerate(["tiles216", "text", "copy", "runs", "random", "repetitive"] * 2)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    for t in range(40):
        sel = [int(x) for x in rng.choice(len(srcs), size=int(rng.integers(1, 9)), replace=False)]
        bad, caps = [], []
        for i in sel:
            c = comps[i].copy()
            for _ in range(int(rng.integers(1, 4))):
                c[rng.integers(0, c.size)] = rng.integers(0, 256)
            bad.append(c)
            caps.append(srcs[i].size + int(rng.integers(-3, 8)))
        st, outs, lens = lz4mi.decompress_blocks(bad, caps)
        for j, c in enumerate(bad):
            est, ew, eo = O.decompress_block(c, caps[j])
            if st[j] == lz4mi.ERR_CROSS_BLOCK:      # batched: reaches before its own block
                assert len(sel) > 1 and est == lz4mi.ERR_DICT_OOB, (t, j)
                continue
            assert st[j] == est, (t, j, st[j], est)
            if est == 0:
                assert lens[j] == ew and np.array_equal(outs[j], eo[:min(ew, caps[j])]), (t, j)


def test_small_batch_mixed_with_unexported_block():
    """A block past the export limit (output capacity above 4 MiB) in the same small batch is
    decoded by the batch kernel as usual, the others by the pointer pipeline."""
    srcs = [O.generate("tiles216", 21, 1 << 20), O.generate("text", 22, (4 << 20) + 1000),
            O.generate("copy", 23, 500000)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    st, outs, lens = lz4mi.decompress_blocks(comps, [s.size for s in srcs])
    for j, s in enumerate(srcs):
        assert st[j] == 0 and lens[j] == s.size and np.array_equal(outs[j], s), j


def _straddle_block(rng, n):
    """Compressible data interleaved with random runs of 2-9 KiB: in the compressed block these
    are long literal runs, so a segment's warm-up parse often starts inside one and guesses a
    wrong entry (phase 1 re-parses it)."""
    parts, size = [], 0
    while size < n:
        if rng.random() < 0.5:
            p = rng.integers(0, 256, int(rng.integers(2048, 9216)), dtype=np.uint8)
        else:
            p = O.generate("tiles216", int(rng.integers(1, 10 ** 6)), int(rng.integers(4096, 40000)))
        parts.append(p)
        size += p.size
    return np.concatenate(parts)[:n]


@pytest.mark.parametrize("force", [0, 1, 2])
def test_small_batch_segment_reparse(force, monkeypatch):
    """Segments whose speculative entry is wrong are re-parsed from the previous segment's exit:
    natural mis-guesses (literal runs across segment starts, text) and, with the test hook
    LZ4MI_SMALL_REPARSE, every first guess past segment 0 wrong (1: phase 2 re-parses them all at
    once) or every guess (2: phase 1 re-parses them in order); errors inside a re-parsed segment
    keep the reference's first-error order."""
    if force:
        monkeypatch.setenv("LZ4MI_SMALL_REPARSE", str(force))
    rng = np.random.default_rng(2718)
    srcs = [_straddle_block(rng, int(n)) for n in (4 << 20, 3 << 20, 1 << 20, 777777)]
    srcs += [O.generate(k, 31, 2 << 20) for k in ("text", "copy", "repetitive", "random")]
    comps = [O.compress_block_bytes(s) for s in srcs]
    st, outs, lens = lz4mi.decompress_blocks(comps, [s.size for s in srcs])
    for j, s in enumerate(srcs):
        assert st[j] == 0 and lens[j] == s.size and np.array_equal(outs[j], s), (force, j)
    bad, caps = [], []
    for j, c in enumerate(comps):   # one corruption late in each block
        c = c.copy()
        c[int(c.size * 0.8) + j] ^= 0x5A
        bad.append(c)
        caps.append(srcs[j].size)
    st, outs, lens = lz4mi.decompress_blocks(bad, caps)
    for j, c in enumerate(bad):
        est, ew, eo = O.decompress_block(c, caps[j])
        if st[j] == lz4mi.ERR_CROSS_BLOCK:
            assert est == lz4mi.ERR_DICT_OOB, (force, j)
            continue
        assert st[j] == est, (force, j, st[j], est)
        if est == 0:
            assert lens[j] == ew and np.array_equal(outs[j], eo[:min(ew, caps[j])]), (force, j)


def test_small_batch_reference_mode_matches_reference_decoder():
    """Reference mode (LZ4MI_JS_EXACT) through the small path: blocks whose output a
    double-copy-tail rewrite changes are decoded again by the batch kernel's fix-up,
    a block past the export limit is decoded in reference mode by the same launch; every result
    equals the reference-exact oracle decode (oracle js_compat), alone and batched."""
    srcs = [O.generate("copy", 61, 1 << 20), O.generate("tiles216", 62, 1 << 20),
            O.generate("copy", 63, (4 << 20) + 4096), O.generate("runs", 64, 700000), O.generate("text", 65, 300000)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    for sel in ([0], [1], [2], [0, 1, 2, 3, 4]):
        st, outs, lens = lz4mi.decompress_blocks([comps[i] for i in sel], [srcs[i].size for i in sel], js_exact=True)
        for j, i in enumerate(sel):
            est, ew, eo = O.decompress_block(comps[i], srcs[i].size, js_compat=True)
            if st[j] == lz4mi.ERR_CROSS_BLOCK:     # batched: the rewrite reaches before the block
                assert len(sel) > 1, (sel, i)
                continue
            assert st[j] == est and lens[j] == ew, (sel, i, st[j], est)
            if est == 0:
                assert np.array_equal(outs[j], eo[:ew]), (sel, i)


def test_small_batch_scratch_allocation_failure():
    """when the small path's scratch cannot be allocated (here a real hipMalloc failure: the
    test hook LZ4MI_TEST_SCRATCH_EXTRA_MB asks for a petabyte more), the call falls back to the batch
    kernel and returns LZ4MI_OK with the right bytes (the failed allocation's error is not the call's);
    with LZ4MI_SMALL_SCRATCH_MB=0 (the cap) the batch kernel runs too. Each in a fresh process: the cap
    is read once per process."""
    import subprocess
    import sys
    code = r"""
import os, sys
sys.path[:0] = [os.path.join(%r, "oracle"), os.path.join(%r, "divortio-lz4_amd")]
import numpy as np, oracle as O, lz4mi
lz4mi.init(0)
srcs = [O.generate(k, 60 + i, n) for i, (k, n) in enumerate([("tiles216", 1 << 20), ("text", 300000), ("random", 70000)])]
comps = [O.compress_block_bytes(x) for x in srcs]
for rep in range(2):
    st, outs, lens = lz4mi.decompress_blocks(comps, [x.size for x in srcs])
    assert (st == 0).all() and all(np.array_equal(o, x) for o, x in zip(outs, srcs))
    for c, x in zip(comps, srcs):      # reference mode, one block per output array
        st, outs, lens = lz4mi.decompress_blocks([c], [x.size], js_exact=True)
        est, ew, eo = O.decompress_block(c, x.size, js_compat=True)
        assert st[0] == est == 0 and lens[0] == ew and np.array_equal(outs[0], eo[:x.size])
print("ok")
""" % (ROOT, ROOT)
    for env in ({"LZ4MI_TEST_SCRATCH_EXTRA_MB": str(1 << 30)}, {"LZ4MI_SMALL_SCRATCH_MB": "0"}):
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (env, r.stdout[-500:], r.stderr[-1500:])
