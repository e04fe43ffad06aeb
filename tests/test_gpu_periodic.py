"""Periodic matches (match offset < match length) through every place the
single-pass decoder writes them: lane-sized runs, whole-wave runs in round 1
(the pattern buffer is the pending list), in rounds 2+ (the staged-literal
buffer) and in the cut path (a length varint too long for the parse window:
all of LDS, or all but the sequence tables with the F1 check on), for periods
either side of each buffer's limit and periods done in several slices. Blocks are hand-assembled from
sequence lists so the paths are hit on purpose, plus oracle-compressed data of
the same shape; every block is checked bit-exact against the CPU oracle
(spec and reference/JS-compat decode) and against the byte-level expectation.

Sequence layout per the LZ4 block format (the reference's decoder,
src/block/blockDecompress.js:30, reads the same fields).
"""
import numpy as np
import pytest

import oracle as O


def _varint(n):
    out = []
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)
    return out


def encode_block(seqs, final_lits):
    """seqs: [(literals bytes, offset, match length)], then the literal-only tail."""
    out = []
    for lits, off, ml in seqs:
        assert ml >= 4 and 1 <= off <= 65535
        ll = len(lits)
        out.append((min(ll, 15) << 4) | min(ml - 4, 15))
        if ll >= 15:
            out += _varint(ll - 15)
        out += list(lits)
        out += [off & 255, off >> 8]
        if ml - 4 >= 15:
            out += _varint(ml - 4 - 15)
    ll = len(final_lits)
    out.append(min(ll, 15) << 4)
    if ll >= 15:
        out += _varint(ll - 15)
    out += list(final_lits)
    return np.array(out, dtype=np.uint8)


def expected_output(seqs, final_lits):
    out = bytearray()
    for lits, off, ml in seqs:
        out += lits
        s = len(out) - off
        assert s >= 0
        for j in range(ml):                      # byte by byte: overlap repeats the period
            out.append(out[s + j])
    out += final_lits
    return np.frombuffer(bytes(out), dtype=np.uint8)


def crafted_blocks():
    rng = np.random.default_rng(2024)
    rb = lambda n: bytes(rng.integers(0, 256, n, dtype=np.uint8))
    blocks = []
    # cut path: one literal run of `per` bytes, then a match too long for the parse window
    for per in (1, 5, 15, 16, 17, 251, 1000, 3000, 3507, 3508, 3509, 3600, 8000, 10151, 10152, 10153, 40000, 65535):
        for ml in (70000, 200001, 600007):
            blocks.append(([(rb(per), per, ml)], rb(20)))
    # round 1: long literals first so the periodic match opens a later table; its
    # source ends before that table
    for per in (3, 16, 100, 1331, 1332, 1333, 2000):
        for ml in (1025, 1100, 5000, 40000):
            blocks.append(([(rb(3000), per, ml), (rb(7), 9, 30)], rb(16)))
    # rounds 2+: the periodic match reads output of a match in the same table,
    # followed by > 64 short self-overlapping matches (pending in round 2 too)
    for per in (7, 20, 50, 64, 120, 1000, 1068, 1069, 1100):
        for ml in (1025, 3000, 20000):
            seqs = [(rb(150), 150, 1200), (b"", per, ml)]
            seqs += [(rb(2), 3, 10) for _ in range(100)]
            seqs += [(rb(1), per % 700 + 1, 2000)]
            blocks.append((seqs, rb(13)))
    return [(encode_block(s, f), expected_output(s, f)) for s, f in blocks]


def natural_blocks():
    """Oracle-compressed data: random headers, then a pattern repeated."""
    rng = np.random.default_rng(7)
    srcs = []
    for per in (2, 16, 17, 63, 251, 1024, 2500, 3300, 3600, 9000):
        parts = []
        total = 0
        while total < (1 << 20):
            parts.append(rng.integers(0, 256, int(rng.integers(20, 400)), dtype=np.uint8))
            pat = rng.integers(0, 256, per, dtype=np.uint8)
            parts.append(np.tile(pat, int(rng.integers(2, 200000 // per + 3))))
            total += parts[-2].size + parts[-1].size
        srcs.append(np.concatenate(parts)[: 1 << 20])
    return [(O.compress_block_bytes(s), s) for s in srcs]


def test_crafted_blocks_decode_on_oracle():
    """CPU: the hand-assembled blocks are valid and decode to the byte-level expectation."""
    for comp, exp in crafted_blocks():
        for js in (False, True):
            st, n, out = O.decompress_block(comp, exp.size, js_compat=js)
            assert st == 0 and n == exp.size
            if not js:
                assert np.array_equal(out, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["crafted", "natural"])
def test_periodic_runs_single_pass(source):
    lz4mi = pytest.importorskip("lz4mi")
    lz4mi.init(0)
    cases = crafted_blocks() if source == "crafted" else natural_blocks()
    comps = [c for c, _ in cases]
    exps = [e for _, e in cases]
    st, outs, lens = lz4mi.decompress_blocks(comps, [e.size for e in exps])
    for i, (k, o, n, e) in enumerate(zip(st, outs, lens, exps)):
        assert k == 0 and n == e.size, i
        assert np.array_equal(o, e), i
    for i, (c, e) in enumerate(zip(comps, exps)):   # reference decode (serial and in-kernel F1), one block per array
        ref = O.decompress_block(c, e.size, js_compat=True)
        for mode in ({"js_compat": True}, {"js_exact": True}):
            st1, outs1, _ = lz4mi.decompress_blocks([c], [e.size], **mode)
            assert st1[0] == ref[0] and np.array_equal(outs1[0], ref[2]), (i, mode)


def json_blocks():
    """The reference benchmark's data shape (tools/json_data.mjs: one JSON record repeated):
    short F1-eligible matches inside the first record, then one periodic match running to
    the block end as the chunk's cut sequence — the F1 replay and the long match in one chunk."""
    import json
    rec = json.dumps({"seq": 42, "kind": "sample_record", "labels": ["alpha", "beta", "gamma", "delta", "epsilon"],
                      "stats": {"ok": True, "values": [12, 240, 3600, 48000, 510000]},
                      "note": "One small record, repeated until the buffer is full, compresses very well."},
                     separators=(",", ":"))
    out = []
    for n in (1 << 16, 1 << 20, 4 << 20):
        raw = np.frombuffer((rec * (n // len(rec) + 1)).encode()[:n], dtype=np.uint8)
        out.append((O.compress_block_bytes(raw), raw))
    return out


@pytest.mark.gpu
def test_json_repeat_reference_mode_matches_reference_decoder():
    lz4mi = pytest.importorskip("lz4mi")
    lz4mi.init(0)
    cases = json_blocks()
    comps = [c for c, _ in cases]
    sizes = [r.size for _, r in cases]
    refs = [O.decompress_block(c, n, js_compat=True) for c, n in zip(comps, sizes)]
    assert any(not np.array_equal(r[2], raw) for r, (_, raw) in zip(refs, cases))   # the reference corrupts it (F1)
    st, outs, _ = lz4mi.decompress_blocks(comps, sizes, js_exact=True)          # batched, in-kernel replay
    for k, o, r in zip(st, outs, refs):
        assert k == r[0] and np.array_equal(o, r[2])
    for c, n, r in zip(comps, sizes, refs):                                     # one block per call
        st1, outs1, _ = lz4mi.decompress_blocks([c], [n], js_exact=True)
        assert st1[0] == r[0] and np.array_equal(outs1[0], r[2])
    st, outs, _ = lz4mi.decompress_blocks(comps, sizes)                          # spec
    for k, o, (_, raw) in zip(st, outs, cases):
        assert k == 0 and np.array_equal(o, raw)

