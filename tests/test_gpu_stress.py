"""Seeded, bounded versions of the randomized stress tools (tools/small_fuzz.py, tools/enc_fuzz.py;
the long runs are in profiles/r05_edge): every decode path (small batches and the batch kernel,
spec and reference mode) on corrupted encoder output and on random valid streams, statuses and
bytes equal to the oracle's decode; GPU compressed bytes equal to the oracle's compressBlock on
mixed-piece blocks."""
import numpy as np
import pytest

import oracle as O

lz4mi = pytest.importorskip("lz4mi")
pytestmark = pytest.mark.gpu

GENS = ["tiles216", "text", "copy", "runs", "random", "repetitive"]


def _len_field(v):
    r = v - 15
    return [255] * (r // 255) + [r % 255]


def _random_stream(rng, target):
    out, produced = bytearray(), 0
    while True:
        ll = int(rng.choice([0, 0, 1, 14, 15, 16, 200, 269, 270, int(rng.integers(0, 3000))]))
        if produced + ll + 16 > target:
            ll = max(target - produced, 5)
            out += bytes([min(ll, 15) << 4] + (_len_field(ll) if ll >= 15 else [])) + \
                rng.integers(0, 256, ll, dtype=np.uint8).tobytes()
            return np.frombuffer(bytes(out), dtype=np.uint8), produced + ll
        hist = produced + ll
        if hist == 0:
            ll, hist = 8, produced + 8
        off = min(int(rng.choice([1, 3, 8, 17, 64, 65535, int(rng.integers(1, 65536))])), hist)
        ml = min(int(rng.choice([4, 5, 18, 19, 270, int(rng.integers(4, 9000))])), max(4, target - hist - 12))
        mc = ml - 4
        out += bytes([(min(ll, 15) << 4) | min(mc, 15)] + (_len_field(ll) if ll >= 15 else [])) + \
            rng.integers(0, 256, ll, dtype=np.uint8).tobytes() + bytes([off & 255, off >> 8]) + \
            (bytes(_len_field(mc)) if mc >= 15 else b"")
        produced = hist + ml


def _check(comps, caps, js_exact):
    if js_exact:   # reference mode: one block per output array (positions absolute in it)
        res = [lz4mi.decompress_blocks([c], [k], js_exact=True) for c, k in zip(comps, caps)]
        st, outs, lens = [r[0][0] for r in res], [r[1][0] for r in res], [r[2][0] for r in res]
    else:
        st, outs, lens = lz4mi.decompress_blocks(comps, caps)
    for j, c in enumerate(comps):
        est, ew, eo = O.decompress_block(c, caps[j], js_compat=js_exact)
        if st[j] == lz4mi.ERR_CROSS_BLOCK and est == lz4mi.ERR_DICT_OOB:
            continue
        assert st[j] == est, (j, st[j], est)
        if est == 0:
            assert lens[j] == ew and np.array_equal(outs[j], eo[:min(ew, caps[j])]), j


@pytest.mark.parametrize("path", ["small", "batch"])
@pytest.mark.parametrize("source", ["corrupted", "random_streams"])
def test_decode_stress(path, source):
    rng = np.random.default_rng({"small": 1, "batch": 2}[path] * 10 + (source == "random_streams"))
    pool = []
    for t in range(12):
        n = int(rng.choice([100, 5000, 65536, 300000, 1 << 20]))
        if source == "random_streams":
            c, m = _random_stream(rng, n)
            pool.append((c, m))
        else:
            s = O.generate(GENS[t % len(GENS)], 700 + t, n)
            pool.append((O.compress_block_bytes(s), s.size))
    for it in range(3):
        lim = lz4mi.SMALL_BLOCKS
        k = int(rng.integers(1, lim + 1)) if path == "small" else int(rng.integers(lim + 1, lim + 35))
        comps, caps = [], []
        for i in rng.integers(0, len(pool), k):
            c, m = pool[int(i)]
            c = c.copy()
            for _ in range(int(rng.choice([0, 0, 1, 2])) if source == "corrupted" else 0):
                c[rng.integers(0, c.size)] = rng.integers(0, 256)
            comps.append(c)
            caps.append(m + int(rng.choice([0, 0, 7])))
        _check(comps, caps, js_exact=False)
        if path == "small":
            _check(comps[:6], caps[:6], js_exact=True)


def test_encoder_stress():
    rng = np.random.default_rng(99)

    def block(n):
        out, w = np.empty(n + 70000, dtype=np.uint8), 0
        while w < n:
            kind, m = int(rng.integers(0, 4)), int(rng.choice([1, 15, 300, 2048, 9000, 40000]))
            if kind == 0 or w == 0:
                piece = O.generate(GENS[int(rng.integers(0, len(GENS)))], int(rng.integers(1, 1 << 30)), m)
            elif kind == 1:
                d = int(rng.integers(1, min(w, 70000) + 1))
                piece = np.resize(out[w - d:w], m)
            elif kind == 2:
                piece = np.full(m, rng.integers(0, 256), dtype=np.uint8)
            else:
                piece = rng.integers(0, 256, m, dtype=np.uint8)
            out[w:w + m] = piece.astype(np.uint8)
            w += m
        return out[:n].copy()

    for sizes in ([int(x) for x in rng.choice([0, 13, 5000, 65536, 1 << 20, 4 << 20], 12)],
                  [int(x) for x in rng.choice([0, 13, 5000, 65536], 780)]):   # (> 768: global-table kernel)
        srcs = [block(n) for n in sizes]
        comps = lz4mi.compress_blocks(srcs)
        for j, (s, c) in enumerate(zip(srcs, comps)):
            assert np.array_equal(c, O.compress_block_bytes(s)), (j, s.size)



def _seg_geom(in_len):
    """csrc/lz4mi_decompress.h seg_geom: S segments of L compressed bytes (the small path's waves)."""
    s = max(1, min(256, -(-in_len // 8192)))
    L = max(4096, (-(-in_len // s) + 1023) & ~1023)
    return s, L


def _ext(v):
    return 0 if v < 15 else 1 + (v - 15) // 255


def _boundary_stream(rng, comp_len):
    """A valid LZ4 block of exactly comp_len compressed bytes whose sequences straddle the small path's
    segment starts k*L (seg_geom) and warm-up starts k*L - 3072: before each such mark a filler sequence
    puts the next token 0..6 bytes before it, so the mark falls on a token, a literal length byte, a
    literal, an offset byte or a match length byte. Returns (compressed, decoded size, marks placed)."""
    S, L = _seg_geom(comp_len)
    marks = sorted({m for k in range(1, S) for m in (k * L, k * L - 3072) if 64 < m < comp_len - 1200})
    out, produced, placed = bytearray(), 0, 0

    def seq(ll, ml, off):
        mc = ml - 4
        return bytes([(min(ll, 15) << 4) | min(mc, 15)] + (_len_field(ll) if ll >= 15 else [])) + \
            rng.integers(0, 256, ll, dtype=np.uint8).tobytes() + bytes([off & 255, off >> 8]) + \
            (bytes(_len_field(mc)) if mc >= 15 else b"")

    def add(ll, ml):
        nonlocal produced
        off = int(rng.choice([1, 3, 8, 17, int(rng.integers(1, 65536))]))
        out.extend(seq(ll, ml, max(1, min(off, produced + ll, 65535))))
        produced += ll + ml

    add(16, 4)
    for m in marks:
        t = m - int(rng.integers(0, 7))          # the next token's position
        while t - len(out) > 700:                # ordinary sequences up to near the mark
            add(int(rng.choice([0, 1, 3, 15, 40, 200])), int(rng.choice([4, 16, 19, 64, 120, 300, 1000])))
        gap = t - len(out)                       # a filler of exactly `gap` bytes: 3 + ext(ll) + ll (ml < 19)
        ll = next((x for x in range(gap - 3, -1, -1) if x + _ext(x) == gap - 3), None)
        if ll is None:
            continue
        add(ll, int(rng.integers(4, 19)))
        placed += 1
        add(int(rng.choice([0, 15, 300])), int(rng.choice([4, 19, 270, 600])))   # the straddling sequence
    while comp_len - len(out) > 250:
        add(int(rng.choice([0, 3, 40])) if comp_len - len(out) > 300 else 0, int(rng.choice([4, 64, 300])))
    ll = comp_len - len(out) - 2                 # the final literal run: 1 + 1 + ll bytes (15 <= ll <= 269)
    out.extend(bytes([0xF0] + _len_field(ll)) + rng.integers(0, 256, ll, dtype=np.uint8).tobytes())
    assert len(out) == comp_len
    return np.frombuffer(bytes(out), dtype=np.uint8), produced + ll, placed


@pytest.mark.parametrize("force", [0, 1, 2])
def test_small_path_segment_boundaries(force, monkeypatch):
    """random valid streams whose sequences straddle the small path's segment starts
    and 3 KiB warm-up starts (every field of a sequence on the mark, 0..6 bytes of slack), in the three
    re-parse modes (LZ4MI_SMALL_REPARSE 0: the guesses as they come, 1: every guess past segment 0 wrong
    in phase 0, 2: in phases 0 and 2), spec and reference mode, statuses and bytes == the oracle's."""
    monkeypatch.setenv("LZ4MI_SMALL_REPARSE", str(force))
    rng = np.random.default_rng(40 + force)
    comps, caps, placed = [], [], 0
    for n in [20000, 65536, 131071, 300000, 700001]:
        c, m, p = _boundary_stream(rng, n)
        comps.append(c)
        caps.append(m)
        placed += p
    assert placed >= 100
    _check(comps, caps, js_exact=False)
    _check(comps, caps, js_exact=True)


def test_global_table_encoder_on_large_blocks_of_every_generator():
    """The batch encoder above kLdsTableMaxBlocks (768) keeps its tables in global memory, 15-bit entries
    with 2-bit epoch codes in LDS relabelled every 32 KiB (csrc/lz4mi_compress.hip). The bench batch
    covers it with 4 MiB tiles216 blocks and the stress tool with blocks of <= 96 KiB; here 4 MiB blocks
    of every generator (and a copy of far windows, and a block with a period just under 64 KiB, whose matches sit at the window edge across every
    epoch edge) go through it in one batch beside 770 tiny blocks: compressed bytes == the oracle's
    compressBlock, byte for byte, and the round trip decodes."""
    rng = np.random.default_rng(7)
    big = [O.generate(g, 31 + k, 4 << 20) for k, g in enumerate(GENS + ["copy", "text"])]
    far = np.empty(4 << 20, dtype=np.uint8)
    far[:65536] = rng.integers(0, 256, 65536, dtype=np.uint8)
    pos = 65536
    while pos < far.size:
        ln = min(int(rng.integers(8192, 49152)), far.size - pos)
        src = pos - int(rng.integers(ln, 65536))
        far[pos:pos + ln] = far[src:src + ln]
        pos += ln
    per = np.resize(rng.integers(0, 256, 65533, dtype=np.uint8), 4 << 20)
    big += [far, per]
    tiny = [O.generate("text", 900 + k, int(rng.integers(0, 300))) for k in range(770)]
    srcs = big + tiny
    comps = lz4mi.compress_blocks(srcs)
    for j, (s, c) in enumerate(zip(srcs, comps)):
        assert np.array_equal(c, O.compress_block_bytes(s)), (j, s.size)
    st, outs, _ = lz4mi.decompress_blocks(comps[:len(big)], [s.size for s in big])
    assert (st == 0).all() and all(np.array_equal(o, s) for o, s in zip(outs, big))
