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
        k = int(rng.integers(1, 97)) if path == "small" else int(rng.integers(97, 131))
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
