"""Structured fuzz of both kernels against the oracle (GPU, bit-exact).

Encoder: blocks assembled from random segments -- incompressible runs of log-uniform length
(1 B .. 70 KiB: literal runs of every size, across the output ring and the direct-copy
threshold), constant runs, short periods, copies from 1 B .. 64 KiB back and from beyond the
window -- compressed in one batch; every block's bytes == the oracle's compressBlock
(oracle/lz4mi_oracle.c, the reference's LZ4.compressBlock parse) and the GPU decode returns
the source.

Decoder: valid streams the greedy parse never makes (any offset 1..65535 with any overlap,
long length fields, back-to-back zero-literal sequences, the last 5 bytes as literals) built
from random sequences; the GPU decode == the oracle decoder (status, length, bytes).
"""
import numpy as np
import pytest

import oracle as O

lz4mi = pytest.importorskip("lz4mi")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    lz4mi.init(0)


def _segmented_block(rng, n):
    out = np.empty(n, dtype=np.uint8)
    pos = 0
    while pos < n:
        kind = rng.integers(0, 6)
        ln = int(np.exp(rng.uniform(0, np.log(70000))))
        ln = min(max(ln, 1), n - pos)
        if kind == 0 or pos < 16:                       # incompressible
            out[pos:pos + ln] = rng.integers(0, 256, ln, dtype=np.uint8)
        elif kind == 1:                                 # constant run
            out[pos:pos + ln] = rng.integers(0, 256)
        elif kind == 2:                                 # short period
            per = int(rng.integers(1, 300))
            out[pos:pos + ln] = np.resize(rng.integers(0, 256, per, dtype=np.uint8), ln)
        elif kind in (3, 4):                            # copy from within the window (may overlap)
            d = int(rng.integers(1, min(pos, 65535) + 1))
            for k in range(pos, pos + ln, d):           # overlapping copy, d bytes at a time
                m = min(d, pos + ln - k)
                out[k:k + m] = out[k - d:k - d + m]
        else:                                           # copy from beyond the window
            if pos > 70000:
                s = int(rng.integers(0, pos - 66000))
                ln = min(ln, pos - s)
                out[pos:pos + ln] = out[s:s + ln]
            else:
                out[pos:pos + ln] = rng.integers(0, 256, ln, dtype=np.uint8)
        pos += ln
    return out


def test_encoder_segment_fuzz():
    rng = np.random.default_rng(20261018)
    sizes = [int(x) for x in rng.choice([13, 100, 5000, 65536, 200000, 1 << 20, 3 << 20], 40)]
    blocks = [_segmented_block(rng, n) for n in sizes]
    comps = lz4mi.compress_blocks(blocks)
    for k, (b, c) in enumerate(zip(blocks, comps)):
        ref = O.compress_block_bytes(b)
        assert c.size == ref.size and np.array_equal(c, ref), (k, b.size)
    st, outs, lens = lz4mi.decompress_blocks(comps, [b.size for b in blocks])
    for k, (b, o) in enumerate(zip(blocks, outs)):
        assert st[k] == 0 and np.array_equal(o, b), k


def _len_field(v):
    """Extension bytes of an LZ4 length field value v >= 15 (v - 15 as 255s and a remainder)."""
    r = v - 15
    return [255] * (r // 255) + [r % 255]


def _random_stream(rng, target):
    """A valid LZ4 block of about `target` decoded bytes from random sequences."""
    out = bytearray()
    produced = 0
    while True:
        ll = int(rng.choice([0, 0, 0, 1, 3, 14, 15, 16, 300, int(rng.integers(0, 5000))]))
        if produced + ll + 4 + 12 > target:             # the last sequence: literals only (>= 5 end bytes)
            ll = max(target - produced, 5)
            tok = [min(ll, 15) << 4] + (_len_field(ll) if ll >= 15 else [])
            out += bytes(tok) + rng.integers(0, 256, ll, dtype=np.uint8).tobytes()
            return np.frombuffer(bytes(out), dtype=np.uint8), produced + ll
        hist = produced + ll
        off = int(rng.choice([1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 64, 65535, int(rng.integers(1, 65536))]))
        off = min(off, hist) if hist > 0 else 0
        if off == 0:                                    # no history yet: force literals
            ll = max(ll, 8)
            hist = produced + ll
            off = int(rng.integers(1, hist + 1))
        ml = int(rng.choice([4, 5, 18, 19, 20, 270, 300, int(rng.integers(4, 20000))]))
        ml = min(ml, max(4, target - hist - 12))
        mc = ml - 4
        tok = [(min(ll, 15) << 4) | min(mc, 15)]
        if ll >= 15:
            tok += _len_field(ll)
        out += bytes(tok) + rng.integers(0, 256, ll, dtype=np.uint8).tobytes() + bytes([off & 255, off >> 8])
        if mc >= 15:
            out += bytes(_len_field(mc))
        produced = hist + ml


@pytest.mark.parametrize("path", ["small", "batch"])
def test_decoder_random_stream_fuzz(path):
    """Random valid streams (every length-field shape, offsets 1..65535, overlapping copies)
    through the small-batch path (lz4mi.SMALL_BLOCKS blocks) and the batch kernel (8 more: past the
    small path's limit), equal to the oracle's decode."""
    rng = np.random.default_rng(55)
    streams, sizes = [], []
    for t in range(lz4mi.SMALL_BLOCKS if path == "small" else lz4mi.SMALL_BLOCKS + 8):
        target = int(rng.choice([20, 300, 4096, 70000, 500000, 1 << 20]))
        s, n = _random_stream(rng, target)
        streams.append(s)
        sizes.append(n)
    st, outs, lens = lz4mi.decompress_blocks(streams, sizes)
    for t, (s, n) in enumerate(zip(streams, sizes)):
        est, ew, eo = O.decompress_block(s, n)
        assert est == 0 and ew == n, t                   # the generator makes valid streams
        assert st[t] == 0 and lens[t] == n, (t, st[t], lens[t], n)
        assert np.array_equal(outs[t], eo[:n]), t


def test_chain_encoder_segment_fuzz():
    """lz4mi_compress_chain (dependent blocks, carried table) on segmented data == the oracle's
    compressBlock per block with the table carried."""
    rng = np.random.default_rng(7)
    data = _segmented_block(rng, 3 << 20)
    start, length, bs = 5000, data.size - 5000 - 777, 1 << 19
    t_ref = np.zeros(16384, dtype=np.int32)
    t_gpu = t_ref.copy()
    got = lz4mi.compress_chain(data, start, length, bs, t_gpu)
    pos, b = start, 0
    while pos < start + length:
        n = min(bs, start + length - pos)
        w, out, _ = O.compress_block(data, pos, n, t_ref)
        assert np.array_equal(got[b], out[:w]), b
        pos += n
        b += 1
    assert b == len(got)
    assert np.array_equal(t_gpu, t_ref)
