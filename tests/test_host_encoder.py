"""The host-CPU block encoder of the drop-in's routing (lz4mi_host_compress_block /
lz4mi_host_compress_chain, csrc/lz4mi_host.cpp; SURVEY.md §8b "Routing"): product code
written fresh, checked here on CPU against the reference-generated golden vectors —
the same fixtures that pin the oracle — with no GPU and no oracle in the path under test
(the oracle only regenerates seeded inputs)."""
import numpy as np
import pytest

import oracle as O
from conftest import cases_of, golden_bytes

lz4mi = pytest.importorskip("lz4mi")


def _src_of(case):
    if "gen" in case:
        g = case["gen"]
        return O.generate(g["gen"], g["seed"], g["n"])
    return golden_bytes(case["src_file"]).copy()


def _host_block(src):
    out = np.zeros(lz4mi.compress_bound(src.size), dtype=np.uint8)
    t = np.zeros(16384, dtype=np.int32)
    n = lz4mi.host_compress_raw(src, out, 0, src.size, t, 0)
    return out[:n]


def test_host_blocks_match_reference(manifest):
    for c in cases_of(manifest, "block"):
        comp = _host_block(_src_of(c))
        assert comp.size == c["comp_len"], c["name"]
        assert "%08x" % lz4mi.xxh32(comp) == c["comp_xxh"], c["name"]
        if c["comp_file"]:
            assert np.array_equal(comp, golden_bytes(c["comp_file"])), c["name"]


def test_host_chain_with_carried_table(manifest):
    """blockCompress.js with one table carried over three calls into one output buffer."""
    (c,) = cases_of(manifest, "block_chain")
    g = c["gen"]
    src = O.generate(g["gen"], g["seed"], g["n"])
    out = np.zeros(400000, dtype=np.uint8)
    table = np.full(16384, c["table_init"], dtype=np.int32)
    pos = c["out_off0"]
    for i, (start, n, expect) in enumerate(c["segments"]):
        w = lz4mi.host_compress_raw(src, out, start, n, table, pos)
        assert w == expect
        pos += w
        if i == 0:
            assert np.array_equal(table.view(np.uint8), golden_bytes(c["table1_file"]))
    assert np.array_equal(out[:pos], golden_bytes(c["out_file"]))
    assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_final_file"]))


def test_host_raw_edges_rangeerror_and_drops(manifest):
    """Output too small: the reference's RangeError of output.set (bytes and table entries
    written before it kept) and byte stores past the end dropped; F7 (five arguments) = 0."""
    (g,) = cases_of(manifest, "compress_raw_edges")
    for c in g["cases"]:
        src = golden_bytes(c["src_file"]).copy()
        out = np.zeros(c["out_len"], dtype=np.uint8)
        table = np.zeros(16384, dtype=np.int32)
        try:
            v = lz4mi.host_compress_raw(src, out, c["start"], c["len"], table, None if c["five_args"] else c["out_off"])
            assert c["ok"] and v == c["value"], c["name"]
        except lz4mi.Lz4miError as e:
            assert not c["ok"] and e.status == lz4mi.ERR_RANGE and c["error_name"] == "RangeError", c["name"]
        assert np.array_equal(out, golden_bytes(c["out_file"])), c["name"]
        assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_file"])), c["name"]


def test_host_dependent_frames_match_reference(manifest):
    """LZ4.compress's default (dependent blocks, one table carried across the frame) through
    the host chain: every dependent golden frame without a dictionary, byte for byte."""
    (g,) = cases_of(manifest, "frames")
    inputs = {"text": ("text", 5, 300000), "copy": ("copy", 6, 150000), "tiles216": ("tiles216", 8, 1 << 20),
              "random": ("random", 9, 70000)}
    from lz4mi import frame as F, shard
    done = 0
    for f in g["frames"]:
        if f["indep"] or "dict" in f or "dict_text" in f or f["input"] not in inputs:
            continue
        data = O.generate(*inputs[f["input"]])[: f["n"]]
        table = np.zeros(16384, dtype=np.int32)
        blocks = lz4mi.compress_chain(data, 0, data.size, f["block"], table, host=True)
        raws = [data[p:p + f["block"]] for p in range(0, data.size, f["block"])]
        body = shard.block_records(raws, blocks)
        add = f.get("add_size", True)
        hdr = F.header(f["block"], False, f["checksum"], data.size if add else None)
        frame = np.concatenate([np.frombuffer(hdr, dtype=np.uint8), body, np.zeros(4, dtype=np.uint8)] +
                               ([np.array([lz4mi.xxh32(data)], dtype="<u4").view(np.uint8)] if f["checksum"] else []))
        assert frame.size == f["frame_len"], f
        assert "%08x" % lz4mi.xxh32(frame) == f["frame_xxh"], f
        done += 1
    assert done >= 8


@pytest.mark.parametrize("kind", ["random", "repetitive", "tiles216"])
def test_host_digest_manifest_4mib(manifest, kind):
    (g,) = cases_of(manifest, "digest_4mib")
    for r in [r for r in g["rows"] if r["gen"] == kind][:4]:
        comp = _host_block(O.generate(kind, r["seed"], r["n"]))
        assert comp.size == r["comp_len"] and "%08x" % lz4mi.xxh32(comp) == r["comp_xxh"], r


# ---- the host decoder of the same routing (lz4mi_host_decompress_block) ----------------

MESSAGES = {-1: "LZ4: Output Buffer Too Small", -2: "LZ4: Malformed Input", -3: "LZ4: Invalid Offset 0",
            -4: "LZ4: Dictionary Offset Out of Bounds"}


def test_host_decoder_reference_blocks(manifest):
    """Every golden block decoded with the reference's semantics: its written count and its
    bytes (the reference decoder's own output, F1 corruption included), and in spec mode the
    input back."""
    for c in cases_of(manifest, "block"):
        src = _src_of(c)
        comp = golden_bytes(c["comp_file"]) if c["comp_file"] else _host_block(src)
        out = np.zeros(src.size, dtype=np.uint8)
        w = lz4mi.host_decompress_raw(comp, 0, comp.size, out, 0)
        assert w == c["js_dec_written"], c["name"]
        if c["js_dec_equals_input"]:
            assert np.array_equal(out, src), c["name"]
        else:
            assert "%08x" % lz4mi.xxh32(out) == c["js_dec_xxh"], c["name"]
        spec = np.zeros(src.size, dtype=np.uint8)
        assert lz4mi.host_decompress_raw(comp, 0, comp.size, spec, 0, spec=True) == src.size
        assert np.array_equal(spec, src), c["name"]


def test_host_decoder_edge_and_error_cases(manifest):
    """The reference decoder's own results on the edge / corruption vectors: bytes, counts,
    dictionary reads, and the four error messages in its check order."""
    (g,) = cases_of(manifest, "decode_cases")
    for c in g["cases"]:
        comp = np.array(c["comp"], dtype=np.uint8)
        dic = None if c["dict"] is None else np.array(c["dict"], dtype=np.uint8)
        out = np.zeros(c["out_len"], dtype=np.uint8)
        try:
            w = lz4mi.host_decompress_raw(comp, 0, comp.size, out, c["out_off"], dictionary=dic)
            assert c["ok"] and w == c["written"] and out.tolist() == c["out"], c["name"]
        except lz4mi.Lz4miError as e:
            assert not c["ok"] and MESSAGES.get(e.status) == c["error"], (c["name"], e.status)


def test_host_decoder_dependent_frames(manifest):
    """The golden dependent-block frames (one table carried, blocks reading earlier blocks'
    output) decoded block by block in order by the host decoder into one result buffer, as
    bufferDecompress.js does with a content size: the reference's decoded bytes."""
    (g,) = cases_of(manifest, "frames")
    from lz4mi import shard
    done = 0
    for f in g["frames"]:
        if f["indep"] or not f.get("frame_file") or "dict" in f or "dict_text" in f or not f.get("dec_ok"):
            continue
        fr = golden_bytes(f["frame_file"])
        info, blocks = shard.frame_blocks(fr)
        if info["content_size"] <= 0:
            continue
        out = np.zeros(info["content_size"], dtype=np.uint8)
        pos = 0
        for p, n, stored in blocks:
            if stored:
                out[pos:pos + n] = fr[p:p + n]
                pos += n
            else:
                pos += lz4mi.host_decompress_raw(fr, p, n, out, pos)
        assert pos == f["dec_len"] and "%08x" % lz4mi.xxh32(out[:pos]) == f["dec_xxh"], f
        done += 1
    assert done >= 4


@pytest.mark.parametrize("gen", ["copy", "runs", "text", "tiles216", "random", "repetitive"])
def test_host_decoder_matches_oracle_fuzz(gen):
    """Differential check of the host decoder against the oracle's decoders (reference-exact and
    spec) on seeded blocks, output offsets with bytes already in place (no stray writes), output
    buffers shorter than the block (writes past the end vanish, or the reference's errors), and
    byte-flipped inputs (statuses and every output byte, partial writes included)."""
    rng = np.random.default_rng({"copy": 1, "runs": 2, "text": 3, "tiles216": 4, "random": 5, "repetitive": 6}[gen])
    for seed in range(4):
        n = int(rng.integers(1000, 120000))
        src = O.generate(gen, 100 + seed, n)
        comp = _host_block(src)
        cases = [(comp, n, 0), (comp, n, int(rng.integers(1, 40))), (comp, max(1, n - int(rng.integers(1, 64))), 0)]
        for _ in range(3):
            bad = comp.copy()
            for _ in range(int(rng.integers(1, 4))):
                bad[int(rng.integers(0, bad.size))] ^= np.uint8(1 << int(rng.integers(0, 8)))
            cases.append((bad, n, int(rng.integers(0, 8))))
        for blk, cap, off in cases:
            for spec in (False, True):
                base = rng.integers(0, 256, off + cap, dtype=np.uint8)
                want_out = base.copy()
                st, w, _ = O.decompress_block(blk, cap, out=want_out, out_off=off, js_compat=not spec)
                got_out = base.copy()
                try:
                    got = lz4mi.host_decompress_raw(blk, 0, blk.size, got_out, off, spec=spec)
                    got_st = 0
                except lz4mi.Lz4miError as e:
                    got, got_st = None, e.status
                assert got_st == st, (gen, seed, spec, got_st, st)
                if st == 0:
                    assert got == w, (gen, seed, spec)
                assert np.array_equal(got_out, want_out), (gen, seed, spec, off, cap)


@pytest.mark.parametrize("gen", ["copy", "text", "tiles216", "random"])
def test_host_encoder_matches_oracle_fuzz(gen):
    """Differential check of the host encoder against the oracle's compressBlock restatement:
    seeded sources, a start inside the source, a carried table, an output offset, outputs sized
    to the bound and too small (the RangeError path and dropped stores): return value, every
    output byte and the table after the call."""
    rng = np.random.default_rng({"copy": 11, "text": 12, "tiles216": 13, "random": 14}[gen])
    for seed in range(4):
        n = int(rng.integers(2000, 150000))
        src = O.generate(gen, 200 + seed, n)
        start = int(rng.integers(0, 64))
        length = n - start - int(rng.integers(0, 64))
        table0 = np.zeros(16384, dtype=np.int32)
        if seed & 1:   # a carried table: positions of an earlier call on the same source
            O.compress_raw(src, np.zeros(O.compress_bound(start + 1) + 64, dtype=np.uint8), 0, max(start, 1), table0, 0)
        for cap in (O.compress_bound(length) + 32, length // 3):
            off = int(rng.integers(0, 16))
            want_out = rng.integers(0, 256, cap, dtype=np.uint8)
            got_out = want_out.copy()
            want_t, got_t = table0.copy(), table0.copy()
            want_st, want_n = O.compress_raw(src, want_out, start, length, want_t, off)   # -8: RangeError
            try:
                got_n, got_st = lz4mi.host_compress_raw(src, got_out, start, length, got_t, off), 0
            except lz4mi.Lz4miError as e:
                got_n, got_st = None, e.status
            assert got_st == want_st, (gen, seed, cap, got_st, want_st)
            if want_st == 0:
                assert got_n == want_n, (gen, seed, cap)
            assert np.array_equal(got_out, want_out), (gen, seed, cap)
            assert np.array_equal(got_t, want_t), (gen, seed, cap)


@pytest.mark.parametrize("thp", ["1", "0"])
def test_host_decoder_large_fresh_output(thp, monkeypatch):
    """A block decoded into a fresh (never written) output mapping larger than 4 MiB at an
    unaligned offset: the library advises the range's 2 MiB-aligned interior for huge pages
    (lz4mi_advise_output; LZ4MI_THP=0 skips it). Bytes in the output before the offset and past
    the block stay as they were; the block equals the oracle's decode."""
    import mmap
    monkeypatch.setenv("LZ4MI_THP", thp)
    src = O.generate("tiles216", 77, 9 << 20)
    comp = O.compress_block_bytes(src)
    m = mmap.mmap(-1, (12 << 20) + 4096)
    out = np.frombuffer(m, dtype=np.uint8)
    off = 4096 + 123
    out[:off] = 0xA5
    w = lz4mi.host_decompress_raw(comp, 0, comp.size, out, off, spec=True)
    assert w == src.size and np.array_equal(out[off:off + w], src)
    assert (out[:off] == 0xA5).all() and (out[off + w:] == 0).all()
    del out
    m.close()
