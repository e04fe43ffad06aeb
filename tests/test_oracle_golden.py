"""Pins the CPU oracle (oracle/lz4_oracle.c) to the reference's own outputs.

Every fixture under tests/golden/ was produced by executing the reference
JavaScript (tools/golden/gen_golden.mjs); the oracle must reproduce each one
bit-for-bit. Runs on CPU only.
"""
import numpy as np
import pytest

import oracle as O
from conftest import cases_of, golden_bytes

MESSAGES = {
    -1: "LZ4: Output Buffer Too Small",
    -2: "LZ4: Malformed Input",
    -3: "LZ4: Invalid Offset 0",
    -4: "LZ4: Dictionary Offset Out of Bounds",
    -5: "LZ4: Invalid Magic Number",
    -7: "LZ4: Content Checksum Error",
}


def _src_of(case):
    if "gen" in case:
        g = case["gen"]
        return O.generate(g["gen"], g["seed"], g["n"])
    return golden_bytes(case["src_file"]).copy()


def test_xxh32_known_answers(manifest):
    (c,) = cases_of(manifest, "xxh32")
    base = O.generate(c["input"]["gen"], c["input"]["seed"], c["input"]["n"])
    for n, h0, h1 in c["rows"]:
        assert "%08x" % O.xxh32(base[:n], 0) == h0, n
        assert "%08x" % O.xxh32(base[:n], 12345) == h1, n
    for text, h in c["text"]:
        assert "%08x" % O.xxh32(text.encode()) == h
    assert O.xxh32(b"") == 0x02CC5D05 and O.xxh32(b"Hello World") == 0xB1FD16EE
    assert "%08x" % O.xxh32(base[:1000]) == c["stateful_1000"]


def test_block_compress_matches_reference(manifest):
    cases = cases_of(manifest, "block")
    assert len(cases) > 30
    for c in cases:
        src = _src_of(c)
        assert "%08x" % O.xxh32(src) == c["src_xxh"], c["name"]      # generator parity with the JS one
        comp = O.compress_block_bytes(src)
        assert comp.size == c["comp_len"], c["name"]
        assert "%08x" % O.xxh32(comp) == c["comp_xxh"], c["name"]
        if c["comp_file"]:
            assert np.array_equal(comp, golden_bytes(c["comp_file"])), c["name"]


def test_block_decompress_spec_and_jscompat(manifest):
    for c in cases_of(manifest, "block"):
        src = _src_of(c)
        comp = O.compress_block_bytes(src)
        st, w, out = O.decompress_block(comp, src.size)
        assert st == 0 and w == src.size and np.array_equal(out, src), c["name"]   # spec round trip
        st, w, js = O.decompress_block(comp, src.size, js_compat=True)
        assert st == 0 and w == c["js_dec_written"], c["name"]
        if c["js_dec_equals_input"]:
            assert np.array_equal(js, src), c["name"]
        else:                                                                          # SURVEY F1 divergence
            assert "%08x" % O.xxh32(js) == c["js_dec_xxh"], c["name"]
            if c.get("js_dec_file"):
                assert np.array_equal(js, golden_bytes(c["js_dec_file"])), c["name"]


def test_block_chain_with_carried_table(manifest):
    (c,) = cases_of(manifest, "block_chain")
    g = c["gen"]
    src = O.generate(g["gen"], g["seed"], g["n"])
    out = np.zeros(400000, dtype=np.uint8)
    table = np.full(16384, c["table_init"], dtype=np.int32)
    pos = c["out_off0"]
    for i, (start, n, expect) in enumerate(c["segments"]):
        w, out, table = O.compress_block(src, start, n, table, out, pos)
        assert w == expect
        pos += w
        if i == 0:
            assert np.array_equal(table.view(np.uint8), golden_bytes(c["table1_file"]))
    assert np.array_equal(out[:pos], golden_bytes(c["out_file"]))
    assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_final_file"]))


def test_decode_edge_cases(manifest):
    (g,) = cases_of(manifest, "decode_cases")
    for c in g["cases"]:
        comp = np.array(c["comp"], dtype=np.uint8)
        dic = None if c["dict"] is None else np.array(c["dict"], dtype=np.uint8)
        out = np.zeros(c["out_len"], dtype=np.uint8)
        st, w, out = O.decompress_block(comp, 0, out=out, out_off=c["out_off"], dictionary=dic, js_compat=True)
        if c["ok"]:
            assert st == 0, c["name"]
            assert w == c["written"], c["name"]
            assert out.tolist() == c["out"], c["name"]
        else:
            assert MESSAGES.get(st) == c["error"], (c["name"], st, c["error"])


def test_frames_compress(manifest):
    (g,) = cases_of(manifest, "frames")
    inputs = {"text": ("text", 5, 300000), "copy": ("copy", 6, 150000), "tiles216": ("tiles216", 8, 1 << 20),
              "random": ("random", 9, 70000)}
    for f in g["frames"]:
        name = f["input"]
        if name in inputs:
            data = O.generate(*inputs[name])[: f["n"]]
        elif name == "hello":
            data = b"Hello World"
        elif name == "A10000":
            data = b"A" * 10000
        elif name == "empty":
            data = b""
        elif name == "dictmsg":
            data = f["input_text"].encode()
        dic = None
        if "dict" in f:
            d = f["dict"]
            dic = O.generate(d["gen"], d["seed"], d["n"])
        if "dict_text" in f:
            dic = f["dict_text"].encode()
        frame = O.compress_frame(data, dic, f["block"], f["indep"], f["checksum"], f.get("add_size", True))
        assert frame.size == f["frame_len"], f
        if "frame_hex" in f:
            assert frame.tobytes().hex() == f["frame_hex"]
        else:
            assert "%08x" % O.xxh32(frame) == f["frame_xxh"], f
        if f.get("frame_file"):
            assert np.array_equal(frame, golden_bytes(f["frame_file"]))
        verify = not f.get("noverify", False)
        # js_compat decode reproduces the reference's decoder, including its
        # F1 corruption and the resulting checksum failures
        st, back = O.decompress_frame(frame, dic, verify_checksum=verify, js_compat=True)
        if "dec_ok" in f:
            if f["dec_ok"]:
                assert st == 0, f
                assert back.size == f["dec_len"] and "%08x" % O.xxh32(back) == f["dec_xxh"], f
            else:
                assert MESSAGES.get(st) == f["dec_error"], (st, f)
        # the spec decoder always round-trips the reference's frames
        st, back = O.decompress_frame(frame, dic)
        assert st == 0 and back.tobytes() == bytes(np.frombuffer(bytes(data), dtype=np.uint8)), f


def test_config0_frame(manifest):
    """BASELINE configs[0], the reference benchmark's call (benchWorker.js:47-54):
    LZ4.compress(1 MiB of i % 251, null, 4194304, true, false) — frame bytes and decode."""
    (c,) = cases_of(manifest, "config0")
    i = c["input"]
    data = O.generate(i["gen"], i["seed"], i["n"])
    assert np.array_equal(data, np.arange(i["n"]) % 251)
    frame = O.compress_frame(data, None, c["block"], c["indep"], c["checksum"], True)
    assert c["outbuf_equal"] and frame.size == c["frame_len"] == c["outbuf_len"]
    assert np.array_equal(frame, golden_bytes(c["frame_file"]))
    st, back = O.decompress_frame(frame, None, js_compat=True)
    assert st == 0 and c["dec_equals_input"] and np.array_equal(back, data)
    assert "%08x" % O.xxh32(back) == c["dec_xxh"]


def test_frames_decode_reference_vectors(manifest):
    (g,) = cases_of(manifest, "frames")
    for c in g["decode"]:
        st, out = O.decompress_frame(bytes.fromhex(c["hex"]), verify_checksum=c["verify"], js_compat=True)
        if c["ok"]:
            assert st == 0, c["name"]
            assert out.tobytes().hex() == c["out_hex"], c["name"]
        elif st == -6:
            assert c["error"].startswith("LZ4: Unsupported Version"), c["name"]
        else:
            assert MESSAGES.get(st) == c["error"], (c["name"], st)


@pytest.mark.parametrize("kind", ["random", "repetitive", "tiles216"])
def test_digest_manifest_4mib_subset(manifest, kind):
    (g,) = cases_of(manifest, "digest_4mib")
    rows = [r for r in g["rows"] if r["gen"] == kind][:3]          # full 16 seeds run on the GPU box
    for r in rows:
        src = O.generate(kind, r["seed"], r["n"])
        assert "%08x" % O.xxh32(src) == r["src_xxh"]
        comp = O.compress_block_bytes(src)
        assert comp.size == r["comp_len"] and "%08x" % O.xxh32(comp) == r["comp_xxh"]
        st, w, out = O.decompress_block(comp, src.size, js_compat=True)
        assert st == 0 and w == r["js_dec_written"] and "%08x" % O.xxh32(out) == r["js_dec_xxh"]


def test_compress_raw_edges(manifest):
    """F7 (five-argument call returns 0) and the RangeError of output.set on an
    overflowing literal run > 64 bytes (blockCompress.js:37,100,198,232): the
    oracle reproduces the reference's output bytes and table at return/throw."""
    (g,) = cases_of(manifest, "compress_raw_edges")
    for c in g["cases"]:
        src = golden_bytes(c["src_file"]).copy()
        out = np.zeros(c["out_len"], dtype=np.uint8)
        table = np.zeros(16384, dtype=np.int32)
        st, n = O.compress_raw(src, out, c["start"], c["len"], table, c["out_off"] or 0)
        if c["ok"]:
            assert st == 0, c["name"]
            assert (0 if c["five_args"] else n) == c["value"], c["name"]
        else:
            assert st == -8 and c["error_name"] == "RangeError", c["name"]
        assert np.array_equal(out, golden_bytes(c["out_file"])), c["name"]
        assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_file"])), c["name"]


def test_xxh32_stateful_chunkings(manifest):
    (g,) = cases_of(manifest, "xxh32_stateful")
    base = O.generate(g["input"]["gen"], g["input"]["seed"], g["input"]["n"])
    for n, chunk, seed, h in g["rows"]:
        chunks = [base[p:min(n, p + chunk)] for p in range(0, n, chunk)]
        assert "%08x" % O.xxh32_stateful(chunks, seed) == h, (n, chunk)
    seed, n, h = g["empty_updates"]
    assert "%08x" % O.xxh32_stateful([base[:0], base[:5], base[:0], base[5:n]], seed) == h


def test_block_checksum_frames_are_skipped_like_the_reference(manifest):
    """Frames with FLG bit 0x10 decode exactly as the reference decodes them (it skips the
    checksums, bufferDecompress.js:191)."""
    (g,) = cases_of(manifest, "block_checksum_skip")
    for c in g["cases"]:
        frame = golden_bytes(c["frame_file"])
        st, out = O.decompress_frame(frame, js_compat=True)
        assert st == 0 and c["dec_ok"], c["input"]
        assert "%08x" % O.xxh32(out) == c["dec_xxh"], c["input"]


def _liblz4_decode_frame(frame, cap):
    """Decode an LZ4 frame with the system liblz4 (LZ4F API, verifies block checksums)."""
    import ctypes
    L = ctypes.CDLL("liblz4.so.1")
    ctx = ctypes.c_void_p()
    assert L.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100) == 0
    out = np.zeros(cap, dtype=np.uint8)
    src = np.ascontiguousarray(frame)
    dst_size = ctypes.c_size_t(cap)
    src_size = ctypes.c_size_t(src.size)
    L.LZ4F_decompress.restype = ctypes.c_size_t
    r = L.LZ4F_decompress(ctx, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(dst_size),
                          src.ctypes.data_as(ctypes.c_void_p), ctypes.byref(src_size), None)
    L.LZ4F_isError.restype = ctypes.c_uint
    err = L.LZ4F_isError(ctypes.c_size_t(r))
    L.LZ4F_freeDecompressionContext(ctx)
    return err, out[:dst_size.value]


def test_block_checksum_frames_interoperate_with_liblz4():
    """Block checksums are the LZ4 frame format's (spec XXH32 of the payload): liblz4 1.9.3
    verifies them. A corrupted checksum must be rejected by it."""
    pytest.importorskip("ctypes")
    try:
        import ctypes
        ctypes.CDLL("liblz4.so.1")
    except OSError:
        pytest.skip("liblz4 not installed")
    data = np.concatenate([O.generate("tiles216", 3, 200000), O.generate("random", 4, 70000),
                           O.generate("repetitive", 5, 90000)])
    for bs in (65536, 262144):
        f = O.compress_frame(data, None, bs, True, False, True, block_checksum=True)
        assert f[4] & 0x10
        err, out = _liblz4_decode_frame(f, data.size + 1024)
        assert err == 0 and np.array_equal(out, data), bs
        bad = f.copy()
        bad[-8] ^= 1                      # last block's checksum (before the EndMark)
        err, _ = _liblz4_decode_frame(bad, data.size + 1024)
        assert err != 0, bs
        # the reference-style reader skips them and decodes the same bytes
        st, back = O.decompress_frame(f)
        assert st == 0 and np.array_equal(back, data)


def test_oracle_reference_decode_of_the_bench_batch(manifest):
    """The headline batch (tiles216 seeds 1..4096, 4 MiB) under the reference decoder: the
    reference's own census (gen_golden.mjs section 12: 116 of 4096 blocks decode differently from
    their input) pins the oracle's js_compat decode. Seeds 1..512 here (12 F1 blocks);
    the GPU test (test_gpu_parity.py) runs all 4096 against both."""
    (g,) = cases_of(manifest, "bench_batch_js_decode")
    assert g["seeds"] == [1, 4096] and len(g["rows"]) == 116
    rows = {r["seed"]: r for r in g["rows"]}
    n = 512
    r = O.census("tiles216", 1, n, g["n"], 8)
    assert all(st == 0 for st in r["dec_status"]) and all(w == g["n"] for w in r["dec_len"])
    for s in range(1, n + 1):
        want = rows[s]["js_dec_xxh"] if s in rows else "%08x" % r["src_xxh"][s - 1]
        assert "%08x" % r["dec_xxh"][s - 1] == want, s
        if s in rows:
            assert r["comp_len"][s - 1] == rows[s]["comp_len"] and "%08x" % r["comp_xxh"][s - 1] == rows[s]["comp_xxh"]
    assert sum(1 for s in rows if s <= n) == 12
