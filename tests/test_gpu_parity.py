"""GPU parity: the HIP kernels (through the C-ABI) against the reference's
golden vectors and the pinned CPU oracle. Bit-exact for every byte.

Run on a real MI355X: python -m pytest tests -m gpu
"""
import os

import numpy as np
import pytest

import oracle as O
from conftest import cases_of, golden_bytes

lz4mi = pytest.importorskip("lz4mi")

pytestmark = pytest.mark.gpu

MESSAGES = {
    -1: "LZ4: Output Buffer Too Small",
    -2: "LZ4: Malformed Input",
    -3: "LZ4: Invalid Offset 0",
    -4: "LZ4: Dictionary Offset Out of Bounds",
}


@pytest.fixture(scope="module", autouse=True)
def _device():
    lz4mi.init(0)


def _src_of(case):
    if "gen" in case:
        g = case["gen"]
        return O.generate(g["gen"], g["seed"], g["n"])
    return golden_bytes(case["src_file"]).copy()


def test_compress_matches_reference_golden(manifest):
    cases = cases_of(manifest, "block")
    srcs = [_src_of(c) for c in cases]
    comps = lz4mi.compress_blocks(srcs)          # one batched launch
    for c, comp in zip(cases, comps):
        assert comp.size == c["comp_len"], c["name"]
        assert "%08x" % O.xxh32(comp) == c["comp_xxh"], c["name"]
        if c["comp_file"]:
            assert np.array_equal(comp, golden_bytes(c["comp_file"])), c["name"]


def test_decompress_reference_blocks_spec_and_jscompat(manifest):
    cases = cases_of(manifest, "block")
    srcs = [_src_of(c) for c in cases]
    comps = [O.compress_block_bytes(s) for s in srcs]
    st, outs, lens = lz4mi.decompress_blocks(comps, [s.size for s in srcs])
    for c, s, o, k, n in zip(cases, srcs, outs, st, lens):
        assert k == 0 and n == s.size, c["name"]
        assert np.array_equal(o, s), c["name"]
    # js-compat: each block in its own output array, as the golden vectors were
    # made (batched, a block's rewrite may legitimately touch its predecessor's tail)
    res = [lz4mi.decompress_blocks([cb], [s.size], js_compat=True) for cb, s in zip(comps, srcs)]
    st = [r[0][0] for r in res]
    outs = [r[1][0] for r in res]
    lens = [r[2][0] for r in res]
    for c, s, o, k, n in zip(cases, srcs, outs, st, lens):
        assert k == 0 and n == c["js_dec_written"], c["name"]
        if c["js_dec_equals_input"]:
            assert np.array_equal(o, s), c["name"]
        else:
            assert "%08x" % O.xxh32(o) == c["js_dec_xxh"], c["name"]


def test_decompress_js_exact_batched(manifest):
    """JS_EXACT: the parallel spec kernel flags the blocks where the reference's
    F1 rewrite changes bytes and re-decodes only those serially; one batch must
    reproduce the reference decoder on every golden block (F1 blocks included)."""
    cases = cases_of(manifest, "block")
    srcs = [_src_of(c) for c in cases]
    comps = [O.compress_block_bytes(s) for s in srcs]
    st, outs, lens = lz4mi.decompress_blocks(comps, [s.size for s in srcs], js_exact=True)
    for c, s, o, k, n in zip(cases, srcs, outs, st, lens):
        if k == lz4mi.ERR_CROSS_BLOCK:
            # the F1 rewrite of a match at the block's start reads bytes before the
            # block (the predecessor's output in a shared buffer): batches report it,
            # the caller decodes that block alone (below)
            assert not c["js_dec_equals_input"], c["name"]
            continue
        assert k == 0 and n == c["js_dec_written"], c["name"]
        if c["js_dec_equals_input"]:
            assert np.array_equal(o, s), c["name"]
        else:
            assert "%08x" % O.xxh32(o) == c["js_dec_xxh"], c["name"]
    # single-block calls (decompressRaw) agree too
    for c, cb, s in zip(cases, comps, srcs):
        out = np.zeros(max(1, s.size), dtype=np.uint8)
        w = lz4mi.decompress_raw(cb, 0, cb.size, out, 0, js_exact=True)
        assert w == c["js_dec_written"], c["name"]
        assert "%08x" % O.xxh32(out[:s.size]) == (c["src_xxh"] if c["js_dec_equals_input"] else c["js_dec_xxh"]), c["name"]


def test_decode_edge_cases(manifest):
    (g,) = cases_of(manifest, "decode_cases")
    for c in g["cases"]:
        for js in (False, True):
            comp = np.array(c["comp"], dtype=np.uint8)
            dic = None if c["dict"] is None else np.array(c["dict"], dtype=np.uint8)
            out = np.zeros(c["out_len"], dtype=np.uint8)
            if c["ok"]:
                n = lz4mi.decompress_raw(comp, 0, comp.size, out, c["out_off"], dic, js_compat=js)
                assert n == c["written"], (c["name"], js)
                if js or c["name"] != "f1_trigger":
                    assert out.tolist() == c["out"], (c["name"], js)
            else:
                with pytest.raises(lz4mi.Lz4miError) as ei:
                    lz4mi.decompress_raw(comp, 0, comp.size, out, c["out_off"], dic, js_compat=js)
                assert str(ei.value) == c["error"], (c["name"], js)


def test_compress_raw_chain_with_table(manifest):
    (c,) = cases_of(manifest, "block_chain")
    g = c["gen"]
    src = O.generate(g["gen"], g["seed"], g["n"])
    out = np.zeros(400000, dtype=np.uint8)
    table = np.full(16384, c["table_init"], dtype=np.int32)
    pos = c["out_off0"]
    for i, (start, n, expect) in enumerate(c["segments"]):
        w = lz4mi.compress_raw(src, out, start, n, table, pos)
        assert w == expect
        pos += w
        if i == 0:
            assert np.array_equal(table.view(np.uint8), golden_bytes(c["table1_file"]))
    assert np.array_equal(out[:pos], golden_bytes(c["out_file"]))
    assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_final_file"]))


def test_xxh32_batch_matches_reference(manifest):
    (c,) = cases_of(manifest, "xxh32")
    base = O.generate(c["input"]["gen"], c["input"]["seed"], c["input"]["n"])
    rows = c["rows"]
    h0 = lz4mi.xxh32_blocks([base[:n] for n, _, _ in rows], 0)
    h1 = lz4mi.xxh32_blocks([base[:n] for n, _, _ in rows], 12345)
    for (n, e0, e1), a, b in zip(rows, h0, h1):
        assert "%08x" % a == e0 and "%08x" % b == e1, n
        assert "%08x" % lz4mi.xxh32(base[:n]) == e0
    hs = lz4mi.xxh32_blocks([base[:n] for n, _, _ in rows], 0, standard=True)
    for (n, _, _), a in zip(rows, hs):
        assert a == O.xxh32_std(base[:n])


def test_xxh32_batch_pipeline_edges():
    """Lengths around the kernel's 128-stripe load pipeline (2 x 128 x 16 B) and its
    8-stripe remainder loop, at odd buffer alignments, against the oracle."""
    src = O.generate("random", 11, (1 << 16) + 64)
    lens = [0, 15, 16, 4095, 4096, 4097, 4111, 4112, 4128, 6144 + 7, 8191, 8192, 8193, 12288 + 200,
            (1 << 16) - 1, 1 << 16, (1 << 16) + 17]
    bufs = [src[k % 5:k % 5 + n] for k, n in enumerate(lens)]
    for seed in (0, 12345):
        hs = lz4mi.xxh32_blocks(bufs, seed)
        for n, b, h in zip(lens, bufs, hs):
            assert int(h) == O.xxh32(b, seed), n


def test_generator_matches_oracle():
    torch = pytest.importorskip("torch")
    bs = 1 << 20
    for kind in ("random", "repetitive", "tiles216"):
        buf = torch.empty(3 * bs, dtype=torch.uint8, device="cuda")
        lz4mi.generate_blocks_dev(buf.data_ptr(), kind, 5, bs, 3, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        for b in range(3):
            assert np.array_equal(host[b * bs:(b + 1) * bs], O.generate(kind, 5 + b, bs)), (kind, b)


def test_fuzz_roundtrip_and_corruption():
    rng = np.random.default_rng(1234)
    kinds = ["random", "repetitive", "tiles216", "copy", "runs", "text"]
    srcs = []
    for t in range(48):
        n = int(rng.choice([0, 1, 5, 12, 13, 17, 100, 777, 4096, 20000, 65536, 100003, 300000]))
        srcs.append(O.generate(kinds[t % len(kinds)], 100 + t, n))
    comps = lz4mi.compress_blocks(srcs)
    for s, c in zip(srcs, comps):
        assert np.array_equal(c, O.compress_block_bytes(s))
    st, outs, _ = lz4mi.decompress_blocks(comps, [s.size for s in srcs])
    assert (st == 0).all()
    for s, o in zip(srcs, outs):
        assert np.array_equal(s, o)
    # corrupted streams: status and (on success) bytes must equal the oracle's
    bad, caps = [], []
    for t, c in enumerate(comps):
        c = c.copy()
        if c.size:
            for _ in range(1 + t % 4):
                c[rng.integers(0, c.size)] = rng.integers(0, 256)
        bad.append(c)
        caps.append(srcs[t].size + (t % 3) * 7)
    # spec mode as 48 blocks (the small-batch path) and as the same blocks repeated past the small
    # path's limit (the batch kernel); reference-compatible mode one block at a time
    for js, rep in ((False, 1), (False, lz4mi.SMALL_BLOCKS // 48 + 1), (True, 1)):
        if js:     # one output array per block (see test_decompress_reference_blocks_spec_and_jscompat)
            res = [lz4mi.decompress_blocks([c], [k], js_compat=True) for c, k in zip(bad, caps)]
            st = [r[0][0] for r in res]
            outs = [r[1][0] for r in res]
            lens = [r[2][0] for r in res]
        else:
            st, outs, lens = lz4mi.decompress_blocks(bad * rep, caps * rep)
        for t, c in enumerate(bad * rep):
            est, ew, eo = O.decompress_block(c, caps[t % len(bad)], js_compat=js)
            t0, t = t, t % len(bad)
            st_t, out_t, len_t = st[t0], outs[t0], lens[t0]
            if st_t == lz4mi.ERR_CROSS_BLOCK:          # batched: reaches before its own block
                assert not js and est == lz4mi.ERR_DICT_OOB, (t0, rep)   # standalone at offset 0 that is OOB
                continue
            assert st_t == est, (t0, js, rep)
            if est == 0:
                assert len_t == ew, (t0, js, rep)
                assert np.array_equal(out_t, eo[:min(ew, caps[t])]), (t0, js, rep)


@pytest.mark.parametrize("kind", ["random", "repetitive", "tiles216"])
def test_full_size_digest_manifest(manifest, kind):
    """4 MiB blocks, all 16 reference seeds: generate, compress and decompress on
    the GPU; compressed size and digests must equal the reference's."""
    torch = pytest.importorskip("torch")
    (g,) = cases_of(manifest, "digest_4mib")
    rows = [r for r in g["rows"] if r["gen"] == kind]
    n, bs = len(rows), rows[0]["n"]
    seed0 = rows[0]["seed"]
    assert [r["seed"] for r in rows] == list(range(seed0, seed0 + n))
    dev, s = "cuda", torch.cuda.current_stream().cuda_stream
    raw = torch.empty(n * bs, dtype=torch.uint8, device=dev)
    lz4mi.generate_blocks_dev(raw.data_ptr(), kind, seed0, bs, n, s)
    bound = lz4mi.compress_bound(bs)
    slot = (bound + 255) & ~255
    comp = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    in_off = torch.arange(n, dtype=torch.int64, device=dev) * bs
    in_len = torch.full((n,), bs, dtype=torch.int32, device=dev)
    out_off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    comp_len = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.compress_blocks_dev(raw.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), comp.data_ptr(),
                              out_off.data_ptr(), comp_len.data_ptr(), n, s)
    hashes = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.xxh32_blocks_dev(raw.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), hashes.data_ptr(), n, 0, s)
    ch = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.xxh32_blocks_dev(comp.data_ptr(), out_off.data_ptr(), comp_len.data_ptr(), ch.data_ptr(), n, 0, s)
    dec = torch.zeros(n * bs, dtype=torch.uint8, device=dev)
    cap = torch.full((n,), bs, dtype=torch.int32, device=dev)
    dlen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.decompress_blocks_dev(comp.data_ptr(), out_off.data_ptr(), comp_len.data_ptr(), dec.data_ptr(),
                                in_off.data_ptr(), cap.data_ptr(), dlen.data_ptr(), st.data_ptr(), n, s)
    dh = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.xxh32_blocks_dev(dec.data_ptr(), in_off.data_ptr(), dlen.data_ptr(), dh.data_ptr(), n, 0, s)
    torch.cuda.synchronize()
    for k, r in enumerate(rows):
        assert "%08x" % (int(hashes[k]) & 0xFFFFFFFF) == r["src_xxh"], (kind, r["seed"])
        assert int(comp_len[k]) == r["comp_len"], (kind, r["seed"])
        assert "%08x" % (int(ch[k]) & 0xFFFFFFFF) == r["comp_xxh"], (kind, r["seed"])
        assert int(st[k]) == 0 and int(dlen[k]) == bs
        assert "%08x" % (int(dh[k]) & 0xFFFFFFFF) == r["js_dec_xxh"] == r["src_xxh"]
    assert torch.equal(dec, raw)


def test_bench_batch_decode_vs_oracle_hashes(manifest):
    """The bench's whole headline batch (4096 x 4 MiB tiles216, seeds 1..4096, bench.py Batch):
    generated, compressed and decoded on the GPU, in spec mode and in reference mode
    (LZ4MI_JS_EXACT, the JS layer's default), in the bench's layout (one shared output buffer).
    * spec: every decoded block's XXH32 (GPU) equals the oracle's XXH32 of the oracle's own
      generation of that block on the host - an independent check of all 16 GiB of decoded bytes;
    * compressed bytes (configs[2] at the bench's scale): every block's length and XXH32 equal the
      oracle encoder's;
    * reference mode: every block's status, length and XXH32 equal the oracle's
      js_compat decode (host threads) AND the reference's own census (tests/golden section 12: 116
      blocks whose reference decode differs from their input, and the XXH32 over all 4096 digests).
      A block whose double-copy-tail rewrite reaches before its own output reports
      LZ4MI_ERR_CROSS_BLOCK in the batch and is decoded alone, as the JS layer does."""
    torch = pytest.importorskip("torch")
    (g,) = cases_of(manifest, "bench_batch_js_decode")
    n, bs = 4096, 4 << 20
    assert g["seeds"] == [1, n] and g["n"] == bs
    dev, s = "cuda", torch.cuda.current_stream().cuda_stream
    raw = torch.empty(n * bs, dtype=torch.uint8, device=dev)
    lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 1, bs, n, s)
    slot = (lz4mi.compress_bound(bs) + 255) & ~255
    comp = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    roff = torch.arange(n, dtype=torch.int64, device=dev) * bs
    rlen = torch.full((n,), bs, dtype=torch.int32, device=dev)
    coff = torch.arange(n, dtype=torch.int64, device=dev) * slot
    clen = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(), coff.data_ptr(),
                              clen.data_ptr(), n, s)
    ch = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.xxh32_blocks_dev(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), ch.data_ptr(), n, 0, s)
    del raw                                          # the decode is checked against the host oracle only
    dec = torch.zeros(n * bs, dtype=torch.uint8, device=dev)
    got = {}
    for mode in ("spec", "reference"):
        dec.zero_()
        dlen = torch.zeros(n, dtype=torch.int32, device=dev)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        lz4mi.decompress_blocks_dev(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                    roff.data_ptr(), rlen.data_ptr(), dlen.data_ptr(), st.data_ptr(), n, s,
                                    js_exact=(mode == "reference"))
        dh = torch.zeros(n, dtype=torch.int32, device=dev)
        lz4mi.xxh32_blocks_dev(dec.data_ptr(), roff.data_ptr(), dlen.data_ptr(), dh.data_ptr(), n, 0, s)
        torch.cuda.synchronize()
        got[mode] = ([int(x) for x in st.cpu().tolist()], [int(x) for x in dlen.cpu().tolist()],
                     [int(x) & 0xFFFFFFFF for x in dh.cpu().tolist()])
    got_clen = [int(x) for x in clen.cpu().tolist()]
    got_ch = [int(x) & 0xFFFFFFFF for x in ch.cpu().tolist()]
    del dec
    # blocks the reference-mode batch could not finish alone: decoded alone (decompressRaw semantics)
    st_r, len_r, h_r = got["reference"]
    cross = [b for b in range(n) if st_r[b] == lz4mi.ERR_CROSS_BLOCK]
    for b in cross:
        cb = comp[b * slot:b * slot + got_clen[b]].cpu().numpy()
        out = np.zeros(bs, dtype=np.uint8)
        len_r[b] = lz4mi.decompress_raw(cb, 0, cb.size, out, 0, js_exact=True)
        st_r[b] = 0
        h_r[b] = O.xxh32(out)
    del comp
    threads = min(16, os.cpu_count() or 8)
    want = O.census("tiles216", 1, n, bs, threads, js_compat=True)
    st_s, len_s, h_s = got["spec"]
    assert all(x == 0 for x in st_s) and all(x == bs for x in len_s)
    bad = [b for b in range(n) if h_s[b] != want["src_xxh"][b]]
    assert not bad, bad[:10]
    bad = [b for b in range(n) if got_clen[b] != want["comp_len"][b] or got_ch[b] != want["comp_xxh"][b]]
    assert not bad, bad[:10]
    # reference mode vs the oracle's reference decode ...
    assert all(x == 0 for x in want["dec_status"]) and all(x == 0 for x in st_r)
    bad = [b for b in range(n) if len_r[b] != want["dec_len"][b] or h_r[b] != want["dec_xxh"][b]]
    assert not bad, bad[:10]
    # ... and vs the reference's own census of this batch
    rows = {r["seed"]: r for r in g["rows"]}
    for b in range(n):
        r = rows.get(b + 1)
        assert "%08x" % h_r[b] == (r["js_dec_xxh"] if r else "%08x" % want["src_xxh"][b]), b
    assert "%08x" % O.digest_of_digests(h_r) == g["js_dec_xxh_of_digests"]
    assert sum(1 for b in range(n) if h_r[b] != h_s[b]) == len(rows) == 116


def test_frame_pack_matches_reference_frame():
    """Device-side frame records (lz4mi_frame_pack) == the reference frame's block records."""
    import torch
    from lz4mi import shard
    data = np.concatenate([O.generate("tiles216", 8, 600000), O.generate("random", 9, 70000)])
    bsize = 65536
    ref = O.compress_frame(data, None, bsize, True, False, True)
    info, blocks = shard.frame_blocks(ref)
    first = blocks[0][0] - 4
    nb = len(blocks)
    raw = torch.from_numpy(data.copy()).cuda()
    raw_off = torch.arange(nb, dtype=torch.int64, device="cuda") * bsize
    raw_len = torch.tensor([min(bsize, data.size - b * bsize) for b in range(nb)], dtype=torch.int32, device="cuda")
    slot = (lz4mi.compress_bound(bsize) + 255) & ~255
    comp = torch.empty(nb * slot, dtype=torch.uint8, device="cuda")
    comp_off = torch.arange(nb, dtype=torch.int64, device="cuda") * slot
    comp_len = torch.zeros(nb, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    lz4mi.compress_blocks_dev(raw.data_ptr(), raw_off.data_ptr(), raw_len.data_ptr(), comp.data_ptr(),
                              comp_off.data_ptr(), comp_len.data_ptr(), nb, s)
    rec = shard.record_sizes(comp_len, raw_len)
    rec_off = torch.cumsum(rec, 0) - rec
    out = torch.zeros(int(rec.sum().item()), dtype=torch.uint8, device="cuda")
    lz4mi.frame_pack_dev(raw.data_ptr(), raw_off.data_ptr(), raw_len.data_ptr(), comp.data_ptr(), comp_off.data_ptr(),
                         comp_len.data_ptr(), out.data_ptr(), rec_off.data_ptr(), nb, s)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref[first:ref.size - 4])


@pytest.mark.parametrize("bs", [65536, 262144, 1 << 20])
def test_compress_chain_dependent_blocks_match_oracle(bs):
    """lz4mi_compress_chain (the dependent-block frame mode in one GPU chain, source ring in
    LDS): every block == the oracle's compressBlock(src, scratch, start_b, n_b, table, 0) with
    the table carried, and the final table equal — on mixed data (matches across block
    boundaries, incompressible runs, long repetitive runs past the ring's look-ahead), from a
    start past a 64 KiB history and with a non-empty incoming table."""
    data = np.concatenate([O.generate("text", 41, 300000), O.generate("tiles216", 42, 700000),
                           O.generate("random", 43, 200000), O.generate("repetitive", 44, 500000),
                           O.generate("copy", 45, 400000)])
    for start, init in ((0, 0), (100000, -1), (70001, 5)):
        length = data.size - start - 12345
        t_ref = np.full(16384, init, dtype=np.int32)
        t_gpu = t_ref.copy()
        got = lz4mi.compress_chain(data, start, length, bs, t_gpu)
        pos, b = start, 0
        while pos < start + length:
            n = min(bs, start + length - pos)
            w, out, _ = O.compress_block(data, pos, n, t_ref)
            assert np.array_equal(got[b], out[:w]), (bs, start, b)
            pos += n
            b += 1
        assert b == len(got)
        assert np.array_equal(t_gpu, t_ref), (bs, start)


def _lit_run_blocks():
    """Blocks whose literal runs sweep the batch encoder's 2 KiB output ring: random runs of
    2000..2100 bytes between zero runs (every count of bytes a ring flush leaves pending),
    final runs of 2016..2064 bytes, and the `far` data (8-48 KiB copies from the previous
    64 KiB, tools/microbench.py) that showed a 2034..2048-byte run wrapping the ring."""
    rng = np.random.default_rng(77)
    parts = [rng.integers(0, 256, 4096, dtype=np.uint8)]
    for L in range(2000, 2101):
        parts.append(rng.integers(1, 256, L, dtype=np.uint8))
        parts.append(np.zeros(40 + L % 23, dtype=np.uint8))
    blocks = [np.concatenate(parts)]
    for L in range(2016, 2065, 3):
        head = np.concatenate([rng.integers(0, 256, 3000, dtype=np.uint8), np.zeros(L % 37 + 20, dtype=np.uint8)])
        blocks.append(np.concatenate([head, rng.integers(0, 256, L, dtype=np.uint8)]))
    for _ in range(2):
        b = np.empty(1 << 20, dtype=np.uint8)
        b[:65536] = rng.integers(0, 256, 65536, dtype=np.uint8)
        pos = 65536
        while pos < b.size:
            ln = min(int(rng.integers(8192, 49152)), b.size - pos)
            src = pos - int(rng.integers(ln, 65536))
            b[pos:pos + ln] = b[src:src + ln]
            pos += ln
        blocks.append(b)
    return blocks


def test_compress_literal_runs_around_ring_size():
    """Batch encoder vs the oracle, byte-exact, on literal runs about the output ring's size
    (lz4mi_compress.hip ring_copy), and the GPU decode of its output round-trips."""
    blocks = _lit_run_blocks()
    comps = lz4mi.compress_blocks(blocks)
    for k, (b, c) in enumerate(zip(blocks, comps)):
        ref = O.compress_block_bytes(b)
        assert c.size == ref.size and np.array_equal(c, ref), k
    st, outs, lens = lz4mi.decompress_blocks(comps, [b.size for b in blocks])
    for k, (b, o) in enumerate(zip(blocks, outs)):
        assert st[k] == 0 and np.array_equal(o, b), k


def _window_edge_stream(end, ll=200, off=100):
    """An LZ4 block whose sequence with `ll` literals (one extension byte) ends its offset exactly
    at compressed position `end` (the decoder's first chunk covers [0, 1088)): 8 literals + a
    4-byte match, 3-byte sequences up to the token, the long sequence, literal-only tail."""
    out = bytearray([0x80]) + bytes(range(65, 73)) + bytes([8, 0])          # 8 literals, offset 8, ml 4
    size = 1 + ll - 15                                                       # (token, ext, literals, offset)
    p = end - (1 + 1 + ll + 2)
    r = (p - len(out)) % 3                                                   # r 4-byte sequences (1 literal)
    k = (p - len(out) - 4 * r) // 3
    assert k >= 0
    out += bytes([0x10, 0x2A, 4, 0]) * r + bytes([0x00, 4, 0]) * k          # ml 4, offset 4
    assert len(out) == p
    out += bytes([0xF0, size - 1]) + bytes((i * 7 + 3) & 255 for i in range(ll)) + bytes([off & 255, off >> 8])
    assert len(out) == end
    out += bytes([0x50]) + b"tail!"                                          # the last literals
    return np.frombuffer(bytes(out), dtype=np.uint8)


def test_sequence_ending_on_the_window_edge():
    """A sequence whose offset's last byte is the last byte of the decoder's 1088-byte window
    (kLim) is parsed inside the window, and its offset must be read from the window (it was read
    from the window's first bytes: found by tools/small_fuzz.py); neighbouring alignments too,
    through the small-batch path, the batch kernel and the reference-compatible kernel."""
    streams, sizes = [], []
    for end in (1085, 1086, 1087, 1088, 1089, 1090, 1091):
        for ll in (17, 200, 269):
            try:
                s = _window_edge_stream(end, ll)
            except AssertionError:
                continue
            est, ew, eo = O.decompress_block(s, 1 << 16)
            assert est == 0
            streams.append(s)
            sizes.append(ew)
    assert any(s.size > 1088 for s in streams)
    exp = [O.decompress_block(s, n)[2][:n] for s, n in zip(streams, sizes)]
    for rep in (1, (lz4mi.SMALL_BLOCKS + 8) // len(streams) + 1):     # the small-batch path, then the batch kernel
        st, outs, lens = lz4mi.decompress_blocks(streams * rep, sizes * rep)
        assert (st == 0).all() and all(np.array_equal(o, exp[i % len(exp)]) for i, o in enumerate(outs)), rep
    # reference-compatible mode, one block per output array (its positions are absolute in the
    # array, as test_fuzz_roundtrip_and_corruption does): the reference's bytes, F1 rewrite included
    for s, n in zip(streams, sizes):
        est, ew, eo = O.decompress_block(s, n, js_compat=True)
        st, outs, lens = lz4mi.decompress_blocks([s], [n], js_compat=True)
        assert st[0] == est == 0 and np.array_equal(outs[0], eo[:n]), s.size
