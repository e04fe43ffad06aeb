"""GPU parity for the BASELINE configs beyond the single-GPU block batch, and the
C-ABI behaviours added in round 2. Everything runs through liblz4mi.so and is
checked against the pinned oracle (bit-exact).

  config 4  a complete independent frame (header, device records, EndMark,
            content xxh32) built by lz4mi.frame from device-compressed blocks
  config 5  the 50/50 random/tiles216 mix, shuffled and clustered, compressed and
            decoded on the GPU, per-block digests against the oracle
  plus      compressRaw's RangeError/F7 semantics, block checksums, unaligned
            device xxh32, two concurrent streams
"""
import os

import numpy as np
import pytest

import oracle as O
from conftest import cases_of, golden_bytes

lz4mi = pytest.importorskip("lz4mi")
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
BLOCK = 4 << 20


@pytest.fixture(scope="module", autouse=True)
def _device():
    lz4mi.init(0)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_library_is_built_from_this_tree():
    from test_capi_cpu import source_hash
    assert lz4mi.build_id() == source_hash()


def test_config4_complete_frame_64mib():
    """64 MiB of tiles216 (16 x 4 MiB blocks): lz4mi.frame.compress_frame_sharded (batch
    encoder + lz4mi_frame_pack + header/EndMark/streamed content xxh32) == the oracle's
    LZ4.compress(x, null, 4 MiB, true, true) byte for byte; the sharded decode returns x."""
    from lz4mi import frame as F
    n = 16
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 1, BLOCK, n, _stream())
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    ref = O.compress_frame(host, None, BLOCK, True, True, True)
    got = F.compress_frame_sharded(raw, BLOCK, content_checksum=True)
    torch.cuda.synchronize()
    assert got.numel() == ref.size
    assert np.array_equal(got.cpu().numpy(), ref)
    back = F.decompress_frame_sharded(got, verify_checksum=True)          # device frame: index on the GPU
    assert back.is_cuda and np.array_equal(back.cpu().numpy(), host)
    tim = {}
    back = F.decompress_frame_sharded(ref, verify_checksum=True, timings=tim)   # host frame
    assert np.array_equal(back.cpu().numpy(), host)
    assert {"index", "scatter", "kernel", "checksum_wait", "kernel_device"} <= set(tim)
    # the block index of a ragged frame (4 + 4 + 4 + 3 MiB)
    part = host[:5 * (3 << 20)]
    odd = O.compress_frame(part, None, BLOCK, True, True, True)
    idx_meta, pay, word = F.frame_index(torch.from_numpy(odd).cuda())
    assert idx_meta["content_size"] == part.size and pay.numel() == 4
    assert np.array_equal(F.decompress_frame_sharded(odd).cpu().numpy(), part)
    # a middle block that does not fill block_max (another encoder's layout: 4, 1, 4 MiB):
    # the outputs are compacted, not laid out at block_max strides
    from lz4mi import shard
    pieces = [host[:BLOCK], host[BLOCK:BLOCK + (1 << 20)], host[2 * BLOCK:3 * BLOCK]]
    want = np.concatenate(pieces)
    body = shard.block_records(pieces, [O.compress_block_bytes(x) for x in pieces])
    fr = np.concatenate([np.frombuffer(F.header(BLOCK, True, True, want.size), dtype=np.uint8), body,
                         np.zeros(4, dtype=np.uint8), np.array([O.xxh32(want)], dtype="<u4").view(np.uint8)])
    assert np.array_equal(F.decompress_frame_sharded(torch.from_numpy(fr).cuda()).cpu().numpy(), want)
    corrupt = got.clone()
    corrupt[-1] ^= 0x5A
    with pytest.raises(lz4mi.Lz4miError) as ei:
        F.decompress_frame_sharded(corrupt, verify_checksum=True)
    assert str(ei.value) == "LZ4: Content Checksum Error"


def test_frame_checksum_waits_for_async_producer():
    """compress_frame_sharded's content checksum starts on a side stream at
    once; the shard written by work still queued on the caller's stream (here behind a
    ~0.1 s device sleep, no synchronisation) must be hashed after that work, not before."""
    from lz4mi import frame as F
    n = 4
    src = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(src.data_ptr(), "tiles216", 3, BLOCK, n, _stream())
    torch.cuda.synchronize()
    want = O.compress_frame(src.cpu().numpy(), None, BLOCK, True, True, True)
    raw = torch.zeros(n * BLOCK, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)     # the producer is still queued when the call starts
    raw.copy_(src)
    got = F.compress_frame_sharded(raw, BLOCK, content_checksum=True)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want)


def test_mostly_stored_frame_decodes_on_device():
    """a 16-block frame of 12 random (stored) + 4 tiles216 blocks — the
    GPU frame == the oracle's frame byte for byte, and the sharded device decode (stored blocks
    copied in the batch decode's own launch, LZ4MI_FRAME_WORDS) returns the raw bytes; a stored
    block too large for its slot reports the reference's RangeError."""
    from lz4mi import frame as F
    n = 16
    kinds = ["random"] * 12 + ["tiles216"] * 4
    order = [kinds[(5 * b) % n] for b in range(n)]          # interleaved
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    tmp = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
    for b, k in enumerate(order):
        lz4mi.generate_blocks_dev(tmp.data_ptr(), k, 40 + b, BLOCK, 1, _stream())
        raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    ref = O.compress_frame(host, None, BLOCK, True, True, True)
    got = F.compress_frame_sharded(raw, BLOCK, content_checksum=True)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), ref)
    meta, pay, word = F.frame_index(got)
    assert int(((word & 0x80000000) != 0).sum()) == 12
    dec = F.DeviceDecoder()
    back = F.decompress_frame_sharded(got, verify_checksum=True, decoder=dec)
    assert np.array_equal(back.cpu().numpy(), host)
    assert dec.last_kernel_s is not None and dec.last_kernel_s > 0
    # a stored block whose slot is too small: RangeError status (-8), nothing else touched
    out, st = dec.decode(got, pay, word, BLOCK, BLOCK - 1)
    last = n - 1
    want = -8 if int(word[last]) & 0x80000000 else 0
    assert int(st[last]) in (want, -1) and all(int(x) == 0 for x in st[:last].tolist())


def test_frame_words_flag_contract():
    """LZ4MI_FRAME_WORDS needs device pointers and the batch kernel (not LZ4MI_JS_COMPAT)."""
    L = lz4mi.lib()
    z = torch.zeros(64, dtype=torch.int64, device="cuda")
    p = z.data_ptr()
    fl = lz4mi.DEVICE_PTRS | lz4mi.FRAME_WORDS
    assert L.lz4mi_decompress_blocks(p, p, p, p, p, p, None, 0, p, p, 1, fl | lz4mi.JS_COMPAT, None) == lz4mi.ERR_ARG
    assert L.lz4mi_decompress_blocks(p, p, p, p, p, p, None, 0, p, p, 0, fl, None) == lz4mi.OK


def test_decoder_workspace_aliasing():
    """with a caller's DeviceDecoder the result is a copy (a later call of the same
    shape does not overwrite it) unless zero_copy=True asks for the workspace view."""
    from lz4mi import frame as F
    n = 2
    a = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    b = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(a.data_ptr(), "tiles216", 5, BLOCK, n, _stream())
    lz4mi.generate_blocks_dev(b.data_ptr(), "tiles216", 9, BLOCK, n, _stream())
    torch.cuda.synchronize()
    fa = F.compress_frame_sharded(a, BLOCK)
    fb = F.compress_frame_sharded(b, BLOCK)
    dec = F.DeviceDecoder()
    ra = F.decompress_frame_sharded(fa, decoder=dec)
    rb = F.decompress_frame_sharded(fb, decoder=dec)
    assert torch.equal(ra, a) and torch.equal(rb, b)
    va = F.decompress_frame_sharded(fa, decoder=dec, zero_copy=True)
    assert va.data_ptr() == dec.ws[1].data_ptr() and torch.equal(va, a)


def test_config0_frame_through_device_path(manifest):
    """BASELINE configs[0], the reference benchmark's call (benchWorker.js:47-54,
    LZ4.compress(1 MiB of i % 251, null, 4194304, true, false)): the device frame path writes
    the reference's frame byte for byte and decodes it back; a truncated copy of the frame
    (host and device) is the reference's Malformed Input, not a read past its end."""
    from lz4mi import frame as F
    (c,) = cases_of(manifest, "config0")
    i = c["input"]
    data = O.generate(i["gen"], i["seed"], i["n"])
    want = golden_bytes(c["frame_file"])
    got = F.compress_frame_sharded(torch.from_numpy(data.copy()).cuda(), c["block"], content_checksum=c["checksum"],
                                   add_content_size=True)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want)
    assert np.array_equal(F.decompress_frame_device(got).cpu().numpy(), data)
    assert np.array_equal(F.decompress_frame_sharded(got).cpu().numpy(), data)
    cut = want[:want.size - 100].copy()
    for fr in (cut, torch.from_numpy(cut).cuda()):
        with pytest.raises(lz4mi.Lz4miError) as ei:
            F.decompress_frame_sharded(fr)
        assert str(ei.value) == "LZ4: Malformed Input"


def test_frame_with_block_checksums_matches_oracle():
    """Device records with FLG 0x10 block checksums (lz4mi_frame_pack + in-place XXH32) ==
    the oracle's frame; a ragged last block and a stored (random) block included."""
    from lz4mi import frame as F
    data = np.concatenate([O.generate("tiles216", 21, 700000), O.generate("random", 22, 300000),
                           O.generate("repetitive", 23, 90001)])
    raw = torch.from_numpy(data.copy()).cuda()
    for bs, cs in ((65536, False), (262144, True)):
        ref = O.compress_frame(data, None, bs, True, cs, True, block_checksum=True)
        got = F.compress_frame_sharded(raw, bs, content_checksum=cs, block_checksum=True)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), ref), bs


def _mix_kinds(n, clustered):
    if clustered:
        from lz4mi import shard
        return shard.clustered_mix_kinds(n)
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench.mix_order(n)


@pytest.mark.parametrize("clustered", [False, True])
def test_config5_mix_encode_decode_vs_oracle(clustered):
    """Config 5's 50/50 random/tiles216 mix (Fisher-Yates by xorshift32(0x5EED), or the
    first half random): GPU compressed bytes == the oracle's for every block, GPU decode
    == the input, in one batch each."""
    n = 32
    kinds = _mix_kinds(n, clustered)
    assert kinds.count("random") == n // 2
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    tmp = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
    for b, k in enumerate(kinds):
        lz4mi.generate_blocks_dev(tmp.data_ptr(), k, 1 + b, BLOCK, 1, _stream())
        raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
    torch.cuda.synchronize()
    host = raw.cpu().numpy()
    # oracle: all blocks on host threads
    in_off = np.arange(n, dtype=np.uint64) * np.uint64(BLOCK)
    in_len = np.full(n, BLOCK, dtype=np.uint32)
    slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
    oc = np.zeros(n * slot, dtype=np.uint8)
    o_off = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    o_cap = np.full(n, slot, dtype=np.uint32)
    o_len, st = O.blocks_mt(1, host, in_off, in_len, oc, o_off, o_cap, 8)
    assert (st == 0).all()
    # GPU
    dev = "cuda"
    r_off = torch.arange(n, dtype=torch.int64, device=dev) * BLOCK
    r_len = torch.full((n,), BLOCK, dtype=torch.int32, device=dev)
    comp = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    c_off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    c_len = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.compress_blocks_dev(raw.data_ptr(), r_off.data_ptr(), r_len.data_ptr(), comp.data_ptr(), c_off.data_ptr(),
                              c_len.data_ptr(), n, _stream())
    dec = torch.zeros(n * BLOCK, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(n, dtype=torch.int32, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    lz4mi.decompress_blocks_dev(comp.data_ptr(), c_off.data_ptr(), c_len.data_ptr(), dec.data_ptr(), r_off.data_ptr(),
                                r_len.data_ptr(), d_len.data_ptr(), d_st.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    cl = c_len.cpu().numpy()
    ch = comp.cpu().numpy()
    for b in range(n):
        assert cl[b] == o_len[b], (b, kinds[b])
        s = int(o_off[b])
        assert np.array_equal(ch[b * slot:b * slot + cl[b]], oc[s:s + o_len[b]]), (b, kinds[b])
    assert (d_st == 0).all() and (d_len == BLOCK).all()
    assert torch.equal(dec, raw)


def test_compress_raw_rangeerror_and_five_args(manifest):
    """compressBlock's throw (RangeError of output.set on a literal run > 64 that does not
    fit, blockCompress.js:100,198) and F7 (no outputOffset -> returns 0): the GPU table
    kernel leaves the same output bytes and table as the reference."""
    (g,) = cases_of(manifest, "compress_raw_edges")
    for c in g["cases"]:
        src = golden_bytes(c["src_file"]).copy()
        out = np.zeros(c["out_len"], dtype=np.uint8)
        table = np.zeros(16384, dtype=np.int32)
        if c["ok"]:
            r = lz4mi.compress_raw(src, out, c["start"], c["len"], table, None if c["five_args"] else c["out_off"])
            assert r == c["value"], c["name"]
        else:
            with pytest.raises(lz4mi.Lz4miError) as ei:
                lz4mi.compress_raw(src, out, c["start"], c["len"], table, c["out_off"])
            assert ei.value.status == lz4mi.ERR_RANGE and str(ei.value) == c["error"], c["name"]
        assert np.array_equal(out, golden_bytes(c["out_file"])), c["name"]
        assert np.array_equal(table.view(np.uint8), golden_bytes(c["table_file"])), c["name"]


def test_xxh32_device_unaligned_buffers():
    """lz4mi_xxh32_blocks on device pointers at odd offsets (the kernel's byte-load path)."""
    src = O.generate("random", 12, 70000)
    lens = [4095, 4096, 4111, 4112, 8191, 8192, 8193, 12345, 0, 1, 15, 16, 17]
    stride = 9000
    buf = np.zeros(stride * len(lens) + 64, dtype=np.uint8)
    offs = []
    for b, n in enumerate(lens):
        o = b * stride + (b % 4) + (1 if b % 3 == 0 else 0)
        buf[o:o + n] = src[b * 100:b * 100 + n]
        offs.append(o)
    d = torch.from_numpy(buf).cuda()
    off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
    for std in (False, True):
        h = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
        lz4mi.xxh32_blocks_dev(d.data_ptr(), off.data_ptr(), ln.data_ptr(), h.data_ptr(), len(lens), 7, _stream(),
                               standard=std)
        torch.cuda.synchronize()
        for b, n in enumerate(lens):
            want = (O.xxh32_std if std else O.xxh32)(buf[offs[b]:offs[b] + n], 7)
            assert (int(h[b]) & 0xFFFFFFFF) == want, (b, n, std)


def test_two_streams_concurrently_bit_exact():
    """Device-pointer calls on two streams at once: per-stream scratch (hash tables) keeps both exact; no call blocks the host (the include/lz4mi.h contract)."""
    n = 24
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    jobs = []
    for k, (s, kind) in enumerate(((s1, "tiles216"), (s2, "repetitive"))):
        raw = torch.empty(n * (1 << 20), dtype=torch.uint8, device="cuda")
        lz4mi.generate_blocks_dev(raw.data_ptr(), kind, 40 + k, 1 << 20, n, s.cuda_stream)
        jobs.append((s, kind, raw))
    torch.cuda.synchronize()
    outs = []
    for s, kind, raw in jobs:
        bs = 1 << 20
        slot = (lz4mi.compress_bound(bs) + 255) & ~255
        with torch.cuda.stream(s):
            r_off = torch.arange(n, dtype=torch.int64, device="cuda") * bs
            r_len = torch.full((n,), bs, dtype=torch.int32, device="cuda")
            comp = torch.zeros(n * slot, dtype=torch.uint8, device="cuda")
            c_off = torch.arange(n, dtype=torch.int64, device="cuda") * slot
            c_len = torch.zeros(n, dtype=torch.int32, device="cuda")
            dec = torch.zeros(n * bs, dtype=torch.uint8, device="cuda")
            d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
            d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
        outs.append((s, raw, r_off, r_len, comp, c_off, c_len, dec, d_len, d_st))
    torch.cuda.synchronize()
    for _ in range(3):      # interleave the two streams' enqueues
        for s, raw, r_off, r_len, comp, c_off, c_len, dec, d_len, d_st in outs:
            lz4mi.compress_blocks_dev(raw.data_ptr(), r_off.data_ptr(), r_len.data_ptr(), comp.data_ptr(),
                                      c_off.data_ptr(), c_len.data_ptr(), n, s.cuda_stream)
        for s, raw, r_off, r_len, comp, c_off, c_len, dec, d_len, d_st in outs:
            lz4mi.decompress_blocks_dev(comp.data_ptr(), c_off.data_ptr(), c_len.data_ptr(), dec.data_ptr(),
                                        r_off.data_ptr(), r_len.data_ptr(), d_len.data_ptr(), d_st.data_ptr(), n,
                                        s.cuda_stream)
    torch.cuda.synchronize()
    for (s, kind, _), (_, raw, r_off, r_len, comp, c_off, c_len, dec, d_len, d_st) in zip(jobs, outs):
        assert (d_st == 0).all() and torch.equal(dec, raw), kind
        host = raw[: 1 << 20].cpu().numpy()
        assert np.array_equal(comp[:int(c_len[0])].cpu().numpy(), O.compress_block_bytes(host)), kind


@pytest.mark.parametrize("kind", ["copy", "runs", "text", "tiles216"])
def test_js_exact_fixup_matches_reference_decoder(kind):
    """LZ4MI_JS_EXACT (the JS layer's default): the parallel kernel's in-chunk replay of the
    reference's double-copy-tail rewrites (F1) gives the reference decoder's bytes on
    F1-heavy data (copy: ~19% of sequences), batched and per block."""
    sizes = [1 << 20, 4 << 20, 300001]
    srcs = [O.generate(kind, 70 + k, n) for k, n in enumerate(sizes)]
    comps = [O.compress_block_bytes(s) for s in srcs]
    st, outs, lens = lz4mi.decompress_blocks(comps, sizes, js_exact=True)
    for k, (s, c) in enumerate(zip(srcs, comps)):
        est, ew, eo = O.decompress_block(c, sizes[k], js_compat=True)
        assert est == 0
        if st[k] == lz4mi.ERR_CROSS_BLOCK:       # its first rewrite reaches the previous block's bytes
            out = np.zeros(sizes[k], dtype=np.uint8)
            w = lz4mi.decompress_raw(c, 0, c.size, out, 0, js_exact=True)
            assert w == ew and np.array_equal(out, eo[:sizes[k]]), (kind, k)
            continue
        assert st[k] == 0 and lens[k] == ew, (kind, k)
        assert np.array_equal(outs[k], eo[:sizes[k]]), (kind, k)


def test_frame_decompress_on_device_matches_reference():
    """lz4mi_frame_decompress: header + size-word walk on the device, stored blocks copied,
    compressed blocks batched (dependent blocks re-decoded in order); == the oracle's frame
    decode for independent/dependent frames, with stored blocks, block checksums and the
    content checksum; the reference's errors for a bad magic and a corrupted checksum."""
    from lz4mi import frame as F
    data = np.concatenate([O.generate("tiles216", 31, 900000), O.generate("random", 32, 300000),
                           O.generate("text", 33, 500000), O.generate("repetitive", 34, 77777)])
    cases = [(65536, True, True, False), (262144, False, True, False), (1048576, True, False, True),
             (4194304, True, True, False), (65536, False, False, True)]
    for bs, indep, cs, bcs in cases:
        f = O.compress_frame(data, None, bs, indep, cs, True, block_checksum=bcs)
        st, ref_spec = O.decompress_frame(f, verify_checksum=False)
        assert st == 0 and np.array_equal(ref_spec, data)
        dev = torch.from_numpy(f.copy()).cuda()
        got = F.decompress_frame_device(dev, js_exact=False, verify_checksum=cs)
        assert np.array_equal(got.cpu().numpy(), data), (bs, indep, cs, bcs)
        # reference-exact: the oracle's reference decode (F1 on the text part); checksum as the reference checks it
        est, eref = O.decompress_frame(f, verify_checksum=cs, js_compat=True)
        if est == 0:
            got = F.decompress_frame_device(dev, js_exact=True, verify_checksum=cs)
            assert np.array_equal(got.cpu().numpy(), eref), (bs, indep, cs, bcs)
        else:
            with pytest.raises(lz4mi.Lz4miError) as ei:
                F.decompress_frame_device(dev, js_exact=True, verify_checksum=cs)
            assert ei.value.status == est
    # frames the device walk declines go through the host-buffer path, same bytes: no content
    # size (the rolling 64 KiB window layout), and the empty input's frame (content size 0)
    for bs, indep in ((65536, False), (4194304, True)):
        f = O.compress_frame(data, None, bs, indep, True, False)
        got = F.decompress_frame_device(torch.from_numpy(f.copy()).cuda())
        assert np.array_equal(got.cpu().numpy(), data), (bs, indep)
    f = O.compress_frame(np.zeros(0, dtype=np.uint8), None, 65536, True, True, True)
    assert F.decompress_frame_device(torch.from_numpy(f.copy()).cuda()).numel() == 0
    bad = torch.from_numpy(np.frombuffer(bytes(range(6)), dtype=np.uint8).copy()).cuda()
    with pytest.raises(lz4mi.Lz4miError) as ei:
        F.decompress_frame_device(bad)
    assert str(ei.value) == "LZ4: Invalid Magic Number"


def test_js_exact_tiles216_f1_blocks_match_reference_census(manifest):
    """tiles216 4 MiB blocks whose reference decode differs from their input (the reference's census
    of the bench batch, tests/golden section 12): seeds 33 and 62 and two with a single
    rewritten 4-byte group, batched with two F1-free seeds and one at a time, in reference mode
    (LZ4MI_JS_EXACT) == the reference decoder's digest; in spec mode == the input."""
    (g,) = cases_of(manifest, "bench_batch_js_decode")
    rows = {r["seed"]: r for r in g["rows"]}
    seeds = [33, 62, 969, 1426, 1, 2]
    bs = g["n"]
    srcs = [O.generate("tiles216", sd, bs) for sd in seeds]
    comps = [O.compress_block_bytes(x) for x in srcs]
    for sd, c in zip(seeds, comps):
        if sd in rows:
            assert c.size == rows[sd]["comp_len"] and "%08x" % O.xxh32(c) == rows[sd]["comp_xxh"]
    want = ["%08x" % (int(rows[sd]["js_dec_xxh"], 16) if sd in rows else O.xxh32(x)) for sd, x in zip(seeds, srcs)]
    st, outs, lens = lz4mi.decompress_blocks(comps, [bs] * len(seeds), js_exact=True)
    for k, sd in enumerate(seeds):
        if st[k] == lz4mi.ERR_CROSS_BLOCK:
            continue
        assert st[k] == 0 and lens[k] == bs and "%08x" % O.xxh32(outs[k]) == want[k], sd
    for k, (sd, c) in enumerate(zip(seeds, comps)):
        out = np.zeros(bs, dtype=np.uint8)
        assert lz4mi.decompress_raw(c, 0, c.size, out, 0, js_exact=True) == bs
        assert "%08x" % O.xxh32(out) == want[k], sd
        out[:] = 0
        assert lz4mi.decompress_raw(c, 0, c.size, out, 0) == bs and np.array_equal(out, srcs[k]), sd


def test_frame_past_4gib():
    """a frame whose compressed bytes exceed 2^32 (configs[3] at 8 GPUs is ~8.6 GB):
    1280 x 4 MiB blocks, 7 of 8 random (stored records) and every 8th tiles216 (compressed, some past the
    4 GiB mark), through compress_frame_sharded (content checksum) and decompress_frame_sharded (index,
    scatter, batch decode with stored blocks in the same launch, checksum verified) and the single-GPU
    device frame path; payload positions past 2^32 in the index, the content checksum equal to the
    oracle's XXH32 of the raw bytes, the last compressed block equal to the oracle encoder's."""
    from lz4mi import frame as F
    n = 1280
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    lz4mi.generate_blocks_dev(raw.data_ptr(), "random", 7000, BLOCK, n, _stream())
    tiles = [b for b in range(n) if b % 8 == 7]
    tmp = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
    for b in tiles:
        lz4mi.generate_blocks_dev(tmp.data_ptr(), "tiles216", 9000 + b, BLOCK, 1, _stream())
        raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
    del tmp
    torch.cuda.synchronize()
    frame = F.compress_frame_sharded(raw, BLOCK, content_checksum=True, add_content_size=True)
    torch.cuda.synchronize()
    assert frame.numel() > (1 << 32)
    meta, pay, word = F.frame_index(frame)
    assert pay.numel() == n and meta["content_size"] == n * BLOCK and int(pay[-1]) > (1 << 32)
    stored = ((word & 0x80000000) != 0).cpu().numpy()
    assert stored.sum() == n - len(tiles) and not stored[tiles].any()
    # the content checksum (the frame's last 4 bytes) == the oracle's XXH32 of all raw bytes
    host = raw.cpu().numpy()
    assert int.from_bytes(frame[-4:].cpu().numpy().tobytes(), "little") == O.xxh32(host)
    # the last compressed record (past 2^32) == the oracle encoder's bytes
    b = tiles[-1]
    p, w = int(pay[b]), int(word[b])
    assert p > (1 << 32)
    want = O.compress_block_bytes(host[b * BLOCK:(b + 1) * BLOCK])
    assert w == want.size and np.array_equal(frame[p:p + w].cpu().numpy(), want)
    del host
    back = F.decompress_frame_sharded(frame, verify_checksum=True)
    assert back.numel() == n * BLOCK and torch.equal(back, raw)
    del back
    dev = F.decompress_frame_device(frame, verify_checksum=True)
    assert dev.numel() == n * BLOCK and torch.equal(dev, raw)
