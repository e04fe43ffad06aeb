"""Device-resident LZ4 frames over one or many GPUs (SURVEY.md §8e/§8f rank 1;
BASELINE config 4: an independent-block frame with content checksum, sharded).

The frame layout is the reference writer's (src/buffer/bufferCompress.js:100-259):

    header (:147-178)  magic, FLG, BD, [content size u64], [dictId], HC
    records (:209-239) per block: LE32 size + payload (compressed when 0 < c < n,
                       else n | 0x80000000 + the raw bytes)  [+ LE32 block checksum]
    EndMark (:244), [content checksum (:248-252): xxHash32 of the whole input]

Each rank holds a contiguous shard of the input (every shard but the last a whole
number of blocks), compresses it with the batch encoder and packs its records on
its GPU (`lz4mi_frame_pack`). The records are concatenated on the root in rank
order: an all-gather of the record byte counts, then point-to-point sends of
exactly those bytes (RCCL over xGMI with the nccl backend; any torch.distributed
backend works). The content checksum is one serial XXH32 chain over the whole
input: it runs on root's host over host-staged shards (the ranks share
the host: each copies its shard into /dev/shm, nothing crosses xGMI for it), the
chain on a worker thread while the next piece is copied.

`codec` is the per-rank block compressor: the GPU kernels by default
(DeviceCodec). Tests on CPU pass a stand-in with the same two methods so the
collectives, layout and checksum path (this module) run under gloo.
"""
import os
import tempfile
import threading

import numpy as np

from . import shard

MAGIC = b"\x04\x22\x4d\x18"
CHECKSUM_PIECE = 64 << 20        # content-checksum streaming granularity


def block_id(nbytes):
    """getBlockId (bufferCompress.js:77-82)."""
    if not nbytes or nbytes <= 65536:
        return 4
    if nbytes <= 262144:
        return 5
    if nbytes <= 1048576:
        return 6
    return 7


def header(block_size, independent=True, content_checksum=False, content_size=None, dict_id=None,
           block_checksum=False):
    """Frame header bytes exactly as bufferCompress.js:147-178 writes them (FLG bit 0x10 when
    block_checksum, which the reference never sets)."""
    import lz4mi
    bd = block_id(block_size)
    flg = 0x40
    if independent:
        flg |= 0x20
    if block_checksum:
        flg |= 0x10
    if content_checksum:
        flg |= 0x04
    if dict_id is not None:
        flg |= 0x01
    if content_size is not None:
        flg |= 0x08
    h = bytearray(MAGIC) + bytes([flg, (bd & 7) << 4])
    if content_size is not None:
        h += int(content_size).to_bytes(8, "little")
    if dict_id is not None:
        h += int(dict_id & 0xFFFFFFFF).to_bytes(4, "little")
    h.append((lz4mi.xxh32(bytes(h[4:])) >> 8) & 0xFF)
    return bytes(h)


class DeviceCodec:
    """The GPU path: batch encoder + device frame records (one stream)."""

    def __init__(self, stream=None):
        import torch
        self.torch = torch
        self.stream = stream if stream is not None else torch.cuda.current_stream()

    def records(self, raw, block_size, block_checksum):
        """This rank's frame records (uint8 device tensor) for raw (uint8 device tensor)."""
        import lz4mi
        torch = self.torch
        s = self.stream.cuda_stream
        n = raw.numel()
        nb = -(-n // block_size)
        if nb == 0:
            return torch.empty(0, dtype=torch.uint8, device=raw.device)
        dev = raw.device
        raw_off = torch.arange(nb, dtype=torch.int64, device=dev) * block_size
        raw_len = torch.clamp(n - raw_off, max=block_size).to(torch.int32)
        slot = (lz4mi.compress_bound(block_size) + 255) & ~255
        comp = torch.empty(nb * slot, dtype=torch.uint8, device=dev)
        comp_off = torch.arange(nb, dtype=torch.int64, device=dev) * slot
        comp_len = torch.zeros(nb, dtype=torch.int32, device=dev)
        with torch.cuda.stream(self.stream):
            lz4mi.compress_blocks_dev(raw.data_ptr(), raw_off.data_ptr(), raw_len.data_ptr(), comp.data_ptr(),
                                      comp_off.data_ptr(), comp_len.data_ptr(), nb, s)
            rec = shard.record_sizes(comp_len, raw_len) + (4 if block_checksum else 0)
            rec_off = torch.cumsum(rec, 0) - rec
            total = int(rec.sum().item())
            out = torch.empty(total, dtype=torch.uint8, device=dev)
            lz4mi.frame_pack_dev(raw.data_ptr(), raw_off.data_ptr(), raw_len.data_ptr(), comp.data_ptr(),
                                 comp_off.data_ptr(), comp_len.data_ptr(), out.data_ptr(), rec_off.data_ptr(), nb, s,
                                 block_checksum=block_checksum)
        self.stream.synchronize()
        return out


class _ChecksumWorker:
    """Host streaming XXH32 on a worker thread (ctypes calls drop the GIL), fed in order."""

    def __init__(self, seed=0):
        import queue
        import lz4mi
        self.h = lz4mi.XXHash32(seed, len64=True)
        self.q = queue.Queue(maxsize=2)
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            a = self.q.get()
            if a is None:
                return
            self.h.update(a)

    def feed(self, host_bytes):
        self.q.put(host_bytes)

    def digest(self):
        self.q.put(None)
        self.t.join()
        return self.h.digest()


_STAGE_PIECE = 256 << 20
_stage_calls = [0]


def _dist_ctx(group):
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    return dist, multi, world, rank


def _shm_dir():
    return "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()


def _shm_free():
    try:
        st = os.statvfs(_shm_dir())
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


def _sent_checksum(shard, sizes, dist, group, world, rank, root, seed):
    """staged_checksum's route when the shared memory filesystem cannot hold the shards:
    every other rank sends its shard to root in _STAGE_PIECE pieces over the group (device
    tensors over RCCL with the nccl backend), root hashes them in rank order as they come."""
    import torch
    g = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    if rank != root:
        n = shard.numel()
        for p in range(0, n, _STAGE_PIECE):
            dist.send(shard[p:p + _STAGE_PIECE].contiguous(), dst=g(root), group=group)
        return None
    w = _ChecksumWorker(seed)
    for r in range(world):
        if r == root:
            for a in _host_pieces(shard):
                w.feed(a)
            continue
        if not sizes[r]:
            continue
        buf = torch.empty(min(_STAGE_PIECE, sizes[r]), dtype=torch.uint8, device=shard.device)
        for p in range(0, sizes[r], _STAGE_PIECE):
            m = min(_STAGE_PIECE, sizes[r] - p)
            dist.recv(buf[:m], src=g(r), group=group)
            for a in _host_pieces(buf[:m]):
                w.feed(a.copy())     # the pinned piece is reused by the next recv
    return w.digest()


def _host_pieces(t, piece=_STAGE_PIECE, nbuf=4):
    """Numpy views of consecutive pieces of a 1-D uint8 tensor. A device tensor goes through
    `nbuf` rotating pinned buffers (full-rate device-to-host copies); a piece's buffer is
    reused `nbuf` pieces later, after _ChecksumWorker (at most 3 pieces queued or in
    hand) has finished with it."""
    import torch
    n = t.numel()
    if t.device.type != "cuda":
        for p in range(0, n, piece):
            yield t[p:p + piece].numpy()
        return
    bufs = [torch.empty(min(piece, n), dtype=torch.uint8, pin_memory=True) for _ in range(min(nbuf, -(-n // piece)))]
    for k, p in enumerate(range(0, n, piece)):
        m = min(piece, n - p)
        b = bufs[k % len(bufs)][:m]
        b.copy_(t[p:p + m])
        yield b.numpy()


def staged_checksum(shard, group=None, root=0, seed=0):
    """XXH32 (the reference's variant, 64-bit length) of every rank's shard concatenated in
    rank order, computed on root's host: the content checksum is one serial chain,
    so it runs on one core, but the bytes need not cross xGMI — the ranks share the host.
    Each other rank copies its shard (1-D uint8 tensor, device or host) into a /dev/shm
    segment; root hashes its own shard meanwhile (device-to-host piece by piece, the chain on
    a worker thread), then each rank's segment in order. Returns the digest on root, None
    elsewhere."""
    import torch
    dist, multi, world, rank = _dist_ctx(group)
    n = shard.numel()
    if not multi:
        w = _ChecksumWorker(seed)
        for a in _host_pieces(shard):
            w.feed(a)
        return w.digest()
    dev = shard.device
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    all_n = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(all_n, t, group=group)
    sizes = [int(x.item()) for x in all_n]
    # every rank must agree on the staging route before anyone writes: the segments of all
    # non-root ranks must fit the shared memory filesystem (a memmap write past a full tmpfs
    # is a SIGBUS, not an exception), else the shards go to root piece by piece over the group
    need = sum(sizes[r] for r in range(world) if r != root)
    ok = torch.tensor([1 if _shm_free() >= need + (1 << 30) else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if not int(ok.item()):
        return _sent_checksum(shard, sizes, dist, group, world, rank, root, seed)
    _stage_calls[0] += 1
    tag = torch.tensor([os.getpid(), _stage_calls[0]], dtype=torch.int64, device=dev)
    dist.broadcast(tag, src=dist.get_global_rank(group, root) if group is not None else root, group=group)
    tag = [int(x) for x in tag.tolist()]
    path = lambda r: os.path.join(_shm_dir(), f"lz4mi_stage_{tag[0]}_{tag[1]}_{r}.bin")
    if rank != root:
        try:
            if n:
                mm = np.memmap(path(rank), dtype=np.uint8, mode="w+", shape=(n,))
                for p in range(0, n, _STAGE_PIECE):
                    m = min(_STAGE_PIECE, n - p)
                    torch.from_numpy(mm[p:p + m]).copy_(shard[p:p + m])
                mm.flush()
                del mm
            dist.barrier(group=group)       # staged
            dist.barrier(group=group)       # root has read it
        finally:
            if os.path.exists(path(rank)):
                os.unlink(path(rank))
        return None
    w = _ChecksumWorker(seed)
    staged = False
    for r in range(world):
        if r == root:
            for a in _host_pieces(shard):
                w.feed(a)
            continue
        if not staged:
            dist.barrier(group=group)
            staged = True
        if sizes[r]:
            mm = np.memmap(path(r), dtype=np.uint8, mode="r", shape=(sizes[r],))
            for p in range(0, sizes[r], _STAGE_PIECE):
                w.feed(mm[p:p + _STAGE_PIECE])
    d = w.digest()
    if not staged:
        dist.barrier(group=group)
    dist.barrier(group=group)
    return d


def _phase(timings, key, t0, dev):
    """Close a timed phase: device work done, all ranks through it (barrier)."""
    import time
    import torch
    import torch.distributed as dist
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    t = time.perf_counter()
    if timings is not None:
        timings[key] = timings.get(key, 0.0) + (t - t0)
    return t


def compress_frame_sharded(raw, block_size=4194304, content_checksum=True, add_content_size=True,
                           block_checksum=False, codec=None, group=None, root=0, timings=None):
    """One LZ4 frame of every rank's shard, concatenated in rank order, on `root`.

    raw: this rank's shard, a 1-D uint8 tensor (device tensor for the GPU codec). Every
    shard but the last rank's must be a whole number of blocks. Returns the frame as a
    uint8 tensor on root's device (None on the other ranks). Without torch.distributed
    initialised this is the single-GPU frame. Every collective moves tensors of raw's
    device (RCCL over xGMI for CUDA tensors, gloo for CPU ones). `timings` (dict) gets the
    phases, each closed by a barrier: kernel (compress + records), collective (records to
    root), checksum (host-staged content checksum), assemble (header + EndMark on root)."""
    import time
    import torch
    block_size = {4: 65536, 5: 262144, 6: 1048576, 7: 4194304}[block_id(block_size)]
    codec = codec or DeviceCodec()
    dist, multi, world, rank = _dist_ctx(group)
    n = raw.numel()
    dev = raw.device
    t0 = time.perf_counter()
    if multi:
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        all_n = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(all_n, t, group=group)
        sizes = [int(x.item()) for x in all_n]
    else:
        sizes = [n]
    for r in range(world - 1):
        if sizes[r] % block_size:
            raise ValueError("lz4mi: every shard but the last must hold whole blocks")
    t0 = _phase(timings, "setup", t0, dev)
    records = codec.records(raw, block_size, block_checksum)
    t0 = _phase(timings, "kernel", t0, dev)
    body = shard.gather_records_to_root(records, root=root, group=group) if multi else records
    t0 = _phase(timings, "collective", t0, dev)
    csum = staged_checksum(raw, group, root) if content_checksum else None
    t0 = _phase(timings, "checksum", t0, dev)
    if rank != root:
        _phase(timings, "assemble", t0, dev)
        return None
    total = sum(sizes)
    hdr = header(block_size, True, content_checksum, total if add_content_size else None, None, block_checksum)
    tail = b"\x00\x00\x00\x00" + (int(csum).to_bytes(4, "little") if content_checksum else b"")
    out = torch.empty(len(hdr) + body.numel() + len(tail), dtype=torch.uint8, device=dev)
    out[:len(hdr)] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).to(dev)
    out[len(hdr):len(hdr) + body.numel()] = body
    out[len(hdr) + body.numel():] = torch.frombuffer(bytearray(tail), dtype=torch.uint8).to(dev)
    _phase(timings, "assemble", t0, dev)
    return out


def frame_index(frame):
    """(info, pay_off, size_word) of a frame: the payload position and raw size word of every
    block in order (bufferDecompress.js:133-192). A CUDA frame is walked on its device
    (lz4mi_frame_index), a host one on the host. info: flg, content_size, block_max, end."""
    import torch
    if frame.device.type == "cuda":
        import lz4mi
        dev = frame.device
        n = frame.numel()
        cap = n // 4 + 2
        pay = torch.empty(cap, dtype=torch.int64, device=dev)
        word = torch.empty(cap, dtype=torch.int32, device=dev)
        info = torch.zeros(8, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev)
        lz4mi.frame_index_dev(frame.data_ptr(), n, pay.data_ptr(), word.data_ptr(), cap, info.data_ptr(),
                              s.cuda_stream)
        h = info.cpu().tolist()
        if h[0]:
            raise lz4mi.Lz4miError(int(h[0]))
        nb = int(h[3])
        meta = {"flg": int(h[1]), "content_size": int(h[2]), "block_max": int(h[6]), "end": int(h[5]),
                "overflow": int(h[7])}
        return meta, pay[:nb], word[:nb].to(torch.int64) & 0xFFFFFFFF
    info, blocks = shard.frame_blocks(frame.numpy())
    pay = torch.tensor([p for p, _, _ in blocks], dtype=torch.int64)
    word = torch.tensor([(nb | (0x80000000 if st else 0)) for _, nb, st in blocks], dtype=torch.int64)
    meta = {"flg": info["flg"], "content_size": info["content_size"], "block_max": info["block_max"],
            "end": info["end"], "overflow": 0}
    return meta, pay, word


class DeviceDecoder:
    """The GPU path of a rank's share of a frame: one batched decode of its compressed
    blocks (lz4mi_decompress_blocks, device pointers), stored blocks copied."""

    def __init__(self, stream=None):
        self.stream = stream

    def decode(self, rng, pay_rel, word, block_max, last_cap):
        """rng: this rank's frame bytes (device); pay_rel/word: its blocks' payload positions in
        rng and size words (int64 tensors). Returns (output, statuses): output = the blocks'
        decoded bytes concatenated in order; status 0 or the reference's error code."""
        import torch
        import lz4mi
        if rng.device.type != "cuda":          # a host frame: its bytes go to the current GPU once
            rng = rng.to("cuda")
            pay_rel, word = pay_rel.to("cuda"), word.to("cuda")
        dev = rng.device
        nb = pay_rel.numel()
        s = self.stream if self.stream is not None else torch.cuda.current_stream(dev)
        size = word & 0x7FFFFFFF
        stored = (word & 0x80000000) != 0
        cap = torch.full((nb,), block_max, dtype=torch.int64, device=dev)
        if nb:
            cap[-1] = last_cap
        slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * block_max
        out = torch.empty(max(1, nb * block_max), dtype=torch.uint8, device=dev)
        status = torch.zeros(nb, dtype=torch.int32, device=dev)
        out_len = torch.zeros(nb, dtype=torch.int32, device=dev)
        ci = torch.nonzero(~stored).flatten()
        if ci.numel():
            c_in_off = pay_rel[ci].contiguous()
            c_in_len = size[ci].to(torch.int32).contiguous()
            c_out_off = slot_off[ci].contiguous()
            c_cap = cap[ci].to(torch.int32).contiguous()
            c_len = torch.zeros(ci.numel(), dtype=torch.int32, device=dev)
            c_st = torch.zeros(ci.numel(), dtype=torch.int32, device=dev)
            with torch.cuda.stream(s):
                lz4mi.decompress_blocks_dev(rng.data_ptr(), c_in_off.data_ptr(), c_in_len.data_ptr(), out.data_ptr(),
                                            c_out_off.data_ptr(), c_cap.data_ptr(), c_len.data_ptr(), c_st.data_ptr(),
                                            ci.numel(), s.cuda_stream)
                out_len[ci] = c_len
                status[ci] = c_st
        for b in torch.nonzero(stored).flatten().tolist():      # stored blocks (rare): plain copies
            p, m = int(pay_rel[b]), int(size[b])
            if m > int(cap[b]):
                status[b] = -8                                  # the reference's RangeError (result.set)
                continue
            out[b * block_max:b * block_max + m].copy_(rng[p:p + m])
            out_len[b] = m
        if nb == 0:
            return torch.zeros(0, dtype=torch.uint8, device=dev), status
        # every block but the last filled its slot (the reference encoder's layout): the slots
        # are the output already; otherwise close the gaps
        lens = out_len.to(torch.int64)
        if bool((lens[:-1] == block_max).all()):
            return out[:(nb - 1) * block_max + int(lens[-1])], status
        ll = lens.tolist()
        res = torch.cat([out[b * block_max:b * block_max + ll[b]] for b in range(nb)])
        return res, status


def decompress_frame_sharded(frame, verify_checksum=True, group=None, root=0, decoder=None, gather=True,
                             timings=None, device=None):
    """Decode an independent-block frame with its blocks shared out over the ranks.

    frame: the whole frame on root (1-D uint8 tensor; a CUDA tensor is indexed and scattered
    on the device), ignored on the other ranks. Root indexes the size words, every rank gets
    the index (broadcast) and a contiguous run of blocks — the frame bytes of its run, sent
    point to point (RCCL over xGMI for CUDA tensors) — decodes them in one batch on its
    device, and the outputs are gathered to root in block order (`gather`), else each rank
    returns its own part. The content checksum (FLG 0x04) is verified on root's host from
    host-staged shards. Returns root's output (uint8 tensor), None on the other ranks (their
    part with gather=False). The frame's first error in block order is raised on every rank
    with the reference's message. `decoder` replaces DeviceDecoder (CPU tests); `timings`
    gets index / scatter / kernel / gather / checksum phases, each closed by a barrier.
    `device`: where this rank's tensors live (default: frame's device on root, else the
    backend's: CUDA for nccl, host for gloo)."""
    import time
    import torch
    import lz4mi
    dist, multi, world, rank = _dist_ctx(group)
    if isinstance(frame, np.ndarray):
        frame = torch.from_numpy(np.ascontiguousarray(frame, dtype=np.uint8))
        if device is None and not multi:
            device = frame.device
    if device is not None:
        dev = torch.device(device)
    elif frame is not None:
        dev = frame.device
    else:   # the backend's device: RCCL moves CUDA tensors, gloo host ones
        nccl = multi and dist.get_backend(group) == "nccl"
        dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    decoder = decoder or DeviceDecoder()
    src = dist.get_global_rank(group, root) if (multi and group is not None) else root
    t0 = time.perf_counter()
    # ---- index on root, broadcast
    if rank == root:
        meta, pay, word = frame_index(frame)
        hdr = torch.tensor([pay.numel(), meta["flg"], meta["content_size"], meta["block_max"], meta["end"],
                            meta["overflow"]], dtype=torch.int64, device=dev)
    else:
        hdr = torch.zeros(6, dtype=torch.int64, device=dev)
    if multi:
        dist.broadcast(hdr, src=src, group=group)
    nb, flg, csize, bmax, end, overflow = [int(x) for x in hdr.tolist()]
    if overflow:
        raise lz4mi.Lz4miError(lz4mi.ERR_MALFORMED)
    if not flg & 0x20:
        raise ValueError("lz4mi: dependent-block frames decode serially (LZ4.decompress)")
    if rank != root:
        pay = torch.zeros(nb, dtype=torch.int64, device=dev)
        word = torch.zeros(nb, dtype=torch.int64, device=dev)
    if multi and nb:
        dist.broadcast(pay, src=src, group=group)
        dist.broadcast(word, src=src, group=group)
    t0 = _phase(timings, "index", t0, dev)
    # ---- contiguous runs of blocks: rank r's frame bytes [a_r, b_r)
    bsum = 4 if flg & 0x10 else 0
    size = word & 0x7FFFFFFF
    runs = [shard.shard_range(nb, r, world) for r in range(world)]

    def span(lo, hi):
        if hi <= lo:
            return 0, 0
        return int(pay[lo]), int(pay[hi - 1] + size[hi - 1]) + bsum

    lo, hi = runs[rank]
    a, b = span(lo, hi)
    if multi:
        if rank == root:
            reqs = []
            for r in range(world):
                ra, rb = span(*runs[r])
                if r != root and rb > ra:
                    reqs.append(dist.isend(frame[ra:rb].contiguous(), dst=dist.get_global_rank(group, r)
                                           if group is not None else r, group=group))
            rng = frame[a:b]
            for q in reqs:
                q.wait()
        else:
            rng = torch.empty(max(1, b - a), dtype=torch.uint8, device=dev)[:b - a]
            if b > a:
                dist.recv(rng, src=src, group=group)
    else:
        rng = frame[a:b]
    t0 = _phase(timings, "scatter", t0, dev)
    # ---- decode this rank's run
    # each block decodes into block_max bytes (a block's output position depends on the sizes
    # before it, which only the decode gives); the content size is checked on the sum below
    last_cap = bmax
    out, status = decoder.decode(rng, pay[lo:hi] - a, word[lo:hi], bmax, last_cap)
    bad = torch.nonzero(status != 0).flatten()
    first = torch.tensor([lo + int(bad[0]) if bad.numel() else nb, int(status[bad[0]]) if bad.numel() else 0],
                         dtype=torch.int64, device=dev)
    if multi:
        allf = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(allf, first, group=group)
        first = min(allf, key=lambda x: int(x[0]))
    total = torch.tensor([out.numel()], dtype=torch.int64, device=dev)
    if multi:
        dist.all_reduce(total, group=group)
    t0 = _phase(timings, "kernel", t0, dev)
    if int(first[0]) < nb:
        raise lz4mi.Lz4miError(int(first[1]))
    if csize > 0 and int(total.item()) != csize:
        raise lz4mi.Lz4miError(lz4mi.ERR_MALFORMED, "lz4mi: decoded size differs from the frame's content size")
    # ---- content checksum from host-staged shards (before the gather: the shards are local)
    if verify_checksum and flg & 0x04:
        d = staged_checksum(out, group, root)
        ok = torch.tensor([1], dtype=torch.int64, device=dev)
        if rank == root:
            want = int.from_bytes(frame[end:end + 4].cpu().numpy().tobytes(), "little")
            ok[0] = int(d == want)
        if multi:
            dist.broadcast(ok, src=src, group=group)
        t0 = _phase(timings, "checksum", t0, dev)
        if not int(ok[0]):
            raise lz4mi.Lz4miError(lz4mi.ERR_CHECKSUM)
    if not gather or not multi:
        return out if (rank == root or not gather) else None
    got = shard.gather_records_to_root(out, root=root, group=group)
    _phase(timings, "gather", t0, dev)
    return got


def decompress_frame_device(frame, js_exact=False, verify_checksum=True, stream=None):
    """Decode a device-resident frame (1-D uint8 CUDA tensor) on its GPU: the header and the
    block walk run on the device (lz4mi_frame_decompress), stored blocks are copied and the
    compressed ones decoded in one batch; the content checksum (FLG 0x04) is verified on the
    host, streamed piece by piece. Frames the device walk declines (no content size, content
    size 0, a block layout other than the reference encoder's) are decoded block by block
    through the host-buffer path, as bufferDecompress.js does. Returns the content as a
    uint8 CUDA tensor. Raises lz4mi.Lz4miError with the reference's message for the frame's
    first error."""
    import torch
    import lz4mi
    lz4mi.init(frame.device.index if frame.device.index is not None else torch.cuda.current_device())
    s = stream if stream is not None else torch.cuda.current_stream(frame.device)
    head = frame[:19].cpu().numpy()
    if head.size < 4 or int.from_bytes(head[:4].tobytes(), "little") != 0x184D2204:
        raise lz4mi.Lz4miError(lz4mi.ERR_MAGIC)
    size = int.from_bytes(head[6:14].tobytes(), "little") if head.size >= 14 and head[4] & 0x08 else 0
    out = torch.empty(max(1, size), dtype=torch.uint8, device=frame.device)
    try:
        info = lz4mi.frame_decompress_dev(frame.data_ptr(), frame.numel(), out.data_ptr(), size, s.cuda_stream,
                                          js_exact=js_exact)
    except lz4mi.Lz4miError as e:
        if e.status != lz4mi.ERR_ARG:
            raise
        host = decompress_frame_host(frame.cpu().numpy(), js_exact=js_exact, verify_checksum=verify_checksum)
        return torch.from_numpy(host).to(frame.device)
    if info["status"]:
        raise lz4mi.Lz4miError(info["status"])
    out = out[:info["written"]]
    if verify_checksum and info["flg"] & 0x04:
        pos = info["checksum_pos"]
        want = int.from_bytes(frame[pos:pos + 4].cpu().numpy().tobytes(), "little")
        w = _ChecksumWorker()
        for p in range(0, out.numel(), CHECKSUM_PIECE):
            w.feed(out[p:p + CHECKSUM_PIECE].cpu().numpy())
        if w.digest() != want:
            raise lz4mi.Lz4miError(lz4mi.ERR_CHECKSUM)
    return out


def decompress_frame_host(frame, js_exact=False, verify_checksum=True):
    """A frame in host memory decoded block by block through the host-buffer C-ABI path,
    with the reference's two layouts (bufferDecompress.js:97-186): with a content size every
    block is decoded straight into the result at its position (back-references into earlier
    blocks resolve there); without one, each block is decoded behind the last 64 KiB of output
    (the reference's rolling window). Returns the content (numpy uint8)."""
    import lz4mi
    f = np.asarray(frame, dtype=np.uint8)
    try:
        info, blocks = shard.frame_blocks(f)
    except ValueError:
        raise lz4mi.Lz4miError(lz4mi.ERR_MAGIC)
    if ((info["flg"] & 0xC0) >> 6) != 1:
        raise lz4mi.Lz4miError(lz4mi.ERR_VERSION)
    bmax = info["block_max"]
    size = info["content_size"]
    if size > 0:
        out = np.zeros(size, dtype=np.uint8)
        pos = 0
        for p, n, stored in blocks:
            if stored:
                if pos + n > size:
                    raise lz4mi.Lz4miError(lz4mi.ERR_RANGE)
                out[pos:pos + n] = f[p:p + n]
                pos += n
            else:
                pos += lz4mi.decompress_raw(f, p, n, out, pos, js_exact=js_exact)
        out = out[:pos]
    else:
        parts, window = [], np.zeros(0, dtype=np.uint8)
        for p, n, stored in blocks:
            if stored:
                piece = f[p:p + n].copy()
            else:
                buf = np.concatenate([window, np.zeros(bmax, dtype=np.uint8)])
                m = lz4mi.decompress_raw(f, p, n, buf, window.size, js_exact=js_exact)
                piece = buf[window.size:window.size + m].copy()
            parts.append(piece)
            window = np.concatenate([window, piece])[-65536:]
        out = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
    if verify_checksum and info["checksum"]:
        end = info["end"]
        want = int.from_bytes(f[end:end + 4].tobytes(), "little")
        if lz4mi.XXHash32(0, len64=True).update(out).digest() != want:
            raise lz4mi.Lz4miError(lz4mi.ERR_CHECKSUM)
    return out
