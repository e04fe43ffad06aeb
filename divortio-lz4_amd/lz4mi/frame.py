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
input: the root streams every rank's raw shard, in order, through
the host streaming XXH32 (lz4mi.XXHash32) on a worker thread while the next piece
is in flight, so the chain overlaps the transfers.

`codec` is the per-rank block compressor: the GPU kernels by default
(DeviceCodec). Tests on CPU pass a stand-in with the same two methods so the
collectives, layout and checksum path (this module) run under gloo.
"""
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


def _content_checksum(raw, group, root, rank, world, sizes, dist):
    """XXH32 of the concatenation of every rank's raw shard (in rank order) on root: the
    root's own shard and, piece by piece, each other rank's shard sent to it; the host
    chain runs on a worker thread while the next piece travels."""
    import torch
    piece = CHECKSUM_PIECE
    if rank != root:
        for p in range(0, raw.numel(), piece):
            dist.send(raw[p:p + piece].contiguous(), dst=root, group=group)
        return None
    w = _ChecksumWorker()
    bufs = [torch.empty(piece, dtype=torch.uint8, device=raw.device) for _ in range(2)]
    k = 0
    for r in range(world):
        n = sizes[r]
        for p in range(0, n, piece):
            m = min(piece, n - p)
            if r == root:
                host = raw[p:p + m].cpu().numpy()
            else:
                b = bufs[k % 2][:m]
                dist.recv(b, src=r, group=group)
                # a copy even for a CPU buffer: b is reused while the worker may still hash this piece
                host = b.to("cpu", copy=True).numpy()
            k += 1
            w.feed(host)
    return w.digest()


def compress_frame_sharded(raw, block_size=4194304, content_checksum=True, add_content_size=True,
                           block_checksum=False, codec=None, group=None, root=0):
    """One LZ4 frame of every rank's shard, concatenated in rank order, on `root`.

    raw: this rank's shard, a 1-D uint8 tensor (device tensor for the GPU codec). Every
    shard but the last rank's must be a whole number of blocks. Returns the frame as a
    uint8 tensor on root's device (None on the other ranks). Without torch.distributed
    initialised this is the single-GPU frame."""
    import torch
    import torch.distributed as dist
    block_size = {4: 65536, 5: 262144, 6: 1048576, 7: 4194304}[block_id(block_size)]
    codec = codec or DeviceCodec()
    multi = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    n = raw.numel()
    dev = raw.device
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
    records = codec.records(raw, block_size, block_checksum)
    body = shard.gather_records_to_root(records, root=root, group=group) if multi else records
    csum = None
    if content_checksum:
        csum = _content_checksum(raw, group, root, rank, world, sizes, dist) if multi else None
        if not multi:
            w = _ChecksumWorker()
            for p in range(0, n, CHECKSUM_PIECE):
                w.feed(raw[p:p + CHECKSUM_PIECE].cpu().numpy())
            csum = w.digest()
    if rank != root:
        return None
    total = sum(sizes)
    hdr = header(block_size, True, content_checksum, total if add_content_size else None, None, block_checksum)
    tail = b"\x00\x00\x00\x00" + (int(csum).to_bytes(4, "little") if content_checksum else b"")
    out = torch.empty(len(hdr) + body.numel() + len(tail), dtype=torch.uint8, device=dev)
    out[:len(hdr)] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).to(dev)
    out[len(hdr):len(hdr) + body.numel()] = body
    out[len(hdr) + body.numel():] = torch.frombuffer(bytearray(tail), dtype=torch.uint8).to(dev)
    return out


def decompress_frame_sharded(frame, verify_checksum=True, group=None, root=0, decode=None):
    """Decode an independent-block frame with its blocks shared out over the ranks.

    frame: the whole frame on every rank (host numpy uint8). The host walks the size
    words (bufferDecompress.js:133-192; shard.frame_blocks), rank r takes every
    world-th block (interleaved: per-block cost varies) and decodes them in
    one batch into its slots of the output. Returns (output on root as a uint8 tensor
    in block order, or None elsewhere). `decode(blocks) -> list of uint8 arrays`
    replaces the GPU decoder in CPU tests."""
    import torch
    import torch.distributed as dist
    multi = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    info, blocks = shard.frame_blocks(frame)
    if not info["independent"]:
        raise ValueError("lz4mi: dependent-block frames decode serially (LZ4.decompress)")
    mine = shard.shard_interleaved(len(blocks), rank, world)
    f = np.asarray(frame, dtype=np.uint8)
    comp = [(f[p:p + n], stored) for p, n, stored in (blocks[b] for b in mine)]
    outs = (decode or _gpu_decode)([c for c in comp], info["block_max"])
    local = [torch.from_numpy(np.ascontiguousarray(o)) for o in outs]
    if not multi:
        parts = local
    else:
        # gather every rank's decoded blocks to root, then lay them out in block order
        flat = torch.cat(local) if local else torch.zeros(0, dtype=torch.uint8)
        got = shard.gather_records_to_root(flat, root=root, group=group)
        lens_all = [None] * world
        dist.all_gather_object(lens_all, [o.numel() for o in local], group=group)
        if rank != root:
            return None
        parts = [None] * len(blocks)
        pos = 0
        for r in range(world):
            for b, m in zip(shard.shard_interleaved(len(blocks), r, world), lens_all[r]):
                parts[b] = got[pos:pos + m]
                pos += m
    out = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8)
    if info["checksum"] and verify_checksum:
        import lz4mi
        end = info["end"]
        want = int.from_bytes(f[end:end + 4].tobytes(), "little")
        h = lz4mi.XXHash32(0, len64=True)
        for p in range(0, out.numel(), CHECKSUM_PIECE):
            h.update(out[p:p + CHECKSUM_PIECE].numpy())
        if h.digest() != want:
            raise ValueError("LZ4: Content Checksum Error")
    return out


def decompress_frame_device(frame, js_exact=False, verify_checksum=True, stream=None):
    """Decode a device-resident frame (1-D uint8 CUDA tensor) on its GPU: the header and the
    block walk run on the device (lz4mi_frame_decompress), stored blocks are copied and the
    compressed ones decoded in one batch; the content checksum (FLG 0x04) is verified on the
    host, streamed piece by piece. Returns the content as a uint8 CUDA tensor. Raises
    lz4mi.Lz4miError with the reference's message for the frame's first error."""
    import torch
    import lz4mi
    s = stream if stream is not None else torch.cuda.current_stream()
    head = frame[:19].cpu().numpy()
    if head.size < 4 or int.from_bytes(head[:4].tobytes(), "little") != 0x184D2204:
        raise lz4mi.Lz4miError(lz4mi.ERR_MAGIC)
    size = int.from_bytes(head[6:14].tobytes(), "little") if head.size >= 14 and head[4] & 0x08 else 0
    out = torch.empty(max(1, size), dtype=torch.uint8, device=frame.device)
    info = lz4mi.frame_decompress_dev(frame.data_ptr(), frame.numel(), out.data_ptr(), size, s.cuda_stream,
                                      js_exact=js_exact)
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


def _gpu_decode(comp, block_max):
    import lz4mi
    payloads = [c for c, stored in comp if not stored]
    st, dec, _ = lz4mi.decompress_blocks(payloads, [block_max] * len(payloads)) if payloads else ([], [], [])
    out, k = [], 0
    for c, stored in comp:
        if stored:
            out.append(np.asarray(c))
        else:
            if int(st[k]) != 0:
                raise lz4mi.Lz4miError(int(st[k]))
            out.append(dec[k])
            k += 1
    return out
