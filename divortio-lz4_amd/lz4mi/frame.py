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
    """The GPU path: batch encoder + device frame records (one stream). Its buffers are kept
    for the next call of the same shape (allocation is not part of a frame's kernel time);
    `last_kernel_s` is the encoder + record packing time from HIP events on the stream. The
    returned records are a view of that workspace, valid until the next call."""

    def __init__(self, stream=None):
        import torch
        self.torch = torch
        self.stream = stream if stream is not None else torch.cuda.current_stream()
        self.ws = None
        self.last_kernel_s = None

    def _workspace(self, nb, n, block_size, block_checksum, dev):
        import lz4mi
        torch = self.torch
        key = (nb, n, block_size, block_checksum, str(dev))
        if self.ws is None or self.ws["key"] != key:
            self.ws = None
            raw_off = torch.arange(nb, dtype=torch.int64, device=dev) * block_size
            raw_len = torch.clamp(n - raw_off, max=block_size).to(torch.int32)
            slot = (lz4mi.compress_bound(block_size) + 255) & ~255
            rec_max = int((4 + raw_len.to(torch.int64) + (4 if block_checksum else 0)).sum().item())
            self.ws = {"key": key, "raw_off": raw_off, "raw_len": raw_len,
                       "comp": torch.empty(nb * slot, dtype=torch.uint8, device=dev),
                       "comp_off": torch.arange(nb, dtype=torch.int64, device=dev) * slot,
                       "comp_len": torch.zeros(nb, dtype=torch.int32, device=dev),
                       "out": torch.empty(max(1, rec_max), dtype=torch.uint8, device=dev)}
        return self.ws

    def records(self, raw, block_size, block_checksum):
        """This rank's frame records (uint8 device tensor) for raw (uint8 device tensor)."""
        import lz4mi
        torch = self.torch
        s = self.stream.cuda_stream
        n = raw.numel()
        nb = -(-n // block_size)
        self.last_kernel_s = None
        if nb == 0:
            return torch.empty(0, dtype=torch.uint8, device=raw.device)
        w = self._workspace(nb, n, block_size, block_checksum, raw.device)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.stream):
            e0.record(self.stream)
            lz4mi.compress_blocks_dev(raw.data_ptr(), w["raw_off"].data_ptr(), w["raw_len"].data_ptr(),
                                      w["comp"].data_ptr(), w["comp_off"].data_ptr(), w["comp_len"].data_ptr(), nb, s)
            rec = shard.record_sizes(w["comp_len"], w["raw_len"]) + (4 if block_checksum else 0)
            rec_off = torch.cumsum(rec, 0) - rec
            lz4mi.frame_pack_dev(raw.data_ptr(), w["raw_off"].data_ptr(), w["raw_len"].data_ptr(), w["comp"].data_ptr(),
                                 w["comp_off"].data_ptr(), w["comp_len"].data_ptr(), w["out"].data_ptr(),
                                 rec_off.data_ptr(), nb, s, block_checksum=block_checksum)
            e1.record(self.stream)
        self.stream.synchronize()
        self.last_kernel_s = e0.elapsed_time(e1) / 1e3
        total = int((rec_off[-1] + rec[-1]).item())
        return w["out"][:total]


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


def _host_id():
    """This host's identity as an int64 (host name + boot id): ranks whose ids match share a
    /dev/shm, the precondition of the host-staged checksum route."""
    import hashlib
    import socket
    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    h = hashlib.sha256((socket.gethostname() + "|" + boot).encode()).digest()
    return int.from_bytes(h[:8], "little") & 0x7FFFFFFFFFFFFFFF


class ContentChecksum:
    """The frame's content checksum: XXH32 (the reference's variant, 64-bit length) of every
    rank's shard concatenated in rank order, on root's host (one serial chain, so one
    core). Three steps, so the chain can run beside other work:

      ContentChecksum(n, dev, group, root)   collectives, main thread: shard sizes, whether
                                             all ranks share root's host and /dev/shm has room
      .start(shard)                          no collectives: a background thread; on root it
                                             hashes root's shard (device-to-host through pinned
                                             buffers on a side stream, the chain on a worker
                                             thread), then each other rank's /dev/shm segment
                                             as soon as that rank's done-marker appears; on the
                                             other ranks it writes the shard into its segment
      .finish()                              joins, then one all-reduce of a success flag, so a
                                             failure on any rank raises on every rank

    When the ranks do not share a host (or tmpfs lacks room: a memmap written past a full tmpfs
    is a SIGBUS, not an exception), the shards go to root over the group in finish() instead
    (_sent_checksum), which is not overlapped. Returns the digest on root, None elsewhere."""

    POLL_S = 0.0005
    DEADLINE_S = 900.0

    def __init__(self, n, dev, group=None, root=0, seed=0):
        import torch
        self.dist, self.multi, self.world, self.rank = _dist_ctx(group)
        self.group, self.root, self.seed, self.dev = group, root, seed, dev
        self.n = n
        self.error = None
        self.digest = None
        self.thread = None
        self.elapsed = 0.0
        self.route = "single"
        if not self.multi:
            self.sizes = [n]
            return
        dist = self.dist
        mine = torch.tensor([n, _host_id()], dtype=torch.int64, device=dev)
        allv = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(self.world)]
        dist.all_gather(allv, mine, group=group)
        allv = [[int(x) for x in v.tolist()] for v in allv]
        self.sizes = [v[0] for v in allv]
        same_host = all(v[1] == allv[0][1] for v in allv)
        need = sum(self.sizes[r] for r in range(self.world) if r != root)
        ok = torch.tensor([1 if same_host and _shm_free() >= need + (1 << 30) else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if not int(ok.item()):
            self.route = "send"
            return
        self.route = "shm"
        if self.rank == root:    # abort markers of this process's earlier calls
            import glob
            for f in glob.glob(os.path.join(_shm_dir(), f"lz4mi_stage_{os.getpid()}_*.abort")):
                try:
                    os.unlink(f)
                except OSError:
                    pass
        _stage_calls[0] += 1
        tag = torch.tensor([os.getpid(), _stage_calls[0]], dtype=torch.int64, device=dev)
        dist.broadcast(tag, src=self._g(root), group=group)
        self.tag = [int(x) for x in tag.tolist()]

    def _g(self, r):
        return self.dist.get_global_rank(self.group, r) if self.group is not None else r

    def _path(self, r, suffix=""):
        return os.path.join(_shm_dir(), f"lz4mi_stage_{self.tag[0]}_{self.tag[1]}_{r}.bin{suffix}")

    def start(self, shard):
        """Start the chain on `shard`. Work already queued on the caller's current stream that
        writes `shard` is waited for (an event recorded here, waited on by the side stream), so
        the caller need not synchronise first."""
        self.shard = shard
        self.ready = None
        self.cancel = False
        if self.route == "send":
            return self
        if shard.device.type == "cuda":
            import torch
            self.ready = torch.cuda.Event()
            self.ready.record(torch.cuda.current_stream(shard.device))
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()
        return self

    def abort(self):
        """Stop the chain after an error between start() and finish() (no collectives): the
        thread ends at its next poll or staging piece (a writer stops between pieces and writes
        no marker), and this call's staging files of this rank (all ranks' on root) are removed."""
        self.cancel = True
        if self.route == "shm" and self.rank == self.root:
            # the other ranks' writers may still be copying: a marker tells them to stop between
            # pieces and remove their own file; the files of ranks already done are removed here
            # (zero bytes, removed by root's next ContentChecksum)
            with open(self._path(self.root, ".abort"), "w"):
                pass
        if getattr(self, "thread", None) is not None:
            self.thread.join()
        if self.route == "shm":
            for r in (range(self.world) if self.rank == self.root else [self.rank]):
                for suf in ("", ".done", ".err", ".done.tmp", ".err.tmp"):
                    if r != self.rank and suf == "" and not (os.path.exists(self._path(r, ".done")) or
                                                             os.path.exists(self._path(r, ".err"))):
                        continue   # still being written: its writer removes it on seeing the marker
                    try:
                        os.unlink(self._path(r, suf))
                    except OSError:
                        pass

    def _run(self):
        import time
        import torch
        t0 = time.perf_counter()
        try:
            ctx = torch.cuda.device(self.shard.device) if self.shard.device.type == "cuda" else None
            side = torch.cuda.Stream(self.shard.device) if ctx is not None else None
            if side is not None and self.ready is not None:
                side.wait_event(self.ready)      # the shard's producers on the caller's stream
            if ctx is not None:
                ctx.__enter__()
            try:
                if ctx is not None:
                    with torch.cuda.stream(side):
                        self._work()
                else:
                    self._work()
            finally:
                if ctx is not None:
                    ctx.__exit__(None, None, None)
        except BaseException as e:     # reported by finish() on every rank
            self.error = e
        self.elapsed = time.perf_counter() - t0

    def _work(self):
        import time
        import torch
        shard = self.shard
        if self.route == "single" or self.rank == self.root:
            w = _ChecksumWorker(self.seed)
            try:
                for r in range(self.world):
                    if r == self.root or self.route == "single":
                        for a in _host_pieces(shard):
                            w.feed(a)
                        continue
                    deadline = time.perf_counter() + self.DEADLINE_S
                    while not os.path.exists(self._path(r, ".done")):
                        if self.cancel:
                            raise RuntimeError("lz4mi: content checksum aborted")
                        if os.path.exists(self._path(r, ".err")):
                            raise RuntimeError(f"lz4mi: rank {r} failed to stage its shard for the content checksum")
                        if time.perf_counter() > deadline:
                            raise TimeoutError(f"lz4mi: rank {r} did not stage its shard for the content checksum")
                        time.sleep(self.POLL_S)
                    if self.sizes[r]:
                        mm = np.memmap(self._path(r), dtype=np.uint8, mode="r", shape=(self.sizes[r],))
                        for p in range(0, self.sizes[r], _STAGE_PIECE):
                            w.feed(mm[p:p + _STAGE_PIECE])
                        del mm
            finally:
                self.digest = w.digest()
            return
        n = shard.numel()
        marker = ".err"
        try:
            if n:
                mm = np.memmap(self._path(self.rank), dtype=np.uint8, mode="w+", shape=(n,))
                for p in range(0, n, _STAGE_PIECE):
                    # abort() on this rank, or on root (its marker): stop between pieces, leave no files
                    if self.cancel or os.path.exists(self._path(self.root, ".abort")):
                        del mm
                        marker = None
                        raise RuntimeError("lz4mi: content checksum aborted")
                    m = min(_STAGE_PIECE, n - p)
                    torch.from_numpy(mm[p:p + m]).copy_(shard[p:p + m])
                mm.flush()
                del mm
            marker = ".done"
        except BaseException:
            if os.path.exists(self._path(self.rank)):
                os.unlink(self._path(self.rank))
            raise
        finally:
            if marker is not None and not self.cancel and not os.path.exists(self._path(self.root, ".abort")):
                tmp = self._path(self.rank, marker + ".tmp")
                with open(tmp, "w") as f:
                    f.write(marker)
                os.rename(tmp, self._path(self.rank, marker))

    def finish(self):
        """Join the background chain; raises on every rank if any rank failed. Returns the
        digest on root (None elsewhere)."""
        import torch
        if self.route == "send":
            return _sent_checksum(self.shard, self.sizes, self.dist, self.group, self.world, self.rank, self.root,
                                  self.seed)
        if self.thread is not None:
            self.thread.join()
        if self.multi:
            ok = torch.tensor([0 if self.error is not None else 1], dtype=torch.int32, device=self.dev)
            self.dist.all_reduce(ok, op=self.dist.ReduceOp.MIN, group=self.group)
            if self.rank == self.root:          # every rank is past its writes: remove what is left
                for r in range(self.world):
                    for suf in ("", ".done", ".err"):
                        if os.path.exists(self._path(r, suf)):
                            os.unlink(self._path(r, suf))
            if not int(ok.item()):
                raise self.error if self.error is not None else RuntimeError(
                    "lz4mi: the content checksum failed on another rank")
        elif self.error is not None:
            raise self.error
        return self.digest if (self.rank == self.root or not self.multi) else None


def staged_checksum(shard, group=None, root=0, seed=0):
    """XXH32 (the reference's variant, 64-bit length) of every rank's shard concatenated in
    rank order, on root's host (ContentChecksum, run to completion). Returns the digest on
    root, None elsewhere."""
    return ContentChecksum(shard.numel(), shard.device, group, root, seed).start(shard).finish()


def _phase(timings, key, t0, dev, group=None):
    """Close a timed phase: device work done, all ranks of `group` through it (barrier). Without
    `timings` nothing is synchronised."""
    import time
    import torch
    import torch.distributed as dist
    if timings is None:
        return t0
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)
    t = time.perf_counter()
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
    # the content checksum reads only the raw input: its chain starts now, beside the
    # kernel and the collective (bufferCompress.js:244-252 hashes the same bytes at the end)
    ck = ContentChecksum(n, dev, group, root).start(raw) if content_checksum else None
    try:
        t0 = _phase(timings, "setup", t0, dev, group)
        records = codec.records(raw, block_size, block_checksum)
        if timings is not None and getattr(codec, "last_kernel_s", None) is not None:
            timings["kernel_device"] = timings.get("kernel_device", 0.0) + codec.last_kernel_s
        t0 = _phase(timings, "kernel", t0, dev, group)
        body = shard.gather_records_to_root(records, root=root, group=group) if multi else records
        t0 = _phase(timings, "collective", t0, dev, group)
    except BaseException:
        if ck is not None:
            ck.abort()
        raise
    csum = ck.finish() if ck is not None else None
    if timings is not None and ck is not None:
        timings["checksum_chain"] = timings.get("checksum_chain", 0.0) + ck.elapsed
    t0 = _phase(timings, "checksum_wait", t0, dev, group)
    if rank != root:
        _phase(timings, "assemble", t0, dev, group)
        return None
    total = sum(sizes)
    hdr = header(block_size, True, content_checksum, total if add_content_size else None, None, block_checksum)
    tail = b"\x00\x00\x00\x00" + (int(csum).to_bytes(4, "little") if content_checksum else b"")
    out = torch.empty(len(hdr) + body.numel() + len(tail), dtype=torch.uint8, device=dev)
    out[:len(hdr)] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).to(dev)
    out[len(hdr):len(hdr) + body.numel()] = body
    out[len(hdr) + body.numel():] = torch.frombuffer(bytearray(tail), dtype=torch.uint8).to(dev)
    _phase(timings, "assemble", t0, dev, group)
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
    import lz4mi
    f = frame.numpy()
    try:
        info, blocks = shard.frame_blocks(f)
    except ValueError:
        raise lz4mi.Lz4miError(lz4mi.ERR_MAGIC)
    if ((info["flg"] & 0xC0) >> 6) != 1:
        raise lz4mi.Lz4miError(lz4mi.ERR_VERSION)
    pay = torch.tensor([p for p, _, _ in blocks], dtype=torch.int64)
    word = torch.tensor([(nb | (0x80000000 if st else 0)) for _, nb, st in blocks], dtype=torch.int64)
    # as lz4mi_frame_index_kernel: the walk ran past the frame's end (a payload, its block
    # checksum or the EndMark missing): the blocks cannot be cut out of it
    meta = {"flg": info["flg"], "content_size": info["content_size"], "block_max": info["block_max"],
            "end": info["end"], "overflow": int(info["end"] > f.size)}
    return meta, pay, word


class DeviceDecoder:
    """The GPU path of a rank's share of a frame: one batched decode of its compressed
    blocks (lz4mi_decompress_blocks, device pointers), stored blocks copied. The output
    buffer is kept for the next call of the same shape; `last_kernel_s` is the decode
    launch's time from HIP events on the stream."""

    def __init__(self, stream=None):
        self.stream = stream
        self.ws = None
        self.last_kernel_s = None

    def decode(self, rng, pay_rel, word, block_max, last_cap):
        """rng: this rank's frame bytes (device); pay_rel/word: its blocks' payload positions in
        rng and size words (int64 tensors). Returns (output, statuses): output = the blocks'
        decoded bytes concatenated in order; status 0 or the reference's error code. The output
        is a view of the decoder's workspace, valid until the next call."""
        import torch
        import lz4mi
        if rng.device.type != "cuda":          # a host frame: its bytes go to the current GPU once
            rng = rng.to("cuda")
            pay_rel, word = pay_rel.to("cuda"), word.to("cuda")
        dev = rng.device
        nb = pay_rel.numel()
        s = self.stream if self.stream is not None else torch.cuda.current_stream(dev)
        self.last_kernel_s = None
        cap = torch.full((nb,), block_max, dtype=torch.int64, device=dev)
        if nb:
            cap[-1] = last_cap
        slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * block_max
        key = (nb, block_max, str(dev))
        if self.ws is None or self.ws[0] != key:
            self.ws = None
            self.ws = (key, torch.empty(max(1, nb * block_max), dtype=torch.uint8, device=dev))
        out = self.ws[1]
        status = torch.zeros(nb, dtype=torch.int32, device=dev)
        out_len = torch.zeros(nb, dtype=torch.int32, device=dev)
        # every block in one launch: the size words go in as they are (LZ4MI_FRAME_WORDS), so a stored
        # block (bit 31) is copied by its own wave beside the compressed ones (bufferDecompress.js:173-180;
        # larger than its slot: the reference's RangeError, status -8)
        if nb:
            w32 = torch.where(word >= 2 ** 31, word - 2 ** 32, word).to(torch.int32).contiguous()
            in_off = pay_rel.contiguous()
            c_cap = cap.to(torch.int32).contiguous()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            s.wait_stream(torch.cuda.current_stream(dev))   # the tensors above were made on the current stream
            with torch.cuda.stream(s):
                e0.record(s)
                lz4mi.decompress_blocks_dev(rng.data_ptr(), in_off.data_ptr(), w32.data_ptr(), out.data_ptr(),
                                            slot_off.data_ptr(), c_cap.data_ptr(), out_len.data_ptr(),
                                            status.data_ptr(), nb, s.cuda_stream, frame_words=True)
                e1.record(s)
            s.synchronize()
            self.last_kernel_s = e0.elapsed_time(e1) / 1e3
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
                             timings=None, device=None, zero_copy=False):
    """Decode an independent-block frame with its blocks shared out over the ranks.

    frame: the whole frame on root (1-D uint8 tensor; a CUDA tensor is indexed and scattered
    on the device), ignored on the other ranks. Root indexes the size words, every rank gets
    the index (broadcast) and a contiguous run of blocks of about equal decode cost
    (shard.balanced_runs) — the frame bytes of its run, sent
    point to point (RCCL over xGMI for CUDA tensors) — decodes them in one batch on its
    device, and the outputs are gathered to root in block order (`gather`), else each rank
    returns its own part. The content checksum (FLG 0x04) is verified on root's host from
    host-staged shards. Returns root's output (uint8 tensor), None on the other ranks (their
    part with gather=False). The frame's first error in block order is raised on every rank
    with the reference's message. `decoder` replaces DeviceDecoder (CPU tests); `timings`
    gets index / scatter / kernel / gather / checksum_wait phases, each closed by a barrier,
    plus kernel_device (the decoder's HIP-event time) and checksum_chain (the chain's own
    duration: it runs beside the gather, so checksum_wait is what it adds).
    `device`: where this rank's tensors live (default: frame's device on root, else the
    backend's: CUDA for nccl, host for gloo). With a caller's `decoder` the un-gathered result
    is a copy unless `zero_copy`: then it is a view of that decoder's workspace, overwritten
    by the decoder's next call of the same shape (bench.py keeps one decoder and opts in)."""
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
    own_decoder = decoder is None
    decoder = decoder or DeviceDecoder()
    src = dist.get_global_rank(group, root) if (multi and group is not None) else root
    t0 = time.perf_counter()
    # ---- index on root, broadcast (a malformed frame raises on every rank, not only on root)
    status = 0
    meta = None
    if rank == root:
        try:
            meta, pay, word = frame_index(frame)
        except lz4mi.Lz4miError as e:
            status = e.status
    if meta is not None:
        hdr = torch.tensor([0, pay.numel(), meta["flg"], meta["content_size"], meta["block_max"], meta["end"],
                            meta["overflow"]], dtype=torch.int64, device=dev)
    else:
        hdr = torch.zeros(7, dtype=torch.int64, device=dev)
        hdr[0] = status
    if multi:
        dist.broadcast(hdr, src=src, group=group)
    status, nb, flg, csize, bmax, end, overflow = [int(x) for x in hdr.tolist()]
    if status:
        raise lz4mi.Lz4miError(status)
    if overflow:
        raise lz4mi.Lz4miError(lz4mi.ERR_MALFORMED)
    if not flg & 0x20:
        raise ValueError("lz4mi: dependent-block frames decode serially (LZ4.decompress)")
    if rank != root:
        pay = torch.zeros(nb, dtype=torch.int64, device=dev)
        word = torch.zeros(nb, dtype=torch.int64, device=dev)
    else:
        pay, word = pay.to(dev), word.to(dev)
    if multi and nb:
        dist.broadcast(pay, src=src, group=group)
        dist.broadcast(word, src=src, group=group)
    t0 = _phase(timings, "index", t0, dev, group)
    # ---- contiguous runs of blocks of about equal decode cost (shard.balanced_runs): rank r's
    # frame bytes [a_r, b_r)
    bsum = 4 if flg & 0x10 else 0
    size = word & 0x7FFFFFFF
    word_h = word.tolist()
    runs = shard.balanced_runs(word_h, bmax, world)
    pay_h, size_h = pay.tolist(), size.tolist()

    def span(lo, hi):
        if hi <= lo:
            return 0, 0
        return int(pay_h[lo]), int(pay_h[hi - 1] + size_h[hi - 1]) + bsum

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
    t0 = _phase(timings, "scatter", t0, dev, group)
    # ---- decode this rank's run
    # each block decodes into block_max bytes (a block's output position depends on the sizes
    # before it, which only the decode gives); the content size is checked on the sum below
    last_cap = bmax
    out, status = decoder.decode(rng, pay[lo:hi] - a, word[lo:hi], bmax, last_cap)
    if timings is not None and getattr(decoder, "last_kernel_s", None) is not None:
        timings["kernel_device"] = timings.get("kernel_device", 0.0) + decoder.last_kernel_s
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
    t0 = _phase(timings, "kernel", t0, dev, group)
    if int(first[0]) < nb:
        raise lz4mi.Lz4miError(int(first[1]))
    if csize > 0 and int(total.item()) != csize:
        raise lz4mi.Lz4miError(lz4mi.ERR_MALFORMED, "lz4mi: decoded size differs from the frame's content size")
    # ---- content checksum (bufferDecompress.js:213-217) from the decoded shards, its chain on
    # root's host beside the gather of the outputs to root (the chain reads each rank's shard
    # where it was decoded: host-staged, nothing crosses xGMI for it)
    ck = None
    if verify_checksum and flg & 0x04:
        ck = ContentChecksum(out.numel(), dev, group, root).start(out)
    got = None
    if gather and multi:
        try:
            got = shard.gather_records_to_root(out, root=root, group=group)
        except BaseException:
            if ck is not None:
                ck.abort()
            raise
        t0 = _phase(timings, "gather", t0, dev, group)
    if ck is not None:
        d = ck.finish()
        if timings is not None:
            timings["checksum_chain"] = timings.get("checksum_chain", 0.0) + ck.elapsed
        ok = torch.tensor([1], dtype=torch.int64, device=dev)
        if rank == root:
            want = int.from_bytes(frame[end:end + 4].cpu().numpy().tobytes(), "little")
            ok[0] = int(d == want)
        if multi:
            dist.broadcast(ok, src=src, group=group)
        t0 = _phase(timings, "checksum_wait", t0, dev, group)
        if not int(ok[0]):
            raise lz4mi.Lz4miError(lz4mi.ERR_CHECKSUM)
    if not gather or not multi:
        if rank != root and gather:
            return None
        caller_ws = decoder is not None and getattr(decoder, "ws", None) is not None and \
            out.numel() and out.data_ptr() >= decoder.ws[1].data_ptr() and \
            out.data_ptr() < decoder.ws[1].data_ptr() + decoder.ws[1].numel()
        return out.clone() if (caller_ws and not zero_copy and not own_decoder) else out
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
    # the library binds one device per process: a frame on another device raises ERR_ARG here
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
