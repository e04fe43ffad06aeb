"""Multi-GPU sharding of independent LZ4 frame blocks.

One process per GPU. Independent blocks need no exchange to be compressed or
decoded: each rank takes its own range (`shard_range`), or every world-th block
(`shard_interleaved`) when per-block cost is clustered by position. The frame is the one
real exchange step: the compressed blocks of all ranks are concatenated, in
block order, between the header and the EndMark. `gather_frame` does that with
two collectives over `torch.distributed` (RCCL over xGMI with the nccl backend,
gloo on CPU):

  1. all-gather of each rank's record byte count (one int64 per rank);
  2. all-gather of the records, padded to the largest rank's count.

Each rank's records are already laid out exactly as the reference's block loop
writes them (bufferCompress.js:209-239): LE32 size + payload when
0 < compSize < blockSize, else LE32 (blockSize | 0x80000000) + the raw block.
`gather_records_to_root` is the device-resident variant used when one rank
writes the frame: records packed on each GPU by `lz4mi_frame_pack`, byte counts
all-gathered, then exactly those bytes sent point-to-point to the root (no
padding, no copy to every rank).
`frame_blocks` is the inverse walk for decoding (bufferDecompress.js:133-192).
"""
import numpy as np

BLOCK_MAX_SIZES = {4: 65536, 5: 262144, 6: 1048576, 7: 4194304}


def shard_range(nblocks, rank, world):
    """Contiguous block range [lo, hi) of `rank`: ceil(N / world) blocks each."""
    per = -(-nblocks // world)
    lo = min(nblocks, rank * per)
    return lo, min(nblocks, lo + per)


def block_cost(size_word, block_max):
    """Relative decode cost of a frame block from its size word: a compressed block of
    ratio above 2 is one latency-bound chain of short copies (tiles216: ~10 ms for 4 MiB whatever
    else runs beside it), 1.0; a stored or barely compressed block is a bandwidth-bound copy (a
    random 4 MiB block ~1/4 of a chain in the batch decode: 2.5-5 ms against 10-12 ms), 0.25 per
    block_max bytes."""
    n = size_word & 0x7FFFFFFF
    if not size_word & 0x80000000 and 2 * n < block_max:
        return 1.0
    return 0.25 * max(n, 1) / block_max


def balanced_runs(size_words, block_max, world):
    """Contiguous block runs [lo, hi) for every rank with about equal decode cost (block_cost):
    a clustered frame (the first half stored random blocks) gives the first ranks
    more of the cheap blocks instead of all of them to rank 0. Runs stay contiguous so each rank's
    frame bytes are one range and the gathered output is the ranks' outputs in rank order. Every
    rank computes the same runs from the broadcast size words."""
    costs = np.array([block_cost(int(w), block_max) for w in size_words], dtype=np.float64)
    nb = costs.size
    if world <= 1 or nb == 0:
        return [(0, nb)] + [(nb, nb)] * max(0, world - 1)
    cum = np.concatenate([[0.0], np.cumsum(costs)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, total * r / world, side="left"))
        cuts.append(min(nb, max(cuts[-1], c)))
    cuts.append(nb)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_interleaved(nblocks, rank, world):
    """Global block indices of `rank` under interleaved assignment (b = rank, rank + world, ...).

    For batches whose per-block cost is skewed by position (a clustered random/tiles216 mix,
    where a contiguous split would give one rank all the cheap blocks), every rank gets the same share of
    each cluster. Blocks stay independent: each decodes into its own output slot, no exchange."""
    return list(range(rank, nblocks, world)) if 0 <= rank < world else []


def clustered_mix_kinds(nblocks):
    """SURVEY.md §8d config (5), clustered variant: the first half random blocks, then tiles216."""
    return ["random"] * (nblocks // 2) + ["tiles216"] * (nblocks - nblocks // 2)


def block_records(raw_blocks, comp_blocks):
    """The frame bytes of consecutive blocks: size word + payload, stored fallback."""
    parts = []
    for raw, comp in zip(raw_blocks, comp_blocks):
        n, c = int(raw.size), int(comp.size)
        if 0 < c < n:
            parts.append(np.array([c], dtype="<u4").view(np.uint8))
            parts.append(np.asarray(comp, dtype=np.uint8))
        else:
            parts.append(np.array([(n | 0x80000000) & 0xFFFFFFFF], dtype="<u4").view(np.uint8))
            parts.append(np.asarray(raw, dtype=np.uint8))
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)


def gather_frame(local_records, header, trailer, group=None, device="cpu"):
    """All ranks' block records in rank order, framed: header + records + EndMark + trailer.

    local_records: uint8 numpy array (this rank's consecutive blocks, from block_records).
    Returns the frame (numpy uint8) on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([int(local_records.size)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(1, max(sizes))
    buf = torch.zeros(cap, dtype=torch.uint8, device=device)
    if local_records.size:
        buf[: local_records.size] = torch.from_numpy(np.ascontiguousarray(local_records)).to(device)
    parts = [torch.empty(cap, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    body = [p[:s].cpu().numpy() for p, s in zip(parts, sizes)]
    end = np.zeros(4, dtype=np.uint8)
    return np.concatenate([np.frombuffer(bytes(header), dtype=np.uint8)] + body +
                          [end, np.frombuffer(bytes(trailer), dtype=np.uint8)])


def record_sizes(comp_len, raw_len):
    """Per-block frame record sizes (torch int64): 4 + payload (compressed when 0 < comp < raw)."""
    import torch
    comp = comp_len.to(torch.int64)
    raw = raw_len.to(torch.int64)
    return 4 + torch.where((comp > 0) & (comp < raw), comp, raw)


def gather_records_to_root(records, root=0, group=None):
    """Concatenate every rank's record bytes (1-D uint8 tensor, any device the
    backend supports) on `root`, in rank order: an all-gather of the byte
    counts, then point-to-point sends of exactly those bytes (RCCL over xGMI with
    the nccl backend). Returns the concatenation on root, None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = records.device
    n = torch.tensor([records.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    if rank != root:
        if sizes[rank]:
            dist.send(records, dst=root, group=group)
        return None
    out = torch.empty(sum(sizes), dtype=torch.uint8, device=dev)
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    reqs = []
    for r in range(world):
        if r == root:
            out[offs[r]:offs[r + 1]].copy_(records)
        elif sizes[r]:
            reqs.append(dist.irecv(out[offs[r]:offs[r + 1]], src=r, group=group))
    for q in reqs:
        q.wait()
    return out


def frame_blocks(frame):
    """Walk a frame's blocks like the reference's decoder: returns (header_info, blocks)
    with blocks = [(payload_pos, size, stored)] in order and the position after the EndMark."""
    f = np.asarray(frame, dtype=np.uint8)
    rd = lambda p: int(f[p]) | int(f[p + 1]) << 8 | int(f[p + 2]) << 16 | int(f[p + 3]) << 24 if p + 4 <= f.size else 0
    if f.size < 4 or rd(0) != 0x184D2204:
        raise ValueError("LZ4: Invalid Magic Number")
    flg, bd = int(f[4]), int(f[5])
    pos = 6
    content_size = 0
    if flg & 0x08:
        content_size = rd(pos) + rd(pos + 4) * 4294967296
        pos += 8
    if flg & 0x01:
        pos += 4
    pos += 1
    blocks = []
    while pos < f.size:
        bs = rd(pos)
        pos += 4
        if bs == 0:
            break
        n = bs & 0x7FFFFFFF
        blocks.append((pos, n, bool(bs & 0x80000000)))
        pos += n + (4 if flg & 0x10 else 0)
    info = {"flg": flg, "independent": bool(flg & 0x20), "checksum": bool(flg & 0x04),
            "content_size": content_size, "block_max": BLOCK_MAX_SIZES.get((bd >> 4) & 7, 4194304), "end": pos}
    return info, blocks
