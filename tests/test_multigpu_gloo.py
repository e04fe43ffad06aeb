"""Multi-rank frame path on CPU (gloo, world size 2): each rank compresses its
shard of independent blocks, the frame is assembled with lz4mi.shard's
collectives, and must equal the reference frame byte for byte; the inverse
(each rank decoding its shard of a frame's blocks, then gathering) must
reproduce the input. The per-rank block codec here is the oracle (test
infrastructure standing in for each rank's GPU); the collectives, sharding and
frame layout are the product code that runs over RCCL on the GPU box."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "divortio-lz4_amd")]
    import torch.distributed as dist
    import oracle as O
    from lz4mi import shard
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        data = np.concatenate([O.generate("tiles216", 8, 600000), O.generate("random", 9, 70000)])
        bsize = 65536
        nb = -(-data.size // bsize)
        lo, hi = shard.shard_range(nb, rank, world)
        raws = [data[b * bsize:(b + 1) * bsize] for b in range(lo, hi)]
        comps = [O.compress_block_bytes(r) for r in raws]
        recs = shard.block_records(raws, comps)
        ref = O.compress_frame(data, None, bsize, True, True, True)
        info, _ = shard.frame_blocks(ref)
        first = shard.frame_blocks(ref)[1][0][0] - 4          # header = bytes before the first size word
        trailer = ref[-4:].tobytes()                           # content checksum
        frame = shard.gather_frame(recs, ref[:first].tobytes(), trailer)
        ok_frame = bool(np.array_equal(frame, ref))
        # decode side: blocks of the frame sharded over ranks, gathered back in order
        info, blocks = shard.frame_blocks(frame)
        lo, hi = shard.shard_range(len(blocks), rank, world)
        outs = []
        for pos, n, stored in blocks[lo:hi]:
            if stored:
                outs.append(frame[pos:pos + n])
            else:
                st, w, out = O.decompress_block(frame[pos:pos + n], info["block_max"])
                assert st == 0
                outs.append(out[:w])
        local = np.concatenate(outs) if outs else np.zeros(0, dtype=np.uint8)
        back = shard.gather_frame(local, b"", b"")[:-4]        # reuse the gather: no header, EndMark stripped
        ok_back = bool(np.array_equal(back, data))
        # records gathered to rank 0 by byte counts + point-to-point (the RCCL path's code)
        import torch
        got = shard.gather_records_to_root(torch.from_numpy(recs.copy()), root=0)
        if rank == 0:
            body = ref[first:ref.size - 8]                      # records between the header and EndMark+checksum
            ok_frame = ok_frame and bool(np.array_equal(got.numpy(), body))
        q.put((rank, ok_frame, ok_back, int(info["independent"])))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, False, repr(e)))


def test_shard_range_covers_blocks():
    from lz4mi import shard
    for n in (0, 1, 7, 16, 4096):
        for w in (1, 2, 3, 8):
            got = [b for r in range(w) for b in range(*shard.shard_range(n, r, w))]
            assert got == list(range(n))


def test_shard_interleaved_balances_clustered_mix():
    from lz4mi import shard
    for n in (0, 1, 7, 16, 4096):
        for w in (1, 2, 3, 8):
            parts = [shard.shard_interleaved(n, r, w) for r in range(w)]
            assert sorted(b for p in parts for b in p) == list(range(n))
            kinds = shard.clustered_mix_kinds(n)
            rnd = [sum(kinds[b] == "random" for b in p) for p in parts]
            assert max(rnd) - min(rnd) <= 1 + (n % w != 0)   # each rank gets an even share of each cluster


def test_frame_gather_and_sharded_decode_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    for r in res:
        assert r[1] is True and r[2] is True, r
