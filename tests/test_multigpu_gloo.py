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


class _OracleCodec:
    """Each rank's block codec stand-in on CPU (the GPU path is lz4mi.frame.DeviceCodec):
    the oracle compresses the blocks; lz4mi.shard lays out the records."""

    def records(self, raw, block_size, block_checksum):
        import torch
        import oracle as O
        from lz4mi import shard
        a = raw.numpy()
        parts = []
        for p in range(0, a.size, block_size):
            blk = a[p:p + block_size]
            rec = shard.block_records([blk], [O.compress_block_bytes(blk)])
            parts.append(rec)
            if block_checksum:
                parts.append(np.array([O.xxh32_std(rec[4:])], dtype="<u4").view(np.uint8))
        return torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8))


class _OracleDecoder:
    """Each rank's decoder stand-in on CPU (the GPU path is lz4mi.frame.DeviceDecoder): the
    same interface, the oracle decoding each block of the rank's run of frame bytes."""

    def decode(self, rng, pay_rel, word, block_max, last_cap):
        import torch
        import oracle as O
        f = rng.numpy()
        outs, status = [], []
        nb = pay_rel.numel()
        for b in range(nb):
            p, w = int(pay_rel[b]), int(word[b])
            n, cap = w & 0x7FFFFFFF, (block_max if b + 1 < nb else last_cap)
            if w & 0x80000000:
                outs.append(f[p:p + n])
                status.append(0)
            else:
                st, m, out = O.decompress_block(f[p:p + n], cap)
                outs.append(out[:m] if st == 0 else np.zeros(0, dtype=np.uint8))
                status.append(st)
        cat = np.concatenate(outs) if outs else np.zeros(0, dtype=np.uint8)
        return torch.from_numpy(np.ascontiguousarray(cat)), torch.tensor(status, dtype=torch.int32)


def _frame_worker(rank, world, port, q):
    """lz4mi.frame (the product's sharded frame path) under gloo: records gathered to the
    root, header, EndMark and the streamed content checksum must give the reference frame."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "divortio-lz4_amd")]
    import torch
    import torch.distributed as dist
    import oracle as O
    from lz4mi import frame as F, shard
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        F.CHECKSUM_PIECE = 100003                      # several pieces per shard, odd size
        data = np.concatenate([O.generate("tiles216", 18, 700000), O.generate("random", 19, 300000),
                               O.generate("repetitive", 20, 90000)])
        res = []
        for bsize, bcs in ((65536, False), (262144, True)):
            nb = -(-data.size // bsize)
            lo, hi = shard.shard_range(nb, rank, world)
            mine = torch.from_numpy(data[lo * bsize:min(data.size, hi * bsize)].copy())
            tim = {}
            got = F.compress_frame_sharded(mine, bsize, True, True, bcs, codec=_OracleCodec(), timings=tim)
            ref = O.compress_frame(data, None, bsize, True, True, True, block_checksum=bcs)
            ok = all(k in tim for k in ("kernel", "collective", "checksum_wait", "checksum_chain", "assemble"))
            if rank == 0:
                ok = ok and got is not None and np.array_equal(got.numpy(), ref)
            else:
                ok = ok and got is None
            tim = {}
            fr = torch.from_numpy(ref.copy()) if rank == 0 else None
            back = F.decompress_frame_sharded(fr, True, decoder=_OracleDecoder(), timings=tim)
            ok_back = (back is not None and np.array_equal(back.numpy(), data)) if rank == 0 else back is None
            ok_back = ok_back and all(k in tim for k in ("index", "scatter", "kernel", "checksum_wait", "gather"))
            # a corrupted content checksum: the reference's error on every rank
            bad = ref.copy()
            bad[-1] ^= 0x5A
            try:
                F.decompress_frame_sharded(torch.from_numpy(bad) if rank == 0 else None, True,
                                           decoder=_OracleDecoder())
                ok_back = False
            except Exception as e:
                ok_back = ok_back and "Content Checksum Error" in str(e)
            # a bad magic number and a truncated frame (a block payload running past the end): the
            # reference's errors on every rank, found on root (no rank may hang in a collective)
            for broken, want in ((np.concatenate([np.zeros(4, np.uint8), ref[4:]]), "Invalid Magic Number"),
                                 (ref[:ref.size // 2].copy(), "Malformed Input")):
                try:
                    F.decompress_frame_sharded(torch.from_numpy(broken) if rank == 0 else None, True,
                                               decoder=_OracleDecoder())
                    ok_back = False
                except Exception as e:
                    ok_back = ok_back and want in str(e)
            # the host-staged content checksum alone == the oracle's XXH32 of the whole input
            d = F.staged_checksum(mine)
            ok = ok and (d == O.xxh32(data) if rank == 0 else d is None)
            # the same when the shared memory filesystem is too small: shards sent to the root
            real_free = F._shm_free
            F._shm_free = lambda: 0
            try:
                d = F.staged_checksum(mine)
            finally:
                F._shm_free = real_free
            ok = ok and (d == O.xxh32(data) if rank == 0 else d is None)
            # ranks on different hosts (no shared /dev/shm): the same, over the group
            real_id = F._host_id
            F._host_id = lambda: 1000 + rank
            try:
                d = F.staged_checksum(mine)
            finally:
                F._host_id = real_id
            ok = ok and (d == O.xxh32(data) if rank == 0 else d is None)
            res.append((ok, ok_back))
        q.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_sharded_frame_with_content_checksum_world2():
    """BASELINE config 4's exchange on CPU: a whole independent frame (header + every
    rank's records + EndMark + content xxh32, with and without block checksums) built
    by lz4mi.frame across 2 ranks equals the oracle's frame byte for byte, and the
    sharded decode of it gives the input back on the root."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_frame_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert isinstance(r[1], list), r
        assert all(a and b for a, b in r[1]), r


def test_frame_header_matches_reference_bytes(manifest):
    """lz4mi.frame.header == the header of the reference's frames (bufferCompress.js:147-178)."""
    from lz4mi import frame as F
    from conftest import golden_bytes
    (g,) = [c for c in manifest["cases"] if c["kind"] == "frames"]
    seen = 0
    for f in g["frames"]:
        if not f.get("frame_file") or "dict" in f or "dict_text" in f:
            continue
        fr = golden_bytes(f["frame_file"])
        size = f["n"] if f.get("add_size", True) else None
        h = F.header(f["block"], f["indep"], f["checksum"], size)
        assert bytes(fr[:len(h)]) == h, f
        seen += 1
    assert seen > 20


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


def _scaling_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "divortio-lz4_amd")]
    import importlib.util
    import torch
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        spec = importlib.util.spec_from_file_location("bench", os.path.join(root, "bench.py"))
        bench = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(bench)
        from lz4mi import shard
        n_total = 16
        mine = shard.shard_interleaved(n_total, rank, world)
        kinds = shard.clustered_mix_kinds(n_total)
        # a stand-in timing: random blocks cost 1, tiles216 blocks 3 (the skew the interleave evens out)
        kern = sum(1.0 if kinds[b] == "random" else 3.0 for b in mine) / 1000.0
        wall = kern * 5 + 0.001 * rank
        walls, value, per_rank = bench.weak_scaling(torch, dist, (wall, 2 * wall), (kern, 2 * kern),
                                                    len(mine) * (4 << 20), 5, "cpu")
        q.put((rank, walls, value, per_rank, kern))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None, None))


def test_weak_scaling_value_formula_world2():
    """bench.py's aggregation at world 2 on the clustered mix dealt out interleaved: the
    walls are max-reduced on every rank, value = all ranks' bytes x steps / the slowest wall,
    and every rank's kernel time is reported (equal shares of each cluster: balanced)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_scaling_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[2] is not None for r in res), res
    kerns = [r[4] for r in res]
    walls = [k * 5 + 0.001 * i for i, k in enumerate(kerns)]
    for rank, mx, value, per_rank, _ in res:
        assert abs(mx[0] - max(walls)) < 1e-12 and abs(mx[1] - 2 * max(walls)) < 1e-12
        assert abs(value - 2 * 8 * (4 << 20) * 5 / max(walls) / 1e9) < 1e-6
        assert per_rank[0] == [round(k * 1e3, 3) for k in kerns]
    assert kerns[0] == kerns[1]          # interleaving gave both ranks the same mix


def test_balanced_runs_cover_and_balance():
    """shard.balanced_runs: contiguous runs covering every block once, in order, each rank's
    decode cost (shard.block_cost) within one block of an equal share; on a clustered mix (stored
    random blocks first) the first rank takes the cheap blocks plus some chains."""
    from lz4mi import shard
    bmax = 4 << 20
    for n in (0, 1, 7, 16, 4096):
        words = [(bmax | 0x80000000) if b < n // 2 else 520000 for b in range(n)]
        for w in (1, 2, 3, 8):
            runs = shard.balanced_runs(words, bmax, w)
            assert len(runs) == w and runs[0][0] == 0 and runs[-1][1] == n
            assert all(runs[r][1] == runs[r + 1][0] and runs[r][0] <= runs[r][1] for r in range(w - 1))
            costs = [sum(shard.block_cost(words[b], bmax) for b in range(lo, hi)) for lo, hi in runs]
            assert max(costs) - min(costs) <= 1.0 + 1e-9 or n < w
    words = [(bmax | 0x80000000)] * 2048 + [520000] * 2048
    (a0, b0), (a1, b1) = shard.balanced_runs(words, bmax, 2)
    assert b0 - a0 > 2048 > b1 - a1 and b0 - a0 == 2048 + 768


class _CountingDecoder(_OracleDecoder):
    def __init__(self):
        self.blocks = 0

    def decode(self, rng, pay_rel, word, block_max, last_cap):
        self.blocks += pay_rel.numel()
        return super().decode(rng, pay_rel, word, block_max, last_cap)


def _balanced_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "divortio-lz4_amd")]
    import torch
    import torch.distributed as dist
    import oracle as O
    from lz4mi import frame as F
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        bs = 65536
        data = np.concatenate([O.generate("random", 70 + b, bs) for b in range(16)] +
                              [O.generate("tiles216", 90 + b, bs) for b in range(16)])
        ref = O.compress_frame(data, None, bs, True, True, True)
        dec = _CountingDecoder()
        back = F.decompress_frame_sharded(torch.from_numpy(ref.copy()) if rank == 0 else None, True, decoder=dec)
        ok = (back is not None and np.array_equal(back.numpy(), data)) if rank == 0 else back is None
        part = F.decompress_frame_sharded(torch.from_numpy(ref.copy()) if rank == 0 else None, True,
                                          decoder=_CountingDecoder(), gather=False)
        q.put((rank, ok, dec.blocks, int(part.numel())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), 0, 0))


def test_balanced_sharded_decode_of_clustered_mix_world2():
    """a clustered mix frame (16 stored random blocks, then 16 tiles216) decoded
    sharded over 2 gloo ranks: cost-balanced contiguous runs give rank 0 the 16 stored blocks and 6
    chains (22 blocks) and rank 1 10 chains, instead of 16 + 16; the gathered output is the input and
    the un-gathered parts are the runs' bytes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_balanced_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res
    assert [r[2] for r in res] == [22, 10]
    assert [r[3] for r in res] == [22 * 65536, 10 * 65536]


def _abort_worker(rank, world, port, q):
    import glob
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "divortio-lz4_amd")]
    import torch
    import torch.distributed as dist
    from lz4mi import frame as F
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        F._STAGE_PIECE = 1024                           # 65 536 pieces: the writer is still copying at abort()
        shard = torch.from_numpy(np.random.default_rng(rank).integers(0, 256, 64 << 20, dtype=np.uint8))
        ck = F.ContentChecksum(shard.numel(), torch.device("cpu"))
        ok = ck.route == "shm"
        ck.start(shard)
        if rank == 0:
            t_wait = time.time() + 60
            while not os.path.exists(ck._path(1)) and time.time() < t_wait:
                time.sleep(0.001)                       # rank 1's writer has started its staging file
            ck.abort()                                  # root's error path: no collective; rank 1 still copying
        dist.barrier()
        if rank == 1:
            ck.thread.join()                            # rank 1's writer saw root's marker and stopped
            ok = ok and ck.error is not None and "aborted" in str(ck.error)
        time.sleep(0.2)                                 # a writer that ignored cancel would recreate files now
        left = [x for x in glob.glob(os.path.join(F._shm_dir(), f"lz4mi_stage_{ck.tag[0]}_{ck.tag[1]}_*"))
                if not x.endswith(".abort")]
        q.put((rank, ok, sorted(os.path.basename(x) for x in left)))
        dist.barrier()
        if rank == 0:                                   # (root's zero-byte abort marker)
            for x in glob.glob(os.path.join(F._shm_dir(), f"lz4mi_stage_{ck.tag[0]}_{ck.tag[1]}_*.abort")):
                os.unlink(x)
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), []))


def test_content_checksum_abort_leaves_no_staging_files_world2():
    """ContentChecksum.abort() on root while the other rank is still copying its shard
    into /dev/shm (only root aborts, as when root's kernel fails): the writer sees root's abort marker,
    stops between pieces, removes its file and writes no done/err marker, so no staging file of that
    call is left behind."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_abort_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res
    assert all(r[2] == [] for r in res), res
