#!/usr/bin/env python3
"""bench.py — LZ4 raw-block decompress (+ compress) throughput on MI355X.

Workload (BASELINE.json configs[1]): 4096 independent 4 MiB blocks per GPU
(16 GiB uncompressed), generator tiles216 (~8:1), compressed
on the GPU with the bit-exact encoder, then decompressed device-resident.
A "step" = one lz4mi_decompress_blocks launch over the whole batch.

value = uncompressed GB/s (1e9 B/s) of all ranks; scaling is weak (every rank
decodes its own 4096 blocks, no data-path collective). `--gen mixc` is the
clustered random/tiles216 mix (first half of all ranks' blocks random) dealt
to the ranks interleaved.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--gen tiles216|random|repetitive|mix|mixc]

With --gpus N > 1 and no torch.distributed environment, the script starts N
rank processes itself (torch.distributed.run, one per GPU, before touching the
GPU) and exits with their status; it fails if fewer than N GPUs are visible.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))

HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "LZ4 compress+decompress GB/s on 4 MiB independent blocks; % of HBM peak"   # BASELINE.json
BLOCK = 4 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--gen", default="tiles216")
    ap.add_argument("--compress-steps", type=int, default=2)
    ap.add_argument("--extra", type=int, default=1, help="also time the random/repetitive/mix variants")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-blocks", type=int, default=64, help="4 MiB blocks per CPU thread (pure-JS baseline)")
    ap.add_argument("--napi", type=int, default=1, help="time the JS drop-in end to end (host buffers)")
    ap.add_argument("--frame-blocks", type=int, default=2048,
                    help="4 MiB blocks per rank in the sharded frame workload (configs[3]; 0 = skip)")
    return ap.parse_args()


def visible_gpus():
    """GPUs this process may use, counted without touching HIP: the KFD topology's GPU
    nodes (simd_count > 0) whose render node this user can open, limited by
    HIP/ROCR/CUDA_VISIBLE_DEVICES when one is set."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        nodes = os.listdir(base)
    except OSError:
        nodes = []
    for d in nodes:
        props = {}
        try:
            with open(os.path.join(base, d, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue
        minor = props.get("drm_render_minor")
        if minor is None or os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            n += 1
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args):
    """--gpus N without a distributed environment: one process per GPU via
    torch.distributed.run. This process never initialises HIP (the GPUs are counted
    from the KFD topology), so the ranks are its children, not a re-exec."""
    import socket
    have = visible_gpus()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
        sys.exit(2)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


class Batch:
    """Device-resident batch: raw blocks, compressed slots, decode buffers."""

    def __init__(self, torch, lz4mi, n, gen, seed0, stream, rank=0, world=1):
        self.n = n
        dev = "cuda"
        self.raw = torch.empty(n * BLOCK, dtype=torch.uint8, device=dev)
        if gen in ("mix", "mixc"):
            if gen == "mix":    # 50/50 random + tiles216, Fisher-Yates shuffled by xorshift32(0x5EED)
                order = [(kind, seed0 + b) for b, kind in enumerate(mix_order(n))]
            else:               # clustered 50/50 over all ranks' blocks, dealt out interleaved
                from lz4mi import shard
                kinds = shard.clustered_mix_kinds(n * world)
                order = [(kinds[g], 1 + g) for g in shard.shard_interleaved(n * world, rank, world)]
            tmp = torch.empty(BLOCK, dtype=torch.uint8, device=dev)
            for b, (kind, seed) in enumerate(order):
                lz4mi.generate_blocks_dev(tmp.data_ptr(), kind, seed, BLOCK, 1, stream)
                self.raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
        else:
            lz4mi.generate_blocks_dev(self.raw.data_ptr(), gen, seed0, BLOCK, n, stream)
        self.slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
        self.comp = torch.empty(n * self.slot, dtype=torch.uint8, device=dev)
        self.raw_off = torch.arange(n, dtype=torch.int64, device=dev) * BLOCK
        self.raw_len = torch.full((n,), BLOCK, dtype=torch.int32, device=dev)
        self.comp_off = torch.arange(n, dtype=torch.int64, device=dev) * self.slot
        self.comp_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.dec = torch.empty(n * BLOCK, dtype=torch.uint8, device=dev)
        self.dec_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.status = torch.zeros(n, dtype=torch.int32, device=dev)

    def compress(self, lz4mi, stream):
        lz4mi.compress_blocks_dev(self.raw.data_ptr(), self.raw_off.data_ptr(), self.raw_len.data_ptr(),
                                  self.comp.data_ptr(), self.comp_off.data_ptr(), self.comp_len.data_ptr(),
                                  self.n, stream)

    def decompress(self, lz4mi, stream):
        lz4mi.decompress_blocks_dev(self.comp.data_ptr(), self.comp_off.data_ptr(), self.comp_len.data_ptr(),
                                    self.dec.data_ptr(), self.raw_off.data_ptr(), self.raw_len.data_ptr(),
                                    self.dec_len.data_ptr(), self.status.data_ptr(), self.n, stream)

    def decompress_reference(self, lz4mi, stream):
        """The same launch with the reference decoder's bytes (LZ4MI_JS_EXACT, the JS layer's default)."""
        lz4mi.decompress_blocks_dev(self.comp.data_ptr(), self.comp_off.data_ptr(), self.comp_len.data_ptr(),
                                    self.dec.data_ptr(), self.raw_off.data_ptr(), self.raw_len.data_ptr(),
                                    self.dec_len.data_ptr(), self.status.data_ptr(), self.n, stream, js_exact=True)

    def verify(self, torch, lz4mi, stream):
        """Per-block xxh32 of the decoded bytes == of the generated bytes (GPU)."""
        h1 = torch.zeros(self.n, dtype=torch.int32, device="cuda")
        h2 = torch.zeros(self.n, dtype=torch.int32, device="cuda")
        lz4mi.xxh32_blocks_dev(self.raw.data_ptr(), self.raw_off.data_ptr(), self.raw_len.data_ptr(),
                               h1.data_ptr(), self.n, 0, stream)
        lz4mi.xxh32_blocks_dev(self.dec.data_ptr(), self.raw_off.data_ptr(), self.dec_len.data_ptr(),
                               h2.data_ptr(), self.n, 0, stream)
        torch.cuda.synchronize()
        return bool((self.status == 0).all().item()) and bool(torch.equal(h1, h2)) and \
            bool((self.dec_len == BLOCK).all().item())


def reference_mode(torch, lz4mi, batch, stream_obj, gen, seed0, steps=5):
    """the headline batch decoded with the reference decoder's bytes
    (LZ4MI_JS_EXACT: the spec kernel plus the in-chunk replay of the double-copy-tail rewrites,
    SURVEY F1), timed like the headline (HIP events on the launch stream). Checked against the
    reference's own census of this batch (tests/golden/manifest.json 'bench_batch_js_decode',
    generated by executing the reference: per-block digests of its decode, each block in an array of
    its own): every block's XXH32 (GPU) must equal it. A block whose rewrite reaches before its own
    output reports LZ4MI_ERR_CROSS_BLOCK in the batch and is decoded alone into a scratch block,
    as the JS layer does (`cross_block_ms`)."""
    s = stream_obj.cuda_stream
    _, k = timed(torch, None, lambda: batch.decompress_reference(lz4mi, s), steps, 1, stream_obj)
    n = batch.n
    st = batch.status.cpu().tolist()
    cross = [b for b in range(n) if st[b] == lz4mi.ERR_CROSS_BLOCK]
    h = torch.zeros(n, dtype=torch.int32, device="cuda")
    lz4mi.xxh32_blocks_dev(batch.dec.data_ptr(), batch.raw_off.data_ptr(), batch.dec_len.data_ptr(), h.data_ptr(),
                           n, 0, s)
    hr = torch.zeros(n, dtype=torch.int32, device="cuda")
    lz4mi.xxh32_blocks_dev(batch.raw.data_ptr(), batch.raw_off.data_ptr(), batch.raw_len.data_ptr(), hr.data_ptr(),
                           n, 0, s)
    torch.cuda.synchronize()
    h, hr = [int(x) & 0xFFFFFFFF for x in h.tolist()], [int(x) & 0xFFFFFFFF for x in hr.tolist()]
    lens = batch.dec_len.cpu().tolist()
    cross_ms = 0.0
    if cross:
        one = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
        z64 = torch.zeros(1, dtype=torch.int64, device="cuda")
        cap = torch.full((1,), BLOCK, dtype=torch.int32, device="cuda")
        ol, os_ = torch.zeros(1, dtype=torch.int32, device="cuda"), torch.zeros(1, dtype=torch.int32, device="cuda")
        hh = torch.zeros(1, dtype=torch.int32, device="cuda")
        for b in cross:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream_obj)
            lz4mi.decompress_blocks_dev(batch.comp.data_ptr() + b * batch.slot, z64.data_ptr(),
                                        batch.comp_len.data_ptr() + 4 * b, one.data_ptr(), z64.data_ptr(),
                                        cap.data_ptr(), ol.data_ptr(), os_.data_ptr(), 1, s, js_exact=True)
            e1.record(stream_obj)
            lz4mi.xxh32_blocks_dev(one.data_ptr(), z64.data_ptr(), ol.data_ptr(), hh.data_ptr(), 1, 0, s)
            torch.cuda.synchronize()
            cross_ms += e0.elapsed_time(e1)
            st[b], lens[b], h[b] = int(os_.item()), int(ol.item()), int(hh.item()) & 0xFFFFFFFF
    ok = all(x == 0 for x in st) and all(x == BLOCK for x in lens)
    fixed = sum(1 for b in range(n) if h[b] != hr[b])
    census = None
    try:
        with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
            census = [c for c in json.load(f)["cases"] if c["kind"] == "bench_batch_js_decode"][0]
    except (OSError, ValueError, IndexError):
        pass
    checked = 0
    if census is not None and gen == "tiles216" and census["gen"] == gen:
        rows = {r["seed"]: int(r["js_dec_xxh"], 16) for r in census["rows"]}
        lo, hi = census["seeds"]
        for b in range(n):
            sd = seed0 + b
            if lo <= sd <= hi:
                ok &= h[b] == rows.get(sd, hr[b])
                checked += 1
    comp_bytes = int(batch.comp_len.sum().item())
    return {"kernel_ms": round(k * 1e3, 3), "GBps": round(n * BLOCK / k / 1e9, 1),
            "frac": round((n * BLOCK + comp_bytes) / k / 1e9 / HBM_PEAK_GBPS, 4),
            "blocks_fixed_up": fixed, "cross_block_blocks": len(cross), "cross_block_ms": round(cross_ms, 3),
            "verified": bool(ok and checked == n), "blocks_checked_vs_reference_census": checked,
            "note": "LZ4MI_JS_EXACT (the JS layer's default): the reference decoder's bytes, double-copy-tail "
                    "rewrites (SURVEY F1) included; blocks_fixed_up = blocks whose output differs from their "
                    "input (the reference's own decode of them differs too); every block's XXH32 checked against "
                    "the reference's census of seeds 1..4096 (tests/golden, made by executing the reference)"}


def mix_order(n):
    x = 0x5EED
    kinds = ["random"] * (n // 2) + ["tiles216"] * (n - n // 2)
    for i in range(n - 1, 0, -1):
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        j = x % (i + 1)
        kinds[i], kinds[j] = kinds[j], kinds[i]
    return kinds


def timed(torch, dist, fn, steps, warmup, stream_obj):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream_obj)
    for _ in range(steps):
        fn()
    ev1.record(stream_obj)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = ev0.elapsed_time(ev1) / 1e3 / steps       # average launch duration on the launch stream
    return wall, kern


def frame_workload(torch, dist, lz4mi, stream_obj, world, rank, blocks_per_rank):
    """BASELINE.json configs[3]: one LZ4 frame (independent 4 MiB blocks, content size and
    content checksum: FLG 0x6C, BD 0x70) over every rank's tiles216 shard, assembled on rank 0,
    then decoded with its blocks shared out again (lz4mi.frame). 2048 blocks per rank make
    the 64 GiB frame of configs[3] at 8 GPUs. One untimed warm-up frame (no checksums) first, so
    the codec's buffers and the library's scratch exist before the timed frame. Each phase is
    closed by a barrier and reported separately; `kernel_ms` is the kernels' HIP-event time on
    the codec stream (max over ranks), `phases_ms` the barrier-closed wall times. The content
    checksum (one serial XXH32 chain on rank 0's host) runs beside the kernel and the collective
    in compress, beside the output gather in decompress: `checksum_chain_ms` is its own
    duration, `checksum_wait` what it adds after the other work."""
    from lz4mi import frame as F
    dev = torch.device("cuda", torch.cuda.current_device())
    n = blocks_per_rank
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device=dev)
    lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 1 + rank * n, BLOCK, n, stream_obj.cuda_stream)
    torch.cuda.synchronize()
    codec = F.DeviceCodec(stream_obj)
    decoder = F.DeviceDecoder(stream_obj)
    # warm-up: the same frame without checksums (allocations, scratch growth, first launches)
    w = F.compress_frame_sharded(raw, BLOCK, content_checksum=False, add_content_size=True, codec=codec)
    w = F.decompress_frame_sharded(w, verify_checksum=False, decoder=decoder, device=dev, gather=True, zero_copy=True)
    del w
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    tc = {}
    t0 = time.perf_counter()
    frame = F.compress_frame_sharded(raw, BLOCK, content_checksum=True, add_content_size=True, codec=codec, timings=tc)
    c_total = time.perf_counter() - t0
    fbytes = torch.tensor([frame.numel() if frame is not None else 0], dtype=torch.int64, device=dev)
    if dist is not None:
        dist.all_reduce(fbytes)
        dist.barrier()
    ts = {}     # sharded result (gather=False): each rank keeps its decoded run
    t0 = time.perf_counter()
    part = F.decompress_frame_sharded(frame, verify_checksum=True, decoder=decoder, timings=ts, device=dev, gather=False, zero_copy=True)
    d_sharded = time.perf_counter() - t0
    del part
    if dist is not None:
        dist.barrier()
    td = {}
    t0 = time.perf_counter()
    out = F.decompress_frame_sharded(frame, verify_checksum=True, decoder=decoder, timings=td, device=dev, gather=True, zero_copy=True)
    d_total = time.perf_counter() - t0
    total_raw = world * n * BLOCK
    ok = torch.tensor([1], dtype=torch.int32, device=dev)
    if rank == 0:   # the checksum inside the decode checked every byte; the root's own shard once more
        ok[0] = int(out.numel() == total_raw and bool(torch.equal(out[:n * BLOCK], raw)))
    kd = torch.tensor([tc.get("kernel_device", 0.0), td.get("kernel_device", 0.0)], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.broadcast(ok, src=0)
        dist.all_reduce(kd, op=dist.ReduceOp.MAX)
    del out, frame, raw, codec, decoder
    torch.cuda.empty_cache()
    ms = lambda v: round(v * 1e3, 2)
    gbps = lambda v: round(total_raw / v / 1e9, 2) if v > 0 else None
    ck, dk = float(kd[0]), float(kd[1])
    c_coll = tc.get("kernel", 0.0) + tc.get("collective", 0.0)
    d_coll = td.get("index", 0.0) + td.get("scatter", 0.0) + td.get("kernel", 0.0)
    phases = lambda t: {k: ms(v) for k, v in t.items() if k not in ("kernel_device", "checksum_chain")}
    return {
        "workload": f"LZ4 frame (independent 4 MiB blocks, content size + content xxh32), {n} tiles216 blocks "
                    f"per rank x {world} rank(s) = {total_raw / 2**30:.0f} GiB; assembled on rank 0, then decoded "
                    f"sharded (contiguous block runs of equal decode cost) and gathered back to rank 0 (BASELINE.json configs[3])",
        "raw_bytes": total_raw, "frame_bytes": int(fbytes.item()), "verified": bool(ok.item()),
        "compress": {"kernel_ms": ms(ck), "kernel_collective_ms": ms(c_coll),
                     "checksum_chain_ms": ms(tc.get("checksum_chain", 0.0)),
                     "end_to_end_ms": ms(c_total), "phases_ms": phases(tc),
                     "kernel_GBps": gbps(ck), "kernel_collective_GBps": gbps(c_coll),
                     "end_to_end_GBps": gbps(c_total)},
        "decompress": {"kernel_ms": ms(dk), "kernel_collective_ms": ms(d_coll),
                       "checksum_chain_ms": ms(td.get("checksum_chain", 0.0)),
                       "end_to_end_ms": ms(d_total), "end_to_end_sharded_ms": ms(d_sharded),
                       "phases_ms": phases(td), "phases_sharded_ms": phases(ts),
                       "kernel_GBps": gbps(dk), "kernel_collective_GBps": gbps(d_coll),
                       "end_to_end_GBps": gbps(d_total), "end_to_end_sharded_GBps": gbps(d_sharded)},
        "collective": ("all_gather(byte counts) + send/recv of records to rank 0; decode: broadcast of the block "
                       "index, send of each rank's frame bytes, send/recv of outputs to rank 0") if world > 1 else None,
        "checksum": "serial XXH32 on rank 0's host over host-staged shards (/dev/shm), one core, overlapped: "
                    "from t0 beside the compress kernel + collective, beside the output gather in decompress",
        "sharded_note": "end_to_end_sharded: a second timed decode of the same frame with gather=False (each rank "
                        "keeps its decoded run: the natural sharded result), checksum verified as in the gathered one",
    }


def latency_curve(torch, lz4mi, batch, stream_obj, counts=(1, 16, 64, 128, 192, 256, 2048, 4096), reps=3):
    """device-resident time (HIP events on the launch stream, median of `reps`)
    of the first b blocks of the headline batch, decode and compress. Decode of <= 192 blocks takes
    the small-batch path (a wave per ~8 KiB segment: segment-parallel parse, output by pointer jumping,
    csrc/lz4mi_expand.hip); larger batches the batch kernel (one wave per block, every block
    resident: the time is one block's chain latency under the CU's contention). Compress is one
    wave per block at every size."""
    s = stream_obj.cuda_stream
    res = {"blocks": [], "decompress_ms": [], "decompress_reference_ms": [], "compress_ms": []}

    def med(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream_obj)
            fn()
            e1.record(stream_obj)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(sorted(ts)[len(ts) // 2], 3)
    scratch = torch.empty(batch.comp.numel(), dtype=torch.uint8, device="cuda")
    slen = torch.zeros(batch.n, dtype=torch.int32, device="cuda")
    for b in counts:
        if b > batch.n:
            continue
        res["blocks"].append(b)
        res["decompress_ms"].append(med(lambda: lz4mi.decompress_blocks_dev(
            batch.comp.data_ptr(), batch.comp_off.data_ptr(), batch.comp_len.data_ptr(), batch.dec.data_ptr(),
            batch.raw_off.data_ptr(), batch.raw_len.data_ptr(), batch.dec_len.data_ptr(), batch.status.data_ptr(), b, s)))
        res["decompress_reference_ms"].append(med(lambda: lz4mi.decompress_blocks_dev(   # (the JS layer's default)
            batch.comp.data_ptr(), batch.comp_off.data_ptr(), batch.comp_len.data_ptr(), batch.dec.data_ptr(),
            batch.raw_off.data_ptr(), batch.raw_len.data_ptr(), batch.dec_len.data_ptr(), batch.status.data_ptr(), b, s,
            js_exact=True)))
        res["compress_ms"].append(med(lambda: lz4mi.compress_blocks_dev(
            batch.raw.data_ptr(), batch.raw_off.data_ptr(), batch.raw_len.data_ptr(), scratch.data_ptr(),
            batch.comp_off.data_ptr(), slen.data_ptr(), b, s)))
    del scratch
    torch.cuda.empty_cache()
    thr = lz4mi.SMALL_BLOCKS   # (the library's default, lz4mi_capi.cpp, or LZ4MI_SMALL_BLOCKS)
    res["decompress_path"] = ["small-batch" if b <= thr else "batch kernel" for b in res["blocks"]]
    res["note"] = (f"device-resident, HIP events; the first b blocks of the headline batch; decode of <= {thr} "
                   "blocks: small-batch path (LZ4MI_SMALL_BLOCKS), else the batch kernel; decompress_reference_ms: "
                   "LZ4MI_JS_EXACT, the reference decoder's bytes (the JS layer's default)")
    return res


def mix_frame(torch, lz4mi, stream_obj, n):
    """a frame of the 50/50 random/tiles216 mix (n blocks: the random ones are
    stored blocks) decoded by DeviceDecoder (compressed blocks in one batch, stored ones in one
    copy launch: `frame_kernel_ms` spans both) beside the batch decode of the same blocks
    (every block an LZ4 block, one lz4mi_decompress_blocks launch)."""
    from lz4mi import frame as F
    s = stream_obj.cuda_stream
    raw = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    tmp = torch.empty(BLOCK, dtype=torch.uint8, device="cuda")
    for b, kind in enumerate(mix_order(n)):
        lz4mi.generate_blocks_dev(tmp.data_ptr(), kind, 1 + b, BLOCK, 1, s)
        raw[b * BLOCK:(b + 1) * BLOCK].copy_(tmp)
    del tmp
    torch.cuda.synchronize()
    codec = F.DeviceCodec(stream_obj)
    dec = F.DeviceDecoder(stream_obj)
    frame = F.compress_frame_sharded(raw, BLOCK, content_checksum=False, codec=codec)
    meta, pay, word = F.frame_index(frame)
    stored = int(((word & 0x80000000) != 0).sum().item())
    ks = []
    ok = True
    for _ in range(4):
        out = F.decompress_frame_sharded(frame, verify_checksum=False, decoder=dec, gather=False, zero_copy=True)
        ks.append(dec.last_kernel_s * 1e3)
    ok = bool(torch.equal(out, raw))
    del out, frame, codec, dec
    torch.cuda.empty_cache()
    b2 = Batch.__new__(Batch)
    b2.n, b2.raw = n, raw
    b2.slot = (lz4mi.compress_bound(BLOCK) + 255) & ~255
    b2.comp = torch.empty(n * b2.slot, dtype=torch.uint8, device="cuda")
    b2.raw_off = torch.arange(n, dtype=torch.int64, device="cuda") * BLOCK
    b2.raw_len = torch.full((n,), BLOCK, dtype=torch.int32, device="cuda")
    b2.comp_off = torch.arange(n, dtype=torch.int64, device="cuda") * b2.slot
    b2.comp_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    b2.dec = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    b2.dec_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    b2.status = torch.zeros(n, dtype=torch.int32, device="cuda")
    b2.compress(lz4mi, s)
    torch.cuda.synchronize()
    _, kb = timed(torch, None, lambda: b2.decompress(lz4mi, s), 3, 1, stream_obj)
    ok = ok and b2.verify(torch, lz4mi, s)
    del b2, raw
    torch.cuda.empty_cache()
    fk = sorted(ks[1:])[1]
    return {"blocks": n, "stored_blocks": stored, "frame_kernel_ms": round(fk, 3),
            "batch_kernel_ms": round(kb * 1e3, 3), "frame_over_batch": round(fk / (kb * 1e3), 3), "verified": ok}


def weak_scaling(torch, dist, walls, kern_s, bytes_per_rank, steps, device):
    """The bench's aggregation: every rank's timed-region wall times (`walls`, seconds) are
    max-reduced, value = all ranks' bytes / the slowest rank's wall (weak scaling: each rank
    has its own fixed batch); the per-rank kernel times are gathered so imbalance (the
    skewed mix) shows. Returns (max walls, value GB/s, per-rank kernel ms lists)."""
    world = dist.get_world_size() if dist is not None else 1
    t = torch.tensor(list(walls), dtype=torch.float64, device=device)
    k = torch.tensor(list(kern_s), dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ks = [torch.zeros_like(k) for _ in range(world)]
        dist.all_gather(ks, k)
    else:
        ks = [k]
    mx = [float(x) for x in t.tolist()]
    value = world * bytes_per_rank * steps / mx[0] / 1e9
    per_rank = [[round(float(x) * 1e3, 3) for x in kk.tolist()] for kk in ks]
    return mx, value, [list(col) for col in zip(*per_rank)]


def cpu_threads():
    """The host cores this job may use: the box exports OMP_NUM_THREADS (its CPU share)."""
    n = os.environ.get("OMP_NUM_THREADS")
    return max(1, int(n)) if n and n.isdigit() else (os.cpu_count() or 1)


def js_cpu_baseline(gen, blocks):
    """The pure-JS path (oracle/lz4_js.mjs: our restatement of the reference's
    compressBlock/decompressBlock, checked against the reference's digests first) on
    worker_threads over the host's cores, `blocks` distinct 4 MiB blocks per thread."""
    threads = cpu_threads()
    r = subprocess.run(["node", "--no-warnings", os.path.join(ROOT, "oracle", "js_cpu_baseline.mjs"), gen,
                        str(threads), str(blocks), os.path.join(ROOT, "tests", "golden", "manifest.json")],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": d["decompress_GBps"], "unit": "GB/s", "cores": threads, "kind": "port",
            "compress_GBps": d["compress_GBps"], "roundtrip_GBps": d["roundtrip_GBps"],
            "sample": f"pure-JS block codec (oracle/lz4_js.mjs, restatement of blockCompress.js/blockDecompress.js, "
                      f"bit-exact on {d['golden_digests_checked']} reference 4 MiB digests), {threads} worker_threads "
                      f"x {blocks} distinct 4 MiB {gen} blocks each, compress then decompress; node {d['node']}, "
                      f"{d['cpu_model']}; verified={d['verified']}"}


def c_cpu_baseline(batch, threads, target_s=1.5):
    """The C oracle decoder (restatement of blockDecompress.js) on host cores over a
    bounded sample of the same compressed blocks (second baseline key)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    nb = min(batch.n, 256)
    lens = batch.comp_len[:nb].cpu().numpy().astype(np.uint32)
    comp = batch.comp[:nb * batch.slot].cpu().numpy()
    in_off = (np.arange(nb, dtype=np.uint64) * np.uint64(batch.slot))
    out = np.empty(nb * BLOCK, dtype=np.uint8)
    out_off = np.arange(nb, dtype=np.uint64) * np.uint64(BLOCK)
    out_cap = np.full(nb, BLOCK, dtype=np.uint32)
    reps, t0 = 0, time.perf_counter()
    while True:
        _, st = O.blocks_mt(0, comp, in_off, lens, out, out_off, out_cap, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    assert (st == 0).all()
    gbps = reps * nb * BLOCK / el / 1e9
    # the baseline doubles as a checker of the GPU's results at the bench's scale: its decode of
    # the GPU-compressed blocks equals the generated bytes, and the oracle encoder's bytes for a
    # few of those blocks equal the GPU encoder's (compressBlock is deterministic)
    raw = batch.raw[:nb * BLOCK].cpu().numpy()
    dec_ok = bool(np.array_equal(out, raw))
    ncmp = min(nb, 8)
    comp_ok = all(np.array_equal(O.compress_block_bytes(raw[b * BLOCK:(b + 1) * BLOCK]),
                                 comp[b * batch.slot:b * batch.slot + int(lens[b])]) for b in range(ncmp))
    return {"value": round(gbps, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"oracle C decoder, {nb} x 4 MiB blocks of the same compressed batch, {reps} passes, "
                      f"{threads} pthreads, {el:.1f} s wall",
            "oracle_check": {"decoded_equal_generated_blocks": nb, "decoded_ok": dec_ok,
                             "compressed_equal_oracle_blocks": ncmp, "compressed_ok": bool(comp_ok)}}


def napi_e2e(batch, nblocks=128):
    """LZ4.compress/decompress of the JS drop-in on host buffers (N-API -> liblz4mi), on
    the first `nblocks` generated blocks: PCIe-inclusive, reported beside the bench."""
    import tempfile
    path = os.path.join(tempfile.gettempdir(), f"lz4mi_napi_{os.getpid()}.bin")
    try:
        batch.raw[:nblocks * BLOCK].cpu().numpy().tofile(path)
        r = subprocess.run(["node", "--no-warnings", "--expose-gc", os.path.join(ROOT, "tools", "napi_e2e.mjs"), path, "3"],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr[-500:]}
        return json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        if os.path.exists(path):
            os.remove(path)


def reference_benchmark(with_js):
    """The reference's own published benchmark shape (docs/BENCHMARKS.md: LZ4.compress /
    decompress of 25 MB of repeated JSON, 4 MiB independent blocks) through the drop-in
    (tools/json_workload.mjs, host buffers, PCIe-inclusive), the pure-JS block codec on one
    core of this box on the same data (cpu_baseline leg), and the published numbers."""
    r = subprocess.run(["node", "--no-warnings", os.path.join(ROOT, "tools", "json_workload.mjs"), "25", "5"],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    out = {"workload": "LZ4.compress(x, null, 4194304, true, false) / LZ4.decompress of 25 MiB of one JSON record "
                       "repeated (the shape of the reference's benchmark data), host buffers through N-API; MB = 2^20 B",
           "routes": "drop_in.auto: the default routing (7 blocks: below both crossovers, so the host codec; the "
                     "*_route counts say which side each call took); drop_in.gpu: every block call forced onto the "
                     "GPU kernels (LZ4.setRouting('gpu')) - the GPU's figure for this call size",
           "drop_in": json.loads(r.stdout.strip().splitlines()[-1]),
           "published_reference_MBps": {"compress_25MB": 484, "decompress_25MB": 459,
                                        "hardware": "MacBook Pro mid-2015 (i7 quad, Node 24), docs/BENCHMARKS.md"}}
    if with_js:
        j = subprocess.run(["node", "--no-warnings", os.path.join(ROOT, "oracle", "js_cpu_baseline.mjs"), "json", "1", "6"],
                           capture_output=True, text=True, timeout=600)
        if j.returncode == 0:
            d = json.loads(j.stdout.strip().splitlines()[-1])
            out["pure_js_1core_MBps"] = {"compress": round(d["compress_GBps"] * 1e9 / (1 << 20), 1),
                                         "decompress": round(d["decompress_GBps"] * 1e9 / (1 << 20), 1),
                                         "sample": "oracle/lz4_js.mjs block codec, 6 x 4 MiB blocks, 1 worker_thread, "
                                                   f"{d['cpu_model']}, node {d['node']}"}
    return out


def single_block(torch, lz4mi, batch, reps=5):
    """Raw-block calls through the C-ABI with host buffers (LZ4.compressRaw / LZ4.decompressRaw:
    lz4mi_compress_block_table — the chain kernel with the caller's table in LDS — and
    lz4mi_decompress_blocks with nblocks = 1), PCIe included, median of `reps` calls, beside the
    host encoder/decoder (lz4mi_host_compress_block / lz4mi_host_decompress_block, the layer's
    route for serial-chain calls) on the same bytes, at 64 KiB, 1 MiB and 4 MiB (prefixes of one
    tiles216 block): the GPU/host crossover of DESIGN §5. Latency, not throughput: one block is
    one wave."""
    import numpy as np
    src_all = batch.raw[:BLOCK].cpu().numpy()

    def med(fn):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        return r, round(sorted(ts)[len(ts) // 2] * 1e3, 3)

    res, ok = {}, True
    for size in (65536, 1 << 20, BLOCK):
        src = np.ascontiguousarray(src_all[:size])
        out = np.zeros(lz4mi.compress_bound(size), dtype=np.uint8)
        row, comp = {}, None
        for name, fn in (("compressRaw_gpu", lz4mi.compress_raw), ("compressRaw_host", lz4mi.host_compress_raw)):
            n, row[name + "_ms"] = med(lambda: fn(src, out, 0, size, np.zeros(16384, dtype=np.int32), 0))
            if comp is None:
                comp = out[:n].copy()
            ok &= bool(np.array_equal(out[:n], comp))
        dec = np.zeros(size, dtype=np.uint8)
        for name, fn in (("decompressRaw_gpu", lambda: lz4mi.decompress_raw(comp, 0, comp.size, dec, 0)),
                         ("decompressRaw_host", lambda: lz4mi.host_decompress_raw(comp, 0, comp.size, dec, 0))):
            dec[:] = 0
            w, row[name + "_ms"] = med(fn)
            ok &= bool(w == size and np.array_equal(dec, src))
        if size == BLOCK:
            res.update(row)
        else:
            res["%d_KiB" % (size >> 10)] = row
    res["verified"] = ok
    res["workload"] = ("one tiles216 block of the bench's batch (and its 64 KiB / 1 MiB prefixes), host buffers, "
                       "fresh table, median of %d calls" % reps)
    return res


def pmc_traffic(lz4mi, n, gen, name="pmc_traffic.json"):
    """HBM bytes per launch (decode: pmc_traffic.json, compress: pmc_traffic_compress.json)
    from the committed rocprofv3 PMC passes, used only when they were measured on this exact
    build and workload (else null)."""
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, None
    if pm.get("workload_blocks") == n and pm.get("generator") == gen and pm.get("build_id") == lz4mi.build_id():
        return pm.get("hbm_bytes_per_launch"), pm.get("source")
    return None, None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args)
    import torch
    import lz4mi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        # (rehearsal hook: LZ4MI_BENCH_SHARE_GPU=1 puts every rank on the GPUs there are, round robin, so the
        # multi-rank path runs on a 1-GPU box; LZ4MI_BENCH_BACKEND picks the process group backend)
        if os.environ.get("LZ4MI_BENCH_SHARE_GPU") == "1":
            local %= torch.cuda.device_count()
        torch.cuda.set_device(local)
        dist_mod.init_process_group(os.environ.get("LZ4MI_BENCH_BACKEND", "nccl"), device_id=torch.device("cuda", local))
        dist = dist_mod
    else:
        torch.cuda.set_device(0)
    lz4mi.init(torch.cuda.current_device())
    # a dedicated stream: the kernels and the timing events share it
    stream_obj = torch.cuda.Stream()
    torch.cuda.set_stream(stream_obj)
    stream = stream_obj.cuda_stream

    n = args.blocks
    batch = Batch(torch, lz4mi, n, args.gen, 1 + rank * n, stream, rank, world)
    # compress (bit-exact encoder) — timed too, it is the other half of the metric
    batch.compress(lz4mi, stream)
    torch.cuda.synchronize()
    c_wall, c_kern = timed(torch, dist, lambda: batch.compress(lz4mi, stream), args.compress_steps, 0, stream_obj)
    comp_bytes = int(batch.comp_len.sum().item())
    raw_bytes = n * BLOCK

    d_wall, d_kern = timed(torch, dist, lambda: batch.decompress(lz4mi, stream), args.steps, args.warmup, stream_obj)
    ok = batch.verify(torch, lz4mi, stream)
    ref_mode = reference_mode(torch, lz4mi, batch, stream_obj, args.gen, 1 + rank * n) if rank == 0 else None

    okt = torch.tensor([0 if ok else 1], dtype=torch.int32, device="cuda")
    if dist is not None:
        dist.all_reduce(okt, op=dist.ReduceOp.MAX)
    (d_wall, c_wall), value, per_rank_ms = weak_scaling(torch, dist, (d_wall, c_wall), (d_kern, c_kern), raw_bytes,
                                                        args.steps, "cuda")
    ms_per_step = d_wall / args.steps * 1e3

    lat = latency_curve(torch, lz4mi, batch, stream_obj) if args.extra and rank == 0 and world == 1 else None
    napi = napi_e2e(batch) if args.napi and rank == 0 and world == 1 else None
    single = single_block(torch, lz4mi, batch) if args.napi and rank == 0 and world == 1 else None
    c_base = c_cpu_baseline(batch, cpu_threads()) if args.cpu_baseline and rank == 0 and world == 1 else None

    extra = {}
    if args.extra and rank == 0 and world == 1:
        del batch.dec
        for g in (["random", "repetitive", "mix", "mixc"] if args.gen == "tiles216" else []):
            nb = n                      # same occupancy as the headline workload
            b2 = Batch(torch, lz4mi, nb, g, 1, stream)
            b2.compress(lz4mi, stream)
            torch.cuda.synchronize()
            w, k = timed(torch, None, lambda: b2.decompress(lz4mi, stream), 5, 1, stream_obj)
            cw, ck = timed(torch, None, lambda: b2.compress(lz4mi, stream), 1, 0, stream_obj)
            cb = int(b2.comp_len.sum().item())
            extra[g] = {"blocks": nb, "ratio": round(nb * BLOCK / cb, 3),
                        "decompress_GBps": round(nb * BLOCK / k / 1e9, 1),
                        "decompress_hbm_frac": round((nb * BLOCK + cb) / k / 1e9 / HBM_PEAK_GBPS, 4),
                        "compress_GBps": round(nb * BLOCK / ck / 1e9, 2),
                        "roundtrip_GBps": round(nb * BLOCK / (ck + k) / 1e9, 2),
                        "verified": b2.verify(torch, lz4mi, stream)}
            # the batch's first block alone (the small-batch decode path)
            _, k1 = timed(torch, None, lambda: lz4mi.decompress_blocks_dev(
                b2.comp.data_ptr(), b2.comp_off.data_ptr(), b2.comp_len.data_ptr(), b2.dec.data_ptr(),
                b2.raw_off.data_ptr(), b2.raw_len.data_ptr(), b2.dec_len.data_ptr(), b2.status.data_ptr(), 1,
                stream), 3, 1, stream_obj)
            extra[g]["lone_block_decompress_ms"] = round(k1 * 1e3, 3)
            del b2
            torch.cuda.empty_cache()
        batch.dec = torch.empty(1, dtype=torch.uint8, device="cuda")

    frame = None
    if args.frame_blocks > 0:
        del batch
        torch.cuda.empty_cache()
        try:
            frame = frame_workload(torch, dist, lz4mi, stream_obj, world, rank, args.frame_blocks)
        except Exception as e:    # reported, not fatal: every rank raises the same error (lz4mi.frame)
            frame = {"error": repr(e)[-500:]}
        if world == 1 and args.extra:
            try:
                frame["mix_frame"] = mix_frame(torch, lz4mi, stream_obj, args.frame_blocks)
            except Exception as e:
                frame["mix_frame"] = {"error": repr(e)[-500:]}
    achieved = (raw_bytes + comp_bytes) / d_kern / 1e9
    traffic, traffic_src = pmc_traffic(lz4mi, n, args.gen)
    c_traffic, _ = pmc_traffic(lz4mi, n, args.gen, "pmc_traffic_compress.json")
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic ({args.gen} generator, SURVEY.md §8d), generated and compressed on device",
        "config": {"workload": f"raw block decompress, {n} x 4 MiB independent blocks per GPU ({args.gen}), "
                               f"device-resident (BASELINE.json configs[1])",
                   "blocks_per_gpu": n, "block_bytes": BLOCK, "generator": args.gen,
                   "compression_ratio": round(raw_bytes / comp_bytes, 3), "parallelism": f"blocks sharded x{world}"},
        "verified": okt.item() == 0,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "kernel": "lz4mi_decompress_kernel", "kernel_ms": round(d_kern * 1e3, 3),
                     "algorithmic_bytes_per_launch": raw_bytes + comp_bytes},
        "value_is": "decompress GB/s of uncompressed bytes (the north-star target); compress and the "
                    "round trip (compress then decompress of the same bytes) are under 'compress' and "
                    "'roundtrip_GBps'",
        "compress": {"GBps": round(world * raw_bytes / c_wall * args.compress_steps / 1e9, 2),
                     "kernel": "lz4mi_compress_gts_kernel", "kernel_ms": round(c_kern * 1e3, 3),
                     "hbm_frac": round((raw_bytes + comp_bytes) / c_kern / 1e9 / HBM_PEAK_GBPS, 4),
                     "algorithmic_bytes_per_launch": raw_bytes + comp_bytes, "traffic": c_traffic},
        "roundtrip_GBps": round(world * raw_bytes / (c_wall / args.compress_steps + d_wall / args.steps) / 1e9, 2),
        "build_id": lz4mi.build_id(),
    }
    if traffic_src:
        line["roofline"]["traffic_source"] = traffic_src
    if ref_mode is not None:
        line["reference_mode"] = ref_mode
    if world > 1:   # every rank's average launch time: the imbalance the max hides
        line["per_rank_kernel_ms"] = {"decompress": per_rank_ms[0], "compress": per_rank_ms[1]}
    if frame is not None:
        line["frame"] = frame
    if extra:
        line["variants"] = extra
    if lat is not None:
        line["latency_curve"] = lat
    if single is not None:
        line["single_block"] = single
    if napi is not None:
        line["napi_end_to_end"] = napi
        line["reference_benchmark"] = reference_benchmark(bool(args.cpu_baseline))
    if args.cpu_baseline and rank == 0 and world == 1:
        line["cpu_baseline"] = js_cpu_baseline(args.gen if args.gen in ("tiles216", "random", "repetitive")
                                               else "tiles216", args.cpu_blocks)
        line["cpu_baseline_c_oracle"] = c_base
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
