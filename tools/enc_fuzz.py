"""Randomized encoder stress (tool): batches of blocks built from pieces of every generator,
repeats of earlier bytes at random distances, runs and literal stretches, compressed on the GPU and
by the oracle's compressBlock, byte for byte; batches of <= 768 blocks (LDS-table kernel) and of
more (global-table kernel, smaller blocks). `--seconds` of batches."""
import argparse, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
import oracle as O  # noqa: E402
import lz4mi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=60)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--big", action="store_true", help="batches of 769..900 blocks of <= 96 KiB (global-table kernel)")
args = ap.parse_args()
rng = np.random.default_rng(args.seed)
gens = ["tiles216", "text", "copy", "runs", "random", "repetitive"]


def block(n):
    out = np.empty(n + 70000, dtype=np.uint8)
    w = 0
    while w < n:
        kind = int(rng.integers(0, 4))
        m = int(rng.choice([1, 3, 15, 64, 300, 2048, 9000, 40000, int(rng.integers(1, 70000))]))
        if kind == 0 or w == 0:
            piece = O.generate(gens[int(rng.integers(0, len(gens)))], int(rng.integers(1, 1 << 30)), m)
        elif kind == 1:   # a repeat of earlier bytes (a match at a random distance)
            d = int(rng.integers(1, min(w, 70000) + 1))
            piece = np.resize(out[w - d:w], m)
        elif kind == 2:   # a run
            piece = np.full(m, rng.integers(0, 256), dtype=np.uint8)
        else:             # incompressible
            piece = rng.integers(0, 256, m, dtype=np.uint8)
        out[w:w + m] = piece.astype(np.uint8)
        w += m
    return out[:n].copy()


t0, batches, blocks, bad = time.time(), 0, 0, 0
t_log = t0
while time.time() - t0 < args.seconds:
    if args.big:
        k = int(rng.integers(769, 901))
        sizes = [int(x) for x in rng.choice([0, 1, 13, 100, 5000, 65536, 98304], k)]
    else:
        k = int(rng.integers(1, 33))
        sizes = [int(x) for x in rng.choice([0, 13, 5000, 65536, 300000, 1 << 20, 4 << 20], k)]
    srcs = [block(n) for n in sizes]
    comps = lz4mi.compress_blocks(srcs)
    for j, (s, c) in enumerate(zip(srcs, comps)):
        ref = O.compress_block_bytes(s)
        if c.size != ref.size or not np.array_equal(c, ref):
            bad += 1
            print("MISMATCH batch", batches, "block", j, "size", s.size, "gpu", c.size, "oracle", ref.size, flush=True)
            np.save(os.path.join(ROOT, "gpurun_out", f"enc_mismatch_{args.seed}_{batches}_{j}.npy"), s)
    batches += 1
    blocks += k
    if time.time() - t_log > 30:   # progress (a run longer than 3 minutes must keep writing)
        t_log = time.time()
        print({"batches": batches, "blocks": blocks, "mismatches": bad}, flush=True)
print({"big": args.big, "batches": batches, "blocks": blocks, "mismatches": bad}, flush=True)
sys.exit(1 if bad else 0)
