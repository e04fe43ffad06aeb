"""Randomized stress of the small-batch decode path (tool): batches of 1..96 blocks from every
generator, sizes up to 4 MiB, 0..3 corrupted bytes per block, statuses and bytes against the
oracle's decode; `--seconds` of batches per run. LZ4MI_SMALL_REPARSE (0/1/2) in the environment
selects the re-parse test mode."""
import argparse, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
import oracle as O  # noqa: E402
import lz4mi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=60)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--dump", default="", help="directory: the first mismatching block's input and outputs (.npz), then stop")
args = ap.parse_args()
rng = np.random.default_rng(args.seed)
gens = ["tiles216", "text", "copy", "runs", "random", "repetitive"]
pool = []
for t in range(24):   # a pool of compressed blocks, reused with fresh corruptions
    n = int(rng.choice([100, 5000, 65536, 300000, 1 << 20, 3 << 20, 4 << 20]))
    s = O.generate(gens[t % len(gens)], 500 + t, n)
    pool.append((s, O.compress_block_bytes(s)))
t0, batches, blocks, bad = time.time(), 0, 0, 0
while time.time() - t0 < args.seconds:
    k = int(rng.integers(1, 97))
    sel = rng.integers(0, len(pool), k)
    comps, caps, srcs = [], [], []
    for i in sel:
        s, c = pool[int(i)]
        c = c.copy()
        for _ in range(int(rng.choice([0, 0, 1, 2, 3]))):
            if c.size:
                c[rng.integers(0, c.size)] = rng.integers(0, 256)
        comps.append(c)
        caps.append(s.size + int(rng.choice([0, 0, 0, 7, -3 if s.size > 3 else 0])))
        srcs.append(s)
    st, outs, lens = lz4mi.decompress_blocks(comps, caps)
    for j, c in enumerate(comps):
        est, ew, eo = O.decompress_block(c, caps[j])
        if st[j] == lz4mi.ERR_CROSS_BLOCK and est == lz4mi.ERR_DICT_OOB:
            continue
        ok = st[j] == est and (est != 0 or (lens[j] == ew and np.array_equal(outs[j], eo[:min(ew, caps[j])])))
        if not ok:
            bad += 1
            print("MISMATCH batch", batches, "block", j, "status", int(st[j]), "oracle", int(est),
                  "len", int(lens[j]), int(ew), flush=True)
            if args.dump:
                os.makedirs(args.dump, exist_ok=True)
                np.savez(os.path.join(args.dump, "mismatch.npz"), comp=c, cap=np.array([caps[j]]), got=outs[j],
                         want=eo[:min(ew, caps[j])], batch_comps=np.array([x.size for x in comps]), j=np.array([j]))
                print({"dumped": True, "batch_blocks": len(comps)}, flush=True)
                sys.exit(1)
    batches += 1
    blocks += k
print({"mode": os.environ.get("LZ4MI_SMALL_REPARSE", "0"), "batches": batches, "blocks": blocks, "mismatches": bad}, flush=True)
sys.exit(1 if bad else 0)
