"""Randomized stress of the small-batch decode path (tool): batches of 1..192 blocks from every
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
ap.add_argument("--min-blocks", type=int, default=1)
ap.add_argument("--max-blocks", type=int, default=192, help="above 192 (LZ4MI_SMALL_BLOCKS): the batch kernel")
ap.add_argument("--js-exact", action="store_true", help="reference mode (LZ4MI_JS_EXACT)")
ap.add_argument("--random-streams", action="store_true", help="pool of random valid streams (every field shape)")
ap.add_argument("--dump", default="", help="directory: the first mismatching block's input and outputs (.npz), then stop")
args = ap.parse_args()
rng = np.random.default_rng(args.seed)
gens = ["tiles216", "text", "copy", "runs", "random", "repetitive"]
def _len_field(v):
    r = v - 15
    return [255] * (r // 255) + [r % 255]


def random_stream(target):
    """A valid LZ4 block of about `target` decoded bytes from random sequences (as
    tests/test_gpu_fuzz.py's generator): (compressed, decoded size)."""
    out = bytearray()
    produced = 0
    while True:
        ll = int(rng.choice([0, 0, 0, 1, 3, 14, 15, 16, 100, 200, 269, 270, 300, int(rng.integers(0, 5000))]))
        if produced + ll + 4 + 12 > target:
            ll = max(target - produced, 5)
            tok = [min(ll, 15) << 4] + (_len_field(ll) if ll >= 15 else [])
            out += bytes(tok) + rng.integers(0, 256, ll, dtype=np.uint8).tobytes()
            return np.frombuffer(bytes(out), dtype=np.uint8), produced + ll
        hist = produced + ll
        off = int(rng.choice([1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 64, 65535, int(rng.integers(1, 65536))]))
        off = min(off, hist) if hist > 0 else 0
        if off == 0:
            ll = max(ll, 8)
            hist = produced + ll
            off = int(rng.integers(1, hist + 1))
        ml = int(rng.choice([4, 5, 18, 19, 20, 270, 300, int(rng.integers(4, 20000))]))
        ml = min(ml, max(4, target - hist - 12))
        mc = ml - 4
        tok = [(min(ll, 15) << 4) | min(mc, 15)]
        if ll >= 15:
            tok += _len_field(ll)
        out += bytes(tok) + rng.integers(0, 256, ll, dtype=np.uint8).tobytes() + bytes([off & 255, off >> 8])
        if mc >= 15:
            out += bytes(_len_field(mc))
        produced = hist + ml


pool = []
for t in range(24):   # a pool of compressed blocks, reused with fresh corruptions
    n = int(rng.choice([100, 5000, 65536, 300000, 1 << 20, 3 << 20, 4 << 20]))
    if args.random_streams:
        c, m = random_stream(n)
        pool.append((np.zeros(m, dtype=np.uint8), c))   # (only the size of the source is used)
    else:
        s = O.generate(gens[t % len(gens)], 500 + t, n)
        pool.append((s, O.compress_block_bytes(s)))
t0, batches, blocks, bad = time.time(), 0, 0, 0
t_log = t0
while time.time() - t0 < args.seconds:
    k = int(rng.integers(args.min_blocks, args.max_blocks + 1))
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
    if args.js_exact:   # reference mode, one block per output array (positions absolute in it)
        res = [lz4mi.decompress_blocks([c], [cp], js_exact=True) for c, cp in zip(comps, caps)] if k <= 8 else None
        if res is None:
            st, outs, lens = lz4mi.decompress_blocks(comps, caps, js_exact=True)
        else:
            st = np.array([r[0][0] for r in res]); outs = [r[1][0] for r in res]; lens = [r[2][0] for r in res]
    else:
        st, outs, lens = lz4mi.decompress_blocks(comps, caps)
    for j, c in enumerate(comps):
        est, ew, eo = O.decompress_block(c, caps[j], js_compat=args.js_exact)
        if st[j] == lz4mi.ERR_CROSS_BLOCK and (args.js_exact or est == lz4mi.ERR_DICT_OOB):
            continue   # (batched: reaches before its own block -- the caller decodes it alone)
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
    if time.time() - t_log > 30:   # progress (a run longer than 3 minutes must keep writing)
        t_log = time.time()
        print({"batches": batches, "blocks": blocks, "mismatches": bad}, flush=True)
print({"mode": os.environ.get("LZ4MI_SMALL_REPARSE", "0"), "blocks_range": [args.min_blocks, args.max_blocks],
       "js_exact": args.js_exact, "random_streams": args.random_streams, "batches": batches, "blocks": blocks, "mismatches": bad}, flush=True)
sys.exit(1 if bad else 0)
