"""Runs tools/batch_status_check.mjs on 16 generated 4 MiB tiles216 blocks, then the same check through
the C-ABI from Python (tool)."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
import oracle as O  # noqa: E402
blocks = [O.generate("tiles216", 1 + i, 4 << 20) for i in range(16)]
path = "/tmp/lz4mi_bsc_%d.bin" % os.getpid()
np.concatenate(blocks).tofile(path)
try:
    for mode in ("spec", "reference"):
        r = subprocess.run(["node", "--no-warnings", os.path.join(ROOT, "tools", "batch_status_check.mjs"), path, "16", "30", mode],
                           capture_output=True, text=True, timeout=200)
        print(mode, r.stdout.strip()[-3000:], r.stderr[-800:], flush=True)
finally:
    os.remove(path)
import lz4mi  # noqa: E402
comps = [O.compress_block_bytes(b) for b in blocks]
bad = 0
for r in range(30):
    st, outs, lens = lz4mi.decompress_blocks(comps, [4 << 20] * 16)
    if not ((st == 0).all() and all(np.array_equal(o, b) for o, b in zip(outs, blocks))):
        bad += 1
        print("python rep", r, st.tolist(), lens.tolist(), flush=True)
print("python bad", bad)
