import sys, os, numpy as np
sys.path[:0] = ["oracle", "divortio-lz4_amd"]
import oracle as O, lz4mi
lz4mi.init(0)
text = O.generate("text", 5, 300000)
for bs in (65536, 262144, 1 << 20):
    blocks = [text[o:o + bs] for o in range(0, text.size, bs)]
    for rep in range(3):
        comps = lz4mi.compress_blocks(blocks)
        bad = [(i, c.size, O.compress_block_bytes(b).size) for i, (b, c) in enumerate(zip(blocks, comps))
               if not np.array_equal(c, O.compress_block_bytes(b))]
        print("bs", bs, "rep", rep, "nblocks", len(blocks), "bad", bad, flush=True)
