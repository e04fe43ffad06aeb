import sys, os, numpy as np
sys.path[:0] = ["oracle", "divortio-lz4_amd"]
import oracle as O, lz4mi
lz4mi.init(0)
text = O.generate("text", 5, 300000)
copy = O.generate("copy", 6, 150000)
bad = 0
for rep in range(10):
    for data in (text, copy):
        for bs in (65536, 262144):
            blocks = [data[o:o + bs] for o in range(0, data.size, bs)]
            comps = lz4mi.compress_blocks(blocks)
            for b, c in zip(blocks, comps):
                if not np.array_equal(c, O.compress_block_bytes(b)):
                    bad += 1
                    print("rep", rep, "bs", bs, "size", c.size, "ref", O.compress_block_bytes(b).size, flush=True)
            # interleave a decode like the JS test does
            st, outs, _ = lz4mi.decompress_blocks(comps, [b.size for b in blocks], js_exact=True)
print("total bad", bad)
