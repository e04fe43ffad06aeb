import sys, numpy as np
sys.path[:0] = ["oracle", "divortio-lz4_amd"]
import oracle as O, lz4mi
lz4mi.init(0)
srcs = [O.generate("tiles216", 1 + b, 4 << 20) for b in range(16)]
comps = lz4mi.compress_blocks(srcs)
for name, kw in (("spec", {}), ("exact", {"js_exact": True}), ("compat", {"js_compat": True})):
    if name == "compat":
        srcs2, comps2 = srcs[:2], comps[:2]
    else:
        srcs2, comps2 = srcs, comps
    st, outs, lens = lz4mi.decompress_blocks(comps2, [s.size for s in srcs2], **kw)
    bad = [i for i, (s, o) in enumerate(zip(srcs2, outs)) if not np.array_equal(s, o)]
    print(name, "status", set(st.tolist()), "bad blocks", bad[:10], flush=True)
    for i in bad[:2]:
        d = np.nonzero(srcs2[i] != outs[i][:srcs2[i].size])[0] if outs[i].size == srcs2[i].size else None
        print("  block", i, "len", outs[i].size, "first diffs", None if d is None else d[:8])
