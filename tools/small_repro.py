"""Re-decodes a dumped mismatching block (tools/small_fuzz.py --dump) alone through the small path in
the re-parse mode of LZ4MI_SMALL_REPARSE and reports the first differing output byte (tool)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "divortio-lz4_amd"))
import oracle as O  # noqa: E402
import lz4mi  # noqa: E402
d = np.load(sys.argv[1])
comp, cap = d["comp"], int(d["cap"][0])
est, ew, eo = O.decompress_block(comp, cap)
for rep in range(3):
    st, outs, lens = lz4mi.decompress_blocks([comp], [cap])
    got = outs[0]
    want = eo[:min(ew, cap)]
    same = got.size == want.size and np.array_equal(got, want)
    first = -1
    if not same and got.size == want.size:
        first = int(np.argmax(got != want))
    ndiff = int((got != want).sum()) if got.size == want.size else -1
    print({"mode": os.environ.get("LZ4MI_SMALL_REPARSE", "0"), "rep": rep, "status": int(st[0]), "oracle": int(est),
           "len": int(lens[0]), "olen": int(ew), "same": bool(same), "first_diff": first, "ndiff": ndiff,
           "comp_len": int(comp.size)}, flush=True)
