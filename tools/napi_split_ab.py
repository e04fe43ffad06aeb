"""tools/napi_split.mjs (where the JS GPU route's decode time goes) for this tree and another tree's copy
(e.g. tools/variants/r05), alternating, on the same generated tiles216 blocks (tool)."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
other, counts = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "16,32,64,128"
n = max(int(x) for x in counts.split(","))
path = "/tmp/lz4mi_split_ab_%d.bin" % os.getpid()
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(16) as ex:
    np.concatenate(list(ex.map(lambda b: O.generate("tiles216", 1 + b, 4 << 20), range(n)))).tofile(path)
try:
    for rep in range(2):
        for tree in (ROOT, os.path.abspath(other)):
            r = subprocess.run(["node", "--no-warnings", "--expose-gc", os.path.join(tree, "tools", "napi_split.mjs"), path,
                                counts], capture_output=True, text=True, timeout=600)
            print(os.path.basename(tree.rstrip("/")), r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-800:],
                  flush=True)
finally:
    os.remove(path)
