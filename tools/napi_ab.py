"""A/B of the JS drop-in end to end (tool): tools/napi_e2e.mjs of this tree and of another tree's copy
(e.g. tools/variants/r05: its js/, lz4mi.node and liblz4mi.so), alternating, on the same generated
tiles216 blocks. Prints each run's JSON line."""
import json, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
other = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 128
path = "/tmp/lz4mi_napi_ab_%d.bin" % os.getpid()
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(16) as ex:
    np.concatenate(list(ex.map(lambda b: O.generate("tiles216", 1 + b, 4 << 20), range(n)))).tofile(path)
try:
    for rep in range(int(sys.argv[3]) if len(sys.argv) > 3 else 2):
        for tree in (ROOT, os.path.abspath(other)):
            r = subprocess.run(["node", "--no-warnings", "--expose-gc", os.path.join(tree, "tools", "napi_e2e.mjs"), path, "3"],
                               capture_output=True, text=True, timeout=600)
            d = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-800:]}
            print(os.path.basename(tree.rstrip("/")), json.dumps({k: d.get(k) for k in ("decompress_spec_GBps", "decompress_reference_GBps", "compress_independent_GBps", "crossover", "error")}), flush=True)
finally:
    os.remove(path)
