"""Runs tools/napi_split.mjs on 16 generated 4 MiB tiles216 blocks (tool)."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
path = "/tmp/lz4mi_split_%d.bin" % os.getpid()
np.concatenate([O.generate("tiles216", 1 + i, 4 << 20) for i in range(16)]).tofile(path)
try:
    r = subprocess.run(["node", "--no-warnings", "--expose-gc", os.path.join(ROOT, "tools", "napi_split.mjs"), path] + sys.argv[1:],
                       capture_output=True, text=True, timeout=250)
    print(r.stdout.strip()[-4000:])
    print(r.stderr[-1500:], file=sys.stderr)
    sys.exit(r.returncode)
finally:
    os.remove(path)
