"""Runs tools/exact_status.mjs on 128 generated 4 MiB tiles216 blocks."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (generator only)

path = "/tmp/lz4mi_exact_%d.bin" % os.getpid()
np.concatenate([O.generate("tiles216", 1 + i, 4 << 20) for i in range(128)]).tofile(path)
try:
    r = subprocess.run(["node", "--no-warnings", os.path.join(ROOT, "tools", "exact_status.mjs"), path],
                       capture_output=True, text=True, timeout=200)
    print(r.stdout.strip()[-2000:], r.stderr[-800:])
    sys.exit(r.returncode)
finally:
    os.remove(path)
