"""Runs tools/napi_e2e.mjs (the JS drop-in through N-API, routing crossover sweep) on 128
generated 4 MiB tiles216 blocks, outside bench.py (prints its JSON line)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (generator only: the input bytes)

path = "/tmp/lz4mi_e2e_%d.bin" % os.getpid()
np.concatenate([O.generate("tiles216", 1 + i, 4 << 20) for i in range(128)]).tofile(path)
try:
    r = subprocess.run(["node", "--no-warnings", "--expose-gc", os.path.join(ROOT, "tools", "napi_e2e.mjs"), path, "3"],
                       capture_output=True, text=True, timeout=280)
    print(r.stdout.strip()[-3000:])
    print(r.stderr[-800:], file=sys.stderr)
    sys.exit(r.returncode)
finally:
    os.remove(path)
