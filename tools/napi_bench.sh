# PCIe-inclusive rate of the JS drop-in: 256 MiB of tiles216 blocks (64 x 4 MiB) and of random bytes
set -e
python - <<'PY'
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as O
for g in ("tiles216", "random"):
    np.concatenate([O.generate(g, 1 + b, 4 << 20) for b in range(64)]).tofile(f"/tmp/napi_{g}.bin")
PY
for g in tiles216 random; do echo -n "$g "; timeout -k 10 300 node --no-warnings tools/napi_bench.mjs /tmp/napi_$g.bin 3 2>&1 | tail -5; done
rm -f /tmp/napi_*.bin
