python - <<'PY'
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as O
O.generate("text", 5, 300000).tofile("/tmp/text.bin")
for bs in (65536, 262144):
    for ck in (0, 1):
        f = O.compress_frame(O.generate("text", 5, 300000), None, bs, True, ck, True)
        print("oracle", bs, ck, f.size, "%08x" % O.xxh32(f))
PY
timeout -k 10 120 node --no-warnings tools/dbg_gt.mjs /tmp/text.bin
