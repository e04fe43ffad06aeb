set -e
python - <<'PY'
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as O
np.concatenate([O.generate("tiles216", 1 + b, 4 << 20) for b in range(int(__import__("os").environ.get("NB", "8")))]).tofile("/tmp/in.bin")
PY
timeout -k 10 300 node --no-warnings tools/dbg_js.mjs /tmp/in.bin /tmp/frame.bin
python - <<'PY'
import sys, numpy as np
sys.path.insert(0, "oracle")
import oracle as O
data = np.fromfile("/tmp/in.bin", dtype=np.uint8)
fr = np.fromfile("/tmp/frame.bin", dtype=np.uint8)
ref = O.compress_frame(data, None, 4194304, True, False, True)
print("frame equal oracle:", fr.size == ref.size and bool(np.array_equal(fr, ref)), fr.size, ref.size)
if fr.size == ref.size:
    d = np.nonzero(fr != ref)[0]; print("frame first diffs", d[:10])
st, back = O.decompress_frame(fr, None)
print("oracle decodes gpu frame:", st, bool(np.array_equal(back, data)))
st, jsb = O.decompress_frame(fr, None, js_compat=True)
g = np.fromfile("/tmp/back_ref.bin", dtype=np.uint8)
print("oracle js-compat decode:", st, "equals input:", bool(np.array_equal(jsb, data)), "equals gpu reference-mode:", bool(np.array_equal(jsb, g)))
PY
