"""Where reference mode (LZ4MI_JS_EXACT) costs more than spec decode (tool).

For b 4 MiB tiles216 blocks (seeds 1..b, the bench's blocks: seeds 33, 62, 87 are F1 blocks):
  device   - one lz4mi_decompress_blocks launch on device pointers, HIP events (median of 5)
  host     - the C-ABI call on host buffers (H2D, kernel, D2H: what the N-API addon calls), ms
  node     - LZ4.decompress through the drop-in (tools/napi_split.mjs style), both modes, ms
Prints one JSON line per b."""
import argparse, json, os, subprocess, sys, tempfile, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "divortio-lz4_amd")]
import torch  # noqa: E402
import oracle as O  # noqa: E402
import lz4mi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--counts", default="16,128")
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
lz4mi.init(0)
BS = 4 << 20
NODE_JS = r"""
import fs from 'fs';
import { LZ4 } from '%s';
const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const now = () => Number(process.hrtime.bigint()) / 1e6;
const gc = globalThis.gc || (() => {});
const frame = LZ4.compress(input, null, 4194304, true, false);
const res = {};
for (const mode of ['spec', 'reference', 'spec', 'reference']) {
    LZ4.setDecodeMode(mode);
    LZ4.decompress(frame);
    const ts = [];
    for (let r = 0; r < %d; r++) { gc(); const t0 = now(); LZ4.decompress(frame); ts.push(now() - t0); }
    ts.sort((a, b) => a - b);
    res[mode] = +ts[(ts.length - 1) >> 1].toFixed(3);
}
LZ4.routeStats(true);
LZ4.decompress(frame);
res.route = LZ4.routeStats(true);
console.log(JSON.stringify(res));
"""
mx = max(int(x) for x in args.counts.split(","))
raw = torch.empty(mx * BS, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
lz4mi.generate_blocks_dev(raw.data_ptr(), "tiles216", 1, BS, mx, s)
slot = (lz4mi.compress_bound(BS) + 255) & ~255
comp = torch.zeros(mx * slot, dtype=torch.uint8, device="cuda")
roff = torch.arange(mx, dtype=torch.int64, device="cuda") * BS
rlen = torch.full((mx,), BS, dtype=torch.int32, device="cuda")
coff = torch.arange(mx, dtype=torch.int64, device="cuda") * slot
clen = torch.zeros(mx, dtype=torch.int32, device="cuda")
lz4mi.compress_blocks_dev(raw.data_ptr(), roff.data_ptr(), rlen.data_ptr(), comp.data_ptr(), coff.data_ptr(),
                          clen.data_ptr(), mx, s)
dec = torch.empty(mx * BS, dtype=torch.uint8, device="cuda")
dlen = torch.zeros(mx, dtype=torch.int32, device="cuda")
st = torch.zeros(mx, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
for b in [int(x) for x in args.counts.split(",")]:
    row = {"blocks": b}
    for mode in ("spec", "reference"):
        ts = []
        for r in range(args.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lz4mi.decompress_blocks_dev(comp.data_ptr(), coff.data_ptr(), clen.data_ptr(), dec.data_ptr(),
                                        roff.data_ptr(), rlen.data_ptr(), dlen.data_ptr(), st.data_ptr(), b, s,
                                        js_exact=(mode == "reference"))
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        row[f"device_{mode}_ms"] = round(sorted(ts)[len(ts) // 2], 3)
        row[f"device_{mode}_status"] = sorted(set(int(x) for x in st[:b].cpu().tolist()))
    # host buffers through the C-ABI (the addon's call)
    cl = clen[:b].cpu().numpy().astype(np.uint32)
    hc = comp[:b * slot].cpu().numpy()
    blocks = [hc[k * slot:k * slot + int(cl[k])] for k in range(b)]
    for mode in ("spec", "reference"):
        ts = []
        for r in range(args.reps + 1):
            t0 = time.perf_counter()
            stt, outs, lens = lz4mi.decompress_blocks(blocks, [BS] * b, js_exact=(mode == "reference"))
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        row[f"host_ptr_{mode}_ms"] = round(sorted(ts)[len(ts) // 2], 3)
    # the drop-in through N-API
    path = os.path.join(tempfile.gettempdir(), f"refsplit_{os.getpid()}.bin")
    js = os.path.join(tempfile.gettempdir(), f"refsplit_{os.getpid()}.mjs")
    try:
        raw[:b * BS].cpu().numpy().tofile(path)
        with open(js, "w") as f:
            f.write(NODE_JS % (os.path.join(ROOT, "divortio-lz4_amd", "js", "lz4mi.mjs"), args.reps))
        r = subprocess.run(["node", "--no-warnings", "--expose-gc", js, path], capture_output=True, text=True,
                           timeout=300)
        row["node"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-400:]
    finally:
        for p in (path, js):
            if os.path.exists(p):
                os.remove(p)
    print(json.dumps(row), flush=True)
