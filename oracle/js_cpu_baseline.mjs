// oracle/js_cpu_baseline.mjs — BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
//
// Times the pure-JS block codec (oracle/lz4_js.mjs, our restatement of the
// reference's compressBlock/decompressBlock) on the host's cores, the shape of the
// reference's own benchmark (benchmark/src/base/benchWorker.js:47-54: 4 MiB
// independent blocks, no checksum): every worker_thread compresses then
// decompresses its own `blocks` distinct 4 MiB blocks (a streaming working set, not
// one cache-resident block), checking the round trip. Prints one JSON line.
//
//   node oracle/js_cpu_baseline.mjs <generator> <threads> <blocks per thread> [golden manifest]
// With a manifest, worker 0 first checks its compressed bytes of seeds 1..4 against
// the reference's 4 MiB digests (comp_len + xxh32 of the compressed block).
import os from 'os';
import fs from 'fs';
import { Worker, isMainThread, parentPort, workerData } from 'worker_threads';
import { compressBlock, decompressBlock, generate as generateBlock } from './lz4_js.mjs';
import { jsonRepeat } from '../tools/json_data.mjs';

// 'json': the reference's benchmark data shape (tools/json_data.mjs), same bytes in every block
const generate = (gen, seed, n) => (gen === 'json' ? jsonRepeat(n) : generateBlock(gen, seed, n));

const BLOCK = 4 << 20;

function xxh32(a) {          // reference variant (xxhash32.js), for the digest check only
    const P1 = 2654435761, P2 = 2246822519, P3 = 3266489917, P4 = 668265263, P5 = 374761393;
    const rotl = (x, r) => ((x << r) | (x >>> (32 - r))) >>> 0;
    const mul = (a, b) => Math.imul(a, b) >>> 0;
    const rd = (p) => (a[p] | (a[p + 1] << 8) | (a[p + 2] << 16) | (a[p + 3] << 24)) >>> 0;
    const n = a.length;
    let p = 0, h;
    if (n >= 16) {
        let v = [(P1 + P2) >>> 0, P2, 0, (0 - P1) >>> 0];
        for (; p + 16 <= n; p += 16) for (let k = 0; k < 4; k++) v[k] = mul(rotl((v[k] + mul(rd(p + 4 * k), P2)) >>> 0, 13), P1);
        h = rotl(v[0], 1);
        h = rotl((h + v[1]) >>> 0, 7);
        h = rotl((h + v[2]) >>> 0, 12);
        h = rotl((h + v[3]) >>> 0, 18);
    } else h = P5;
    h = (h + n) >>> 0;
    for (; p + 4 <= n; p += 4) h = mul(rotl((h + mul(rd(p), P3)) >>> 0, 17), P4);
    for (; p < n; p++) h = mul(rotl((h + mul(a[p], P5)) >>> 0, 11), P1);
    h = mul(h ^ (h >>> 15), P2); h = mul(h ^ (h >>> 13), P3); h = (h ^ (h >>> 16)) >>> 0;
    return h;
}

if (isMainThread) {
    const gen = process.argv[2] || 'tiles216';
    const threads = Number(process.argv[3] || os.cpus().length);
    const blocks = Number(process.argv[4] || 64);
    const manifest = process.argv[5] || null;
    let checked = null;
    if (manifest) {
        const m = JSON.parse(fs.readFileSync(manifest, 'utf8'));
        const rows = m.cases.find((c) => c.kind === 'digest_4mib').rows.filter((r) => r.gen === gen && r.seed <= 4);
        const out = new Uint8Array(BLOCK + (BLOCK / 255 | 0) + 16);
        checked = 0;
        for (const r of rows) {
            const n = compressBlock(generate(gen, r.seed, BLOCK), out, 0, BLOCK, new Int32Array(16384), 0);
            if (n !== r.comp_len || xxh32(out.subarray(0, n)).toString(16).padStart(8, '0') !== r.comp_xxh)
                throw new Error(`JS restatement differs from the reference on ${gen} seed ${r.seed}`);
            checked++;
        }
    }
    const res = [];
    let done = 0;
    const t0 = process.hrtime.bigint();
    for (let w = 0; w < threads; w++) {
        const wk = new Worker(new URL(import.meta.url), { workerData: { gen, seed0: 1000 + w * blocks, blocks } });
        wk.on('message', (m) => {
            res.push(m);
            if (++done === threads) {
                const wall = Number(process.hrtime.bigint() - t0) / 1e9;
                const bytes = threads * blocks * BLOCK;
                const ct = Math.max(...res.map((r) => r.compress_s)), dt = Math.max(...res.map((r) => r.decompress_s));
                console.log(JSON.stringify({
                    generator: gen, threads, blocks_per_thread: blocks, block_bytes: BLOCK,
                    compress_GBps: +(bytes / ct / 1e9).toFixed(3), decompress_GBps: +(bytes / dt / 1e9).toFixed(3),
                    roundtrip_GBps: +(bytes / Math.max(...res.map((r) => r.compress_s + r.decompress_s)) / 1e9).toFixed(3),
                    ratio: +(bytes / res.reduce((a, r) => a + r.comp_bytes, 0)).toFixed(3),
                    verified: res.every((r) => r.ok), golden_digests_checked: checked, wall_s: +wall.toFixed(2),
                    cpu_model: os.cpus()[0].model, node: process.version,
                }));
            }
        });
        wk.on('error', (e) => { console.error(e); process.exit(1); });
    }
} else {
    const { gen, seed0, blocks } = workerData;
    const raw = [], comp = [];
    for (let b = 0; b < blocks; b++) raw.push(generate(gen, seed0 + b, BLOCK));
    const cap = BLOCK + (BLOCK / 255 | 0) + 16;
    let t = process.hrtime.bigint();
    let compBytes = 0;
    for (let b = 0; b < blocks; b++) {
        const out = new Uint8Array(cap);
        const n = compressBlock(raw[b], out, 0, BLOCK, new Int32Array(16384), 0);
        comp.push(out.subarray(0, n));
        compBytes += n;
    }
    const cs = Number(process.hrtime.bigint() - t) / 1e9;
    const dec = new Uint8Array(BLOCK);
    let ok = true;
    let ds = 0;
    for (let b = 0; b < blocks; b++) {
        t = process.hrtime.bigint();
        const w = decompressBlock(comp[b], 0, comp[b].length, dec, 0);
        ds += Number(process.hrtime.bigint() - t) / 1e9;
        if (w !== BLOCK || (b % 8 === 0 && !Buffer.from(dec).equals(Buffer.from(raw[b])))) ok = false;
    }
    parentPort.postMessage({ compress_s: cs, decompress_s: ds, comp_bytes: compBytes, ok });
}
