// Where the JS GPU route's decode time goes (tool): for frames of b independent 4 MiB blocks,
// LZ4.decompress (routing 'gpu' and 'host') against the batched native call alone into a fresh
// and into a reused output array, and the output allocation alone (medians of 5, ms).
import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';

const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const BS = 4194304;
const now = () => Number(process.hrtime.bigint()) / 1e6;
const REPS = Number(process.argv[4] || 5);
const gc = globalThis.gc || (() => {});   // (node --expose-gc: earlier results collected before each call)
const med = (fn, n = REPS) => {
    gc();
    fn();
    const ts = [];
    for (let r = 0; r < n; r++) { gc(); const t0 = now(); fn(); ts.push(now() - t0); }
    ts.sort((a, b) => a - b);
    return +ts[(n - 1) >> 1].toFixed(3);
};
const u32 = (d, p) => (d[p] | (d[p + 1] << 8) | (d[p + 2] << 16) | (d[p + 3] << 24)) >>> 0;
const res = {};
for (const b of (process.argv[3] || '1,2,4,7,16').split(',').map(Number)) {
    const sub = input.subarray(0, b * BS);
    LZ4.setRouting('gpu');
    LZ4.setDecodeMode('spec');
    const frame = LZ4.compress(sub, null, BS, true, false);
    let pos = 15;
    const inOff = new Float64Array(b), inLen = new Uint32Array(b), outOff = new Float64Array(b), outCap = new Uint32Array(b);
    for (let k = 0; k < b; k++) {
        const n = u32(frame, pos) & 0x7FFFFFFF;
        inOff[k] = pos + 4; inLen[k] = n; outOff[k] = k * BS; outCap[k] = BS;
        pos += 4 + n;
    }
    const outLen = new Uint32Array(b), status = new Int32Array(b);
    const reuse = new Uint8Array(b * BS);
    const row = {};
    row.alloc = med(() => new Uint8Array(b * BS));
    row.native_fresh = med(() => LZ4.decompressBlocks(frame, inOff, inLen, new Uint8Array(b * BS), outOff, outCap, outLen, status));
    row.native_reused = med(() => LZ4.decompressBlocks(frame, inOff, inLen, reuse, outOff, outCap, outLen, status));
    row.decompress_gpu = med(() => LZ4.decompress(frame));
    LZ4.setRouting('host');
    row.decompress_host = med(() => LZ4.decompress(frame));
    LZ4.setRouting('auto');
    row.decompress_auto = med(() => LZ4.decompress(frame));
    const back = LZ4.decompress(frame);
    row.ok = Buffer.compare(Buffer.from(back), Buffer.from(sub)) === 0;
    res[b] = row;
    console.log(b, JSON.stringify(row));
}
console.log(JSON.stringify(res));
