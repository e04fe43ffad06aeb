// Repeats the JS layer's batched decode of a b-block frame (tool): reports every call whose
// statuses / output lengths would make batchDirect fall back to block-by-block decoding.
import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';
const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const BS = 4194304, b = Number(process.argv[3] || 16), reps = Number(process.argv[4] || 40);
const u32 = (d, p) => (d[p] | (d[p + 1] << 8) | (d[p + 2] << 16) | (d[p + 3] << 24)) >>> 0;
LZ4.setRouting('gpu');
LZ4.setDecodeMode(process.argv[5] || 'spec');
const sub = input.subarray(0, b * BS);
const frame = LZ4.compress(sub, null, BS, true, false);
let pos = 15;
const inOff = new Float64Array(b), inLen = new Uint32Array(b), outOff = new Float64Array(b), outCap = new Uint32Array(b);
for (let k = 0; k < b; k++) {
    const n = u32(frame, pos) & 0x7FFFFFFF;
    inOff[k] = pos + 4; inLen[k] = n; outOff[k] = k * BS; outCap[k] = BS;
    pos += 4 + n;
}
let bad = 0;
for (let r = 0; r < reps; r++) {
    const outLen = new Uint32Array(b), status = new Int32Array(b);
    const res = new Uint8Array(b * BS);
    LZ4.decompressBlocks(frame, inOff, inLen, res, outOff, outCap, outLen, status);
    const odd = [];
    for (let k = 0; k < b; k++) if (status[k] !== 0 || outLen[k] !== outCap[k]) odd.push([k, status[k], outLen[k]]);
    const same = Buffer.compare(Buffer.from(res), Buffer.from(sub)) === 0;
    if (odd.length || !same) { bad++; console.log('rep', r, 'odd', JSON.stringify(odd), 'bytes equal', same); }
}
console.log(JSON.stringify({ blocks: b, reps, bad }));
