// Diagnostic: the statuses the batched reference-mode decode returns for a 4 MiB-block frame
// of the given file (how many blocks the JS layer must re-decode alone, and why).
import fs from 'fs';
import { createRequire } from 'module';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';
const require = createRequire(import.meta.url);
const native = require('../divortio-lz4_amd/lz4mi.node');
const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const frame = LZ4.compress(input, null, 4194304, true, false);
let pos = 4 + 2 + 8 + 1;   // magic, FLG, BD, content size, HC
const inOff = [], inLen = [];
for (;;) {
    const bs = frame[pos] | (frame[pos + 1] << 8) | (frame[pos + 2] << 16) | (frame[pos + 3] << 24);
    pos += 4;
    if (bs === 0) break;
    inOff.push(pos); inLen.push(bs & 0x7FFFFFFF); pos += bs & 0x7FFFFFFF;
}
const nb = inOff.length, BS = 4194304;
const out = new Uint8Array(nb * BS);
const res = {};
for (const [name, flags] of [['spec', 0], ['exact', native.JS_EXACT]]) {
    const outOff = Float64Array.from({ length: nb }, (_, b) => b * BS), outCap = new Uint32Array(nb).fill(BS);
    const outLen = new Uint32Array(nb), status = new Int32Array(nb);
    const t0 = process.hrtime.bigint();
    native.decompressBlocks(frame, Float64Array.from(inOff), Uint32Array.from(inLen), out, outOff, outCap, outLen, status, null, flags);
    const ms = Number(process.hrtime.bigint() - t0) / 1e6;
    const hist = {};
    for (const s of status) hist[s] = (hist[s] || 0) + 1;
    res[name] = { ms: +ms.toFixed(2), statuses: hist };
    const t1 = process.hrtime.bigint();
    LZ4.setDecodeMode(name === 'spec' ? 'spec' : 'reference');
    LZ4.decompress(frame);
    res[name].layer_ms = +(Number(process.hrtime.bigint() - t1) / 1e6).toFixed(2);
}
console.log(JSON.stringify({ blocks: nb, ...res }));
