// End-to-end rates of the drop-in JS layer (host buffers through N-API: H2D +
// kernels + D2H + JS frame assembly), as a caller of the reference's API sees them.
//   node tools/napi_e2e.mjs <input file> [reps] [dependent-mode bytes]
// Prints one JSON line: LZ4.compress with independent blocks (batched), LZ4.compress
// with the reference's default dependent blocks (the layer's host route: one serial chain,
// the table carried; checked to decode back), LZ4.decompress in 'spec' and 'reference'
// (default) modes, the decode of the dependent frame, all under the default routing; then
// the routing crossover: independent-block compress / decompress (spec) of the first b
// blocks with every call forced to the GPU and to the host codec (DESIGN §5.1).
import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';

const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const reps = Number(process.argv[3] || 3);
const depBytes = Math.min(input.length, Number(process.argv[4] || (16 << 20)));
const BS = 4194304;
const now = () => Number(process.hrtime.bigint()) / 1e9;
const gc = globalThis.gc || (() => {});   // (node --expose-gc: large results of earlier calls collected first)
const secs = (fn, n) => {               // median of n timed calls after a warm-up call
    gc();
    fn();
    const ts = [];
    for (let r = 0; r < n; r++) {
        const t0 = now();
        fn();
        ts.push(now() - t0);
    }
    ts.sort((a, b) => a - b);
    return ts[(n - 1) >> 1];
};
const rate = (bytes, fn, n) => +(bytes / secs(fn, n) / 1e9).toFixed(3);
// calls each side took during a measurement (warm-up included): which codec a rate describes
const routed = (key, fn) => { LZ4.routeStats(true); fn(); out[`${key}_route`] = LZ4.routeStats(true); };
const out = { bytes: input.length, routing: 'auto' };
let frame = LZ4.compress(input, null, BS, true, false);
out.ratio = +(input.length / frame.length).toFixed(3);
routed('compress_independent', () => {
    out.compress_independent_GBps = rate(input.length, () => { frame = LZ4.compress(input, null, BS, true, false); }, reps);
});
const dep = input.subarray(0, depBytes);
let depFrame = null;
routed('compress_dependent_default', () => {
    out.compress_dependent_default_GBps = rate(dep.length, () => { depFrame = LZ4.compress(dep); }, 1);
});
out.dependent_bytes = dep.length;
LZ4.setDecodeMode('spec');
if (Buffer.compare(Buffer.from(LZ4.decompress(depFrame)), Buffer.from(dep)) !== 0)
    throw new Error('dependent frame round trip mismatch');
routed('decompress_dependent', () => {
    out.decompress_dependent_GBps = rate(dep.length, () => LZ4.decompress(depFrame), 1);
});
for (const mode of ['spec', 'reference']) {
    LZ4.setDecodeMode(mode);
    const back = LZ4.decompress(frame);
    // (reference mode reproduces the reference decoder, which corrupts a few blocks: SURVEY F1)
    if (mode === 'spec' && Buffer.compare(Buffer.from(back), Buffer.from(input)) !== 0)
        throw new Error(`${mode} round trip mismatch`);
    routed(`decompress_${mode}`, () => {
        out[`decompress_${mode}_GBps`] = rate(input.length, () => LZ4.decompress(frame), reps);
    });
}
LZ4.setDecodeMode('spec');
const cross = { block_bytes: BS, blocks: [], compress_ms: { gpu: [], host: [] }, decompress_ms: { gpu: [], host: [] } };
for (const b of [1, 4, 16, 32, 64, 128]) {
    if (b * BS > input.length) break;
    const sub = input.subarray(0, b * BS);
    cross.blocks.push(b);
    for (const side of ['gpu', 'host']) {
        LZ4.setRouting(side);
        let f = null;
        cross.compress_ms[side].push(+(secs(() => { f = LZ4.compress(sub, null, BS, true, false); }, 3) * 1e3).toFixed(2));
        cross.decompress_ms[side].push(+(secs(() => LZ4.decompress(f), 3) * 1e3).toFixed(2));
    }
}
LZ4.setRouting('auto');
LZ4.setDecodeMode('reference');
out.crossover = cross;
out.note = 'host buffers through N-API (PCIe-inclusive): not the device-resident bench value';
console.log(JSON.stringify(out));
