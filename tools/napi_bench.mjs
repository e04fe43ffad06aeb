// End-to-end (host buffers, PCIe-inclusive) throughput of the drop-in JS layer:
// LZ4.compress / LZ4.decompress of one input file through N-API -> liblz4mi.
//   node tools/napi_bench.mjs <input file> [reps]
// Decode is timed in both modes: 'reference' (the default: byte-identical to the
// reference decoder, F1 included) and 'spec'; the spec decode must round-trip.
import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';

const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const reps = Number(process.argv[3] || 3);
const t = () => Number(process.hrtime.bigint()) / 1e9;
let frame = LZ4.compress(input, null, 4194304, true, false);        // warm-up (independent blocks)
LZ4.setDecodeMode('spec');
if (Buffer.compare(Buffer.from(LZ4.decompress(frame)), Buffer.from(input)) !== 0) throw new Error('round trip mismatch');
const out = { bytes: input.length, ratio: +(input.length / frame.length).toFixed(3) };
let tc = 0;
for (let r = 0; r < reps; r++) {
    const t0 = t();
    frame = LZ4.compress(input, null, 4194304, true, false);
    tc += t() - t0;
}
out.compress_GBps = +(input.length * reps / tc / 1e9).toFixed(3);
for (const mode of ['spec', 'reference']) {
    LZ4.setDecodeMode(mode);
    LZ4.decompress(frame);
    let td = 0;
    for (let r = 0; r < reps; r++) {
        const t0 = t();
        LZ4.decompress(frame);
        td += t() - t0;
    }
    out[`decompress_${mode}_GBps`] = +(input.length * reps / td / 1e9).toFixed(3);
}
out.note = 'host buffers through N-API: H2D + kernels + D2H + JS frame assembly';
console.log(JSON.stringify(out));
