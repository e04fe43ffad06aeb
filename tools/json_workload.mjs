// The reference's own published benchmark, run through the drop-in: LZ4.compress /
// LZ4.decompress of JSON text made of one small record repeated (the shape of
// benchmark/src/base/benchUtils.js's data; our own record), 4 MiB independent blocks,
// no checksum (benchmark/src/base/benchWorker.js:47-54), host buffers through N-API.
// Rates in MB/s with MB = 2^20 bytes, as the reference's docs/BENCHMARKS.md reports them.
//   node tools/json_workload.mjs [MiB] [reps]
// Prints one JSON line.
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';
import { jsonRepeat } from './json_data.mjs';

if (import.meta.url === `file://${process.argv[1]}`) {
    const mib = Number(process.argv[2] || 25);
    const reps = Number(process.argv[3] || 5);
    const input = jsonRepeat(mib << 20);
    const now = () => Number(process.hrtime.bigint()) / 1e9;
    const rate = (fn) => {
        fn();                                   // warm-up (device init, scratch growth)
        const t0 = now();
        for (let r = 0; r < reps; r++) fn();
        return +(input.length * reps / (now() - t0) / (1 << 20)).toFixed(1);
    };
    // every rate twice: the default routing ('auto': this call size goes to the host codec,
    // DESIGN §5.1) and every block call forced onto the GPU kernels; `route` counts the calls
    // each side took during the timed loop (warm-up included)
    const out = { bytes: input.length, block_size: 4194304 };
    for (const routing of ['auto', 'gpu']) {
        LZ4.setRouting(routing);
        const o = { routing };
        LZ4.routeStats(true);
        let frame = LZ4.compress(input, null, 4194304, true, false);
        o.ratio = +(input.length / frame.length).toFixed(1);
        LZ4.routeStats(true);
        o.compress_MBps = rate(() => { frame = LZ4.compress(input, null, 4194304, true, false); });
        o.compress_route = LZ4.routeStats(true);
        for (const mode of ['spec', 'reference']) {
            LZ4.setDecodeMode(mode);
            const back = LZ4.decompress(frame);
            const same = Buffer.compare(Buffer.from(back), Buffer.from(input)) === 0;
            if (mode === 'spec' && !same) throw new Error('spec round trip mismatch');
            o[`${mode}_round_trip_exact`] = same;
            LZ4.routeStats(true);
            o[`decompress_${mode}_MBps`] = rate(() => LZ4.decompress(frame));
            o[`decompress_${mode}_route`] = LZ4.routeStats(true);
        }
        LZ4.setDecodeMode('reference');
        o.roundtrip_MBps = rate(() => LZ4.decompress(LZ4.compress(input, null, 4194304, true, false)));
        o.roundtrip_route = LZ4.routeStats(true);
        out[routing] = o;
    }
    LZ4.setRouting('auto');
    console.log(JSON.stringify(out));
}
