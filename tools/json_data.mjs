// JSON text made of one small record repeated: the shape of the reference's benchmark
// data (benchmark/src/base/benchUtils.js), with our own record. No imports, so both
// the drop-in timing (tools/json_workload.mjs) and the pure-JS baseline
// (oracle/js_cpu_baseline.mjs) can use it.
export function jsonRepeat(bytes) {
    const rec = JSON.stringify({
        seq: 42, kind: 'sample_record', labels: ['alpha', 'beta', 'gamma', 'delta', 'epsilon'],
        stats: { ok: true, values: [12, 240, 3600, 48000, 510000] },
        note: 'One small record, repeated until the buffer is full, compresses very well.',
    });
    return new TextEncoder().encode(rec.repeat(Math.ceil(bytes / rec.length))).subarray(0, bytes);
}
