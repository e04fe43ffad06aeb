// Runs the golden cases of a job file (written by tests/test_js_shim.py) through
// the drop-in JS layer (divortio-lz4_amd/js/lz4mi.mjs -> N-API -> gfx950) and
// prints one JSON line of results. Digests use the reference's xxHash32.
import fs from 'fs';
import { LZ4 } from '../../divortio-lz4_amd/js/lz4mi.mjs';

const job = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
LZ4.setRouting(process.argv[3] || 'gpu');   // 'gpu': every block call on the kernels; 'auto': the layer's routing
const hex = (v) => (v >>> 0).toString(16).padStart(8, '0');
const read = (p) => (p ? new Uint8Array(fs.readFileSync(p)) : null);
const fromHex = (s) => Uint8Array.from(Buffer.from(s, 'hex'));
const results = [];

function check(id, fn) {
    try {
        const d = fn();
        results.push({ id, ok: d === true, detail: d === true ? '' : String(d) });
    } catch (e) {
        results.push({ id, ok: false, detail: 'threw ' + (e && e.stack ? e.stack : e) });
    }
}

function expectThrow(fn, msg) {
    try { fn(); } catch (e) { return e.message === msg ? true : `threw "${e.message}", expected "${msg}"`; }
    return `did not throw "${msg}"`;
}

for (const c of job.cases) {
    if (c.op === 'block') {
        check(c.id, () => {
            const src = read(c.src);
            const out = new Uint8Array(src.length + ((src.length / 255) | 0) + 16);
            const n = LZ4.compressRaw(src, out, 0, src.length, new Int32Array(16384), 0);
            const comp = out.subarray(0, n);
            if (n !== c.comp_len || hex(LZ4.xxHash32(comp, 0)) !== c.comp_xxh)
                return `compressRaw ${n} ${hex(LZ4.xxHash32(comp, 0))} != ${c.comp_len} ${c.comp_xxh}`;
            const dec = new Uint8Array(src.length);
            const w = LZ4.decompressRaw(comp, 0, n, dec, 0);
            if (w !== c.js_dec_written || hex(LZ4.xxHash32(dec, 0)) !== c.js_dec_xxh)
                return `decompressRaw ${w} ${hex(LZ4.xxHash32(dec, 0))} != ${c.js_dec_written} ${c.js_dec_xxh}`;
            return true;
        });
    } else if (c.op === 'frame') {
        check(c.id, () => {
            const input = read(c.input);
            const dict = read(c.dict);
            const frame = LZ4.compress(input, dict, c.block, c.indep, c.checksum, c.add_size);
            if (frame.length !== c.frame_len || hex(LZ4.xxHash32(frame, 0)) !== c.frame_xxh)
                return `compress ${frame.length} ${hex(LZ4.xxHash32(frame, 0))} != ${c.frame_len} ${c.frame_xxh}`;
            if (c.dec_ok === null || c.dec_ok === undefined) return true;
            if (c.dec_ok) {
                const back = LZ4.decompress(frame, dict, !c.noverify);
                if (back.length !== c.dec_len || hex(LZ4.xxHash32(back, 0)) !== c.dec_xxh)
                    return `decompress ${back.length} ${hex(LZ4.xxHash32(back, 0))} != ${c.dec_len} ${c.dec_xxh}`;
            } else {
                const r = expectThrow(() => LZ4.decompress(frame, dict, !c.noverify), c.dec_error);
                if (r !== true) return r;
            }
            LZ4.setDecodeMode('spec');           // the LZ4-spec decoder round-trips every frame
            try {
                const back = LZ4.decompress(frame, dict, false);
                if (Buffer.compare(Buffer.from(back), Buffer.from(input)) !== 0) return 'spec decode != input';
            } finally {
                LZ4.setDecodeMode('reference');
            }
            return true;
        });
    } else if (c.op === 'decode_vec') {
        check(c.id, () => {
            if (c.ok) {
                const out = LZ4.decompress(fromHex(c.hex), null, c.verify);
                return Buffer.from(out).toString('hex') === c.out_hex.toLowerCase() ? true : 'output mismatch';
            }
            try { LZ4.decompress(fromHex(c.hex), null, c.verify); } catch (e) {
                return e.message === c.error || (c.error.startsWith('LZ4: Unsupported Version') && e.message === c.error)
                    ? true : `threw "${e.message}", expected "${c.error}"`;
            }
            return 'did not throw';
        });
    } else if (c.op === 'raw_decode') {
        check(c.id, () => {
            const out = new Uint8Array(c.out_len);
            const dict = c.dict ? Uint8Array.from(c.dict) : null;
            const comp = Uint8Array.from(c.comp);
            if (!c.ok) return expectThrow(() => LZ4.decompressRaw(comp, 0, comp.length, out, c.out_off, dict), c.error);
            const w = LZ4.decompressRaw(comp, 0, comp.length, out, c.out_off, dict);
            if (w !== c.written) return `written ${w} != ${c.written}`;
            return Buffer.from(out).equals(Buffer.from(c.out)) ? true : 'output mismatch';
        });
    } else if (c.op === 'chain') {
        // compressRaw with a table carried across segments, positions absolute
        check(c.id, () => {
            const src = read(c.src);
            const table = new Int32Array(16384);
            if (c.table_init !== 0) table.fill(c.table_init);
            const out = new Uint8Array(c.out_size);
            let op = c.out_off0;
            for (const [s, n, expect] of c.segments) {
                const w = LZ4.compressRaw(src, out, s, n, table, op);
                if (w !== expect) return `segment at ${s}: ${w} != ${expect}`;
                op += w;
            }
            const want = read(c.out);
            if (!Buffer.from(out.subarray(0, op)).equals(Buffer.from(want.subarray(0, op)))) return 'chain output mismatch';
            const tf = new Int32Array(read(c.table_final).buffer);
            for (let k = 0; k < 16384; k++) if (tf[k] !== table[k]) return `table[${k}] ${table[k]} != ${tf[k]}`;
            return true;
        });
    }
}

function concat(parts) {
    const total = parts.reduce((a, b) => a + b.length, 0);
    const all = new Uint8Array(total);
    let o = 0;
    for (const x of parts) { all.set(x, o); o += x.length; }
    return all;
}

for (const c of job.cases) {
    if (c.op === 'raw_edge') {
        // F7 (five arguments -> 0) and the RangeError of output.set (blockCompress.js:37,100,198,232)
        check(c.id, () => {
            const src = read(c.src);
            const out = new Uint8Array(c.out_len);
            const table = new Int32Array(16384);
            let r, err = null;
            try {
                r = c.five_args ? LZ4.compressRaw(src, out, c.start, c.len, table)
                    : LZ4.compressRaw(src, out, c.start, c.len, table, c.out_off);
            } catch (e) { err = e; }
            if (c.ok) {
                if (err) return 'threw ' + err.message;
                if (r !== c.value) return `returned ${r}, expected ${c.value}`;
            } else {
                if (!err) return 'did not throw';
                if (err.name !== c.error_name || err.message !== c.error) return `threw ${err.name}: ${err.message}`;
            }
            if (!Buffer.from(out).equals(Buffer.from(read(c.out_ref)))) return 'output bytes differ';
            if (!Buffer.from(table.buffer).equals(Buffer.from(read(c.table_ref)))) return 'table differs';
            return true;
        });
    } else if (c.op === 'xxh32_stateful') {
        check(c.id, () => {
            const base = read(c.src);
            for (const [n, chunk, seed, h] of c.rows) {
                const st = new LZ4.XXHash32(seed);
                for (let p = 0; p < n; p += chunk) st.update(base.subarray(p, Math.min(n, p + chunk)));
                if (hex(st.digest()) !== h) return `n=${n} chunk=${chunk}: ${hex(st.digest())} != ${h}`;
            }
            return true;
        });
    } else if (c.op === 'stream') {
        // LZ4Encoder (lz4Encode.js) fed the same chunks: the same pieces, bytes and errors
        check(c.id, () => {
            const input = read(c.src);
            const enc = new LZ4.LZ4Encoder(c.block, c.indep, c.checksum);
            const parts = [];
            let err = null;
            try {
                for (let p = 0; p < input.length; p += c.chunk)
                    for (const x of enc.add(input.subarray(p, Math.min(input.length, p + c.chunk)))) parts.push(x.slice());
                for (const x of enc.finish()) parts.push(x.slice());
            } catch (e) { err = e.name + ': ' + e.message; }
            if (err !== c.error) return `error ${err} != ${c.error}`;
            const lens = parts.map((x) => x.length);
            if (JSON.stringify(lens) !== JSON.stringify(c.part_lens)) return `pieces ${lens} != ${c.part_lens}`;
            if (err) return true;
            const all = concat(parts);
            if (hex(LZ4.xxHash32(all, 0)) !== c.stream_xxh) return 'stream bytes differ';
            // LZ4Decoder (the call lz4Decode.js:232 meant) in 50 KB pieces; spec mode round-trips
            for (const mode of ['reference', 'spec']) {
                LZ4.setDecodeMode(mode);
                try {
                    const d = new LZ4.LZ4Decoder(null, mode === 'spec' || c.roundtrip_equals_input);
                    const outs = [];
                    for (let p = 0; p < all.length; p += 50000)
                        for (const x of d.update(all.subarray(p, Math.min(all.length, p + 50000)))) outs.push(x);
                    const back = concat(outs);
                    if ((mode === 'spec' || c.roundtrip_equals_input) && !Buffer.from(back).equals(Buffer.from(input)))
                        return `LZ4Decoder (${mode}) output differs from the input`;
                    const f = LZ4.decompress(all, null, mode === 'spec' || c.roundtrip_equals_input);
                    if (!Buffer.from(f).equals(Buffer.from(back))) return `LZ4Decoder (${mode}) != decompress`;
                } finally {
                    LZ4.setDecodeMode('reference');
                }
            }
            return true;
        });
    } else if (c.op === 'bcs') {
        // block checksums: skipped by default like the reference; written and verified on request
        check(c.id, () => {
            const g = read(c.frame);
            const back = LZ4.decompress(g);
            if (hex(LZ4.xxHash32(back, 0)) !== c.dec_xxh) return 'skip decode differs from the reference';
            const bad = expectThrow(() => LZ4.decompress(g, null, true, true), 'LZ4: Block Checksum Error');
            if (bad !== true) return 'golden frame (marker checksums): ' + bad;
            const data = read(c.src);
            const f = LZ4.compress(data, null, c.block, true, false, true, null, true);
            if (f.length !== c.ours_len || hex(LZ4.xxHash32(f, 0)) !== c.ours_xxh) return 'frame with block checksums != oracle';
            LZ4.setDecodeMode('spec');
            try {
                const rt = LZ4.decompress(f, null, true, true);
                if (!Buffer.from(rt).equals(Buffer.from(data))) return 'verified round trip differs';
            } finally {
                LZ4.setDecodeMode('reference');
            }
            const f2 = f.slice();
            f2[f2.length - 5] ^= 0x40;      // last block's checksum
            return expectThrow(() => LZ4.decompress(f2, null, true, true), 'LZ4: Block Checksum Error');
        });
    }
}
process.stdout.write(JSON.stringify(results) + '\n');
