// Runs the golden cases of a job file (written by tests/test_js_shim.py) through
// the drop-in JS layer (divortio-lz4_amd/js/lz4mi.mjs -> N-API -> gfx950) and
// prints one JSON line of results. Digests use the reference's xxHash32.
import fs from 'fs';
import { LZ4 } from '../../divortio-lz4_amd/js/lz4mi.mjs';

const job = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
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
process.stdout.write(JSON.stringify(results) + '\n');
