import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';
const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const res = [];
for (const bs of [65536, 262144])
    for (const ck of [false, true])
        for (let r = 0; r < 3; r++) {
            const f = LZ4.compress(input, null, bs, true, ck);
            res.push([bs, ck, r, f.length, LZ4.xxHash32(f, 0)]);
            if (r === 0) { try { LZ4.decompress(f); } catch (e) { } }
        }
console.log(JSON.stringify(res));
