import fs from 'fs';
import { LZ4 } from '../divortio-lz4_amd/js/lz4mi.mjs';
const input = new Uint8Array(fs.readFileSync(process.argv[2]));
const frame = LZ4.compress(input, null, 4194304, true, false);
fs.writeFileSync(process.argv[3], frame);
for (const mode of ['spec', 'reference']) {
    LZ4.setDecodeMode(mode);
    const back = LZ4.decompress(frame);
    let first = -1;
    for (let i = 0; i < input.length; i++) if (back[i] !== input[i]) { first = i; break; }
    console.log(mode, 'len', back.length, 'first diff', first);
    if (mode === 'reference') fs.writeFileSync('/tmp/back_ref.bin', back);
}
