// oracle/lz4_js.mjs — TEST / BASELINE INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
//
// A from-scratch JavaScript restatement of the reference's block codec, used as
// the "pure-JS path" CPU baseline bench.py times beside the GPU (BASELINE.json
// north star) and pinned bit-exact to the golden vectors by
// tests/test_js_baseline.py. The reference itself cannot travel to the GPU box;
// this file is our own code with the same algorithm and the same copy
// strategies (typed-array set/copyWithin/fill for long runs, byte loops for
// short ones), so its speed is representative of the reference's.
//
//   compressBlock    src/block/blockCompress.js:31-233 (greedy parse, 14-bit hash,
//                    skip = count >> 6, insert before verify, forward extension only)
//   decompressBlock  src/block/blockDecompress.js:30-275 on independent blocks (no
//                    dictionary); LZ4-spec output, which equals the reference's on the
//                    benchmark generators (no F1 sequences, SURVEY.md §8d)
//   generate         the seeded generators of SURVEY.md §8d (oracle/lz4_oracle.c)

const K_HASH = 2654435761 | 0;

function le32(a, i) {
    return a[i] | (a[i + 1] << 8) | (a[i + 2] << 16) | (a[i + 3] << 24);
}

// token high nibble + 255-run length bytes; returns the new output position
function putLength(out, op, n) {
    n -= 15;
    while (n >= 255) { out[op++] = 255; n -= 255; }
    out[op++] = n;
    return op;
}

function putLiterals(src, out, op, from, n) {
    if (n > 64) {
        out.set(src.subarray(from, from + n), op);
        return op + n;
    }
    for (let k = 0; k < n; k++) out[op++] = src[from + k];
    return op;
}

export function compressBlock(src, out, start, len, table, outPos) {
    const end = (start + len) | 0;
    const mflimit = (end - 12) | 0;
    const mlimit = (end - 5) | 0;
    let i = start | 0, anchor = start | 0, op = outPos | 0;
    let miss = 67;
    while (i < mflimit) {
        const seq = le32(src, i);
        const h = (Math.imul(seq, K_HASH) >>> 18) & 16383;
        const cand = (table[h] - 1) | 0;
        table[h] = (i + 1) | 0;
        if (cand < 0 || cand === i || ((i - cand) >>> 16) !== 0 || le32(src, cand) !== seq) {
            i = (i + (miss++ >> 6)) | 0;
            continue;
        }
        miss = 67;
        const lit = (i - anchor) | 0;
        const tok = op++;
        if (lit >= 15) { out[tok] = 0xF0; op = putLength(out, op, lit); } else out[tok] = lit << 4;
        op = putLiterals(src, out, op, anchor, lit);
        let e = (i + 4) | 0, m = (cand + 4) | 0;
        while (e < mlimit && src[e] === src[m]) { e++; m++; }
        const off = (i - cand) | 0;
        out[op++] = off & 255;
        out[op++] = off >>> 8;
        const code = (e - i - 4) | 0;
        if (code >= 15) { out[tok] |= 15; op = putLength(out, op, code); } else out[tok] |= code;
        i = e;
        anchor = e;
    }
    const lit = (end - anchor) | 0;
    const tok = op++;
    if (lit >= 15) { out[tok] = 0xF0; op = putLength(out, op, lit); } else out[tok] = lit << 4;
    op = putLiterals(src, out, op, anchor, lit);
    return (op - outPos) | 0;
}

function readLength(inp, p, n) {     // returns [length, position]
    let b;
    do { b = inp[p++]; n += b; } while (b === 255);
    return [n, p];
}

export function decompressBlock(inp, inPos, inLen, out, outPos) {
    const inEnd = (inPos + inLen) | 0;
    const outEnd = out.length;
    const o0 = outPos;
    let ip = inPos | 0, op = outPos | 0;
    while (ip < inEnd) {
        const tok = inp[ip++];
        let lit = tok >>> 4;
        if (lit === 15) [lit, ip] = readLength(inp, ip, lit);
        if (op + lit > outEnd) throw new Error('LZ4: Output Buffer Too Small');
        if (ip + lit > inEnd) throw new Error('LZ4: Malformed Input');
        if (lit > 32) {
            out.set(inp.subarray(ip, ip + lit), op);
            op += lit; ip += lit;
        } else {
            for (let k = 0; k < lit; k++) out[op++] = inp[ip++];
        }
        if (ip >= inEnd) break;
        const off = inp[ip] | (inp[ip + 1] << 8);
        ip += 2;
        if (off === 0) throw new Error('LZ4: Invalid Offset 0');
        let ml = tok & 15;
        if (ml === 15) [ml, ip] = readLength(inp, ip, ml);
        ml += 4;
        let s = op - off;
        if (s < 0) throw new Error('LZ4: Dictionary Offset Out of Bounds');
        if (off === 1) {
            out.fill(out[s], op, op + ml);
            op += ml;
        } else if (off >= ml && ml > 16) {
            out.copyWithin(op, s, s + ml);
            op += ml;
        } else {
            const e = op + ml;
            while (op < e) out[op++] = out[s++];
        }
    }
    return (op - o0) | 0;
}

function xorshift(seed) {
    let x = (seed >>> 0) || 1;
    return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x; };
}

export function generate(kind, seed, n) {
    const r = xorshift(seed), b = new Uint8Array(n);
    if (kind === 'random') {
        for (let i = 0; i < n; i += 4) {
            const v = r();
            for (let k = 0; k < 4 && i + k < n; k++) b[i + k] = (v >>> (8 * k)) & 255;
        }
    } else if (kind === 'repetitive') {
        for (let i = 0; i < n; i++) b[i] = i % 251;
    } else if (kind === 'tiles216') {
        const t = new Uint8Array(216 * 64);
        for (let k = 0; k < t.length; k++) t[k] = r() & 255;
        let i = 0;
        while (i < n) {
            const base = 64 * (r() % 216);
            for (let k = 0; k < 64 && i < n; k++) b[i++] = t[base + k];
        }
    } else {
        throw new Error('generator ' + kind);
    }
    return b;
}
