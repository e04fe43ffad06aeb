/**
 * divortio-lz4_amd/js/lz4mi.mjs — drop-in host layer for the MI355X codec.
 *
 * Mirrors the reference's synchronous LZ4 API surface for the hot path
 * (src/lz4.js:27-35): LZ4.compressRaw / decompressRaw (the raw block
 * functions) and LZ4.compress / decompress (the frame layer), with the same
 * argument lists, defaults, return values and thrown messages. The frame
 * header/descriptor logic stays in JS (as the reference's does); every block
 * is compressed/decompressed by the gfx950 kernels through the N-API addon
 * (../lz4mi.node -> liblz4mi.so), batched whenever the blocks are independent.
 *
 * Results are byte-identical to the reference: the encoder is the reference's
 * greedy parse; the decoder runs the LZ4-spec kernel and re-decodes, with the
 * serial reference-exact kernel, any block where the reference's
 * double-copy-tail rewrite (SURVEY.md F1) would change a byte (flag JS_EXACT).
 * There is no CPU fallback: without the addon or a gfx950 device every call
 * throws.
 */
import { createRequire } from 'module';

const require = createRequire(import.meta.url);
const native = require('../lz4mi.node');

const MAGIC = 0x184D2204;
const HASH_TABLE_SIZE = 16384;
const BLOCK_MAX_SIZES = { 4: 65536, 5: 262144, 6: 1048576, 7: 4194304 };
const WINDOW_SIZE = 65536;

// module-global table, as the reference's GLOBAL_HASH_TABLE (bufferCompress.js:56)
const HASH_TABLE = new Int32Array(HASH_TABLE_SIZE);
let decodeFlags = native.JS_EXACT;

/** Coerce like the reference's ensureBuffer (src/shared/lz4Util.js:13-35). */
export function ensureBuffer(input) {
    if (input instanceof Uint8Array) return input;
    if (typeof input === 'string') return new TextEncoder().encode(input);
    if (ArrayBuffer.isView(input)) return new Uint8Array(input.buffer, input.byteOffset, input.byteLength);
    if (input instanceof ArrayBuffer) return new Uint8Array(input);
    if (Array.isArray(input)) return new Uint8Array(input);
    if (typeof input === 'object' && input !== null) {
        try {
            const json = JSON.stringify(input);
            if (json !== undefined) return new TextEncoder().encode(json);
        } catch (e) { /* fall through */ }
    }
    throw new TypeError('LZ4: Input must be a String, ArrayBuffer, View, Array, or Serializable Object');
}

function writeU32(b, v, n) {
    b[n] = v & 0xFF;
    b[n + 1] = (v >>> 8) & 0xFF;
    b[n + 2] = (v >>> 16) & 0xFF;
    b[n + 3] = (v >>> 24) & 0xFF;
}

function readU32(b, n) {
    return (b[n] | (b[n + 1] << 8) | (b[n + 2] << 16) | (b[n + 3] << 24)) >>> 0;
}

function blockId(bytes) {             // bufferCompress.js:77-82
    if (!bytes || bytes <= 65536) return 4;
    if (bytes <= 262144) return 5;
    if (bytes <= 1048576) return 6;
    return 7;
}

/** compressBlock (src/block/blockCompress.js:31) on the GPU. */
export function compressRaw(src, output, srcStart, srcLen, hashTable, outputOffset) {
    return native.compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset);
}

/** decompressBlock (src/block/blockDecompress.js:30) on the GPU. */
export function decompressRaw(input, inputOffset, inputSize, output, outputOffset, dictionary) {
    return native.decompressBlock(input, inputOffset, inputSize, output, outputOffset, dictionary || null,
        decodeFlags);
}

/**
 * Decoder semantics: 'reference' (default; byte-identical to the reference
 * decoder, F1 included) or 'spec' (LZ4 specification: the parallel kernel only).
 */
export function setDecodeMode(mode) {
    if (mode === 'reference') decodeFlags = native.JS_EXACT;
    else if (mode === 'spec') decodeFlags = 0;
    else throw new TypeError("lz4mi: decode mode must be 'reference' or 'spec'");
}

// Dictionary prewarm of the frame encoder: the reference's Jenkins-style hash
// (bufferCompress.js:186-204), not the block encoder's multiplicative hash.
function prewarm(table, buf, dictLen) {
    const limit = (dictLen - 4) | 0;
    for (let i = 0; i <= limit; i++) {
        let h = (buf[i] | (buf[i + 1] << 8) | (buf[i + 2] << 16) | (buf[i + 3] << 24)) | 0;
        h = (h + 0x7ED55D16 + (h << 12)) | 0;
        h = (h ^ 0xC761C23C ^ (h >>> 19)) | 0;
        h = (h + 0x165667B1 + (h << 5)) | 0;
        h = ((h + 0xD3A2646C) ^ (h << 9)) | 0;
        h = (h + 0xFD7046C5 + (h << 3)) | 0;
        h = (h ^ 0xB55A4F09 ^ (h >>> 16)) | 0;
        table[(h >>> 18) & 16383] = i + 1;
    }
}

/**
 * LZ4 frame compression: same signature, defaults and output bytes as the
 * reference's compressBuffer (src/buffer/bufferCompress.js:100-259).
 */
export function compress(input, dictionary = null, maxBlockSize = 4194304, blockIndependence = false,
    contentChecksum = false, addContentSize = true, outputBuffer = null) {
    const rawInput = ensureBuffer(input);
    let work = rawInput;
    let start = 0;
    let dictLen = 0;
    let dictId = null;
    if (dictionary && dictionary.length > 0) {
        const d = ensureBuffer(dictionary);
        dictId = native.xxHash32(d, 0);
        const win = d.length > 65536 ? d.subarray(d.length - 65536) : d;
        dictLen = win.length;
        work = new Uint8Array(dictLen + rawInput.length);
        work.set(win, 0);
        work.set(rawInput, dictLen);
        start = dictLen;
    }
    const len = rawInput.length | 0;
    const bd = blockId(maxBlockSize);
    const bsize = BLOCK_MAX_SIZES[bd] | 0;
    const output = outputBuffer || new Uint8Array((19 + len + ((len / 255) | 0) + 64 + 8) | 0);
    let op = 0;
    output[op++] = 0x04; output[op++] = 0x22; output[op++] = 0x4D; output[op++] = 0x18;
    let flg = 1 << 6;
    if (blockIndependence) flg |= 0x20;
    if (contentChecksum) flg |= 0x04;
    if (dictId !== null) flg |= 0x01;
    if (addContentSize) flg |= 0x08;
    output[op++] = flg;
    output[op++] = (bd & 7) << 4;
    if (addContentSize) {
        writeU32(output, len >>> 0, op); op += 4;
        writeU32(output, (len / 4294967296) | 0, op); op += 4;
    }
    if (dictId !== null) { writeU32(output, dictId, op); op += 4; }
    output[op] = (native.xxHash32(output.subarray(4, op), 0) >>> 8) & 0xFF;
    op++;

    const table = HASH_TABLE;
    table.fill(0);
    if (dictLen > 0) prewarm(table, work, dictLen);

    const end = start + len;
    const emit = (pos, n, compSize, bytes) => {
        if (compSize > 0 && compSize < n) {
            writeU32(output, compSize, op);
            output.set(bytes, op + 4);
            op += 4 + compSize;
        } else {
            writeU32(output, (n | 0x80000000) >>> 0, op);
            output.set(work.subarray(pos, pos + n), op + 4);
            op += 4 + n;
        }
    };
    let pos = start;
    if (blockIndependence) {
        // The first block sees the (possibly prewarmed) table; every later one a fresh table.
        if (dictLen > 0 && pos < end) {
            const n = Math.min(bsize, end - pos);
            const scratch = new Uint8Array(n + ((n / 255) | 0) + 16);
            const c = native.compressBlock(work, scratch, pos, n, table, 0);
            emit(pos, n, c, scratch.subarray(0, Math.max(0, Math.min(c, scratch.length))));
            table.fill(0);
            pos += n;
        }
        const nb = Math.ceil((end - pos) / bsize);
        if (nb > 0) {
            const srcOff = new Float64Array(nb), srcLen = new Uint32Array(nb);
            const outOff = new Float64Array(nb), outLen = new Uint32Array(nb);
            let slot = 0;
            for (let b = 0; b < nb; b++) {
                srcOff[b] = pos + b * bsize;
                srcLen[b] = Math.min(bsize, end - srcOff[b]);
                outOff[b] = slot;
                slot += srcLen[b] + ((srcLen[b] / 255) | 0) + 16;
            }
            const scratch = new Uint8Array(slot);
            native.compressBlocks(work, srcOff, srcLen, scratch, outOff, outLen);
            for (let b = 0; b < nb; b++)
                emit(srcOff[b], srcLen[b], outLen[b], scratch.subarray(outOff[b], outOff[b] + outLen[b]));
            pos = end;
        }
    } else {
        // Dependent blocks (the reference's default): one table carried across blocks.
        while (pos < end) {
            const n = Math.min(bsize, end - pos);
            const scratch = new Uint8Array(n + ((n / 255) | 0) + 16);
            const c = native.compressBlock(work, scratch, pos, n, table, 0);
            emit(pos, n, c, scratch.subarray(0, Math.max(0, Math.min(c, scratch.length))));
            pos += n;
        }
    }
    writeU32(output, 0, op); op += 4;
    if (contentChecksum) { writeU32(output, native.xxHash32(rawInput, 0), op); op += 4; }
    return output.subarray(0, op);
}

/**
 * LZ4 frame decompression: same signature, strategies (direct write when the
 * content size is known, else a 64 KiB rolling window) and errors as the
 * reference's decompressBuffer (src/buffer/bufferDecompress.js:51-220).
 * Blocks of a known-size frame are decoded in one batched GPU call; a frame
 * whose blocks reference each other is decoded block by block.
 */
export function decompress(input, dictionary = null, verifyChecksum = true) {
    const data = ensureBuffer(input);
    const len = data.length | 0;
    let pos = 0;
    if (len < 4 || readU32(data, 0) !== MAGIC) throw new Error('LZ4: Invalid Magic Number');
    pos = 4;
    const flg = data[pos++];
    const version = (flg & 0xC0) >> 6;
    if (version !== 1) throw new Error(`LZ4: Unsupported Version ${version}`);
    const hasBlockChecksum = (flg & 0x10) !== 0;
    const hasContentSize = (flg & 0x08) !== 0;
    const hasContentChecksum = (flg & 0x04) !== 0;
    const hasDictId = (flg & 0x01) !== 0;
    const bd = data[pos++];
    let expected = 0;
    if (hasContentSize) {
        const lo = readU32(data, pos), hi = readU32(data, pos + 4);
        pos += 8;
        expected = hi * 4294967296 + lo;
    }
    if (hasDictId) pos += 4;
    pos++;

    // the block list, exactly as the reference walks it
    const blocks = [];
    while (pos < len) {
        const bs = readU32(data, pos);
        pos += 4;
        if (bs === 0) break;
        blocks.push({ pos, raw: (bs & 0x80000000) !== 0, n: bs & 0x7FFFFFFF });
        pos += bs & 0x7FFFFFFF;
        if (hasBlockChecksum) pos += 4;
    }

    let result;
    if (expected > 0) {
        result = new Uint8Array(expected);
        const dict = dictionary || null;
        if (!batchDirect(data, blocks, result, dict, BLOCK_MAX_SIZES[(bd >> 4) & 7] || 4194304)) {
            result.fill(0);      // forget whatever the batch attempt wrote
            let rp = 0;
            for (const b of blocks) {
                if (b.raw) {
                    result.set(data.subarray(b.pos, b.pos + b.n), rp);
                    rp += b.n;           // the reference advances by the declared size
                } else {
                    rp += native.decompressBlock(data, b.pos, b.n, result, rp, dict, decodeFlags);
                }
            }
        }
    } else {
        const chunks = [];
        const window = new Uint8Array(WINDOW_SIZE);
        let wpos = 0;
        if (dictionary) {
            const dl = dictionary.length;
            if (dl > WINDOW_SIZE) { window.set(dictionary.subarray(dl - WINDOW_SIZE), 0); wpos = WINDOW_SIZE; }
            else { window.set(dictionary, 0); wpos = dl; }
        }
        const workspace = new Uint8Array(BLOCK_MAX_SIZES[7]);
        for (const b of blocks) {
            let chunk;
            if (b.raw) {
                chunk = data.slice(b.pos, b.pos + b.n);
            } else {
                const w = native.decompressBlock(data, b.pos, b.n, workspace, 0,
                    wpos > 0 ? window.subarray(0, wpos) : null, decodeFlags);
                chunk = workspace.slice(0, w);
            }
            chunks.push(chunk);
            const cl = chunk.length;
            if (cl >= WINDOW_SIZE) { window.set(chunk.subarray(cl - WINDOW_SIZE), 0); wpos = WINDOW_SIZE; }
            else if (wpos + cl <= WINDOW_SIZE) { window.set(chunk, wpos); wpos += cl; }
            else {
                const keep = WINDOW_SIZE - cl;
                window.copyWithin(0, wpos - keep, wpos);
                window.set(chunk, keep);
                wpos = WINDOW_SIZE;
            }
        }
        if (chunks.length === 1) {
            result = chunks[0];
        } else {
            let total = 0;
            for (const c of chunks) total += c.length;
            result = new Uint8Array(total);
            let o = 0;
            for (const c of chunks) { result.set(c, o); o += c.length; }
        }
    }
    if (hasContentChecksum && verifyChecksum) {
        if (readU32(data, pos) !== native.xxHash32(result, 0)) throw new Error('LZ4: Content Checksum Error');
    }
    return result;
}

// Known-size frame: every compressed block is assumed to fill a whole block of
// the descriptor's size (the reference encoder's layout) and all are decoded in
// one batched call. Returns false (nothing committed that the block-by-block
// path does not rewrite) when the assumption or independence does not hold.
function batchDirect(data, blocks, result, dict, bmax) {
    const comp = blocks.filter((b) => !b.raw);
    if (comp.length < 2) return false;
    const nb = comp.length;
    const inOff = new Float64Array(nb), inLen = new Uint32Array(nb);
    const outOff = new Float64Array(nb), outCap = new Uint32Array(nb);
    const outLen = new Uint32Array(nb), status = new Int32Array(nb);
    let rp = 0, k = 0;
    const rawAt = [];
    for (const b of blocks) {
        if (b.raw) {
            const m = Math.min(b.n, Math.max(0, data.length - b.pos));
            if (rp + m > result.length) return false;
            rawAt.push([b, rp, m]);
            rp += b.n;
        } else {
            if (b.pos + b.n > data.length || rp > result.length) return false;
            inOff[k] = b.pos; inLen[k] = b.n; outOff[k] = rp;
            outCap[k] = Math.min(bmax, result.length - rp);
            rp += outCap[k];
            k++;
        }
    }
    for (const [b, at, m] of rawAt) result.set(data.subarray(b.pos, b.pos + m), at);
    native.decompressBlocks(data, inOff, inLen, result, outOff, outCap, outLen, status, dict, decodeFlags);
    for (let b = 0; b < nb; b++) {
        if (status[b] === native.ERR_CROSS_BLOCK) {
            // reads bytes of an earlier block (dependent frame, or the F1 rewrite
            // at a block start): every earlier block is final now, decode it alone
            try {
                outLen[b] = native.decompressBlock(data, inOff[b], inLen[b], result, outOff[b], dict, decodeFlags);
            } catch (e) {
                return false;
            }
            status[b] = 0;
        }
        if (status[b] !== 0) return false;
        if (outLen[b] !== outCap[b] && outOff[b] + outLen[b] !== result.length) return false;
        if (outLen[b] !== outCap[b] && b !== nb - 1) return false;
    }
    return true;
}

export function xxHash32(input, seed = 0) {
    return native.xxHash32(ensureBuffer(input), seed);
}

export function compressBlocks(src, srcOff, srcLen, out, outOff, outLen) {
    return native.compressBlocks(src, srcOff, srcLen, out, outOff, outLen);
}

export function decompressBlocks(input, inOff, inLen, output, outOff, outCap, outLen, status, dictionary = null) {
    return native.decompressBlocks(input, inOff, inLen, output, outOff, outCap, outLen, status, dictionary,
        decodeFlags);
}

export const LZ4 = {
    compressRaw,
    decompressRaw,
    compress,
    decompress,
    // batched raw-block entry points (no reference counterpart: the frame layer's block loops)
    compressBlocks,
    decompressBlocks,
    xxHash32,
    setDecodeMode,
    version: native.version,
};

export default LZ4;
