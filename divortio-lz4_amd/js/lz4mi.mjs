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
 *
 * Routing (SURVEY.md §8b): independent blocks go to the GPU in batches; work that is
 * one serial chain by definition — dependent-block frames (LZ4.compress's default,
 * bufferCompress.js:182-236) and a dictionary frame's first block — runs on the
 * addon's host encoder (csrc/lz4mi_host.cpp), byte-identical, because one GPU wave
 * walks a chain ~10x slower than one CPU core (DESIGN §4.2, §5 "Routing").
 * There is no CPU fallback: without the addon or a gfx950 device every call
 * throws, the host-routed ones included.
 */
import { createRequire } from 'module';

const require = createRequire(import.meta.url);
const native = require('../lz4mi.node');

const MAGIC = 0x184D2204;
const HASH_TABLE_SIZE = 16384;
const BLOCK_MAX_SIZES = { 4: 65536, 5: 262144, 6: 1048576, 7: 4194304 };
const WINDOW_SIZE = 65536;
const DECODE_BATCH_BYTES = 256 * 1024 * 1024;   // output slots per batched decode call (LZ4Decoder)

// module-global table, as the reference's GLOBAL_HASH_TABLE (bufferCompress.js:56)
const HASH_TABLE = new Int32Array(HASH_TABLE_SIZE);
let decodeFlags = native.JS_EXACT;
let deviceChecked = false;

// The host-routed calls still require the device the library serves (no CPU fallback).
function requireDevice() {
    if (deviceChecked) return;
    const st = native.deviceCount() === 0 ? -102 : native.init(-1);
    if (st !== 0) throw new Error(native.statusMessage(st));
    deviceChecked = true;
}

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

// Routing (SURVEY.md §8b, DESIGN §5.1). A compress batch of b independent blocks costs the GPU
// about one block's chain latency (every block is one wave, all resident at once) plus the
// PCIe copies, and the host b blocks one after another, so the GPU wins from a block count on
// that is nearly independent of the block size. The crossovers below are measured on the box
// (bench.py `single_block` and `napi_end_to_end.crossover`; 4 MiB tiles216: compress GPU
// ~29 ms for one block vs host 1.1 ms per block -> 32 blocks). Decode of up to 192 blocks takes
// the small-batch path (a wave per ~8 KiB of compressed block, round 5): through N-API with a
// collection before each call, GPU vs host ms 1 block 0.51 vs 0.26, 4: 1.18 vs 1.05, 8: 2.13 vs
// 2.2-2.4 (profiles/r05_hostio/ab_gc.log), a crossover at ~8 blocks; 8 also keeps frames of a few blocks whose reference-mode decode needs the
// double-copy-tail fix-up (the reference's own 25 MiB JSON benchmark: 7 blocks) on the host.
// A raw-block call is one block: the host's. 'gpu' / 'host' force one side for every call
// (tests, and measuring the crossover).
const HOST_MAX_BLOCKS_COMPRESS = 32;
const HOST_MAX_BLOCKS_DECOMPRESS = 8;
let routing = 'auto';

/** 'auto' (default: the measured crossovers above), 'gpu' or 'host' (every block call on that side). */
export function setRouting(mode) {
    if (mode !== 'auto' && mode !== 'gpu' && mode !== 'host')
        throw new TypeError("lz4mi: routing must be 'auto', 'gpu' or 'host'");
    routing = mode;
}

// Calls routed to each side since the last routeStats(true): what a figure measured through
// this layer actually ran on (bench.py records them beside every drop-in rate).
const routeCount = { host: 0, gpu: 0 };

const hostRoute = (nblocks, max) => {
    if (routing === 'gpu' || (routing === 'auto' && nblocks > max)) {
        routeCount.gpu++;
        return false;
    }
    // The host codec runs on this thread, yet it too requires the device: the drop-in is the
    // GPU codec with a measured crossover, not a CPU library with a GPU option, so every route
    // fails the same way without a gfx950 device (INTEGRATION.md, "Routing").
    requireDevice();
    routeCount.host++;
    return true;
};

/** Calls routed to the host codec and to the GPU since the last reset: { host, gpu }. */
export function routeStats(reset = false) {
    const r = { host: routeCount.host, gpu: routeCount.gpu };
    if (reset) routeCount.host = routeCount.gpu = 0;
    return r;
}

/** compressBlock (src/block/blockCompress.js:31): one serial chain, the host encoder unless routing 'gpu'. */
export function compressRaw(src, output, srcStart, srcLen, hashTable, outputOffset) {
    if (hostRoute(1, HOST_MAX_BLOCKS_COMPRESS))
        return native.compressBlockHost(src, output, srcStart, srcLen, hashTable, outputOffset);
    return native.compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset);
}

/** decompressBlock (src/block/blockDecompress.js:30): one block, the host decoder unless routing 'gpu'. */
export function decompressRaw(input, inputOffset, inputSize, output, outputOffset, dictionary) {
    const f = hostRoute(1, HOST_MAX_BLOCKS_DECOMPRESS) ? native.decompressBlockHost : native.decompressBlock;
    return f(input, inputOffset, inputSize, output, outputOffset, dictionary || null, decodeFlags);
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
 * Streaming XXH32 — class XXHash32 (src/xxhash32/xxhash32Stateful.js:13-152) over the
 * addon's host implementation (16-byte carry, `(totalLen + len) | 0` length). The state
 * is a 56-byte Uint8Array owned by this object.
 */
export class XXHash32 {
    constructor(seed = 0) {
        this.seed = seed | 0;
        this.state = native.xxh32Reset(this.seed >>> 0, 0);
    }

    update(input) {
        native.xxh32Update(this.state, input);
    }

    digest() {
        return native.xxh32Digest(this.state) >>> 0;
    }
}

// Block checksums (FLG bit 0x10): XXH32 (spec convergence, seed 0) of each block's payload,
// computed for all blocks of a frame in one batched GPU call over the frame bytes.
function blockChecksums(buf, payOff, payLen) {
    const n = payLen.length;
    const hashes = new Uint32Array(n);
    if (n > 0) native.xxh32Blocks(buf, payOff, payLen, 0, hashes, native.XXH_STANDARD);
    return hashes;
}

/**
 * LZ4 frame compression: same signature, defaults and output bytes as the
 * reference's compressBuffer (src/buffer/bufferCompress.js:100-259).
 * `blockChecksum` (an addition; the reference never writes them) sets FLG bit 0x10
 * and follows every block with the XXH32 of its payload.
 */
export function compress(input, dictionary = null, maxBlockSize = 4194304, blockIndependence = false,
    contentChecksum = false, addContentSize = true, outputBuffer = null, blockChecksum = false) {
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
    const output = outputBuffer || new Uint8Array((19 + len + ((len / 255) | 0) + 64 + 8 +
        (blockChecksum ? 4 * (Math.ceil(len / bsize) + 1) : 0)) | 0);
    let op = 0;
    output[op++] = 0x04; output[op++] = 0x22; output[op++] = 0x4D; output[op++] = 0x18;
    let flg = 1 << 6;
    if (blockIndependence) flg |= 0x20;
    if (blockChecksum) flg |= 0x10;
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
    const sums = [];    // [payload position, payload length] of every block (block checksums)
    const emit = (pos, n, compSize, bytes) => {
        if (compSize > 0 && compSize < n) {
            writeU32(output, compSize, op);
            output.set(bytes, op + 4);
            if (blockChecksum) sums.push(op + 4, compSize);
            op += 4 + compSize;
        } else {
            writeU32(output, (n | 0x80000000) >>> 0, op);
            output.set(work.subarray(pos, pos + n), op + 4);
            if (blockChecksum) sums.push(op + 4, n);
            op += 4 + n;
        }
        if (blockChecksum) op += 4;
    };
    let pos = start;
    if (blockIndependence) {
        // The first block sees the (possibly prewarmed) table; every later one a fresh table.
        if (dictLen > 0 && pos < end) {
            const n = Math.min(bsize, end - pos);
            const scratch = new Uint8Array(n + ((n / 255) | 0) + 16);
            const c = compressRaw(work, scratch, pos, n, table, 0);     // one chain: the host's unless 'gpu'
            emit(pos, n, c, scratch.subarray(0, Math.max(0, Math.min(c, scratch.length))));
            table.fill(0);
            pos += n;
        }
        const nb = Math.ceil((end - pos) / bsize);
        if (nb > 0 && hostRoute(nb, HOST_MAX_BLOCKS_COMPRESS)) {
            const scratch = new Uint8Array(bsize + ((bsize / 255) | 0) + 16);
            for (; pos < end; pos += bsize) {
                const n = Math.min(bsize, end - pos);
                table.fill(0);
                const c = native.compressBlockHost(work, scratch, pos, n, table, 0);
                emit(pos, n, c, scratch.subarray(0, Math.max(0, Math.min(c, scratch.length))));
            }
        } else if (nb > 0) {
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
        // Dependent blocks (the reference's default): one table carried across blocks, each
        // block exactly compressBlock(work, scratch, pos, n, table, 0), the table updated in
        // place — one serial chain, so the host route (the chain kernel runs it as one GPU
        // wave: 0.12 GB/s on tiles216 against ~1.5 GB/s for the host encoder, DESIGN §5).
        const nb = Math.ceil((end - pos) / bsize);
        if (nb > 0) routeCount[routing === 'gpu' ? 'gpu' : 'host']++;
        if (nb > 0 && routing === 'gpu') {
            let slot = 0;
            const outOff = new Float64Array(nb), compLen = new Uint32Array(nb);
            for (let b = 0; b < nb; b++) {
                const n = Math.min(bsize, end - pos - b * bsize);
                outOff[b] = slot;
                slot += n + ((n / 255) | 0) + 16;
            }
            const scratch = new Uint8Array(slot);
            native.compressChain(work, pos, end - pos, bsize, table, scratch, outOff, compLen);
            for (let b = 0; b < nb; b++) {
                const n = Math.min(bsize, end - pos);
                emit(pos, n, compLen[b], scratch.subarray(outOff[b], outOff[b] + compLen[b]));
                pos += n;
            }
        } else if (nb > 0) {
            const outOff = new Float64Array(nb), compLen = new Uint32Array(nb);
            let slot = 0;
            for (let b = 0; b < nb; b++) {
                const n = Math.min(bsize, end - pos - b * bsize);
                outOff[b] = slot;
                slot += n + ((n / 255) | 0) + 16;
            }
            const scratch = new Uint8Array(slot);
            requireDevice();
            native.compressChainHost(work, pos, end - pos, bsize, table, scratch, outOff, compLen);
            for (let b = 0; b < nb; b++) {
                const n = Math.min(bsize, end - pos);
                emit(pos, n, compLen[b], scratch.subarray(outOff[b], outOff[b] + compLen[b]));
                pos += n;
            }
        }
    }
    if (blockChecksum && sums.length > 0) {
        const nb = sums.length / 2;
        const payOff = new Float64Array(nb), payLen = new Uint32Array(nb);
        for (let b = 0; b < nb; b++) { payOff[b] = sums[2 * b]; payLen[b] = sums[2 * b + 1]; }
        const h = blockChecksums(output, payOff, payLen);
        for (let b = 0; b < nb; b++) writeU32(output, h[b], payOff[b] + payLen[b]);
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
 * Block checksums (FLG 0x10) are skipped like the reference does (:191) unless
 * `verifyBlockChecksum` (an addition) asks to check them: one batched GPU XXH32
 * over all payloads; the first mismatching block throws "LZ4: Block Checksum Error".
 */
export function decompress(input, dictionary = null, verifyChecksum = true, verifyBlockChecksum = false) {
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
    if (hasBlockChecksum && verifyBlockChecksum && blocks.length > 0) {
        const nb = blocks.length;
        const payOff = new Float64Array(nb), payLen = new Uint32Array(nb);
        for (let b = 0; b < nb; b++) {
            payOff[b] = blocks[b].pos;
            payLen[b] = Math.max(0, Math.min(blocks[b].n, len - blocks[b].pos));
        }
        const h = blockChecksums(data, payOff, payLen);
        for (let b = 0; b < nb; b++) {
            const at = blocks[b].pos + blocks[b].n;
            if (at + 4 > len || readU32(data, at) !== h[b]) throw new Error('LZ4: Block Checksum Error');
        }
    }

    // Routing: a frame of dependent blocks (FLG bit 0x20 clear) is one serial chain — each
    // block reads its predecessors' output — so its blocks go through the addon's host
    // decoder in order; independent blocks are decoded on the GPU in one batch.
    const independent = (flg & 0x20) !== 0;
    let ncomp = 0;
    for (const b of blocks) if (!b.raw) ncomp++;
    const host = hostRoute(independent ? ncomp : 0, HOST_MAX_BLOCKS_DECOMPRESS);
    const decodeBlock = host ? native.decompressBlockHost : native.decompressBlock;
    let result;
    if (expected > 0) {
        result = new Uint8Array(expected);
        const dict = dictionary || null;
        if (host || !batchDirect(data, blocks, result, dict, BLOCK_MAX_SIZES[(bd >> 4) & 7] || 4194304)) {
            if (!host) result.fill(0);            // forget whatever the batch attempt wrote
            let rp = 0;
            for (const b of blocks) {
                if (b.raw) {
                    result.set(data.subarray(b.pos, b.pos + b.n), rp);
                    rp += b.n;           // the reference advances by the declared size
                } else {
                    rp += decodeBlock(data, b.pos, b.n, result, rp, dict, decodeFlags);
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
                const w = decodeBlock(data, b.pos, b.n, workspace, 0,
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
            try {   // (one block: the host decoder unless routing 'gpu')
                outLen[b] = decompressRaw(data, inOff[b], inLen[b], result, outOff[b], dict);
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

// ---------------------------------------------------------------------------
// Streaming encoder / decoder (src/shared/lz4Encode.js, src/shared/lz4Decode.js).

// The reference's LZ4Encoder compresses a block into a Uint8Array(blockSize + 1028) at
// offset 4 (lz4Encode.js:232-245); a literal run > 64 bytes that does not fit throws the
// RangeError of output.set (blockCompress.js:100,198). A batch-compressed block is walked
// to find that throw when its output overran the array (incompressible blocks > 261 KiB).
function encoderOverflowThrows(comp, cap) {
    let op = 4, ip = 0;
    const n = comp.length;
    while (ip < n) {
        const tok = comp[ip++];
        op++;
        let lit = tok >>> 4;
        if (lit === 15) {
            let b;
            do { b = comp[ip++]; lit += b; op++; } while (b === 255 && ip < n);
        }
        if (lit > 64 && op + lit > cap) return true;
        op += lit;
        ip += lit;
        if (ip >= n) break;          // the final literals
        ip += 2;
        op += 2;
        if ((tok & 15) === 15) {
            let b;
            do { b = comp[ip++]; op++; } while (b === 255 && ip < n);
        }
    }
    return false;
}

function rangeError() { return new RangeError('Source is too large'); }

function frameHeader(blockIndependence, contentChecksum, bdId, dictId) {   // lz4Encode.js:61-94
    const h = new Uint8Array(15);
    let p = 0;
    writeU32(h, MAGIC, p); p += 4;
    let flg = 1 << 6;
    if (blockIndependence) flg |= 0x20;
    if (contentChecksum) flg |= 0x04;
    if (dictId) flg |= 0x01;
    h[p++] = flg;
    h[p++] = (bdId & 7) << 4;
    if (dictId) { writeU32(h, dictId, p); p += 4; }
    h[p] = (native.xxHash32(h.subarray(4, p), 0) >>> 8) & 0xFF;
    p++;
    return h.subarray(0, p);
}

/**
 * Streaming frame encoder with the reference LZ4Encoder's API and output
 * (src/shared/lz4Encode.js:96-340): add(chunk) returns the frame pieces ready so far
 * (header, then one Uint8Array per block: size word + payload), finish() the rest
 * (remaining blocks, EndMark, content checksum). Independent-block streams compress
 * every block an add() completes in one batched GPU call; dependent streams carry the
 * hash table and the 64 KiB window from block to block like the reference (one GPU call
 * per block, the table rebased after each, :262-290).
 */
export class LZ4Encoder {
    constructor(maxBlockSize = 4194304, blockIndependence = false, contentChecksum = false, dictionary = null) {
        this.blockIndependence = blockIndependence;
        this.contentChecksum = contentChecksum;
        this.blockSize = BLOCK_MAX_SIZES[blockId(maxBlockSize)] || 4194304;
        this.bdId = blockId(this.blockSize);
        this.buffer = new Uint8Array(0);
        this.hasWrittenHeader = false;
        this.isClosed = false;
        this.hashTable = new Int32Array(HASH_TABLE_SIZE);
        this.dictSize = 0;
        if (this.contentChecksum) this.hasher = new XXHash32(0);
        this.dictId = null;
        if (dictionary) {
            // the reference chains digest() on update()'s undefined result (lz4Encode.js:130)
            throw new TypeError("Cannot read property 'digest' of undefined");
        }
    }

    add(chunk) {
        if (this.isClosed) throw new Error('Stream is closed');
        const data = ensureBuffer(chunk);
        if (data.length === 0) return [];
        if (this.contentChecksum) this.hasher.update(data);
        const nb = new Uint8Array(this.buffer.length + data.length);
        nb.set(this.buffer);
        nb.set(data, this.buffer.length);
        this.buffer = nb;
        const results = [];
        if (!this.hasWrittenHeader) {
            results.push(frameHeader(this.blockIndependence, this.contentChecksum, this.bdId, this.dictId));
            this.hasWrittenHeader = true;
        }
        if (this.blockIndependence) {
            const n = Math.floor((this.buffer.length - this.dictSize) / this.blockSize);
            if (n > 0) for (const b of this._flushIndependent(n, false)) results.push(b);
        } else {
            while (this.buffer.length >= this.dictSize + this.blockSize) results.push(this._flushDependent(false));
        }
        return results;
    }

    // n full blocks (or, final, everything left) of an independent stream in one batched call
    _flushIndependent(n, final) {
        const bs = this.blockSize;
        const sizes = [];
        let left = this.buffer.length - this.dictSize;
        for (let b = 0; b < n || (final && left > 0); b++) {
            const k = Math.min(bs, left);
            sizes.push(k);
            left -= k;
        }
        const nb = sizes.length;
        const srcOff = new Float64Array(nb), srcLen = new Uint32Array(nb);
        const outOff = new Float64Array(nb), outLen = new Uint32Array(nb);
        let pos = this.dictSize, slot = 0;
        for (let b = 0; b < nb; b++) {
            srcOff[b] = pos; srcLen[b] = sizes[b]; outOff[b] = slot;
            pos += sizes[b];
            slot += sizes[b] + ((sizes[b] / 255) | 0) + 16;
        }
        const scratch = new Uint8Array(slot);
        if (hostRoute(nb, HOST_MAX_BLOCKS_COMPRESS)) {
            const t = new Int32Array(HASH_TABLE_SIZE);
            for (let b = 0; b < nb; b++) {
                t.fill(0);
                outLen[b] = native.compressBlockHost(this.buffer, scratch.subarray(outOff[b]), srcOff[b], srcLen[b], t, 0);
            }
        } else {
            native.compressBlocks(this.buffer, srcOff, srcLen, scratch, outOff, outLen);
        }
        const out = [];
        for (let b = 0; b < nb; b++) {
            const k = sizes[b], c = outLen[b];
            const comp = scratch.subarray(outOff[b], outOff[b] + c);
            const cap = k + 1024 + 4;               // Uint8Array(maxOutputSize + 4), lz4Encode.js:232-233
            if (c + 4 > cap && encoderOverflowThrows(comp, cap)) throw rangeError();
            let rec;
            if (c > 0 && c < k) {
                rec = new Uint8Array(c + 4);
                writeU32(rec, c, 0);
                rec.set(comp, 4);
            } else {
                rec = new Uint8Array(k + 4);
                writeU32(rec, (k | 0x80000000) >>> 0, 0);
                rec.set(this.buffer.subarray(srcOff[b], srcOff[b] + k), 4);
            }
            out.push(rec);
        }
        this.buffer = this.buffer.subarray(pos);
        this.dictSize = 0;
        return out;
    }

    // lz4Encode.js:215-298 for a dependent stream: one block with the carried table
    _flushDependent(final) {
        const available = this.buffer.length - this.dictSize;
        if (available === 0 && !final) return new Uint8Array(0);
        let blockSize = this.blockSize;
        if (available < blockSize) {
            if (final) blockSize = available;
            else return new Uint8Array(0);
        }
        const srcStart = this.dictSize;
        const output = new Uint8Array(blockSize + 1024 + 4);
        const compSize = compressRaw(this.buffer, output, srcStart, blockSize, this.hashTable, 4);   // one chain
        let rec;
        if (compSize > 0 && compSize < blockSize) {
            writeU32(output, compSize, 0);
            rec = output.subarray(0, compSize + 4);
        } else {
            writeU32(output, (blockSize | 0x80000000) >>> 0, 0);
            output.set(this.buffer.subarray(srcStart, srcStart + blockSize), 4);
            rec = output.subarray(0, blockSize + 4);
        }
        const consumedEnd = srcStart + blockSize;
        const preserveLen = Math.min(consumedEnd, WINDOW_SIZE);
        const shift = consumedEnd - preserveLen;
        this.buffer = this.buffer.subarray(shift);
        this.dictSize = preserveLen;
        const t = this.hashTable;
        for (let i = 0; i < HASH_TABLE_SIZE; i++) t[i] = t[i] > shift ? t[i] - shift : 0;
        return rec;
    }

    finish() {
        if (this.isClosed) return [];
        this.isClosed = true;
        const frames = [];
        if (!this.hasWrittenHeader)
            frames.push(frameHeader(this.blockIndependence, this.contentChecksum, this.bdId, this.dictId));
        if (this.blockIndependence) {
            if (this.buffer.length - this.dictSize > 0) for (const b of this._flushIndependent(0, true)) frames.push(b);
        } else {
            while (this.buffer.length - this.dictSize > 0) frames.push(this._flushDependent(true));
        }
        const end = new Uint8Array(4);
        frames.push(end);
        if (this.contentChecksum && this.hasher) {
            const b = new Uint8Array(4);
            writeU32(b, this.hasher.digest(), 0);
            frames.push(b);
        }
        return frames;
    }
}

/**
 * Streaming frame decoder with the reference LZ4Decoder's state machine and API
 * (src/shared/lz4Decode.js:48-307): update(chunk) returns the decoded chunks of every
 * block the input completes. The reference passes three arguments to decompressBlock
 * (:232) and so throws on every compressed block (SURVEY F6); this decoder makes the
 * six-argument call it evidently meant — decompressBlock(block, 0, n, workspace, 0,
 * window) — so each chunk is what the reference's decompressBlock produces for it.
 * The compressed blocks of an independent frame that one update() completes are
 * decoded in one batched GPU call.
 */
export class LZ4Decoder {
    constructor(dictionary = null, verifyChecksum = true) {
        this.state = 0;
        this.dictionary = dictionary ? ensureBuffer(dictionary) : null;
        this.verifyChecksum = verifyChecksum;
        this.blockIndependence = true;
        this.hasBlockChecksum = false;
        this.hasContentChecksum = false;
        this.buffer = new Uint8Array(0);
        this.hasher = null;
        this.window = new Uint8Array(WINDOW_SIZE);
        this.windowPos = 0;
        if (this.dictionary) {
            const size = Math.min(this.dictionary.length, WINDOW_SIZE);
            this.window.set(this.dictionary.subarray(this.dictionary.length - size), 0);
            this.windowPos = size;
        }
    }

    update(chunk) {
        if (this.buffer.length > 0) {
            const nb = new Uint8Array(this.buffer.length + chunk.length);
            nb.set(this.buffer);
            nb.set(chunk, this.buffer.length);
            this.buffer = nb;
        } else {
            this.buffer = chunk;
        }
        const output = [];
        const pending = [];      // compressed blocks of an independent frame, decoded together
        let pendingBytes = 0;    // their output slots (bounded: one batch <= DECODE_BATCH_BYTES)
        const flush = () => {
            if (pending.length === 0) return;
            pendingBytes = 0;
            const dec = this._decodeIndependent(pending);
            for (let k = 0; k < pending.length; k++) {
                if (pending[k].slot === null) continue;
                output[pending[k].slot] = dec[k];
                if (this.hasher) this.hasher.update(dec[k]);
            }
            pending.length = 0;
        };
        for (;;) {
            if (this.state === 0) {                                   // magic
                if (this.buffer.length < 4) break;
                if (readU32(this.buffer, 0) !== MAGIC) { flush(); throw new Error('LZ4: Invalid Magic Number'); }
                this.buffer = this.buffer.subarray(4);
                this.state = 1;
                this.hasher = this.verifyChecksum ? new XXHash32(0) : null;
            }
            if (this.state === 1) {                                   // header
                if (this.buffer.length < 2) break;
                const flg = this.buffer[0];
                this.blockMax = BLOCK_MAX_SIZES[(this.buffer[1] >> 4) & 7] || BLOCK_MAX_SIZES[7];
                this.blockIndependence = (flg & 0x20) !== 0;
                this.hasBlockChecksum = (flg & 0x10) !== 0;
                const hasContentSize = (flg & 0x08) !== 0;
                this.hasContentChecksum = (flg & 0x04) !== 0;
                const hasDictId = (flg & 0x01) !== 0;
                let need = 2 + (hasContentSize ? 8 : 0) + (hasDictId ? 4 : 0) + 1;
                if (this.buffer.length < need) break;
                if (hasDictId) {
                    const expected = readU32(this.buffer, 2 + (hasContentSize ? 8 : 0));
                    if (!this.dictionary) { flush(); throw new Error('LZ4: Archive requires a Dictionary, but none was provided.'); }
                    const actual = native.xxHash32(this.dictionary, 0) >>> 0;
                    if (actual !== expected) {
                        flush();
                        throw new Error(`LZ4: Dictionary ID Mismatch. Header: 0x${expected.toString(16)}, Provided: 0x${actual.toString(16)}`);
                    }
                }
                this.buffer = this.buffer.subarray(need);
                this.state = 2;
            }
            if (this.state === 2) {                                   // block size
                if (this.buffer.length < 4) break;
                const v = readU32(this.buffer, 0);
                this.buffer = this.buffer.subarray(4);
                if (v === 0) { this.state = 4; continue; }
                this.isUncompressed = (v & 0x80000000) !== 0;
                this.currentBlockSize = v & 0x7FFFFFFF;
                this.state = 3;
            }
            if (this.state === 3) {                                   // block body
                const need = this.currentBlockSize + (this.hasBlockChecksum ? 4 : 0);
                if (this.buffer.length < need) break;
                const blockData = this.buffer.subarray(0, this.currentBlockSize);
                this.buffer = this.buffer.subarray(need);
                if (this.blockIndependence && !this.isUncompressed) {
                    pending.push({ data: blockData, slot: output.length });
                    output.push(null);
                    pendingBytes += this.blockMax;
                    if (pendingBytes >= DECODE_BATCH_BYTES) flush();
                } else {
                    flush();
                    let dec;
                    if (this.isUncompressed) {
                        dec = blockData.slice();
                    } else {
                        const dict = this.windowPos === WINDOW_SIZE ? this.window : this.window.subarray(0, this.windowPos);
                        const ws = new Uint8Array(BLOCK_MAX_SIZES[7]);
                        const w = decompressRaw(blockData, 0, blockData.length, ws, 0,
                            this.blockIndependence ? null : dict);
                        dec = ws.slice(0, w);
                    }
                    output.push(dec);
                    if (this.hasher) this.hasher.update(dec);
                    if (!this.blockIndependence) this._updateWindow(dec);
                }
                this.state = 2;
            }
            if (this.state === 4) {                                   // content checksum
                flush();
                if (this.hasContentChecksum) {
                    if (this.buffer.length < 4) break;
                    if (this.verifyChecksum && this.hasher) {
                        if (readU32(this.buffer, 0) !== this.hasher.digest()) throw new Error('LZ4: Content Checksum Error');
                    }
                    this.buffer = this.buffer.subarray(4);
                }
                this.state = 0;
                this.hasher = null;
                if (this.buffer.length === 0) break;
            }
        }
        flush();
        return output;
    }

    // independent compressed blocks, each as decompressBlock(block, 0, n, workspace, 0) decodes it:
    // batched into slots of the frame's block maximum (BD); a block that does not fit its slot
    // (OUTPUT_TOO_SMALL) is decoded again alone into the reference's 4 MiB workspace below
    _decodeIndependent(blocks) {
        const nb = blocks.length, cap = this.blockMax || BLOCK_MAX_SIZES[7];
        if (hostRoute(nb, HOST_MAX_BLOCKS_DECOMPRESS)) {
            const ws = new Uint8Array(BLOCK_MAX_SIZES[7]);   // the reference's 4 MiB workspace, reused
            return blocks.map((b) => ws.slice(0, native.decompressBlockHost(b.data, 0, b.data.length, ws, 0, null,
                decodeFlags)));
        }
        let total = 0;
        for (const b of blocks) total += b.data.length;
        const input = new Uint8Array(total);
        const inOff = new Float64Array(nb), inLen = new Uint32Array(nb);
        const outOff = new Float64Array(nb), outCap = new Uint32Array(nb);
        const outLen = new Uint32Array(nb), status = new Int32Array(nb);
        let p = 0;
        for (let k = 0; k < nb; k++) {
            input.set(blocks[k].data, p);
            inOff[k] = p; inLen[k] = blocks[k].data.length;
            outOff[k] = k * cap; outCap[k] = cap;
            p += blocks[k].data.length;
        }
        const out = new Uint8Array(nb * cap);
        native.decompressBlocks(input, inOff, inLen, out, outOff, outCap, outLen, status, null, decodeFlags);
        const res = [];
        for (let k = 0; k < nb; k++) {
            if (status[k] === native.ERR_CROSS_BLOCK || status[k] !== 0) {
                // a back-reference (or the F1 rewrite) before the block's start: decode it alone,
                // into a fresh workspace, which also raises the reference's error if it has one
                const ws = new Uint8Array(BLOCK_MAX_SIZES[7]);
                const w = decompressRaw(blocks[k].data, 0, blocks[k].data.length, ws, 0, null);
                res.push(ws.slice(0, w));
            } else {
                res.push(out.slice(outOff[k], outOff[k] + outLen[k]));
            }
        }
        return res;
    }

    _updateWindow(chunk) {                                            // lz4Decode.js:279-306
        const cl = chunk.length;
        if (cl >= WINDOW_SIZE) { this.window.set(chunk.subarray(cl - WINDOW_SIZE), 0); this.windowPos = WINDOW_SIZE; return; }
        if (this.windowPos + cl <= WINDOW_SIZE) { this.window.set(chunk, this.windowPos); this.windowPos += cl; return; }
        const keep = WINDOW_SIZE - cl;
        this.window.copyWithin(0, this.windowPos - keep, this.windowPos);
        this.window.set(chunk, keep);
        this.windowPos = WINDOW_SIZE;
    }
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
    XXHash32,
    LZ4Encoder,
    LZ4Decoder,
    setDecodeMode,
    setRouting,
    routeStats,
    version: native.version,
    buildId: native.buildId,
};

export default LZ4;
