/*
 * include/lz4mi.h — C-ABI of the MI355X-native LZ4 block codec (liblz4mi.so).
 *
 * This is the drop-in boundary the reference's hot path is re-bound to. Each
 * entry point names the reference interface it replaces (paths relative to the
 * divortio-lz4 repository root). The N-API addon (divortio-lz4_amd/napi/) and
 * the Python ctypes binding (divortio-lz4_amd/lz4mi/) are thin shims over it.
 *
 * Conventions
 *  - Plain pointers and sizes; no framework types.
 *  - By default every pointer is HOST memory: the call stages it to the GPU,
 *    runs the kernel and copies results back before returning (synchronous,
 *    like the reference's functions).
 *  - With LZ4MI_DEVICE_PTRS every pointer (data AND the per-block descriptor
 *    arrays) is DEVICE memory, the call only enqueues work on `stream`
 *    (a hipStream_t; NULL = HIP's default stream) and returns without waiting
 *    for the device or reading anything back; status/out_len are valid once the
 *    stream has been synchronised. Scratch memory is per stream, so calls on
 *    different streams may run concurrently.
 *  - Status codes: 0 = OK, negative = the reference's error (one per message,
 *    see lz4mi_status_message), <= -100 = infrastructure failure.
 */
#ifndef LZ4MI_H
#define LZ4MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (per block / per call) ------------------------------- */
#define LZ4MI_OK 0
#define LZ4MI_ERR_OUTPUT_TOO_SMALL (-1) /* "LZ4: Output Buffer Too Small"  src/block/blockDecompress.js:74 */
#define LZ4MI_ERR_MALFORMED (-2)        /* "LZ4: Malformed Input"          src/block/blockDecompress.js:75 */
#define LZ4MI_ERR_OFFSET0 (-3)          /* "LZ4: Invalid Offset 0"         src/block/blockDecompress.js:128 */
#define LZ4MI_ERR_DICT_OOB (-4)         /* "LZ4: Dictionary Offset Out of Bounds" src/block/blockDecompress.js:150-152 */
#define LZ4MI_ERR_MAGIC (-5)            /* "LZ4: Invalid Magic Number"     src/buffer/bufferDecompress.js:60 */
#define LZ4MI_ERR_VERSION (-6)          /* "LZ4: Unsupported Version v"    src/buffer/bufferDecompress.js:67 */
#define LZ4MI_ERR_CHECKSUM (-7)         /* "LZ4: Content Checksum Error"   src/buffer/bufferDecompress.js:216 */
#define LZ4MI_ERR_RANGE (-8)            /* RangeError "Source is too large" of TypedArray.set: a literal run
                                           > 64 bytes that does not fit `output` (blockCompress.js:100,198),
                                           a stored block past the result (bufferDecompress.js) */
#define LZ4MI_ERR_CROSS_BLOCK (-9)      /* batched decode only: a back-reference reaches before the block's
                                           own output (not an independent block); the frame layer then
                                           decodes the frame's blocks in order, one call per block */
#define LZ4MI_ERR_BLOCK_CHECKSUM (-10)  /* a frame block's checksum (FLG bit 0x10) does not match its payload;
                                           reported only when block-checksum verification is asked for (the
                                           reference skips them: src/buffer/bufferDecompress.js:191) */
#define LZ4MI_ERR_HIP (-100)            /* a HIP runtime call failed */
#define LZ4MI_ERR_ARG (-101)            /* invalid argument (size limits, NULL pointers) */
#define LZ4MI_ERR_NO_DEVICE (-102)      /* no usable gfx950 device */
#define LZ4MI_ERR_DEVICE_BOUND (-103)   /* lz4mi_init(d): the library is already bound to another device (one
                                           device per process: its stream and scratch live on the first) */

/* ---- flags --------------------------------------------------------------- */
#define LZ4MI_DEVICE_PTRS 0x1u   /* all pointers are device pointers; async on `stream` */
#define LZ4MI_JS_COMPAT 0x2u     /* decode exactly like the reference JS decoder, including its
                                    double-copy-tail rewrite. Default: LZ4 spec. */
#define LZ4MI_XXH_STANDARD 0x4u  /* spec XXH32 lane convergence instead of the reference's variant */
#define LZ4MI_JS_EXACT 0x8u      /* reference-exact result at spec-decoder speed: blocks are decoded by the
                                    parallel spec kernel, which checks every 1 KiB chunk for a reference
                                    double-copy-tail rewrite (F1) that would change a byte and, only in such
                                    a chunk, replays the chunk's matches with the reference's semantics
                                    before going on (cost proportional to the affected chunks). */

#define LZ4MI_XXH_LEN64 0x10u    /* streaming XXH32: keep the 64-bit total length (streams over 2 GiB);
                                    default: the reference class's `(totalLen + len) | 0` */
#define LZ4MI_BLOCK_CHECKSUM 0x20u /* lz4mi_frame_pack: records carry XXH32 (spec) of their payload (FLG 0x10) */
#define LZ4MI_FRAME_WORDS 0x40u  /* lz4mi_decompress_blocks (device pointers, not with LZ4MI_JS_COMPAT): in_len[b]
                                    is the frame's raw size word; bit 31 set = a stored block, whose bytes are
                                    copied in the same launch (bufferDecompress.js:173-180: LZ4MI_ERR_RANGE when
                                    they exceed out_cap[b], the reference's result.set RangeError) */

/* Largest block the kernels accept (the reference's largest block size is 4 MiB;
 * raw calls may pass more, up to 2^31-1 like the reference's `|0` arithmetic). */
#define LZ4MI_MAX_BLOCK 0x7FFFFFFFu

/* Worst-case compressed size of an n-byte block (n + n/255 + 16). */
static inline uint64_t lz4mi_compress_bound(uint64_t n) { return n + n / 255u + 16u; }

/* Human-readable message of a status (the reference's exact error string). */
const char* lz4mi_status_message(int32_t status);

/* Device selection / info. Returns LZ4MI_OK or LZ4MI_ERR_*. lz4mi_init(-1) keeps the
 * current device (or HIP's current one). The library binds to one device per process (one
 * process per GPU): asking for another device once initialised returns LZ4MI_ERR_ARG. */
int32_t lz4mi_init(int32_t device);
int32_t lz4mi_device_count(void);
const char* lz4mi_version(void);
/* Hash of the sources the library was compiled from (Makefile SRC_HASH): lets a test
 * prove the loaded binary was built from the tree beside it. */
const char* lz4mi_build_id(void);

/*
 * Batched raw-block DECOMPRESS.
 * Replaces: decompressBlock(input, inputOffset, inputSize, output, outputOffset, dictionary)
 *           src/block/blockDecompress.js:30-275 (exported as LZ4.decompressRaw, src/lz4.js:33),
 *           and the per-block loop of decompressBuffer src/buffer/bufferDecompress.js:133-192.
 * Block b reads in[in_off[b] .. +in_len[b]) and writes out[out_off[b] ..
 * +out_cap[b]). Positions are absolute in `out` exactly as in the reference:
 * a back-reference below out[out_off[b]] reads earlier bytes of `out`, and
 * below out[0] reads the tail of `dict` (dict_len bytes, may be 0).
 * out_len[b] = bytes produced (outPos - outputOffset); status[b] per block.
 * With nblocks > 1 the blocks must be independent: a back-reference that
 * reaches before the block's own output start yields LZ4MI_ERR_CROSS_BLOCK
 * for that block (with nblocks == 1 it reads the preceding bytes of `out`,
 * then `dict`, exactly as the reference). LZ4MI_JS_COMPAT decodes the blocks
 * in order on one lane with the reference's byte-level behaviour.
 * Returns LZ4MI_OK when the batch ran (per-block errors are in status[]).
 */
int32_t lz4mi_decompress_blocks(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                const uint8_t* dict, uint32_t dict_len,
                                uint32_t* out_len, int32_t* status, uint32_t nblocks, uint32_t flags,
                                void* stream);

/*
 * Batched raw-block COMPRESS (fresh hash table per block: independent blocks).
 * Replaces: compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset)
 *           src/block/blockCompress.js:31-233 (LZ4.compressRaw, src/lz4.js:32) as called by
 *           compressBuffer's block loop src/buffer/bufferCompress.js:209-239 with
 *           blockIndependence=true. Output is byte-identical to the reference encoder.
 * Block b compresses in[in_off[b] .. +in_len[b]) into out[out_off[b] ..), a slot of
 * at least lz4mi_compress_bound(in_len[b]) bytes; out_len[b] = compressed size.
 * The stored-block decision (bufferCompress.js:221-231) is the caller's.
 */
int32_t lz4mi_compress_blocks(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                              uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                              uint32_t nblocks, uint32_t flags, void* stream);

/*
 * Single raw-block COMPRESS with a caller-owned hash table (LZ4.compressRaw with any table).
 * Replaces: compressBlock src/block/blockCompress.js:31-233 with full semantics:
 * positions are absolute in src[0 .. src_total); the block is
 * src[src_start .. +src_len); `table` (16384 int32, values = position+1, <=0 empty)
 * is read and written back; output written at out[out_off ..) (out_total bytes
 * available in out; writes past it are dropped, as with a typed array).
 * With room for lz4mi_compress_bound(src_len) bytes at out_off the block runs on the GPU
 * (the dependent-chain kernel, one block, the table in LDS); with less, the reference's
 * RangeError of output.set() may interrupt the block, and the call runs the host encoder
 * (lz4mi_host_compress_block), which reproduces that store by store.
 * Returns the number of bytes the reference would report written (>= 0) or a
 * negative status (LZ4MI_ERR_RANGE: the reference threw; what it wrote before stays).
 */
int64_t lz4mi_compress_block_table(const uint8_t* src, uint64_t src_total, int32_t src_start, int32_t src_len,
                                   int32_t* table, uint8_t* out, uint64_t out_total, int32_t out_off,
                                   uint32_t flags, void* stream);

/*
 * XXH32, one buffer, on the host CPU (the frame content checksum is one serial
 * chain). Replaces: xxHash32(input, seed) src/xxhash32/xxhash32.js:21-98.
 * flags & LZ4MI_XXH_STANDARD selects the spec convergence.
 */
uint32_t lz4mi_xxh32(const uint8_t* data, size_t len, uint32_t seed, uint32_t flags);

/*
 * Streaming XXH32, on the host CPU.
 * Replaces: class XXHash32 src/xxhash32/xxhash32Stateful.js:13-152 — update() carries up to
 * 15 bytes between calls (:34-68); digest() (:110-152) does not change the state. The
 * length is kept as the class keeps it, `(totalLen + len) | 0` tested signed (:37, :113),
 * unless flags has LZ4MI_XXH_LEN64; LZ4MI_XXH_STANDARD selects the spec convergence.
 * The state is a plain 56-byte struct owned by the caller (no allocation).
 */
typedef struct lz4mi_xxh32_state {
    uint64_t opaque[7];
} lz4mi_xxh32_state;
void lz4mi_xxh32_reset(lz4mi_xxh32_state* state, uint32_t seed, uint32_t flags);
void lz4mi_xxh32_update(lz4mi_xxh32_state* state, const uint8_t* data, size_t len);
uint32_t lz4mi_xxh32_digest(const lz4mi_xxh32_state* state);

/*
 * Batched XXH32 of independent buffers on the GPU (per-block checksums,
 * dictionary ids, parity digests). hashes[b] = xxHash32(in[off[b] .. +len[b]), seed).
 */
int32_t lz4mi_xxh32_blocks(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                           uint32_t* hashes, uint32_t nblocks, uint32_t flags, void* stream);

/*
 * Frame block records on the device (independent-block frames).
 * Replaces the record writing of compressBuffer's block loop, src/buffer/bufferCompress.js:209-239:
 * block b's record goes to frame[rec_off[b] ..): LE32 comp_len[b] and the compressed bytes
 * comp[comp_off[b] ..) when 0 < comp_len[b] < raw_len[b], else LE32 (raw_len[b] | 0x80000000) and the
 * raw bytes raw[raw_off[b] ..). rec_off is the exclusive prefix sum of the record sizes (4 + payload).
 * flags & LZ4MI_BLOCK_CHECKSUM: each record ends with LE32 XXH32 (spec, seed 0) of its payload,
 * the block checksum of the LZ4 frame format (FLG bit 0x10; record size 8 + payload), which the
 * reference's reader skips (src/buffer/bufferDecompress.js:191) and its writer never emits.
 * Device pointers only (flags must include LZ4MI_DEVICE_PTRS); async on `stream`.
 */
int32_t lz4mi_frame_pack(const uint8_t* raw, const uint64_t* raw_off, const uint32_t* raw_len, const uint8_t* comp,
                         const uint64_t* comp_off, const uint32_t* comp_len, uint8_t* frame, const uint64_t* rec_off,
                         uint32_t nblocks, uint32_t flags, void* stream);

/*
 * LZ4 frame DECOMPRESS of a frame in device memory (content size present).
 * Replaces decompressBuffer src/buffer/bufferDecompress.js:51-220 ("direct write" strategy, :97):
 * the header and the size words are walked on the device (one lane: each record's position
 * depends on the previous size), stored blocks are copied (:146-148), and the compressed blocks
 * are decoded in one batch at the output positions of the reference encoder's layout; a block
 * that reads an earlier block's output (dependent frames) is then decoded alone, in order.
 * out: device buffer of out_cap >= content-size bytes. info (host, 8 x int64): [0] the reference's
 * error for the frame (first failing block in block order: LZ4MI_ERR_* of the block decoder,
 * LZ4MI_ERR_RANGE for a stored block past the content size, LZ4MI_ERR_MAGIC / _VERSION for the
 * header) or 0; [1] FLG; [2] content size; [3] bytes written; [4] stored blocks; [5] position
 * of the content checksum (after the EndMark) when FLG has 0x04; [6] block max size (BD).
 * The content checksum (one serial XXH32 chain) is the caller's to verify.
 * flags: LZ4MI_DEVICE_PTRS (required) | LZ4MI_JS_EXACT (reference-exact; default LZ4 spec).
 * Synchronous (reads the header and the block lists back). Returns LZ4MI_ERR_ARG for frames
 * this path does not take (no content size, a block layout other than the reference encoder's,
 * out_cap too small): decode those with the host-buffer path block by block.
 */
int32_t lz4mi_frame_decompress(const uint8_t* frame, uint64_t len, uint8_t* out, uint64_t out_cap, int64_t* info,
                               uint32_t flags, void* stream);

/*
 * Dependent blocks of one frame (the reference's LZ4.compress default,
 * src/buffer/bufferCompress.js:182-236, which calls compressBlock once per block with one
 * table): block b = src[start + b*block_size, ...) compressed in order on one GPU chain with
 * `table` (Int32Array(16384) semantics, in/out, positions absolute in src) carried across
 * blocks; block b's bytes go to out + out_off[b] (room for lz4mi_compress_bound(n_b)),
 * comp_len[b] = its size, exactly compressBlock(src, scratch, start_b, n_b, table, 0). One
 * launch for the whole frame (one staging of src and the table). Host pointers only.
 */
int32_t lz4mi_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len, int32_t block_size,
                             int32_t* table, uint8_t* out, const uint64_t* out_off, uint32_t* comp_len, uint32_t flags,
                             void* stream);

/*
 * Host-CPU block encoder (the routing of SURVEY.md §8b: serial-chain calls run on the calling
 * thread). Same contract as lz4mi_compress_block_table / lz4mi_compress_chain (host pointers,
 * no device needed); byte-identical output and table. Used by the JS layer for dependent-block
 * frames (LZ4.compress's default) and a dictionary's first block, and by
 * lz4mi_compress_block_table when the output has less room than the worst case.
 */
int64_t lz4mi_host_compress_block(const uint8_t* src, uint64_t src_total, int32_t src_start, int32_t src_len,
                                  int32_t* table, uint8_t* out, uint64_t out_total, int32_t out_off);
int32_t lz4mi_host_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len,
                                  int32_t block_size, int32_t* table, uint8_t* out, const uint64_t* out_off,
                                  uint32_t* comp_len);
/*
 * Host-CPU block decoder of the same routing: decompressBlock(input, inputOffset, inputSize,
 * output, outputOffset, dictionary) (src/block/blockDecompress.js:30-275) on the calling thread,
 * for blocks that read their predecessors' output (dependent-block frames, decoded in order).
 * in[0 .. in_total) is the whole input array, out[0 .. out_total) the whole output array
 * (positions absolute in it; below 0 the tail of dict). flags & (LZ4MI_JS_EXACT | LZ4MI_JS_COMPAT):
 * the reference's bytes, its double-copy-tail rewrite included; else LZ4 spec.
 * Returns bytes written (outPos - outputOffset) or a negative status with the reference's meaning.
 */
int64_t lz4mi_host_decompress_block(const uint8_t* in, uint64_t in_total, int64_t in_off, int64_t in_size,
                                    uint8_t* out, uint64_t out_total, int64_t out_off, const uint8_t* dict,
                                    uint32_t dict_len, uint32_t flags);

/*
 * Block index of a device-resident frame, for decoding its blocks on several devices
 * (the block walk of bufferDecompress.js:133-192 without decoding): one lane walks the
 * header and the size words and writes, per block in frame order, the payload position
 * (pay_off) and the raw size word (size_word, bit 31 = stored). info (8 x int64, device)
 * as lz4mi_frame_decompress's, with [3] = blocks listed, [7] = 1 when the walk ran past
 * the frame or past cap_blocks. Device pointers only (LZ4MI_DEVICE_PTRS); asynchronous
 * on `stream`. Replaces nothing in the reference (its frame loop is serial in one call).
 */
int32_t lz4mi_frame_index(const uint8_t* frame, uint64_t len, uint64_t* pay_off, uint32_t* size_word,
                          uint32_t cap_blocks, int64_t* info, uint32_t flags, void* stream);


/*
 * Synthetic input generator (bench/test support, not a reference interface):
 * block b = generator `kind` with seed seed0 + b, block_size bytes each,
 * written to out[b * block_size ..] (device pointer, async on stream).
 * kind: 0 random, 1 repetitive (i % 251), 2 tiles216.
 */
int32_t lz4mi_generate_blocks(uint8_t* out, uint32_t kind, uint32_t seed0, uint32_t block_size,
                              uint32_t nblocks, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LZ4MI_H */
