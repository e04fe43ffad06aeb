/*
 * oracle/lz4_oracle.c — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * CPU restatement of the divortio-lz4 reference algorithms for the hot path
 * (SURVEY.md §8a rows A1-A7). It is the parity checker for the HIP kernels in
 * divortio-lz4_amd/csrc/. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product library (liblz4mi.so) never links,
 * loads or calls anything in this directory.
 *
 * Pinning: every function here is checked against golden vectors produced by
 * executing the reference JavaScript in the build container
 * (tools/golden/gen_golden.mjs -> tests/golden/, test_oracle_golden.py).
 *
 * Reference citations (paths relative to the reference repo root):
 *   orc_xxh32             src/xxhash32/xxhash32.js:21-98
 *   orc_xxh32_stateful    src/xxhash32/xxhash32Stateful.js:13-152
 *   orc_compress_block    src/block/blockCompress.js:31-233 (constants :13-17)
 *   orc_decompress_block  src/block/blockDecompress.js:30-275
 *   orc_compress_frame    src/buffer/bufferCompress.js:77-82,100-259
 *   orc_decompress_frame  src/buffer/bufferDecompress.js:51-220
 *
 * Integer semantics follow the JS `|0` / `>>>` 32-bit arithmetic. Reads the JS
 * code would perform past the end of a typed array yield `undefined`, which the
 * reference's bitwise ops turn into 0: every out-of-range read below returns 0.
 * Typed-array writes past the end are dropped: every store below is clipped.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* Status codes: identical values to include/lz4mi.h (LZ4MI_ERR_*). */
#define ORC_OK 0
#define ORC_ERR_OUTPUT_TOO_SMALL (-1)   /* "LZ4: Output Buffer Too Small"  blockDecompress.js:74 */
#define ORC_ERR_MALFORMED (-2)          /* "LZ4: Malformed Input"          blockDecompress.js:75 */
#define ORC_ERR_OFFSET0 (-3)            /* "LZ4: Invalid Offset 0"         blockDecompress.js:128 */
#define ORC_ERR_DICT_OOB (-4)           /* "LZ4: Dictionary Offset Out of Bounds" :150-152 */
#define ORC_ERR_MAGIC (-5)              /* "LZ4: Invalid Magic Number"     bufferDecompress.js:60 */
#define ORC_ERR_VERSION (-6)            /* "LZ4: Unsupported Version v"    bufferDecompress.js:67 */
#define ORC_ERR_CHECKSUM (-7)           /* "LZ4: Content Checksum Error"   bufferDecompress.js:216 */
#define ORC_ERR_RANGE (-8)              /* RangeError from TypedArray.set (stored block overflow) */

/* ------------------------------------------------------------------ xxh32 */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* xxhash32.js:21-98 — one-shot XXH32 as the reference computes it. (The JS takes
 * len|0; identical below 2 GiB.) NOTE: for len >= 16 the reference converges its
 * four lanes as rotl(rotl(rotl(rotl(v1,1)+v2,7)+v3,12)+v4,18) (xxhash32.js:59-65,
 * xxhash32Stateful.js:114-120), which is NOT the XXH32 spec's
 * rotl(v1,1)+rotl(v2,7)+rotl(v3,12)+rotl(v4,18). `standard` selects the spec form. */
static uint32_t xxh32_impl(const uint8_t* in, uint64_t len, uint32_t seed, int standard) {
    uint64_t p = 0;
    uint32_t h;
    if (len >= 16) {
        uint32_t acc[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
        while (p + 16 <= len) {
            for (int k = 0; k < 4; ++k)
                acc[k] = rotl32(acc[k] + rd32(in + p + 4 * k) * P2, 13) * P1;
            p += 16;
        }
        if (standard) {
            h = rotl32(acc[0], 1) + rotl32(acc[1], 7) + rotl32(acc[2], 12) + rotl32(acc[3], 18);
        } else {
            h = rotl32(acc[0], 1);
            h = rotl32(h + acc[1], 7);
            h = rotl32(h + acc[2], 12);
            h = rotl32(h + acc[3], 18);
        }
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; p + 4 <= len; p += 4) h = rotl32(h + rd32(in + p) * P3, 17) * P4;
    for (; p < len; ++p) h = rotl32(h + in[p] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}
uint32_t orc_xxh32(const uint8_t* in, uint64_t len, uint32_t seed) { return xxh32_impl(in, len, seed, 0); }
uint32_t orc_xxh32_std(const uint8_t* in, uint64_t len, uint32_t seed) { return xxh32_impl(in, len, seed, 1); }

/* xxhash32Stateful.js:13-152 — class XXHash32 fed `nchunks` consecutive chunks of
 * `in` (chunk k is chunk_len[k] bytes): update() carries up to 15 bytes in a
 * 16-byte memory (:34-68); totalLen is kept as `(totalLen + len) | 0` (:37) and
 * digest() tests it with a signed `>= 16` (:113), exactly as the class does. */
uint32_t orc_xxh32_stateful(const uint8_t* in, const uint64_t* chunk_len, uint32_t nchunks, uint32_t seed) {
    uint32_t v[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
    int32_t total = 0;
    uint32_t mem_size = 0;
    uint8_t mem[16];
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint8_t* b = in;
        const uint64_t len = chunk_len[c];
        in += len;
        total = (int32_t)((uint32_t)total + (uint32_t)len);
        if (mem_size + len < 16) { memcpy(mem + mem_size, b, len); mem_size += (uint32_t)len; continue; }
        uint64_t p = 0;
        if (mem_size > 0) {
            p = 16 - mem_size;
            memcpy(mem + mem_size, b, p);
            for (int k = 0; k < 4; ++k) v[k] = rotl32(v[k] + rd32(mem + 4 * k) * P2, 13) * P1;
            mem_size = 0;
        }
        for (; p + 16 <= len; p += 16)
            for (int k = 0; k < 4; ++k) v[k] = rotl32(v[k] + rd32(b + p + 4 * k) * P2, 13) * P1;
        if (p < len) { memcpy(mem, b + p, len - p); mem_size = (uint32_t)(len - p); }
    }
    uint32_t h;
    if (total >= 16) {
        h = rotl32(v[0], 1);
        h = rotl32(h + v[1], 7);
        h = rotl32(h + v[2], 12);
        h = rotl32(h + v[3], 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)total;
    uint32_t p = 0;
    for (; p + 4 <= mem_size; p += 4) h = rotl32(h + rd32(mem + p) * P3, 17) * P4;
    for (; p < mem_size; ++p) h = rotl32(h + mem[p] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

/* ------------------------------------------------------- block compressor */
/* Output sink with JS typed-array semantics (writes past the end dropped). */
typedef struct { uint8_t* b; int64_t cap; int64_t pos; } sink_t;
static inline void put(sink_t* s, uint8_t v) { if (s->pos >= 0 && s->pos < s->cap) s->b[s->pos] = v; s->pos++; }

static void put_len_ext(sink_t* s, int32_t extra) {           /* 255-run varint tail */
    while (extra >= 255) { put(s, 255); extra -= 255; }
    put(s, (uint8_t)extra);
}

/* blockCompress.js:31-233. `table` holds 16384 int32 entries of (absolute
 * position + 1); entries <= 0 mean empty. Positions are absolute in `src`. */
/* A literal run longer than 64 bytes is copied with output.set() (:100, :198), which
 * throws a RangeError when it would run past the end of `output` (shorter runs use
 * per-byte stores, whose out-of-range writes are dropped). *status = ORC_ERR_RANGE
 * then; the bytes and table entries written before the throw stay written. */
int32_t orc_compress_block_ex(const uint8_t* src, uint64_t src_total, uint8_t* out, uint64_t out_total,
                              int32_t src_start, int32_t src_len, int32_t* table, int32_t out_off,
                              int32_t* status) {
    (void)src_total;
    *status = ORC_OK;
    const int32_t end = src_start + src_len;
    const int32_t mflimit = end - 12;      /* MF_LIMIT  :14 */
    const int32_t matchlimit = end - 5;    /* LAST_LITERALS :13 */
    sink_t s = { out, (int64_t)out_total, out_off };
    int32_t i = src_start, anchor = src_start;
    uint32_t miss = 67;                    /* (1 << 6) + 3, :40 */

    while (i < mflimit) {
        uint32_t seq = rd32(src + i);
        uint32_t h = (seq * P1) >> 18;     /* Math.imul(seq, 2654435761) >>> 18, & 16383 */
        int32_t cand = table[h] - 1;
        table[h] = i + 1;                  /* insert before verify (:55) */
        if (cand < 0 || cand == i || ((uint32_t)(i - cand) >> 16) != 0 || rd32(src + cand) != seq) {
            i += (int32_t)(miss++ >> 6);   /* skip acceleration (:66-67) */
            continue;
        }
        miss = 67;
        int32_t lit = i - anchor;
        int64_t tok = s.pos;
        put(&s, (uint8_t)(lit >= 15 ? 0xF0 : (lit << 4)));
        if (lit >= 15) put_len_ext(&s, lit - 15);
        if (lit > 64 && s.pos + lit > s.cap) { *status = ORC_ERR_RANGE; return (int32_t)(s.pos - out_off); }
        for (int32_t k = 0; k < lit; ++k) put(&s, src[anchor + k]);
        int32_t e = i + 4, m = cand + 4;   /* forward extension only (:147-150) */
        while (e < matchlimit && src[e] == src[m]) { ++e; ++m; }
        int32_t off = i - cand;
        put(&s, (uint8_t)(off & 0xFF));
        put(&s, (uint8_t)((off >> 8) & 0xFF));
        int32_t mcode = e - i - 4;
        if (mcode >= 15) {
            if (tok < s.cap) out[tok] |= 0x0F;
            put_len_ext(&s, mcode - 15);
        } else if (tok < s.cap) {
            out[tok] |= (uint8_t)mcode;
        }
        i = e; anchor = e;                 /* no inserts inside the match */
    }
    int32_t lit = end - anchor;            /* final literals (:179-230) */
    put(&s, (uint8_t)(lit >= 15 ? 0xF0 : (lit << 4)));
    if (lit >= 15) put_len_ext(&s, lit - 15);
    if (lit > 64 && s.pos + lit > s.cap) { *status = ORC_ERR_RANGE; return (int32_t)(s.pos - out_off); }
    for (int32_t k = 0; k < lit; ++k) put(&s, src[anchor + k]);
    return (int32_t)(s.pos - out_off);
}

int32_t orc_compress_block(const uint8_t* src, uint64_t src_total, uint8_t* out, uint64_t out_total,
                           int32_t src_start, int32_t src_len, int32_t* table, int32_t out_off) {
    int32_t st;
    return orc_compress_block_ex(src, src_total, out, out_total, src_start, src_len, table, out_off, &st);
}

/* ----------------------------------------------------- block decompressor */
typedef struct { const uint8_t* b; int64_t total; } src_t;
static inline uint8_t getb(const src_t* s, int64_t i) { return (i >= 0 && i < s->total) ? s->b[i] : 0; }

/* blockDecompress.js:30-275. Positions are absolute in `out` (length
 * out_total). Back-references below out[0] read the dictionary (:145-199).
 * js_compat != 0 reproduces the reference's double-copy-tail rewrite (SURVEY
 * F1, :219-250): a general-path match with offset >= 8 and length < 8 rewrites
 * out[p] = out[p-offset] for p in [end-8, start) (out-of-range reads as 0).
 * Returns a status; *written = bytes produced (outPos - outputOffset). */
int32_t orc_decompress_block(const uint8_t* in, uint64_t in_total, int64_t in_off, int64_t in_size,
                             uint8_t* out, int64_t out_total, int64_t out_off,
                             const uint8_t* dict, int64_t dict_len, int32_t js_compat, int64_t* written) {
    src_t S = { in, (int64_t)in_total };
    int64_t ip = in_off, iend = in_off + in_size, op = out_off;
    if (written) *written = 0;
    while (ip < iend) {
        uint32_t token = getb(&S, ip++);
        int64_t lit = token >> 4;
        if (lit == 15) { uint32_t b; do { b = getb(&S, ip++); lit += b; } while (b == 255); }
        int64_t elit = op + lit;
        if (elit > out_total) return ORC_ERR_OUTPUT_TOO_SMALL;
        if (ip + lit > iend) return ORC_ERR_MALFORMED;
        for (int64_t k = 0; k < lit; ++k) out[op + k] = getb(&S, ip + k);
        op = elit; ip += lit;
        if (ip >= iend) break;
        uint32_t off = (uint32_t)getb(&S, ip) | ((uint32_t)getb(&S, ip + 1) << 8);
        ip += 2;
        if (off == 0) return ORC_ERR_OFFSET0;
        int64_t ml = token & 15;
        if (ml == 15) { uint32_t b; do { b = getb(&S, ip++); ml += b; } while (b == 255); }
        ml += 4;
        int64_t from = op - (int64_t)off;
        if (from < 0) {                     /* dictionary path */
            int64_t nd = -from; if (nd > ml) nd = ml;
            int64_t di = dict_len + from;
            if (di < 0 || di + nd > dict_len) return ORC_ERR_DICT_OOB;
            for (int64_t k = 0; k < nd; ++k) { if (op < out_total) out[op] = dict[di + k]; op++; }
            int64_t rp = op - (int64_t)off;
            for (int64_t k = nd; k < ml; ++k) {
                uint8_t v = (rp >= 0 && rp < out_total) ? out[rp] : 0;
                if (op < out_total) out[op] = v;
                op++; rp++;
            }
            continue;
        }
        int64_t start = op;
        for (int64_t k = 0; k < ml; ++k) {  /* forward byte copy == spec overlap semantics */
            int64_t r = op - (int64_t)off;
            uint8_t v = (r < out_total) ? out[r] : 0;
            if (op < out_total) out[op] = v;
            op++;
        }
        if (js_compat && off >= 8 && ml < 8) {
            for (int64_t p = start + ml - 8; p < start; ++p) {
                int64_t r = p - (int64_t)off;
                uint8_t v = (r >= 0 && r < out_total) ? out[r] : 0;
                if (p >= 0 && p < out_total) out[p] = v;
            }
        }
    }
    if (written) *written = op - out_off;
    return ORC_OK;
}

/* ----------------------------------------------------------------- frames */
static const int32_t kBlockMax[8] = { 0, 0, 0, 0, 65536, 262144, 1048576, 4194304 };

static int block_id(int64_t bytes) {                 /* bufferCompress.js:77-82 */
    if (bytes <= 0 || bytes <= 65536) return 4;
    if (bytes <= 262144) return 5;
    if (bytes <= 1048576) return 6;
    return 7;
}

static inline void wr32(sink_t* s, uint32_t v) { put(s, v & 255); put(s, (v >> 8) & 255); put(s, (v >> 16) & 255); put(s, v >> 24); }

/* Worst-case frame size the reference allocates (bufferCompress.js:140). */
int64_t orc_frame_bound(int64_t len) { return 19 + len + len / 255 + 64 + 8; }

/* bufferCompress.js:100-259: LZ4 frame writer. Dictionary prewarm uses the
 * reference's Jenkins-style hash (:191-203), not the block hash.
 * block_checksum (not in the reference, whose reader skips them, bufferDecompress.js:191):
 * FLG bit 0x10 and, after each block's payload, LE32 XXH32 (spec) of the payload — the
 * LZ4 frame format's block checksum. */
int64_t orc_compress_frame_ex(const uint8_t* in, int64_t len, const uint8_t* dict, int64_t dict_len,
                              int64_t max_block, int32_t indep, int32_t checksum, int32_t add_size,
                              int32_t block_checksum, uint8_t* out, int64_t out_cap) {
    sink_t s = { out, out_cap, 0 };
    int64_t win = 0;
    uint8_t* work = (uint8_t*)in;
    uint32_t dict_id = 0;
    int has_dict = dict && dict_len > 0;
    if (has_dict) {
        dict_id = orc_xxh32(dict, (uint64_t)dict_len, 0);
        const uint8_t* dw = dict_len > 65536 ? dict + dict_len - 65536 : dict;
        win = dict_len > 65536 ? 65536 : dict_len;
        work = (uint8_t*)malloc((size_t)(win + len + 1));
        memcpy(work, dw, (size_t)win);
        if (len) memcpy(work + win, in, (size_t)len);
    }
    int bd = block_id(max_block);
    int32_t bsize = kBlockMax[bd];
    put(&s, 0x04); put(&s, 0x22); put(&s, 0x4D); put(&s, 0x18);
    uint8_t flg = 0x40 | (indep ? 0x20 : 0) | (checksum ? 0x04 : 0) | (has_dict ? 0x01 : 0) | (add_size ? 0x08 : 0) |
                  (block_checksum ? 0x10 : 0);
    put(&s, flg);
    put(&s, (uint8_t)((bd & 7) << 4));
    if (add_size) { wr32(&s, (uint32_t)len); wr32(&s, (uint32_t)((uint64_t)len >> 32)); }
    if (has_dict) wr32(&s, dict_id);
    {
        uint8_t hdr[14]; int64_t n = s.pos - 4;
        for (int64_t k = 0; k < n; ++k) hdr[k] = (4 + k < out_cap) ? out[4 + k] : 0;
        put(&s, (uint8_t)((orc_xxh32(hdr, (uint64_t)n, 0) >> 8) & 0xFF));
    }
    int32_t* table = (int32_t*)calloc(16384, sizeof(int32_t));
    for (int64_t i = 0; i + 4 <= win; ++i) {           /* prewarm (:186-204) */
        int32_t h = (int32_t)rd32(work + i);
        h = (int32_t)((uint32_t)h + 2127912214u + ((uint32_t)h << 12));
        h = (int32_t)((uint32_t)h ^ 0xC761C23Cu ^ ((uint32_t)h >> 19));   /* -949894596 */
        h = (int32_t)((uint32_t)h + 374761393u + ((uint32_t)h << 5));
        h = (int32_t)(((uint32_t)h + 0xD3A2646Cu) ^ ((uint32_t)h << 9));  /* -744332180 */
        h = (int32_t)((uint32_t)h + 0xFD7046C5u + ((uint32_t)h << 3));    /* -42973499 */
        h = (int32_t)((uint32_t)h ^ 0xB55A4F09u ^ ((uint32_t)h >> 16));   /* -1252372727 */
        table[((uint32_t)h >> 18) & 16383] = (int32_t)i + 1;
    }
    int64_t pos = win, tend = win + len;
    while (pos < tend) {
        int64_t e = pos + bsize < tend ? pos + bsize : tend;
        int32_t n = (int32_t)(e - pos);
        int64_t size_pos = s.pos;
        s.pos += 4;
        int32_t c = orc_compress_block(work, (uint64_t)(win + len), out, (uint64_t)out_cap,
                                       (int32_t)pos, n, table, (int32_t)s.pos);
        int64_t save = s.pos;
        if (c > 0 && c < n) {
            s.pos = size_pos; wr32(&s, (uint32_t)c); s.pos = save + c;
        } else {
            s.pos = size_pos; wr32(&s, (uint32_t)n | 0x80000000u);
            for (int32_t k = 0; k < n; ++k) put(&s, work[pos + k]);
        }
        if (block_checksum) {
            const int64_t pay = size_pos + 4, plen = s.pos - pay;
            wr32(&s, (pay + plen <= out_cap) ? orc_xxh32_std(out + pay, (uint64_t)plen, 0) : 0);
        }
        if (indep) memset(table, 0, 16384 * sizeof(int32_t));
        pos = e;
    }
    wr32(&s, 0);
    if (checksum) wr32(&s, orc_xxh32(in, (uint64_t)len, 0));
    free(table);
    if (has_dict) free(work);
    return s.pos;
}

int64_t orc_compress_frame(const uint8_t* in, int64_t len, const uint8_t* dict, int64_t dict_len,
                           int64_t max_block, int32_t indep, int32_t checksum, int32_t add_size,
                           uint8_t* out, int64_t out_cap) {
    return orc_compress_frame_ex(in, len, dict, dict_len, max_block, indep, checksum, add_size, 0, out, out_cap);
}

/* bufferDecompress.js:51-220. Writes into `out` (capacity out_cap) and
 * returns the status; *out_len = result length. The "direct write" strategy
 * is used when a non-zero content size is present (:97), else decoded blocks
 * are chained through a 64 KiB window passed as a dictionary (:157-186). */
int32_t orc_decompress_frame(const uint8_t* data, int64_t len, const uint8_t* dict, int64_t dict_len,
                             int32_t verify, int32_t js_compat, uint8_t* out, int64_t out_cap, int64_t* out_len,
                             int32_t* version_out) {
    src_t S = { data, len };
    int64_t pos = 0;
    *out_len = 0;
    if (len < 4 || rd32(data) != 0x184D2204u) return ORC_ERR_MAGIC;
    pos = 4;
    uint8_t flg = getb(&S, pos++);
    int version = (flg & 0xC0) >> 6;
    if (version_out) *version_out = version;
    if (version != 1) return ORC_ERR_VERSION;
    int has_bcs = (flg & 0x10) != 0, has_size = (flg & 0x08) != 0, has_ccs = (flg & 0x04) != 0, has_did = (flg & 0x01) != 0;
    pos++;                                              /* BD ignored (:75) */
    int64_t expected = 0;
    if (has_size) {
        uint64_t lo = (uint64_t)getb(&S, pos) | ((uint64_t)getb(&S, pos + 1) << 8) | ((uint64_t)getb(&S, pos + 2) << 16) | ((uint64_t)getb(&S, pos + 3) << 24);
        uint64_t hi = (uint64_t)getb(&S, pos + 4) | ((uint64_t)getb(&S, pos + 5) << 8) | ((uint64_t)getb(&S, pos + 6) << 16) | ((uint64_t)getb(&S, pos + 7) << 24);
        pos += 8;
        expected = (int64_t)(hi * 4294967296ull + lo);
    }
    if (has_did) pos += 4;
    pos++;                                              /* header checksum ignored (:92) */
    int direct = expected > 0;
    int64_t rpos = 0;
    uint8_t* window = NULL; int64_t wpos = 0;
    uint8_t* ws = NULL;
    if (direct) {
        if (expected > out_cap) return ORC_ERR_OUTPUT_TOO_SMALL;
        memset(out, 0, (size_t)expected);
    } else {
        window = (uint8_t*)calloc(65536, 1);
        ws = (uint8_t*)malloc(4194304);
        if (dict) {
            if (dict_len > 65536) { memcpy(window, dict + dict_len - 65536, 65536); wpos = 65536; }
            else { memcpy(window, dict, (size_t)dict_len); wpos = dict_len; }
        }
    }
    int32_t st = ORC_OK;
    while (pos < len) {
        uint32_t bs = (uint32_t)getb(&S, pos) | ((uint32_t)getb(&S, pos + 1) << 8) | ((uint32_t)getb(&S, pos + 2) << 16) | ((uint32_t)getb(&S, pos + 3) << 24);
        pos += 4;
        if (bs == 0) break;
        int raw = (bs & 0x80000000u) != 0;
        int64_t n = bs & 0x7FFFFFFF;
        if (direct) {
            if (raw) {
                int64_t avail = len - pos; if (avail < 0) avail = 0;
                int64_t m = n < avail ? n : avail;        /* subarray clamps */
                if (rpos + m > expected) { st = ORC_ERR_RANGE; goto done; }
                memcpy(out + rpos, data + pos, (size_t)m);
                rpos += m;
            } else {
                int64_t w = 0;
                st = orc_decompress_block(data, (uint64_t)len, pos, n, out, expected, rpos, dict, dict ? dict_len : 0, js_compat, &w);
                if (st) goto done;
                rpos += w;
            }
        } else {
            const uint8_t* chunk; int64_t clen;
            if (raw) {
                int64_t avail = len - pos; if (avail < 0) avail = 0;
                clen = n < avail ? n : avail; chunk = data + pos;
            } else {
                int64_t w = 0;
                st = orc_decompress_block(data, (uint64_t)len, pos, n, ws, 4194304, 0, wpos > 0 ? window : NULL, wpos, js_compat, &w);
                if (st) goto done;
                clen = w < 4194304 ? w : 4194304; chunk = ws;
            }
            if (rpos + clen > out_cap) { st = ORC_ERR_OUTPUT_TOO_SMALL; goto done; }
            memcpy(out + rpos, chunk, (size_t)clen);
            rpos += clen;
            if (clen >= 65536) { memcpy(window, chunk + clen - 65536, 65536); wpos = 65536; }
            else if (wpos + clen <= 65536) { memcpy(window + wpos, chunk, (size_t)clen); wpos += clen; }
            else { int64_t keep = 65536 - clen; memmove(window, window + wpos - keep, (size_t)keep); memcpy(window + keep, chunk, (size_t)clen); wpos = 65536; }
        }
        pos += n;
        if (has_bcs) pos += 4;
    }
    {
        int64_t rlen = direct ? expected : rpos;
        *out_len = rlen;
        if (has_ccs && verify) {
            uint32_t stored = (uint32_t)getb(&S, pos) | ((uint32_t)getb(&S, pos + 1) << 8) | ((uint32_t)getb(&S, pos + 2) << 16) | ((uint32_t)getb(&S, pos + 3) << 24);
            if (stored != orc_xxh32(out, (uint64_t)rlen, 0)) st = ORC_ERR_CHECKSUM;
        }
    }
done:
    free(window); free(ws);
    return st;
}

/* ------------------------------------------------------------- generators */
/* Seeded synthetic inputs. xorshift32: x^=x<<13; x^=x>>17; x^=x<<5. */
typedef struct { uint32_t x; } xs32_t;
static inline uint32_t xs_next(xs32_t* r) { uint32_t x = r->x; x ^= x << 13; x ^= x >> 17; x ^= x << 5; r->x = x; return x; }

enum { GEN_RANDOM = 0, GEN_REPETITIVE = 1, GEN_TILES216 = 2, GEN_COPY = 3, GEN_RUNS = 4, GEN_TEXT = 5 };

void orc_generate(int32_t kind, uint32_t seed, uint8_t* b, int64_t n) {
    xs32_t r = { seed ? seed : 1u };
    int64_t i = 0;
    switch (kind) {
    case GEN_RANDOM:
        for (i = 0; i < n; i += 4) { uint32_t v = xs_next(&r); for (int k = 0; k < 4 && i + k < n; ++k) b[i + k] = (uint8_t)(v >> (8 * k)); }
        break;
    case GEN_REPETITIVE:
        for (i = 0; i < n; ++i) b[i] = (uint8_t)(i % 251);
        break;
    case GEN_TILES216: {
        uint8_t tiles[216 * 64];
        for (int k = 0; k < 216 * 64; ++k) tiles[k] = (uint8_t)(xs_next(&r) & 255);
        while (i < n) { const uint8_t* t = tiles + 64 * (xs_next(&r) % 216); for (int k = 0; k < 64 && i < n; ++k) b[i++] = t[k]; }
        break;
    }
    case GEN_COPY:   /* literal runs of 4..8 random bytes, then copies of 48..80 bytes from offsets 16..4096 */
        while (i < n) {
            uint32_t L = 4 + xs_next(&r) % 5;
            for (uint32_t k = 0; k < L && i < n; ++k) b[i++] = (uint8_t)(xs_next(&r) & 255);
            uint32_t M = 48 + xs_next(&r) % 33, off = 16 + xs_next(&r) % 4081;
            if (i - (int64_t)off < 0) continue;
            for (uint32_t k = 0; k < M && i < n; ++k, ++i) b[i] = b[i - off];
        }
        break;
    case GEN_RUNS:   /* runs of one random byte, run length 1..24 */
        while (i < n) { uint8_t v = (uint8_t)(xs_next(&r) & 255); uint32_t L = 1 + xs_next(&r) % 24; for (uint32_t k = 0; k < L && i < n; ++k) b[i++] = v; }
        break;
    case GEN_TEXT: { /* words from a 64-entry vocabulary of 2..9 lowercase letters, space separated */
        static const char* voc = "the of and to in is was for on that with as by at from his an were are which this be or has had not but it its";
        const char* words[64]; int wl[64]; int nw = 0; const char* p = voc;
        while (*p && nw < 64) { words[nw] = p; int l = 0; while (p[l] && p[l] != ' ') ++l; wl[nw++] = l; p += l; while (*p == ' ') ++p; }
        while (i < n) {
            uint32_t v = xs_next(&r);
            int w = (int)(v % (uint32_t)nw);
            for (int k = 0; k < wl[w] && i < n; ++k) b[i++] = (uint8_t)words[w][k];
            if (i < n) b[i++] = (v >> 16) % 11 == 0 ? '\n' : ' ';
        }
        break;
    }
    default:
        memset(b, 0, (size_t)n);
    }
}

/* ----------------------------------------------- multi-threaded CPU baseline */
typedef struct {
    int mode; const uint8_t* in; const uint64_t* in_off; const uint32_t* in_len;
    uint8_t* out; const uint64_t* out_off; const uint32_t* out_cap; uint32_t* out_len;
    int32_t* status; uint32_t nblocks; uint32_t tid, nthreads;
} mt_job_t;

static void* mt_worker(void* arg) {
    mt_job_t* j = (mt_job_t*)arg;
    int32_t* table = (int32_t*)malloc(16384 * sizeof(int32_t));
    for (uint32_t b = j->tid; b < j->nblocks; b += j->nthreads) {
        if (j->mode == 0 || j->mode == 2) {
            int64_t w = 0;
            int32_t st = orc_decompress_block(j->in + j->in_off[b], j->in_len[b], 0, j->in_len[b],
                                              j->out + j->out_off[b], j->out_cap[b], 0, NULL, 0, j->mode == 2, &w);
            j->status[b] = st; j->out_len[b] = (uint32_t)w;
        } else {
            memset(table, 0, 16384 * sizeof(int32_t));
            int32_t c = orc_compress_block(j->in + j->in_off[b], j->in_len[b], j->out + j->out_off[b], j->out_cap[b],
                                           0, (int32_t)j->in_len[b], table, 0);
            j->out_len[b] = (uint32_t)c; j->status[b] = 0;
        }
    }
    free(table);
    return NULL;
}

/* mode 0 = decompress (spec), 1 = compress (fresh table per block), 2 = decompress with the
 * reference decoder's bytes (js_compat: the F1 double-copy tail, blockDecompress.js:234-249),
 * each block in an output array of its own (nothing before its offset 0). Independent
 * blocks spread round-robin over `nthreads` pthreads. */
int32_t orc_blocks_mt(int32_t mode, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, uint32_t* out_len,
                      int32_t* status, uint32_t nblocks, uint32_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    mt_job_t* jobs = (mt_job_t*)malloc(sizeof(mt_job_t) * nthreads);
    for (uint32_t t = 0; t < nthreads; ++t) {
        mt_job_t j = { mode, in, in_off, in_len, out, out_off, out_cap, out_len, status, nblocks, t, nthreads };
        jobs[t] = j;
        pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
    }
    for (uint32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}
