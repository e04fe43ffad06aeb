/*
 * lz4mi_napi.c — Node.js N-API addon over the liblz4mi C-ABI (include/lz4mi.h).
 *
 * This is the thin native layer the reference's JS calls into: every function
 * takes the reference's own argument list (typed arrays + numbers) and maps it
 * 1:1 onto a C-ABI entry point. Buffers are caller-owned JS memory, used only
 * for the duration of the synchronous call (the C-ABI stages them to the GPU
 * and copies results back before returning). Errors are thrown as
 * `new Error(<reference message>)`, exactly the strings the reference throws.
 *
 *   compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset) -> bytes written
 *       src/block/blockCompress.js:31 (LZ4.compressRaw, src/lz4.js:32)
 *   decompressBlock(input, inputOffset, inputSize, output, outputOffset, dictionary?) -> bytes written
 *       src/block/blockDecompress.js:30 (LZ4.decompressRaw, src/lz4.js:33)
 *   compressBlocks(src, srcOff: Float64Array, srcLen: Uint32Array, out, outOff: Float64Array, outLen: Uint32Array)
 *       the independent-block loop of compressBuffer (src/buffer/bufferCompress.js:209-239), batched
 *   decompressBlocks(input, inOff: Float64Array, inLen: Uint32Array, output, outOff: Float64Array,
 *                    outCap: Uint32Array, outLen: Uint32Array, status: Int32Array, dictionary?, flags?)
 *       the block loop of decompressBuffer (src/buffer/bufferDecompress.js:133-192), batched
 *   xxHash32(input, seed, flags?) -> uint32       src/xxhash32/xxhash32.js:21
 *   xxh32Reset(seed, flags?) -> Uint8Array state; xxh32Update(state, input); xxh32Digest(state) -> uint32
 *       class XXHash32 src/xxhash32/xxhash32Stateful.js:13-152 (state in a caller-owned Uint8Array)
 *   xxh32Blocks(input, off: Float64Array, len: Uint32Array, seed, hashes: Uint32Array, flags?)
 *       batched XXH32 of independent buffers on the GPU (frame block checksums, FLG 0x10)
 *   statusMessage(code) -> string; init(device) -> status; version() -> string; buildId() -> string
 *   constants: JS_COMPAT, JS_EXACT, XXH_STANDARD, XXH_LEN64, ERR_CROSS_BLOCK
 *
 * Offsets are passed as Float64Array (exact up to 2^53) so one call can span
 * buffers larger than 4 GiB.
 */
#define NAPI_VERSION 6
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lz4mi.h"

#define CHECK(call)                                                          \
    do {                                                                     \
        if ((call) != napi_ok) {                                             \
            napi_throw_error(env, NULL, "lz4mi: N-API call failed: " #call); \
            return NULL;                                                     \
        }                                                                    \
    } while (0)

typedef struct {
    void* data;
    size_t length;   /* elements */
    napi_typedarray_type type;
} view_t;

/* Typed array (or Buffer / DataView-free Uint8Array) argument; null/undefined -> empty view. */
static int get_view(napi_env env, napi_value v, view_t* out, int required, const char* what) {
    napi_valuetype t;
    memset(out, 0, sizeof *out);
    if (napi_typeof(env, v, &t) != napi_ok) return 0;
    if (t == napi_undefined || t == napi_null) {
        if (required) {
            char msg[128];
            snprintf(msg, sizeof msg, "lz4mi: %s must be a typed array", what);
            napi_throw_type_error(env, NULL, msg);
            return 0;
        }
        return 1;
    }
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) {
        char msg[128];
        snprintf(msg, sizeof msg, "lz4mi: %s must be a typed array", what);
        napi_throw_type_error(env, NULL, msg);
        return 0;
    }
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &out->type, &out->length, &out->data, &ab, &off) != napi_ok) return 0;
    return 1;
}

static int get_i64(napi_env env, napi_value v, int64_t* out) {
    double d = 0;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_undefined || t == napi_null) { *out = 0; return 1; }
    if (napi_get_value_double(env, v, &d) != napi_ok) {
        napi_throw_type_error(env, NULL, "lz4mi: expected a number");
        return 0;
    }
    *out = (int64_t)d;
    return 1;
}

/* The reference's `x | 0` on a number argument. */
static int32_t to_i32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

static napi_value make_i64(napi_env env, int64_t v) {
    napi_value r;
    napi_create_int64(env, v, &r);
    return r;
}

static napi_value throw_status(napi_env env, int64_t st) {
    if (st == LZ4MI_ERR_RANGE)   /* the reference's TypedArray.set RangeError */
        napi_throw_range_error(env, NULL, lz4mi_status_message((int32_t)st));
    else
        napi_throw_error(env, NULL, lz4mi_status_message((int32_t)st));
    return NULL;
}

static int is_undefined(napi_env env, size_t argc, napi_value* argv, size_t i) {
    napi_valuetype t;
    if (argc <= i) return 1;
    if (napi_typeof(env, argv[i], &t) != napi_ok) return 0;
    return t == napi_undefined;
}

/* compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset): lz4mi_compress_block_table;
 * compressBlockHost: the host encoder (lz4mi_host_compress_block) */
static napi_value compress_block_impl(napi_env env, napi_callback_info info, int host) {
    size_t argc = 6;
    napi_value argv[6];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t src, out, tab;
    int64_t start, len, ooff;
    if (!get_view(env, argv[0], &src, 1, "src") || !get_view(env, argv[1], &out, 1, "output")) return NULL;
    if (!get_i64(env, argv[2], &start) || !get_i64(env, argv[3], &len)) return NULL;
    if (!get_view(env, argc > 4 ? argv[4] : NULL, &tab, 0, "hashTable")) return NULL;
    if (!get_i64(env, argc > 5 ? argv[5] : NULL, &ooff)) return NULL;
    int32_t* table = NULL;
    if (tab.data) {
        if (tab.type != napi_int32_array || tab.length < 16384) {
            napi_throw_type_error(env, NULL, "lz4mi: hashTable must be an Int32Array(16384)");
            return NULL;
        }
        table = (int32_t*)tab.data;
    } else {
        table = (int32_t*)calloc(16384, sizeof(int32_t));   /* the reference would fault on a missing table */
        if (!table) return throw_status(env, LZ4MI_ERR_ARG);
    }
    int64_t r = host ? lz4mi_host_compress_block((const uint8_t*)src.data, src.length, to_i32(start), to_i32(len), table,
                                                 (uint8_t*)out.data, out.length, to_i32(ooff))
                     : lz4mi_compress_block_table((const uint8_t*)src.data, src.length, to_i32(start), to_i32(len),
                                                  table, (uint8_t*)out.data, out.length, to_i32(ooff), 0, NULL);
    if (!tab.data) free(table);
    if (r < 0) return throw_status(env, r);
    /* without outputOffset the reference returns (dIndex - undefined) | 0 == 0 (blockCompress.js:37,232) */
    if (is_undefined(env, argc, argv, 5)) return make_i64(env, 0);
    return make_i64(env, r);
}

static napi_value n_compress_block(napi_env env, napi_callback_info info) { return compress_block_impl(env, info, 0); }
static napi_value n_compress_block_host(napi_env env, napi_callback_info info) {
    return compress_block_impl(env, info, 1);
}

/* decompressBlock(input, inputOffset, inputSize, output, outputOffset, dictionary) on the GPU;
 * decompressBlockHost: the same on the host decoder (lz4mi_host_decompress_block, the JS
 * layer's route for the blocks of dependent-block frames) */
static napi_value decompress_block_impl(napi_env env, napi_callback_info info, int host) {
    size_t argc = 7;
    napi_value argv[7];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t in, out, dict;
    int64_t ioff, isz, ooff, flags = LZ4MI_JS_EXACT;
    if (!get_view(env, argv[0], &in, 1, "input") || !get_view(env, argv[3], &out, 1, "output")) return NULL;
    if (!get_i64(env, argv[1], &ioff) || !get_i64(env, argv[2], &isz) || !get_i64(env, argv[4], &ooff)) return NULL;
    if (!get_view(env, argc > 5 ? argv[5] : NULL, &dict, 0, "dictionary")) return NULL;
    if (argc > 6 && !get_i64(env, argv[6], &flags)) return NULL;
    int32_t i0 = to_i32(ioff), n = to_i32(isz), o0 = to_i32(ooff);
    if (i0 < 0 || n < 0 || (uint64_t)i0 + (uint64_t)n > in.length) {
        /* the reference would read undefined bytes there: malformed input */
        return throw_status(env, LZ4MI_ERR_MALFORMED);
    }
    if (o0 < 0 || (uint64_t)o0 > out.length) return throw_status(env, LZ4MI_ERR_OUTPUT_TOO_SMALL);
    if (host) {
        int64_t r = lz4mi_host_decompress_block((const uint8_t*)in.data, in.length, i0, n, (uint8_t*)out.data,
                                                out.length, o0, (const uint8_t*)dict.data, (uint32_t)dict.length,
                                                (uint32_t)flags);
        if (r < 0) return throw_status(env, r);
        return make_i64(env, r);
    }
    uint64_t in_off = (uint64_t)i0, out_off = (uint64_t)o0;
    uint32_t in_len = (uint32_t)n, out_cap = (uint32_t)(out.length - out_off), out_len = 0;
    int32_t status = 0;
    int32_t st = lz4mi_decompress_blocks((const uint8_t*)in.data, &in_off, &in_len, (uint8_t*)out.data, &out_off,
                                         &out_cap, (const uint8_t*)dict.data, (uint32_t)dict.length, &out_len, &status,
                                         1, (uint32_t)flags, NULL);
    if (st) return throw_status(env, st);
    if (status) return throw_status(env, status);
    return make_i64(env, out_len);
}

static napi_value n_decompress_block(napi_env env, napi_callback_info info) { return decompress_block_impl(env, info, 0); }
static napi_value n_decompress_block_host(napi_env env, napi_callback_info info) {
    return decompress_block_impl(env, info, 1);
}

/* Block offsets: a Float64Array whose entries are integers in [0, 2^53) (anything else
 * would be undefined behaviour to convert and could wrap the bounds checks below). */
static int f64_offsets(napi_env env, const view_t* v, uint32_t n, uint64_t* dst, const char* what) {
    char msg[128];
    if (v->type != napi_float64_array || v->length < n) {
        snprintf(msg, sizeof msg, "lz4mi: %s must be a Float64Array of block offsets", what);
        napi_throw_type_error(env, NULL, msg);
        return 0;
    }
    const double* d = (const double*)v->data;
    for (uint32_t b = 0; b < n; ++b) {
        const double x = d[b];
        if (!(x >= 0.0 && x < 9007199254740992.0) || x != (double)(uint64_t)x) {
            snprintf(msg, sizeof msg, "lz4mi: %s[%u] is not an integer offset in [0, 2^53)", what, b);
            napi_throw_range_error(env, NULL, msg);
            return 0;
        }
        dst[b] = (uint64_t)x;
    }
    return 1;
}

/* off + len <= total, without overflow */
static int in_bounds(uint64_t off, uint64_t len, uint64_t total) { return off <= total && len <= total - off; }

static int u32_array(napi_env env, const view_t* v, uint32_t n, int want_int32, const char* what) {
    napi_typedarray_type t = want_int32 ? napi_int32_array : napi_uint32_array;
    if (v->type != t || v->length < n) {
        char msg[128];
        snprintf(msg, sizeof msg, "lz4mi: %s must be a%s with one entry per block", what,
                 want_int32 ? "n Int32Array" : " Uint32Array");
        napi_throw_type_error(env, NULL, msg);
        return 0;
    }
    return 1;
}

/* compressBlocks(src, srcOff, srcLen, out, outOff, outLen) -> status */
static napi_value n_compress_blocks(napi_env env, napi_callback_info info) {
    size_t argc = 6;
    napi_value argv[6];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t src, soff, slen, out, ooff, olen;
    if (!get_view(env, argv[0], &src, 1, "src") || !get_view(env, argv[1], &soff, 1, "srcOff") ||
        !get_view(env, argv[2], &slen, 1, "srcLen") || !get_view(env, argv[3], &out, 1, "out") ||
        !get_view(env, argv[4], &ooff, 1, "outOff") || !get_view(env, argv[5], &olen, 1, "outLen"))
        return NULL;
    uint32_t n = (uint32_t)slen.length;
    if (!u32_array(env, &slen, n, 0, "srcLen") || !u32_array(env, &olen, n, 0, "outLen")) return NULL;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * 2 * (n ? n : 1));
    if (!offs) return throw_status(env, LZ4MI_ERR_ARG);
    if (!f64_offsets(env, &soff, n, offs, "srcOff") || !f64_offsets(env, &ooff, n, offs + n, "outOff")) {
        free(offs);
        return NULL;
    }
    const uint32_t* lens = (const uint32_t*)slen.data;
    for (uint32_t b = 0; b < n; ++b) {
        if (!in_bounds(offs[b], lens[b], src.length) ||
            !in_bounds(offs[n + b], lz4mi_compress_bound(lens[b]), out.length)) {
            free(offs);
            return throw_status(env, LZ4MI_ERR_ARG);
        }
    }
    int32_t st = lz4mi_compress_blocks((const uint8_t*)src.data, offs, lens, (uint8_t*)out.data, offs + n,
                                       (uint32_t*)olen.data, n, 0, NULL);
    free(offs);
    if (st) return throw_status(env, st);
    return make_i64(env, 0);
}

/* compressChain(src, start, len, blockSize, hashTable, out, outOff, compLen) -> 0: the dependent
 * blocks of one frame in one GPU chain (lz4mi_compress_chain); compressChainHost: the same on
 * the host encoder (lz4mi_host_compress_chain, the JS layer's route for dependent frames) */
static napi_value compress_chain_impl(napi_env env, napi_callback_info info, int host) {
    size_t argc = 8;
    napi_value argv[8];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t src, tab, out, ooff, clen;
    int64_t start, len, bs;
    if (!get_view(env, argv[0], &src, 1, "src") || !get_i64(env, argv[1], &start) || !get_i64(env, argv[2], &len) ||
        !get_i64(env, argv[3], &bs) || !get_view(env, argv[4], &tab, 1, "hashTable") ||
        !get_view(env, argv[5], &out, 1, "out") || !get_view(env, argv[6], &ooff, 1, "outOff") ||
        !get_view(env, argv[7], &clen, 1, "compLen"))
        return NULL;
    if (tab.type != napi_int32_array || tab.length < 16384) {
        napi_throw_type_error(env, NULL, "lz4mi: hashTable must be an Int32Array(16384)");
        return NULL;
    }
    if (start < 0 || len < 0 || bs <= 0 || bs > LZ4MI_MAX_BLOCK || start + len > INT32_MAX ||
        !in_bounds((uint64_t)start, (uint64_t)len, src.length))
        return throw_status(env, LZ4MI_ERR_ARG);   /* (positions are int32 in the reference's table) */
    const uint32_t n = (uint32_t)((len + bs - 1) / bs);
    if (!u32_array(env, &clen, n, 0, "compLen")) return NULL;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    if (!offs) return throw_status(env, LZ4MI_ERR_ARG);
    if (!f64_offsets(env, &ooff, n, offs, "outOff")) {
        free(offs);
        return NULL;
    }
    for (uint32_t b = 0; b < n; ++b) {
        const uint64_t nb = (uint64_t)(len - (int64_t)b * bs) < (uint64_t)bs ? (uint64_t)(len - (int64_t)b * bs) : (uint64_t)bs;
        if (!in_bounds(offs[b], lz4mi_compress_bound(nb), out.length)) {
            free(offs);
            return throw_status(env, LZ4MI_ERR_ARG);
        }
    }
    int32_t st = host ? lz4mi_host_compress_chain((const uint8_t*)src.data, src.length, (int32_t)start, (int32_t)len,
                                                  (int32_t)bs, (int32_t*)tab.data, (uint8_t*)out.data, offs,
                                                  (uint32_t*)clen.data)
                      : lz4mi_compress_chain((const uint8_t*)src.data, src.length, (int32_t)start, (int32_t)len,
                                             (int32_t)bs, (int32_t*)tab.data, (uint8_t*)out.data, offs,
                                             (uint32_t*)clen.data, 0, NULL);
    free(offs);
    if (st) return throw_status(env, st);
    return make_i64(env, 0);
}

static napi_value n_compress_chain(napi_env env, napi_callback_info info) { return compress_chain_impl(env, info, 0); }
static napi_value n_compress_chain_host(napi_env env, napi_callback_info info) {
    return compress_chain_impl(env, info, 1);
}

/* decompressBlocks(input, inOff, inLen, output, outOff, outCap, outLen, status, dictionary?, flags?) -> status */
static napi_value n_decompress_blocks(napi_env env, napi_callback_info info) {
    size_t argc = 10;
    napi_value argv[10];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t in, ioff, ilen, out, ooff, ocap, olen, stat, dict;
    int64_t flags = LZ4MI_JS_EXACT;
    if (!get_view(env, argv[0], &in, 1, "input") || !get_view(env, argv[1], &ioff, 1, "inOff") ||
        !get_view(env, argv[2], &ilen, 1, "inLen") || !get_view(env, argv[3], &out, 1, "output") ||
        !get_view(env, argv[4], &ooff, 1, "outOff") || !get_view(env, argv[5], &ocap, 1, "outCap") ||
        !get_view(env, argv[6], &olen, 1, "outLen") || !get_view(env, argv[7], &stat, 1, "status"))
        return NULL;
    if (!get_view(env, argc > 8 ? argv[8] : NULL, &dict, 0, "dictionary")) return NULL;
    if (argc > 9 && !get_i64(env, argv[9], &flags)) return NULL;
    uint32_t n = (uint32_t)ilen.length;
    if (!u32_array(env, &ilen, n, 0, "inLen") || !u32_array(env, &ocap, n, 0, "outCap") ||
        !u32_array(env, &olen, n, 0, "outLen") || !u32_array(env, &stat, n, 1, "status"))
        return NULL;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * 2 * (n ? n : 1));
    if (!offs) return throw_status(env, LZ4MI_ERR_ARG);
    if (!f64_offsets(env, &ioff, n, offs, "inOff") || !f64_offsets(env, &ooff, n, offs + n, "outOff")) {
        free(offs);
        return NULL;
    }
    const uint32_t* il = (const uint32_t*)ilen.data;
    const uint32_t* oc = (const uint32_t*)ocap.data;
    for (uint32_t b = 0; b < n; ++b) {
        if (!in_bounds(offs[b], il[b], in.length) || !in_bounds(offs[n + b], oc[b], out.length)) {
            free(offs);
            return throw_status(env, LZ4MI_ERR_ARG);
        }
    }
    int32_t st = lz4mi_decompress_blocks((const uint8_t*)in.data, offs, il, (uint8_t*)out.data, offs + n, oc,
                                         (const uint8_t*)dict.data, (uint32_t)dict.length, (uint32_t*)olen.data,
                                         (int32_t*)stat.data, n, (uint32_t)flags, NULL);
    free(offs);
    if (st) return throw_status(env, st);
    return make_i64(env, 0);
}

/* xxHash32(input, seed) */
static napi_value n_xxh32(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t in;
    int64_t seed = 0, flags = 0;
    if (!get_view(env, argv[0], &in, 1, "input")) return NULL;
    if (argc > 1 && !get_i64(env, argv[1], &seed)) return NULL;
    if (argc > 2 && !get_i64(env, argv[2], &flags)) return NULL;
    size_t bytes = in.length;
    if (in.type != napi_uint8_array && in.type != napi_uint8_clamped_array && in.type != napi_int8_array) {
        napi_throw_type_error(env, NULL, "lz4mi: input must be a Uint8Array");
        return NULL;
    }
    uint32_t h = lz4mi_xxh32((const uint8_t*)in.data, bytes, (uint32_t)seed, (uint32_t)flags);
    napi_value r;
    CHECK(napi_create_uint32(env, h, &r));
    return r;
}

/* xxh32Reset(seed, flags?) -> Uint8Array holding an lz4mi_xxh32_state */
static napi_value n_xxh32_reset(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    int64_t seed = 0, flags = 0;
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc > 0 && !get_i64(env, argv[0], &seed)) return NULL;
    if (argc > 1 && !get_i64(env, argv[1], &flags)) return NULL;
    napi_value ab, ta;
    void* data = NULL;
    CHECK(napi_create_arraybuffer(env, sizeof(lz4mi_xxh32_state), &data, &ab));
    lz4mi_xxh32_reset((lz4mi_xxh32_state*)data, (uint32_t)seed, (uint32_t)flags);
    CHECK(napi_create_typedarray(env, napi_uint8_array, sizeof(lz4mi_xxh32_state), ab, 0, &ta));
    return ta;
}

static lz4mi_xxh32_state* get_state(napi_env env, napi_value v) {
    view_t st;
    if (!get_view(env, v, &st, 1, "state")) return NULL;
    if (st.type != napi_uint8_array || st.length != sizeof(lz4mi_xxh32_state) || ((uintptr_t)st.data & 7)) {
        napi_throw_type_error(env, NULL, "lz4mi: state must come from xxh32Reset");
        return NULL;
    }
    return (lz4mi_xxh32_state*)st.data;
}

/* xxh32Update(state, input) */
static napi_value n_xxh32_update(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    lz4mi_xxh32_state* st = get_state(env, argv[0]);
    if (!st) return NULL;
    view_t in;
    if (!get_view(env, argv[1], &in, 1, "input")) return NULL;
    if (in.type != napi_uint8_array && in.type != napi_uint8_clamped_array && in.type != napi_int8_array) {
        napi_throw_type_error(env, NULL, "lz4mi: input must be a Uint8Array");
        return NULL;
    }
    lz4mi_xxh32_update(st, (const uint8_t*)in.data, in.length);
    return NULL;
}

/* xxh32Digest(state) -> uint32 */
static napi_value n_xxh32_digest(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    lz4mi_xxh32_state* st = get_state(env, argv[0]);
    if (!st) return NULL;
    napi_value r;
    CHECK(napi_create_uint32(env, lz4mi_xxh32_digest(st), &r));
    return r;
}

/* xxh32Blocks(input, off: Float64Array, len: Uint32Array, seed, hashes: Uint32Array, flags?) -> 0 */
static napi_value n_xxh32_blocks(napi_env env, napi_callback_info info) {
    size_t argc = 6;
    napi_value argv[6];
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    view_t in, off, len, hs;
    int64_t seed = 0, flags = 0;
    if (!get_view(env, argv[0], &in, 1, "input") || !get_view(env, argv[1], &off, 1, "off") ||
        !get_view(env, argv[2], &len, 1, "len") || !get_view(env, argv[4], &hs, 1, "hashes"))
        return NULL;
    if (!get_i64(env, argv[3], &seed)) return NULL;
    if (argc > 5 && !get_i64(env, argv[5], &flags)) return NULL;
    uint32_t n = (uint32_t)len.length;
    if (!u32_array(env, &len, n, 0, "len") || !u32_array(env, &hs, n, 0, "hashes")) return NULL;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    if (!offs) return throw_status(env, LZ4MI_ERR_ARG);
    if (!f64_offsets(env, &off, n, offs, "off")) {
        free(offs);
        return NULL;
    }
    const uint32_t* l = (const uint32_t*)len.data;
    for (uint32_t b = 0; b < n; ++b) {
        if (!in_bounds(offs[b], l[b], in.length)) {
            free(offs);
            return throw_status(env, LZ4MI_ERR_ARG);
        }
    }
    int32_t st = lz4mi_xxh32_blocks((const uint8_t*)in.data, offs, l, (uint32_t)seed, (uint32_t*)hs.data, n,
                                    (uint32_t)flags & LZ4MI_XXH_STANDARD, NULL);
    free(offs);
    if (st) return throw_status(env, st);
    return make_i64(env, 0);
}

static napi_value n_status_message(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    int64_t code = 0;
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (!get_i64(env, argv[0], &code)) return NULL;
    napi_value r;
    CHECK(napi_create_string_utf8(env, lz4mi_status_message((int32_t)code), NAPI_AUTO_LENGTH, &r));
    return r;
}

static napi_value n_init(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    int64_t dev = 0;
    CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc > 0 && !get_i64(env, argv[0], &dev)) return NULL;
    return make_i64(env, lz4mi_init((int32_t)dev));
}

static napi_value n_version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value r;
    CHECK(napi_create_string_utf8(env, lz4mi_version(), NAPI_AUTO_LENGTH, &r));
    return r;
}

static napi_value n_build_id(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value r;
    CHECK(napi_create_string_utf8(env, lz4mi_build_id(), NAPI_AUTO_LENGTH, &r));
    return r;
}

static napi_value n_device_count(napi_env env, napi_callback_info info) {
    (void)info;
    return make_i64(env, lz4mi_device_count());
}

static napi_value Init(napi_env env, napi_value exports) {
    napi_property_descriptor fns[] = {
        {"compressBlock", NULL, n_compress_block, NULL, NULL, NULL, napi_default, NULL},
        {"decompressBlock", NULL, n_decompress_block, NULL, NULL, NULL, napi_default, NULL},
        {"compressBlocks", NULL, n_compress_blocks, NULL, NULL, NULL, napi_default, NULL},
        {"compressChain", NULL, n_compress_chain, NULL, NULL, NULL, napi_default, NULL},
        {"compressBlockHost", NULL, n_compress_block_host, NULL, NULL, NULL, napi_default, NULL},
        {"compressChainHost", NULL, n_compress_chain_host, NULL, NULL, NULL, napi_default, NULL},
        {"decompressBlockHost", NULL, n_decompress_block_host, NULL, NULL, NULL, napi_default, NULL},
        {"decompressBlocks", NULL, n_decompress_blocks, NULL, NULL, NULL, napi_default, NULL},
        {"xxHash32", NULL, n_xxh32, NULL, NULL, NULL, napi_default, NULL},
        {"xxh32Reset", NULL, n_xxh32_reset, NULL, NULL, NULL, napi_default, NULL},
        {"xxh32Update", NULL, n_xxh32_update, NULL, NULL, NULL, napi_default, NULL},
        {"xxh32Digest", NULL, n_xxh32_digest, NULL, NULL, NULL, napi_default, NULL},
        {"xxh32Blocks", NULL, n_xxh32_blocks, NULL, NULL, NULL, napi_default, NULL},
        {"buildId", NULL, n_build_id, NULL, NULL, NULL, napi_default, NULL},
        {"statusMessage", NULL, n_status_message, NULL, NULL, NULL, napi_default, NULL},
        {"init", NULL, n_init, NULL, NULL, NULL, napi_default, NULL},
        {"version", NULL, n_version, NULL, NULL, NULL, napi_default, NULL},
        {"deviceCount", NULL, n_device_count, NULL, NULL, NULL, napi_default, NULL},
    };
    if (napi_define_properties(env, exports, sizeof fns / sizeof fns[0], fns) != napi_ok) return NULL;
    const struct { const char* name; int64_t v; } consts[] = {
        {"JS_COMPAT", LZ4MI_JS_COMPAT}, {"JS_EXACT", LZ4MI_JS_EXACT}, {"XXH_STANDARD", LZ4MI_XXH_STANDARD},
        {"XXH_LEN64", LZ4MI_XXH_LEN64}, {"ERR_CROSS_BLOCK", LZ4MI_ERR_CROSS_BLOCK},
    };
    for (size_t i = 0; i < sizeof consts / sizeof consts[0]; ++i) {
        napi_value v;
        napi_create_int64(env, consts[i].v, &v);
        napi_set_named_property(env, exports, consts[i].name, v);
    }
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
