// lz4mi_host.cpp — the host-CPU block encoder of the drop-in's routing:
// calls that are one serial chain by definition — dependent-block frames (the
// reference's LZ4.compress default, bufferCompress.js:182-236), a dictionary's first
// block, LZ4.compressRaw into an output buffer too small for the worst case — run on
// the calling thread instead of one GPU wave. A GPU wave walks a single chain far more
// slowly than a CPU core (0.12 GB/s vs ~1 GB/s for one core of JS), and
// these calls have no block-level parallelism to offer the GPU.
//
// This is product code, not the oracle: a fresh restatement of compressBlock
// (src/block/blockCompress.js:31-233) with the reference's exact semantics — table
// values absolute position + 1 (<= 0 empty), insert before verify, skip steps
// (c++ >> 6), no inserts inside matches, output writes past the buffer dropped as a
// typed array drops them, and the RangeError output.set() throws for a literal run of
// more than 64 bytes that does not fit (blockCompress.js:100, :198).
#include <climits>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/lz4mi.h"

extern "C" __attribute__((visibility("hidden"))) void lz4mi_advise_output(void* p, uint64_t n);   // (lz4mi_capi.cpp)

namespace {

constexpr uint32_t kMul = 2654435761u;

inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

// Output with the reference's typed-array semantics: writes at or past `cap` vanish.
struct Out {
    uint8_t* p;
    int64_t cap;
    int64_t d;   // next write position (absolute in p)
    inline void put(uint32_t v) {
        if (d < cap) p[d] = (uint8_t)v;
        ++d;
    }
    inline void len_ext(int64_t l) {   // the 255-run tail of a length field
        while (l >= 255) {
            put(255);
            l -= 255;
        }
        put((uint32_t)l);
    }
    // literal bytes src[0, n): in the reference a run of more than 64 is one output.set(),
    // which throws (writing nothing) when it does not fit; shorter runs are byte stores
    inline bool lits(const uint8_t* src, int64_t n) {
        if (n > 64 && d + n > cap) return false;
        if (d + n <= cap) {
            std::memcpy(p + d, src, (size_t)n);
        } else if (d < cap) {
            std::memcpy(p + d, src, (size_t)(cap - d));
        }
        d += n;
        return true;
    }
};

// Length of the common run of a[0..] and b[0..] (a > b), at most lim bytes.
inline int64_t common(const uint8_t* a, const uint8_t* b, int64_t lim) {
    int64_t k = 0;
    while (k + 8 <= lim) {
        uint64_t x, y;
        std::memcpy(&x, a + k, 8);
        std::memcpy(&y, b + k, 8);
        if (x != y) return k + (__builtin_ctzll(x ^ y) >> 3);
        k += 8;
    }
    while (k < lim && a[k] == b[k]) ++k;
    return k;
}

// One compressBlock call. Returns bytes written (dIndex - outputOffset) or LZ4MI_ERR_RANGE.
int64_t compress_block(const uint8_t* src, int32_t start, int32_t len, int32_t* T, Out& o) {
    const int64_t out0 = o.d;
    const int64_t end = (int64_t)start + len;   // callers keep start + len <= INT32_MAX
    const int64_t mflimit = end - 12, matchlimit = end - 5;
    int32_t i = start, anchor = start;
    uint32_t c = 67;
    while (i < mflimit) {
        const uint32_t seq = rd32(src + i);
        const uint32_t h = (seq * kMul) >> 18;
        const int32_t m = (int32_t)((uint32_t)T[h] - 1u);
        T[h] = i + 1;
        // the reference's order: empty, itself, more than 65535 back (or ahead), content
        if (m < 0 || m == i || ((uint32_t)(i - m) >> 16) != 0 || rd32(src + m) != seq) {
            i += (int32_t)(c++ >> 6);
            continue;
        }
        c = 67;
        const int64_t lit = i - anchor;
        const int64_t tok = o.d;
        o.put(lit >= 15 ? 0xF0u : (uint32_t)lit << 4);
        if (lit >= 15) o.len_ext(lit - 15);
        if (!o.lits(src + anchor, lit)) return LZ4MI_ERR_RANGE;
        const int64_t e = i + 4 + common(src + i + 4, src + m + 4, (int64_t)matchlimit - (i + 4) > 0 ? matchlimit - (i + 4) : 0);
        const uint32_t off = (uint32_t)(i - m);
        o.put(off & 255);
        o.put((off >> 8) & 255);
        const int64_t code = e - i - 4;
        if (tok < o.cap) o.p[tok] |= (uint8_t)(code >= 15 ? 15 : code);
        if (code >= 15) o.len_ext(code - 15);
        i = (int32_t)e;
        anchor = (int32_t)e;
    }
    const int64_t lit = end - anchor;   // >= 0: anchor <= end
    o.put(lit >= 15 ? 0xF0u : (uint32_t)lit << 4);
    if (lit >= 15) o.len_ext(lit - 15);
    if (!o.lits(src + anchor, lit)) return LZ4MI_ERR_RANGE;
    return (int64_t)(int32_t)(o.d - out0);
}

}  // namespace

extern "C" {

int64_t lz4mi_host_compress_block(const uint8_t* src, uint64_t src_total, int32_t src_start, int32_t src_len,
                                  int32_t* table, uint8_t* out, uint64_t out_total, int32_t out_off) {
    // positions are int32 (the table holds position + 1): start + len must stay below 2^31
    if ((!src && src_total) || !table || src_start < 0 || src_len < 0 ||
        (uint64_t)src_start + (uint64_t)src_len > src_total || (uint64_t)src_start + (uint64_t)src_len > INT32_MAX ||
        out_off < 0 || (!out && out_total))
        return LZ4MI_ERR_ARG;
    Out o{out, (int64_t)out_total, out_off};
    return compress_block(src, src_start, src_len, table, o);
}

int32_t lz4mi_host_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len,
                                  int32_t block_size, int32_t* table, uint8_t* out, const uint64_t* out_off,
                                  uint32_t* comp_len) {
    if ((!src && src_total) || !table || !out || !out_off || !comp_len || start < 0 || len < 0 || block_size <= 0 ||
        (uint64_t)start + (uint64_t)len > src_total || (uint64_t)start + (uint64_t)len > INT32_MAX)
        return LZ4MI_ERR_ARG;
    const int64_t nb = ((int64_t)len + block_size - 1) / block_size;
    for (int64_t b = 0; b < nb; ++b) {
        const int32_t s = start + (int32_t)(b * block_size);
        const int32_t n = (int32_t)((int64_t)start + len - s < block_size ? (int64_t)start + len - s : block_size);
        Out o{out + out_off[b], (int64_t)lz4mi_compress_bound((uint32_t)n), 0};
        const int64_t w = compress_block(src, s, n, table, o);
        if (w < 0) return (int32_t)w;
        comp_len[b] = (uint32_t)w;
    }
    return LZ4MI_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Host-CPU block decoder of the routing (a dependent-block frame decodes block by block,
// each block reading the previous blocks' output: one serial chain). A fresh
// restatement of decompressBlock (src/block/blockDecompress.js:30-275) with the reference's
// typed-array semantics: reads past an array's end (or before its start) give 0, writes
// past the output's end vanish, and — unless `spec` — the double-copy tail of a short far
// match rewrites the bytes before it (:219-250). `spec` decodes per the LZ4
// format instead (what every other LZ4 implementation writes).
namespace {

struct Arr {
    const uint8_t* p;
    int64_t n;
    inline uint32_t at(int64_t i) const { return (i >= 0 && i < n) ? p[i] : 0u; }
};

struct OutArr {
    uint8_t* p;
    int64_t n;
    inline uint32_t at(int64_t i) const { return (i >= 0 && i < n) ? p[i] : 0u; }
    inline void put(int64_t i, uint32_t v) {
        if (i >= 0 && i < n) p[i] = (uint8_t)v;
    }
};

int64_t decompress_block(Arr in, int64_t in_pos, int64_t in_end, OutArr out, int64_t out_pos, Arr dict, bool spec) {
    const int64_t out0 = out_pos;
    while (in_pos < in_end) {
        const uint32_t token = in.at(in_pos++);
        int64_t ll = token >> 4;
        if (ll == 15) {
            uint32_t s;
            do {
                s = in.at(in_pos++);
                ll += s;
            } while (s == 255);
        }
        const int64_t end_lit = out_pos + ll;
        if (end_lit > out.n) return LZ4MI_ERR_OUTPUT_TOO_SMALL;   // :74
        if (in_pos + ll > in_end) return LZ4MI_ERR_MALFORMED;       // :75
        if (ll > 0) {
            if (in_pos >= 0 && in_pos + ll <= in.n) {
                std::memcpy(out.p + out_pos, in.p + in_pos, (size_t)ll);
            } else {
                for (int64_t k = 0; k < ll; ++k) out.put(out_pos + k, in.at(in_pos + k));
            }
        }
        out_pos = end_lit;
        in_pos += ll;
        if (in_pos >= in_end) break;
        const uint32_t offset = in.at(in_pos) | (in.at(in_pos + 1) << 8);
        in_pos += 2;
        if (offset == 0) return LZ4MI_ERR_OFFSET0;                  // :128
        int64_t ml = token & 15;
        if (ml == 15) {
            uint32_t s;
            do {
                s = in.at(in_pos++);
                ml += s;
            } while (s == 255);
        }
        ml += 4;
        int64_t src = out_pos - (int64_t)offset;
        if (src < 0) {                                              // dictionary (:143-185)
            int64_t from_dict = -src;
            src += dict.n;
            if (from_dict > ml) from_dict = ml;
            if (src < 0 || src + from_dict > dict.n) return LZ4MI_ERR_DICT_OOB;
            for (int64_t k = 0; k < from_dict; ++k) out.put(out_pos + k, dict.p[src + k]);
            out_pos += from_dict;
            const int64_t rest = ml - from_dict;
            for (int64_t k = 0; k < rest; ++k, ++out_pos) out.put(out_pos, out.at(out_pos - (int64_t)offset));
            continue;
        }
        if (offset == 1) {                                          // output.fill (:190)
            const uint32_t v = out.at(src);
            const int64_t a = out_pos < out.n ? out_pos : out.n, b = out_pos + ml < out.n ? out_pos + ml : out.n;
            if (b > a) std::memset(out.p + a, (int)v, (size_t)(b - a));
            out_pos += ml;
            continue;
        }
        if ((int64_t)offset >= ml && ml > 16) {                     // output.copyWithin (:195)
            int64_t cnt = ml;
            if (src + cnt > out.n) cnt = out.n - src;
            if (out_pos + cnt > out.n) cnt = out.n - out_pos;
            if (cnt > 0) std::memmove(out.p + out_pos, out.p + src, (size_t)cnt);
            out_pos += ml;
            continue;
        }
        const int64_t end = out_pos + ml;                           // general copy (:200-268)
        if (end <= out.n && src >= 0) {                             // in bounds: no per-byte checks
            uint8_t* o = out.p;
            if (offset >= 8) {
                int64_t r = src;
                for (; out_pos + 8 <= end; out_pos += 8, r += 8) std::memcpy(o + out_pos, o + r, 8);
                if (out_pos < end) {
                    if (spec) {
                        for (; out_pos < end; ++out_pos, ++r) o[out_pos] = o[r];
                    } else if (end - 8 >= 0) {                      // F1: the last 8 bytes again
                        std::memcpy(o + end - 8, o + r + (end - out_pos) - 8, 8);
                        out_pos = end;
                    } else {
                        const int64_t t_out = end - 8, t_src = r + (end - out_pos) - 8;
                        for (int k = 0; k < 8; ++k) out.put(t_out + k, out.at(t_src + k));
                        out_pos = end;
                    }
                }
            } else {
                for (int64_t r = src; out_pos < end; ++out_pos, ++r) o[out_pos] = o[r];
            }
            continue;
        }
        if (offset >= 8 && !spec) {
            int64_t r = src;
            while (out_pos < end - 8) {
                for (int k = 0; k < 8; ++k) out.put(out_pos + k, out.at(r + k));
                out_pos += 8;
                r += 8;
            }
            if (out_pos < end) {                                    // the double-copy tail (F1)
                const int64_t t_out = end - 8, t_src = r + (end - out_pos) - 8;
                for (int k = 0; k < 8; ++k) out.put(t_out + k, out.at(t_src + k));
                out_pos = end;
            }
        } else {
            for (int64_t r = src; out_pos < end; ++out_pos, ++r) out.put(out_pos, out.at(r));
        }
    }
    return (int64_t)(int32_t)(out_pos - out0);
}

}  // namespace

extern "C" int64_t lz4mi_host_decompress_block(const uint8_t* in, uint64_t in_total, int64_t in_off, int64_t in_size,
                                               uint8_t* out, uint64_t out_total, int64_t out_off, const uint8_t* dict,
                                               uint32_t dict_len, uint32_t flags) {
    if ((!in && in_total) || (!out && out_total) || (!dict && dict_len) || in_off < 0 || in_size < 0 || out_off < 0)
        return LZ4MI_ERR_ARG;
    // only the range this block can write: a length byte adds at most 255 output bytes, so a block of
    // in_size bytes writes fewer than 255 * in_size + 64 (a caller decoding block after block into
    // one large array does not advise the whole rest of it on every call)
    if ((uint64_t)out_off < out_total)
        lz4mi_advise_output(out + out_off, std::min<uint64_t>(out_total - (uint64_t)out_off,
                                                              255ull * (uint64_t)in_size + 64));   // (lz4mi_capi.cpp)
    return decompress_block(Arr{in, (int64_t)in_total}, in_off, in_off + in_size, OutArr{out, (int64_t)out_total},
                            out_off, Arr{dict, (int64_t)dict_len}, !(flags & (LZ4MI_JS_COMPAT | LZ4MI_JS_EXACT)));
}
