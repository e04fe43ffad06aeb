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
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/lz4mi.h"

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
    const int32_t end = start + len;
    const int32_t mflimit = end - 12, matchlimit = end - 5;
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
    const int64_t lit = end - anchor;
    o.put(lit >= 15 ? 0xF0u : (uint32_t)lit << 4);
    if (lit >= 15) o.len_ext(lit - 15);
    if (!o.lits(src + anchor, lit)) return LZ4MI_ERR_RANGE;
    return (int64_t)(int32_t)(o.d - out0);
}

}  // namespace

extern "C" {

int64_t lz4mi_host_compress_block(const uint8_t* src, uint64_t src_total, int32_t src_start, int32_t src_len,
                                  int32_t* table, uint8_t* out, uint64_t out_total, int32_t out_off) {
    if ((!src && src_total) || !table || src_start < 0 || src_len < 0 ||
        (uint64_t)src_start + (uint64_t)src_len > src_total || out_off < 0 || (!out && out_total))
        return LZ4MI_ERR_ARG;
    Out o{out, (int64_t)out_total, out_off};
    return compress_block(src, src_start, src_len, table, o);
}

int32_t lz4mi_host_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len,
                                  int32_t block_size, int32_t* table, uint8_t* out, const uint64_t* out_off,
                                  uint32_t* comp_len) {
    if ((!src && src_total) || !table || !out || !out_off || !comp_len || start < 0 || len < 0 || block_size <= 0 ||
        (uint64_t)start + (uint64_t)len > src_total)
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
