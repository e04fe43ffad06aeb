// lz4mi_capi.cpp — host side of liblz4mi.so: the C-ABI declared in
// include/lz4mi.h. Owns the per-device context (stream, grow-only device
// scratch), stages host buffers for the synchronous entry points and launches
// the gfx950 kernels. No CPU fallback: without a gfx950 device every entry
// point that needs the GPU returns LZ4MI_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/lz4mi.h"

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                              const uint64_t*, const uint32_t*, const uint8_t*, uint32_t, uint32_t*,
                                              int32_t*, uint32_t, int, hipStream_t);
extern "C" hipError_t lz4mi_launch_compress(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                            const uint64_t*, uint32_t*, uint32_t, int32_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_frame_pack(const uint8_t*, const uint64_t*, const uint32_t*, const uint8_t*,
                                              const uint64_t*, const uint32_t*, uint8_t*, const uint64_t*, uint32_t,
                                              hipStream_t);
extern "C" hipError_t lz4mi_launch_compress_table(const uint8_t*, uint64_t, int32_t, int32_t, int32_t*, uint8_t*,
                                                  uint64_t, int32_t, int64_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_xxh32(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint32_t*,
                                         uint32_t, int, hipStream_t);
extern "C" hipError_t lz4mi_launch_generate(uint8_t*, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);

namespace {

struct Scratch {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1 << 20);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct Ctx {
    int device = -1;
    hipStream_t stream = nullptr;
    Scratch in, out, meta, aux;
    Scratch tables;   // batch encoder hash tables (64 KiB per block)
    std::mutex mu;
};

Ctx g_ctx;
std::mutex g_init_mu;

#define LZ4MI_TRY(expr)                           \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return LZ4MI_ERR_HIP; \
    } while (0)

int32_t ensure_init() {
    if (g_ctx.device >= 0) return LZ4MI_OK;
    return lz4mi_init(-1);
}

hipStream_t pick_stream(void* s) { return s ? static_cast<hipStream_t>(s) : g_ctx.stream; }

// ---- host XXH32 (reference variant by default, see lz4mi_xxh32.hip) -------
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t le32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

}  // namespace

extern "C" {

const char* lz4mi_status_message(int32_t s) {
    switch (s) {
        case LZ4MI_OK: return "OK";
        case LZ4MI_ERR_OUTPUT_TOO_SMALL: return "LZ4: Output Buffer Too Small";
        case LZ4MI_ERR_MALFORMED: return "LZ4: Malformed Input";
        case LZ4MI_ERR_OFFSET0: return "LZ4: Invalid Offset 0";
        case LZ4MI_ERR_DICT_OOB: return "LZ4: Dictionary Offset Out of Bounds";
        case LZ4MI_ERR_MAGIC: return "LZ4: Invalid Magic Number";
        case LZ4MI_ERR_VERSION: return "LZ4: Unsupported Version";
        case LZ4MI_ERR_CHECKSUM: return "LZ4: Content Checksum Error";
        case LZ4MI_ERR_RANGE: return "offset is out of bounds";
        case LZ4MI_ERR_CROSS_BLOCK: return "lz4mi: block references data before its start (not an independent block)";
        case LZ4MI_ERR_HIP: return "lz4mi: HIP runtime error";
        case LZ4MI_ERR_ARG: return "lz4mi: invalid argument";
        case LZ4MI_ERR_NO_DEVICE: return "lz4mi: no gfx950 (MI355X) device available";
        default: return "lz4mi: unknown status";
    }
}

const char* lz4mi_version(void) { return "lz4mi 0.1 (gfx950)"; }

int32_t lz4mi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int32_t lz4mi_init(int32_t device) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return LZ4MI_ERR_NO_DEVICE;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= n) return LZ4MI_ERR_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return LZ4MI_ERR_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LZ4MI_ERR_NO_DEVICE;
    if (g_ctx.device == device) return LZ4MI_OK;
    LZ4MI_TRY(hipSetDevice(device));
    if (g_ctx.stream) (void)hipStreamDestroy(g_ctx.stream);
    LZ4MI_TRY(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
    g_ctx.device = device;
    return LZ4MI_OK;
}

uint32_t lz4mi_xxh32(const uint8_t* in, size_t len, uint32_t seed, uint32_t flags) {
    size_t p = 0;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        for (; p + 16 <= len; p += 16) {
            v1 = rotl(v1 + le32(in + p) * P2, 13) * P1;
            v2 = rotl(v2 + le32(in + p + 4) * P2, 13) * P1;
            v3 = rotl(v3 + le32(in + p + 8) * P2, 13) * P1;
            v4 = rotl(v4 + le32(in + p + 12) * P2, 13) * P1;
        }
        if (flags & LZ4MI_XXH_STANDARD) {
            h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        } else {   // the reference's chained convergence (xxhash32.js:59-65)
            h = rotl(rotl(rotl(rotl(v1, 1) + v2, 7) + v3, 12) + v4, 18);
        }
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; p + 4 <= len; p += 4) h = rotl(h + le32(in + p) * P3, 17) * P4;
    for (; p < len; ++p) h = rotl(h + in[p] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

int32_t lz4mi_decompress_blocks(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict,
                                uint32_t dict_len, uint32_t* out_len, int32_t* status, uint32_t nblocks,
                                uint32_t flags, void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    const int js = (flags & LZ4MI_JS_COMPAT) ? 1 : 0;
    const int mode = js ? 1 : ((flags & LZ4MI_JS_EXACT) ? 2 : 0);
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        LZ4MI_TRY(lz4mi_launch_decompress(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status,
                                          nblocks, mode, pick_stream(stream)));
        return LZ4MI_OK;
    }
    if (!in || !out || !in_off || !in_len || !out_off || !out_cap || !out_len || !status) return LZ4MI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    // Pack the compressed blocks; stage the output image [lo - hist, hi) so
    // back-references into bytes preceding a block (reference semantics:
    // positions are absolute in `out`) see the caller's bytes.
    uint64_t in_total = 0, lo = UINT64_MAX, hi = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        in_total += (in_len[b] + 15u) & ~15ull;
        lo = std::min<uint64_t>(lo, out_off[b]);
        hi = std::max<uint64_t>(hi, out_off[b] + out_cap[b]);
    }
    uint64_t hist = std::min<uint64_t>(lo, 65536);
    uint64_t base = lo - hist, img = hi - base;
    std::vector<uint64_t> d_in_off(nblocks), d_out_off(nblocks);
    uint64_t pos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        d_in_off[b] = pos;
        pos += (in_len[b] + 15u) & ~15ull;
        d_out_off[b] = out_off[b] - base;
    }
    // Dictionary bytes are only reachable when the image starts at out[0].
    uint32_t dlen = (base == 0 && dict) ? dict_len : 0;
    LZ4MI_TRY(g_ctx.in.ensure(in_total + 64));
    LZ4MI_TRY(g_ctx.out.ensure(img + 64));
    LZ4MI_TRY(g_ctx.aux.ensure((size_t)dlen + 64));
    const size_t meta_bytes = (size_t)nblocks * (8 + 4 + 8 + 4 + 4 + 4);
    LZ4MI_TRY(g_ctx.meta.ensure(meta_bytes + 64));
    uint8_t* m = g_ctx.meta.as<uint8_t>();
    uint64_t* m_in_off = (uint64_t*)m;
    uint64_t* m_out_off = m_in_off + nblocks;
    uint32_t* m_in_len = (uint32_t*)(m_out_off + nblocks);
    uint32_t* m_out_cap = m_in_len + nblocks;
    uint32_t* m_out_len = m_out_cap + nblocks;
    int32_t* m_status = (int32_t*)(m_out_len + nblocks);
    for (uint32_t b = 0; b < nblocks; ++b)
        LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.as<uint8_t>() + d_in_off[b], in + in_off[b], in_len[b],
                                 hipMemcpyHostToDevice, s));
    // js-compat may rewrite bytes anywhere before a match and its result is
    // copied back whole: stage the whole image so untouched bytes survive.
    const uint64_t up = js ? img : hist;
    if (up) LZ4MI_TRY(hipMemcpyAsync(g_ctx.out.p, out + base, up, hipMemcpyHostToDevice, s));
    if (dlen) LZ4MI_TRY(hipMemcpyAsync(g_ctx.aux.p, dict, dlen, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_in_off, d_in_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_out_off, d_out_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_in_len, in_len, 4ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_out_cap, out_cap, 4ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(lz4mi_launch_decompress(g_ctx.in.as<uint8_t>(), m_in_off, m_in_len, g_ctx.out.as<uint8_t>(), m_out_off,
                                      m_out_cap, dlen ? g_ctx.aux.as<uint8_t>() : nullptr, dlen, m_out_len, m_status,
                                      nblocks, mode, s));
    LZ4MI_TRY(hipMemcpyAsync(out_len, m_out_len, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipMemcpyAsync(status, m_status, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    // copy back what each successful block wrote (js-compat may also rewrite up
    // to 7 bytes before a match: copy its whole image range instead)
    if (js) {   // like the reference, bytes written before an error stay written
        LZ4MI_TRY(hipMemcpyAsync(out + base, g_ctx.out.p, img, hipMemcpyDeviceToHost, s));
    } else {
        for (uint32_t b = 0; b < nblocks; ++b) {
            if (status[b] != 0) continue;
            uint64_t n = std::min<uint64_t>(out_len[b], out_cap[b]);
            // a lone block re-decoded reference-exactly may rewrite up to 7 bytes
            // before its start (F1 at the block's first match): copy those back too
            const uint64_t pre = (mode == 2 && nblocks == 1) ? std::min<uint64_t>(d_out_off[b], 8) : 0;
            if (n + pre) LZ4MI_TRY(hipMemcpyAsync(out + out_off[b] - pre, g_ctx.out.as<uint8_t>() + d_out_off[b] - pre,
                                                  n + pre, hipMemcpyDeviceToHost, s));
        }
    }
    LZ4MI_TRY(hipStreamSynchronize(s));
    return LZ4MI_OK;
}

int32_t lz4mi_compress_blocks(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                              const uint64_t* out_off, uint32_t* out_len, uint32_t nblocks, uint32_t flags,
                              void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        // the table scratch is the context's: launches through it are serialised on the context's lock
        // and ordered on one stream per context use (see include/lz4mi.h)
        std::lock_guard<std::mutex> lk(g_ctx.mu);
        LZ4MI_TRY(g_ctx.tables.ensure((size_t)nblocks * 16384 * sizeof(int32_t)));
        LZ4MI_TRY(lz4mi_launch_compress(in, in_off, in_len, out, out_off, out_len, nblocks, g_ctx.tables.as<int32_t>(),
                                        pick_stream(stream)));
        return LZ4MI_OK;
    }
    if (!in || !out || !in_off || !in_len || !out_off || !out_len) return LZ4MI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    std::vector<uint64_t> d_in_off(nblocks), d_out_off(nblocks);
    uint64_t ipos = 0, opos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        d_in_off[b] = ipos;
        ipos += (in_len[b] + 15u) & ~15ull;
        d_out_off[b] = opos;
        opos += (lz4mi_compress_bound(in_len[b]) + 15u) & ~15ull;
    }
    LZ4MI_TRY(g_ctx.in.ensure(ipos + 64));
    LZ4MI_TRY(g_ctx.out.ensure(opos + 64));
    LZ4MI_TRY(g_ctx.meta.ensure((size_t)nblocks * 24 + 64));
    uint64_t* m_in_off = g_ctx.meta.as<uint64_t>();
    uint64_t* m_out_off = m_in_off + nblocks;
    uint32_t* m_in_len = (uint32_t*)(m_out_off + nblocks);
    uint32_t* m_out_len = m_in_len + nblocks;
    for (uint32_t b = 0; b < nblocks; ++b)
        LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.as<uint8_t>() + d_in_off[b], in + in_off[b], in_len[b],
                                 hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_in_off, d_in_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_out_off, d_out_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_in_len, in_len, 4ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(g_ctx.tables.ensure((size_t)nblocks * 16384 * sizeof(int32_t)));
    LZ4MI_TRY(lz4mi_launch_compress(g_ctx.in.as<uint8_t>(), m_in_off, m_in_len, g_ctx.out.as<uint8_t>(), m_out_off,
                                    m_out_len, nblocks, g_ctx.tables.as<int32_t>(), s));
    LZ4MI_TRY(hipMemcpyAsync(out_len, m_out_len, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    for (uint32_t b = 0; b < nblocks; ++b)
        if (out_len[b])
            LZ4MI_TRY(hipMemcpyAsync(out + out_off[b], g_ctx.out.as<uint8_t>() + d_out_off[b], out_len[b],
                                     hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    return LZ4MI_OK;
}

int64_t lz4mi_compress_block_table(const uint8_t* src, uint64_t src_total, int32_t src_start, int32_t src_len,
                                   int32_t* table, uint8_t* out, uint64_t out_total, int32_t out_off, uint32_t flags,
                                   void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    if (src_start < 0 || src_len < 0 || (uint64_t)src_start + (uint64_t)src_len > src_total || !table)
        return LZ4MI_ERR_ARG;
    if (flags & LZ4MI_DEVICE_PTRS) return LZ4MI_ERR_ARG;   // host-only entry point (see header)
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = pick_stream(stream);
    // Candidates never reach further back than 65535 bytes: stage only
    // src[base, start+len) and shift table values by `base` (int32 wrap keeps
    // untouched entries exact; shifted-out entries stay rejected).
    int64_t base = std::max<int64_t>(0, (int64_t)src_start - 65536);
    uint64_t sbytes = (uint64_t)src_start + src_len - base;
    uint64_t obytes = out_total > (uint64_t)out_off ? out_total - (uint64_t)out_off : 0;
    LZ4MI_TRY(g_ctx.in.ensure(sbytes + 64));
    LZ4MI_TRY(g_ctx.out.ensure(obytes + 64));
    LZ4MI_TRY(g_ctx.meta.ensure(16384 * 4 + 64));
    std::vector<int32_t> t(16384);
    for (int k = 0; k < 16384; ++k) t[k] = (int32_t)((uint32_t)table[k] - (uint32_t)base);
    int32_t* d_table = g_ctx.meta.as<int32_t>();
    int64_t* d_ret = (int64_t*)(d_table + 16384);
    if (sbytes) LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.p, src + base, sbytes, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(d_table, t.data(), 16384 * 4, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(lz4mi_launch_compress_table(g_ctx.in.as<uint8_t>(), sbytes, (int32_t)(src_start - base), src_len,
                                          d_table, g_ctx.out.as<uint8_t>(), obytes, 0, d_ret, s));
    int64_t ret = 0;
    LZ4MI_TRY(hipMemcpyAsync(&ret, d_ret, 8, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipMemcpyAsync(t.data(), d_table, 16384 * 4, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    uint64_t n = std::min<uint64_t>((uint64_t)ret, obytes);
    if (n) LZ4MI_TRY(hipMemcpy(out + out_off, g_ctx.out.p, n, hipMemcpyDeviceToHost));
    for (int k = 0; k < 16384; ++k) table[k] = (int32_t)((uint32_t)t[k] + (uint32_t)base);
    return ret;
}

int32_t lz4mi_xxh32_blocks(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                           uint32_t* hashes, uint32_t nblocks, uint32_t flags, void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    const int stdv = (flags & LZ4MI_XXH_STANDARD) ? 1 : 0;
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        LZ4MI_TRY(lz4mi_launch_xxh32(in, off, len, seed, hashes, nblocks, stdv, pick_stream(stream)));
        return LZ4MI_OK;
    }
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    std::vector<uint64_t> d_off(nblocks);
    uint64_t pos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) { d_off[b] = pos; pos += (len[b] + 15u) & ~15ull; }
    LZ4MI_TRY(g_ctx.in.ensure(pos + 64));
    LZ4MI_TRY(g_ctx.meta.ensure((size_t)nblocks * 16 + 64));
    uint64_t* m_off = g_ctx.meta.as<uint64_t>();
    uint32_t* m_len = (uint32_t*)(m_off + nblocks);
    uint32_t* m_h = m_len + nblocks;
    for (uint32_t b = 0; b < nblocks; ++b)
        LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.as<uint8_t>() + d_off[b], in + off[b], len[b], hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_off, d_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_len, len, 4ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(lz4mi_launch_xxh32(g_ctx.in.as<uint8_t>(), m_off, m_len, seed, m_h, nblocks, stdv, s));
    LZ4MI_TRY(hipMemcpyAsync(hashes, m_h, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    return LZ4MI_OK;
}

int32_t lz4mi_frame_pack(const uint8_t* raw, const uint64_t* raw_off, const uint32_t* raw_len, const uint8_t* comp,
                         const uint64_t* comp_off, const uint32_t* comp_len, uint8_t* frame, const uint64_t* rec_off,
                         uint32_t nblocks, uint32_t flags, void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    if (!(flags & LZ4MI_DEVICE_PTRS)) return LZ4MI_ERR_ARG;
    LZ4MI_TRY(lz4mi_launch_frame_pack(raw, raw_off, raw_len, comp, comp_off, comp_len, frame, rec_off, nblocks,
                                      pick_stream(stream)));
    return LZ4MI_OK;
}

int32_t lz4mi_generate_blocks(uint8_t* out, uint32_t kind, uint32_t seed0, uint32_t block_size, uint32_t nblocks,
                              void* stream) {
    int32_t st = ensure_init();
    if (st) return st;
    if (kind > 2) return LZ4MI_ERR_ARG;
    LZ4MI_TRY(lz4mi_launch_generate(out, kind, seed0, block_size, nblocks, pick_stream(stream)));
    return LZ4MI_OK;
}

}  // extern "C"
