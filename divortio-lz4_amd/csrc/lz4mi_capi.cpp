// lz4mi_capi.cpp — host side of liblz4mi.so: the C-ABI declared in
// include/lz4mi.h. Owns the per-device context (stream, grow-only device
// scratch), stages host buffers for the synchronous entry points and launches
// the gfx950 kernels. No CPU fallback: without a gfx950 device every entry
// point that needs the GPU returns LZ4MI_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/lz4mi.h"

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                              const uint64_t*, const uint32_t*, const uint8_t*, uint32_t, uint32_t*,
                                              int32_t*, uint32_t, int, hipStream_t);
extern "C" hipError_t lz4mi_launch_decompress_pending(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                                      const uint64_t*, const uint32_t*, const uint8_t*, uint32_t,
                                                      uint32_t*, int32_t*, uint32_t, const uint64_t*, const uint32_t*,
                                                      hipStream_t);
extern "C" hipError_t lz4mi_launch_token_map(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*,
                                             uint32_t, const uint32_t*, uint64_t*, uint32_t, uint32_t, hipStream_t);
extern "C" hipError_t lz4mi_launch_ring_decode(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                               const uint64_t*, const uint32_t*, uint32_t*, int32_t*, const uint32_t*,
                                               const uint64_t*, uint32_t, uint32_t*, uint32_t, hipStream_t);
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
    // two-pass decoder: per-block chunk index, token bitmaps (128 B per 1 KiB chunk), counters
    Scratch chunk_base, bitmap, stats;
    std::vector<uint32_t> h_len, h_base;
    uint32_t* h_pin = nullptr;   // pinned staging for the block lengths of device-pointer calls
    size_t h_pin_cap = 0;
    hipEvent_t ring_done = nullptr;   // the two-pass scratch is free once this has fired
    std::mutex mu, ring_mu;
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

constexpr uint32_t kRingChunk = 1024;   // lz4mi_decompress_ring.hip kC

// Decoder selection (LZ4MI_DECODER): "auto" (default) = the two-pass ring decoder for
// blocks compressed at least kRingRatio:1 (long matches: it writes them from LDS), the
// single-pass kernel for the rest; "ring" = every block through the ring decoder;
// "single" = the single-pass kernel only.
constexpr uint32_t kRingRatio = 32;
int g_ring_mode = -1;
uint32_t g_ring_ratio = kRingRatio;
bool ring_enabled() {
    if (g_ring_mode < 0) {
        const char* e = std::getenv("LZ4MI_DECODER");
        g_ring_mode = (e && std::strcmp(e, "single") == 0) ? 0 : 1;
        g_ring_ratio = (e && std::strcmp(e, "ring") == 0) ? 0u : kRingRatio;
    }
    return g_ring_mode == 1;
}

// Spec-mode decode of a batch whose pointers are all device pointers: the
// two-pass ring decoder, then the single-pass kernel for the blocks it hands
// back. h_in_len: the block lengths if the caller has them on the host (else
// they are read back from the device, one small synchronous copy).
hipError_t ring_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* h_in_len,
                       uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict,
                       uint32_t dict_len, uint32_t* out_len, int32_t* status, uint32_t nblocks, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_ctx.ring_mu);
    hipError_t e;
    if (!g_ctx.ring_done) {
        if ((e = hipEventCreateWithFlags(&g_ctx.ring_done, hipEventDisableTiming)) != hipSuccess) return e;
    } else if ((e = hipStreamWaitEvent(s, g_ctx.ring_done, 0)) != hipSuccess) {
        return e;
    }
    const uint32_t* lens = h_in_len;
    if (!lens) {
        if (g_ctx.h_pin_cap < nblocks) {
            if (g_ctx.h_pin) (void)hipHostFree(g_ctx.h_pin);
            g_ctx.h_pin = nullptr;
            g_ctx.h_pin_cap = 0;
            if ((e = hipHostMalloc((void**)&g_ctx.h_pin, 4ull * nblocks, 0)) != hipSuccess) return e;
            g_ctx.h_pin_cap = nblocks;
        }
        if ((e = hipMemcpyAsync(g_ctx.h_pin, in_len, 4ull * nblocks, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        lens = g_ctx.h_pin;
    }
    g_ctx.h_base.resize(nblocks);
    uint64_t total = 0;
    uint32_t maxc = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        const uint32_t c = (lens[b] + kRingChunk - 1) / kRingChunk;
        g_ctx.h_base[b] = (uint32_t)total;
        total += c;
        maxc = std::max(maxc, c);
    }
    if (total >= 0xFFFFFFFFull) return hipErrorInvalidValue;
    if ((e = g_ctx.chunk_base.ensure(4ull * nblocks + 64)) != hipSuccess) return e;
    if ((e = g_ctx.bitmap.ensure(128ull * total + 64)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(g_ctx.chunk_base.p, g_ctx.h_base.data(), 4ull * nblocks, hipMemcpyHostToDevice, s)) !=
        hipSuccess)
        return e;
    uint32_t* stats = nullptr;
    if (std::getenv("LZ4MI_RING_STATS")) {
        if (!g_ctx.stats.p) {
            if ((e = g_ctx.stats.ensure(64)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(g_ctx.stats.p, 0, 64, s)) != hipSuccess) return e;
        }
        stats = g_ctx.stats.as<uint32_t>();
    }
    // LZ4MI_BITMAP=1: pass 1 maps every block and the single-pass kernel takes its token starts from it
    static const bool bm_mode = std::getenv("LZ4MI_BITMAP") && std::getenv("LZ4MI_BITMAP")[0] == '1';
    if ((e = lz4mi_launch_token_map(in, in_off, in_len, out_cap, bm_mode ? 0u : g_ring_ratio, g_ctx.chunk_base.as<uint32_t>(),
                                    g_ctx.bitmap.as<uint64_t>(), nblocks, maxc, s)) != hipSuccess)
        return e;
    if ((e = lz4mi_launch_ring_decode(in, in_off, in_len, out, out_off, out_cap, out_len, status,
                                      g_ctx.chunk_base.as<uint32_t>(), g_ctx.bitmap.as<uint64_t>(), g_ring_ratio, stats,
                                      nblocks, s)) != hipSuccess)
        return e;
    if ((e = lz4mi_launch_decompress_pending(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len,
                                             status, nblocks, bm_mode ? g_ctx.bitmap.as<uint64_t>() : nullptr,
                                             g_ctx.chunk_base.as<uint32_t>(), s)) != hipSuccess)
        return e;
    return hipEventRecord(g_ctx.ring_done, s);
}

hipError_t decode_launch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* h_in_len,
                         uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict,
                         uint32_t dict_len, uint32_t* out_len, int32_t* status, uint32_t nblocks, int mode,
                         hipStream_t s) {
    if (mode == 0 && ring_enabled())
        return ring_decode(in, in_off, in_len, h_in_len, out, out_off, out_cap, dict, dict_len, out_len, status,
                           nblocks, s);
    return lz4mi_launch_decompress(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status,
                                   nblocks, mode, s);
}

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

// Debug counters of the two-pass decoder (enabled by LZ4MI_RING_STATS=1):
// [0] chunks whose token bitmap was rebuilt, [1] sequences written directly,
// [2] blocks handed to the single-pass kernel. Reads and resets.
// [3..5] why blocks were handed back: malformed token, sequence error, direct-sequence error.
int32_t lz4mi_debug_ring_stats(uint32_t* out6) {
    for (int i = 0; i < 6; ++i) out6[i] = 0;
    if (!g_ctx.stats.p) return LZ4MI_OK;
    if (hipDeviceSynchronize() != hipSuccess) return LZ4MI_ERR_HIP;
    if (hipMemcpy(out6, g_ctx.stats.p, 24, hipMemcpyDeviceToHost) != hipSuccess) return LZ4MI_ERR_HIP;
    if (hipMemset(g_ctx.stats.p, 0, 24) != hipSuccess) return LZ4MI_ERR_HIP;
    return LZ4MI_OK;
}

// Decoder selection for tests / tools: mode 0 single-pass only, 1 ring decoder for blocks
// compressed at least `ratio`:1 (0: every block). Overrides LZ4MI_DECODER.
int32_t lz4mi_debug_set_decoder(int32_t mode, uint32_t ratio) {
    g_ring_mode = mode ? 1 : 0;
    g_ring_ratio = ratio;
    return LZ4MI_OK;
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
        LZ4MI_TRY(decode_launch(in, in_off, in_len, nullptr, out, out_off, out_cap, dict, dict_len, out_len, status,
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
    LZ4MI_TRY(decode_launch(g_ctx.in.as<uint8_t>(), m_in_off, m_in_len, in_len, g_ctx.out.as<uint8_t>(), m_out_off,
                            m_out_cap, dlen ? g_ctx.aux.as<uint8_t>() : nullptr, dlen, m_out_len, m_status, nblocks,
                            mode, s));
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
