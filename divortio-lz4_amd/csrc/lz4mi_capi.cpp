// lz4mi_capi.cpp — host side of liblz4mi.so: the C-ABI declared in
// include/lz4mi.h. Owns the per-device context (library stream, staging buffers
// of the synchronous host-pointer entry points) and one scratch set per HIP
// stream for the asynchronous device-pointer entry points, and launches the
// gfx950 kernels. No CPU fallback: without a gfx950 device every entry point
// that needs the GPU returns LZ4MI_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <memory>
#include <atomic>
#include <mutex>
#include <vector>

#include <sys/mman.h>

#include "../../include/lz4mi.h"
#include "lz4mi_decompress.h"

#ifndef LZ4MI_SRC_HASH
#define LZ4MI_SRC_HASH "unknown"
#endif

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                              const uint64_t*, const uint32_t*, const uint8_t*, uint32_t, uint32_t*,
                                              int32_t*, uint32_t, int, uint32_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_decompress_small(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                                    const uint64_t*, const uint32_t*, const uint8_t*, uint32_t,
                                                    uint32_t*, int32_t*, uint32_t, uint32_t, uint32_t, void*, int,
                                                    int, hipStream_t);
extern "C" size_t lz4mi_small_scratch_bytes(uint32_t, uint32_t, uint32_t);
extern "C" hipError_t lz4mi_launch_compress(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                            const uint64_t*, uint32_t*, uint32_t, int32_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_frame_pack(const uint8_t*, const uint64_t*, const uint32_t*, const uint8_t*,
                                              const uint64_t*, const uint32_t*, uint8_t*, const uint64_t*, uint32_t,
                                              uint64_t*, uint64_t*, uint32_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_compress_chain(const uint8_t*, uint64_t, int32_t, int32_t, int32_t, int32_t*,
                                                  uint8_t*, const uint64_t*, uint32_t*, uint32_t, hipStream_t);
extern "C" hipError_t lz4mi_launch_xxh32(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint32_t*,
                                         uint32_t, int, uint8_t*, const uint64_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_generate(uint8_t*, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);
extern "C" hipError_t lz4mi_launch_frame_scan(const uint8_t*, uint64_t, uint32_t, uint64_t*, uint32_t*, uint64_t*,
                                              uint32_t*, uint64_t*, uint32_t*, uint64_t*, uint32_t*, uint32_t*,
                                              int64_t*, hipStream_t);
extern "C" hipError_t lz4mi_launch_frame_index(const uint8_t*, uint64_t, uint32_t, uint64_t*, uint32_t*, int64_t*,
                                               hipStream_t);
extern "C" hipError_t lz4mi_launch_frame_stored(const uint8_t*, uint64_t, const uint64_t*, const uint32_t*,
                                                const uint64_t*, uint8_t*, uint64_t, uint32_t, hipStream_t);

namespace {

// Grow-only device buffer. Work using the old buffer may still be queued on
// `s` (the only stream that uses it), so the old one is freed stream-ordered.
struct Scratch {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n, hipStream_t s) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFreeAsync(p, s);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n + n / 4, 1 << 20);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Scratch of the work enqueued on one stream: kernels on one stream run in
// order, so the device never sees two users of it at once; different streams
// never share. Host threads can still call in on the same stream (the NULL
// stream is torch's default), so `mu` is held from the first ensure() of a call
// until its last launch that uses the scratch: a concurrent grow cannot free a
// buffer another thread has read but not yet enqueued.
struct StreamCtx {
    hipStream_t stream = nullptr;
    std::mutex mu;
    Scratch tables;       // batch encoder hash tables (64 KiB per block)
    Scratch frame_meta;   // block-checksum payload offsets / lengths of frame_pack
    Scratch scan;         // frame_decompress: block lists of the device frame walk
    Scratch order;        // batch decode: the blocks' dispatch order (lz4mi_block_order_kernel)
    Scratch small;        // small-batch decode: exported sequences and output pointers (lz4mi_expand.hip)
    void release() {
        tables.release();
        frame_meta.release();
        scan.release();
        order.release();
        small.release();
    }
};

struct Ctx {
    std::atomic<int> device{-1};   // set once by init_locked, never changed after
    hipStream_t stream = nullptr;
    Scratch in, out, meta, aux, order, small;   // staging of the synchronous host-pointer entry points
    std::mutex mu;                // serialises the host-pointer entry points (their staging is shared)
    std::mutex streams_mu;
    std::vector<std::unique_ptr<StreamCtx>> streams;
    Scratch stats;
};

Ctx g_ctx;
std::mutex g_init_mu;

#define LZ4MI_TRY(expr)                           \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return LZ4MI_ERR_HIP; \
    } while (0)

// Every entry point runs on the library's device and leaves the calling thread's
// current device as it found it (HIP's current device is per host thread, and
// torch allocates on it).
class DeviceGuard {
  public:
    DeviceGuard() {
        if (g_ctx.device < 0) {
            status_ = lz4mi_init(-1);
            if (status_) return;
        }
        if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
        if (prev_ != g_ctx.device && hipSetDevice(g_ctx.device) != hipSuccess) status_ = LZ4MI_ERR_HIP;
    }
    ~DeviceGuard() {
        if (prev_ >= 0 && prev_ != g_ctx.device) (void)hipSetDevice(prev_);
    }
    int32_t status() const { return status_; }

  private:
    int prev_ = -1;
    int32_t status_ = LZ4MI_OK;
};

// Device-pointer calls run on the caller's stream; NULL is HIP's default stream (what
// torch reports for its default stream), so work is ordered with the caller's kernels.
hipStream_t pick_stream(void* s) { return static_cast<hipStream_t>(s); }

StreamCtx* stream_ctx(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_ctx.streams_mu);
    for (auto& c : g_ctx.streams)
        if (c->stream == s) return c.get();
    g_ctx.streams.emplace_back(new StreamCtx());
    g_ctx.streams.back()->stream = s;
    return g_ctx.streams.back().get();
}

// Small batches (at most this many blocks, LZ4 spec or reference mode) decode with a wave per
// ~8 KiB of each compressed block (a segment-parallel parse) and the output by pointer jumping
// over the whole GPU (lz4mi_expand.hip) instead of one wave per block: a lone 4 MiB tiles216
// block 0.21 ms instead of 7.9. The batch kernel is a flat 8.4 ms up to 4096 tiles216 blocks; the small path grows
// ~0.03 ms per block (192 blocks: 5.7 ms, 256: 7.8, 320: 9.2; the 50/50 mix 6.3 / 8.4 / 10.4 against 8.3; text
// 192 blocks 18 ms against 153, profiles/r06k2), so the default is 192 blocks. Blocks
// of long runs (ratio >= 32) are decoded by one wave in the same launch. LZ4MI_SMALL_BLOCKS=0
// turns the path off.
// Scratch (lz4mi_small_scratch_bytes): ~16 B per potential sequence of the largest compressed
// block plus 4 B per output byte of the largest output, per block of the batch. Host-pointer calls
// size it from the batch's real maxima (rounded up to 64 KiB, the output's to a power of two); device-pointer calls cannot read
// in_len/out_cap without a sync, so they size it for the largest block the path exports (a 4 MiB
// block: ~47 MB per block). Either way the total is capped (LZ4MI_SMALL_SCRATCH_MB, default 9216 =
// 192 worst-case blocks): a batch above the cap goes to the batch kernel. A block larger than the
// sizing is decoded by one wave inside the same launch (the kernel's export limits).
constexpr uint32_t kSmallInMax = (4u << 20) + (4u << 20) / 255 + 16;   // a 4 MiB block's compress bound
constexpr uint32_t kSmallOutMax = 4u << 20;
uint32_t small_blocks() {
    static const uint32_t n = [] {
        const char* e = std::getenv("LZ4MI_SMALL_BLOCKS");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 192u;
    }();
    return n;
}
size_t small_scratch_cap() {
    static const size_t n = [] {
        const char* e = std::getenv("LZ4MI_SMALL_SCRATCH_MB");
        return (e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)9216) << 20;
    }();
    return n;
}
int small_reparse_hook() {   // (test hook, read per call: LZ4MI_SMALL_REPARSE forces re-parses, tests/test_gpu_small.py)
    const char* e = std::getenv("LZ4MI_SMALL_REPARSE");
    return e ? std::atoi(e) : 0;
}

// `order`: scratch of nblocks words for the dispatch order, owned by the caller's lock
// (nullptr: the blocks go in index order); `small`: the small-batch path's scratch (nullptr:
// never taken); in_max / out_max: the batch's largest compressed block and output capacity when
// the caller knows them (host pointers), 0 = unknown (device pointers: the path's limits)
}  // namespace

// Output memory of the host-pointer entry points is usually fresh (a new Uint8Array from the JS
// layer): every 4 KiB page faults on its first write, inside the D2H copy. A 16 MiB copy into fresh
// 4 KiB pages takes 1.79 ms, into 2 MiB pages 0.31 ms, and registering or staging through pinned
// memory does not help (tools/d2h_options.py, profiles/r05_hostio). The 2 MiB-aligned interior of
// an output range of at least 4 MiB is advised for transparent huge pages: a hint on the caller's
// mapping, no change to its contents. LZ4MI_THP=0 leaves the caller's memory alone.
extern "C" __attribute__((visibility("hidden"))) void lz4mi_advise_output(void* p, uint64_t n) {
    constexpr uintptr_t kHuge = 2u << 20;
    const char* e = std::getenv("LZ4MI_THP");
    if ((e && e[0] == '0') || !p || n < 2 * kHuge) return;
    const uintptr_t a0 = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1), a1 = ((uintptr_t)p + n) & ~(kHuge - 1);
    if (a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
}

namespace {

hipError_t decode_launch(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                         const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict, uint32_t dict_len,
                         uint32_t* out_len, int32_t* status, uint32_t nblocks, int mode, hipStream_t s,
                         Scratch* order, Scratch* small = nullptr, uint32_t in_max = 0, uint32_t out_max = 0) {
    if (small && (mode == 0 || mode == 2) && nblocks <= small_blocks()) {
        // (the output limit is a power of two: lz4mi_launch_expand tiles it)
        constexpr uint32_t kGrain = 64u << 10;
        const uint32_t xi = in_max ? std::min(kSmallInMax, (in_max + kGrain - 1) / kGrain * kGrain) : kSmallInMax;
        uint32_t xo = kGrain;
        while (xo < out_max && xo < kSmallOutMax) xo <<= 1;
        if (!out_max) xo = kSmallOutMax;
        const size_t need = lz4mi_small_scratch_bytes(nblocks, xi, xo);
        if (need <= small_scratch_cap()) {
            // (test hook, read per call: LZ4MI_TEST_SCRATCH_EXTRA_MB asks for that much more, so that the
            // allocation really fails -- tests/test_gpu_small.py::test_small_batch_scratch_allocation_failure)
            const char* xe = std::getenv("LZ4MI_TEST_SCRATCH_EXTRA_MB");
            const size_t extra = xe ? (size_t)std::strtoull(xe, nullptr, 10) << 20 : 0;
            if (small->ensure(need + extra, s) == hipSuccess)
                return lz4mi_launch_decompress_small(in, in_off, in_len, out, out_off, out_cap, dict, dict_len,
                                                     out_len, status, nblocks, xi, xo, small->p, small_reparse_hook(),
                                                     mode == 2 ? 1 : 0, s);
            (void)hipGetLastError();   // the failed allocation is not this call's error: the batch kernel runs
        }
    }
    uint32_t* ord = nullptr;
    if (order && nblocks > 1) {
        if (order->ensure((size_t)nblocks * 4, s) == hipSuccess) ord = order->as<uint32_t>();
        else (void)hipGetLastError();   // index order instead
    }
    return lz4mi_launch_decompress(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status,
                                   nblocks, mode, ord, s);
}

inline uint64_t round16(uint64_t n) { return (n + 15u) & ~15ull; }

// ---- host XXH32 (reference variant by default, see lz4mi_xxh32.hip) -------
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t le32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

inline uint32_t converge(const uint32_t v[4], uint32_t flags) {
    if (flags & LZ4MI_XXH_STANDARD) return rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
    return rotl(rotl(rotl(rotl(v[0], 1) + v[1], 7) + v[2], 12) + v[3], 18);   // xxhash32.js:59-65
}

inline uint32_t tail_mix(uint32_t h, const uint8_t* p, size_t n) {
    size_t k = 0;
    for (; k + 4 <= n; k += 4) h = rotl(h + le32(p + k) * P3, 17) * P4;
    for (; k < n; ++k) h = rotl(h + p[k] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

inline void stripes(uint32_t v[4], const uint8_t* p, size_t n16) {
    uint32_t a = v[0], b = v[1], c = v[2], d = v[3];
    for (size_t k = 0; k < n16; ++k, p += 16) {
        a = rotl(a + le32(p) * P2, 13) * P1;
        b = rotl(b + le32(p + 4) * P2, 13) * P1;
        c = rotl(c + le32(p + 8) * P2, 13) * P1;
        d = rotl(d + le32(p + 12) * P2, 13) * P1;
    }
    v[0] = a; v[1] = b; v[2] = c; v[3] = d;
}

// Streaming state (include/lz4mi.h lz4mi_xxh32_state): v[4], seed, mem_size,
// total (u64), mem[16], flags.
struct XxhState {
    uint32_t v[4];
    uint32_t seed;
    uint32_t mem_size;
    uint64_t total;
    uint8_t mem[16];
    uint32_t flags;
    uint32_t pad;
};
static_assert(sizeof(XxhState) == sizeof(lz4mi_xxh32_state), "lz4mi_xxh32_state layout");

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
        case LZ4MI_ERR_RANGE: return "Source is too large";
        case LZ4MI_ERR_CROSS_BLOCK: return "lz4mi: block references data before its start (not an independent block)";
        case LZ4MI_ERR_BLOCK_CHECKSUM: return "LZ4: Block Checksum Error";
        case LZ4MI_ERR_HIP: return "lz4mi: HIP runtime error";
        case LZ4MI_ERR_ARG: return "lz4mi: invalid argument";
        case LZ4MI_ERR_NO_DEVICE: return "lz4mi: no gfx950 (MI355X) device available";
        case LZ4MI_ERR_DEVICE_BOUND: return "lz4mi: library already bound to another device (one device per process)";
        default: return "lz4mi: unknown status";
    }
}

const char* lz4mi_version(void) { return "lz4mi 0.2 (gfx950) src " LZ4MI_SRC_HASH; }

const char* lz4mi_build_id(void) { return LZ4MI_SRC_HASH; }

int32_t lz4mi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int32_t init_locked(int32_t device);

// Selects (and on first use sets up) the library's device; the calling thread's
// current device is restored before returning.
int32_t lz4mi_init(int32_t device) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    const int32_t st = init_locked(device);
    if (prev >= 0) (void)hipSetDevice(prev);
    return st;
}

static int32_t init_locked(int32_t device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return LZ4MI_ERR_NO_DEVICE;
    if (device < 0) {
        if (g_ctx.device >= 0) return LZ4MI_OK;
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= n) return LZ4MI_ERR_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return LZ4MI_ERR_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LZ4MI_ERR_NO_DEVICE;
    if (g_ctx.device == device) return LZ4MI_OK;
    // the context is bound to one device for the life of the process: another thread may
    // hold a StreamCtx* (and its lock) of this device, so nothing of it is ever released
    if (g_ctx.device >= 0) return LZ4MI_ERR_DEVICE_BOUND;
    LZ4MI_TRY(hipSetDevice(device));
    LZ4MI_TRY(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking));
    g_ctx.device = device;
    return LZ4MI_OK;
}

uint32_t lz4mi_xxh32(const uint8_t* in, size_t len, uint32_t seed, uint32_t flags) {
    uint32_t h;
    const size_t n16 = len / 16;
    if (len >= 16) {
        uint32_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        stripes(v, in, n16);
        h = converge(v, flags);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    const size_t p = len >= 16 ? n16 * 16 : 0;
    return tail_mix(h, in + p, len - p);
}

void lz4mi_xxh32_reset(lz4mi_xxh32_state* st, uint32_t seed, uint32_t flags) {
    XxhState* s = reinterpret_cast<XxhState*>(st);
    std::memset(s, 0, sizeof *s);
    s->v[0] = seed + P1 + P2;
    s->v[1] = seed + P2;
    s->v[2] = seed;
    s->v[3] = seed - P1;
    s->seed = seed;
    s->flags = flags;
}

void lz4mi_xxh32_update(lz4mi_xxh32_state* st, const uint8_t* in, size_t len) {
    XxhState* s = reinterpret_cast<XxhState*>(st);
    s->total += len;
    if (s->mem_size + len < 16) {                       // xxhash32Stateful.js:40-44
        if (len) std::memcpy(s->mem + s->mem_size, in, len);
        s->mem_size += (uint32_t)len;
        return;
    }
    size_t p = 0;
    if (s->mem_size > 0) {                              // :46-54
        p = 16 - s->mem_size;
        std::memcpy(s->mem + s->mem_size, in, p);
        stripes(s->v, s->mem, 1);
        s->mem_size = 0;
    }
    const size_t n16 = (len - p) / 16;                  // :57-61
    stripes(s->v, in + p, n16);
    p += n16 * 16;
    if (p < len) {                                      // :64-67
        std::memcpy(s->mem, in + p, len - p);
        s->mem_size = (uint32_t)(len - p);
    }
}

uint32_t lz4mi_xxh32_digest(const lz4mi_xxh32_state* st) {
    const XxhState* s = reinterpret_cast<const XxhState*>(st);
    // the class keeps totalLen as `(totalLen + len) | 0` (:37) and tests it signed (:113);
    // LZ4MI_XXH_LEN64 keeps the full length (streams over 2 GiB)
    const bool big = (s->flags & LZ4MI_XXH_LEN64) ? s->total >= 16 : (int32_t)(uint32_t)s->total >= 16;
    uint32_t h = big ? converge(s->v, s->flags) : s->seed + P5;
    h += (uint32_t)s->total;
    return tail_mix(h, s->mem, s->mem_size);
}

int32_t lz4mi_decompress_blocks(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict,
                                uint32_t dict_len, uint32_t* out_len, int32_t* status, uint32_t nblocks,
                                uint32_t flags, void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    const int js = (flags & LZ4MI_JS_COMPAT) ? 1 : 0;
    int mode = js ? 1 : ((flags & LZ4MI_JS_EXACT) ? 2 : 0);
    if (flags & LZ4MI_FRAME_WORDS) {   // frame size words (stored bit): the batch kernel, device pointers
        if (js || !(flags & LZ4MI_DEVICE_PTRS)) return LZ4MI_ERR_ARG;
        mode |= 4;
    }
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        // the order scratch belongs to the stream: kernels of one stream use it in order
        hipStream_t s = pick_stream(stream);
        StreamCtx* c = stream_ctx(s);
        std::lock_guard<std::mutex> sl(c->mu);
        LZ4MI_TRY(decode_launch(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                                mode, s, &c->order, &c->small));
        return LZ4MI_OK;
    }
    if (!in || !out || !in_off || !in_len || !out_off || !out_cap || !out_len || !status) return LZ4MI_ERR_ARG;
    for (uint32_t b = 0; b < nblocks; ++b)
        if (in_len[b] > LZ4MI_MAX_BLOCK || out_cap[b] > LZ4MI_MAX_BLOCK) return LZ4MI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    // Pack the compressed blocks; stage the output image [lo - hist, hi) so
    // back-references into bytes preceding a block (reference semantics:
    // positions are absolute in `out`) see the caller's bytes.
    uint64_t in_total = 0, lo = UINT64_MAX, hi = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        in_total += round16(in_len[b]);
        lo = std::min<uint64_t>(lo, out_off[b]);
        hi = std::max<uint64_t>(hi, out_off[b] + out_cap[b]);
    }
    uint64_t hist = std::min<uint64_t>(lo, 65536);
    uint64_t base = lo - hist, img = hi - base;
    lz4mi_advise_output(out + lo, hi - lo);
    std::vector<uint64_t> d_in_off(nblocks), d_out_off(nblocks);
    uint64_t pos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        d_in_off[b] = pos;
        pos += round16(in_len[b]);
        d_out_off[b] = out_off[b] - base;
    }
    // Dictionary bytes are only reachable when the image starts at out[0].
    uint32_t dlen = (base == 0 && dict) ? dict_len : 0;
    LZ4MI_TRY(g_ctx.in.ensure(in_total + 64, s));
    LZ4MI_TRY(g_ctx.out.ensure(img + 64, s));
    LZ4MI_TRY(g_ctx.aux.ensure((size_t)dlen + 64, s));
    const size_t meta_bytes = (size_t)nblocks * (8 + 4 + 8 + 4 + 4 + 4);
    LZ4MI_TRY(g_ctx.meta.ensure(meta_bytes + 64, s));
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
    const uint32_t in_max = *std::max_element(in_len, in_len + nblocks);
    const uint32_t out_max = *std::max_element(out_cap, out_cap + nblocks);
    LZ4MI_TRY(decode_launch(g_ctx.in.as<uint8_t>(), m_in_off, m_in_len, g_ctx.out.as<uint8_t>(), m_out_off, m_out_cap,
                            dlen ? g_ctx.aux.as<uint8_t>() : nullptr, dlen, m_out_len, m_status, nblocks, mode, s,
                            &g_ctx.order, &g_ctx.small, std::max(in_max, 1u), std::max(out_max, 1u)));
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
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        // the hash-table scratch belongs to the stream: kernels of one stream use it in order
        hipStream_t s = pick_stream(stream);
        StreamCtx* c = stream_ctx(s);
        std::lock_guard<std::mutex> sl(c->mu);
        LZ4MI_TRY(c->tables.ensure((size_t)nblocks * 16384 * sizeof(int32_t), s));
        LZ4MI_TRY(lz4mi_launch_compress(in, in_off, in_len, out, out_off, out_len, nblocks, c->tables.as<int32_t>(), s));
        return LZ4MI_OK;
    }
    if (!in || !out || !in_off || !in_len || !out_off || !out_len) return LZ4MI_ERR_ARG;
    for (uint32_t b = 0; b < nblocks; ++b)
        if (in_len[b] > LZ4MI_MAX_BLOCK) return LZ4MI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    std::vector<uint64_t> d_in_off(nblocks), d_out_off(nblocks);
    uint64_t ipos = 0, opos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) {
        d_in_off[b] = ipos;
        ipos += round16(in_len[b]);
        d_out_off[b] = opos;
        opos += round16(lz4mi_compress_bound(in_len[b]));
    }
    LZ4MI_TRY(g_ctx.in.ensure(ipos + 64, s));
    LZ4MI_TRY(g_ctx.out.ensure(opos + 64, s));
    LZ4MI_TRY(g_ctx.meta.ensure((size_t)nblocks * 24 + 64, s));
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
    StreamCtx* c = stream_ctx(s);
    std::unique_lock<std::mutex> sl(c->mu);
    LZ4MI_TRY(c->tables.ensure((size_t)nblocks * 16384 * sizeof(int32_t), s));
    LZ4MI_TRY(lz4mi_launch_compress(g_ctx.in.as<uint8_t>(), m_in_off, m_in_len, g_ctx.out.as<uint8_t>(), m_out_off,
                                    m_out_len, nblocks, c->tables.as<int32_t>(), s));
    LZ4MI_TRY(hipMemcpyAsync(out_len, m_out_len, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    uint64_t olo = UINT64_MAX, ohi = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
        if (out_len[b]) {
            olo = std::min<uint64_t>(olo, out_off[b]);
            ohi = std::max<uint64_t>(ohi, out_off[b] + out_len[b]);
        }
    if (ohi > olo) lz4mi_advise_output(out + olo, ohi - olo);
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
    if (src_start < 0 || src_len < 0 || (uint64_t)src_start + (uint64_t)src_len > src_total || !table || out_off < 0 ||
        (uint64_t)src_start + (uint64_t)src_len > INT32_MAX)   // int32 positions (table values position + 1)
        return LZ4MI_ERR_ARG;
    if (flags & LZ4MI_DEVICE_PTRS) return LZ4MI_ERR_ARG;   // host-only entry point (see header)
    {
        DeviceGuard dg;   // no device: the call fails like every other block call
        if (dg.status()) return dg.status();
    }
    // Room for the worst case: the GPU chain kernel (the dependent-frame kernel with one
    // block: the caller's table in LDS). Otherwise the reference's output.set() may throw
    // mid-block (blockCompress.js:100, :198) with the bytes and table entries written up to
    // that point kept, and writes past the buffer vanish: the host encoder, which follows
    // the reference store by store.
    const uint64_t room = out_total > (uint64_t)out_off ? out_total - (uint64_t)out_off : 0;
    if (src_len == 0 || room < lz4mi_compress_bound((uint64_t)src_len))
        return lz4mi_host_compress_block(src, src_total, src_start, src_len, table, out, out_total, out_off);
    const uint64_t off0 = (uint64_t)out_off;
    uint32_t clen = 0;
    const int32_t st = lz4mi_compress_chain(src, src_total, src_start, src_len, src_len, table, out, &off0, &clen, 0,
                                            stream);
    if (st) return st;
    return (int64_t)clen;
}

int32_t lz4mi_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len, int32_t block_size,
                             int32_t* table, uint8_t* out, const uint64_t* out_off, uint32_t* comp_len, uint32_t flags,
                             void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (flags & LZ4MI_DEVICE_PTRS) return LZ4MI_ERR_ARG;   // host-only entry point (see header)
    if (!src || !table || !out || !out_off || !comp_len || start < 0 || len < 0 || block_size <= 0 ||
        (uint64_t)start + (uint64_t)len > src_total || block_size > (int32_t)LZ4MI_MAX_BLOCK)
        return LZ4MI_ERR_ARG;
    const uint32_t nb = (uint32_t)(((int64_t)len + block_size - 1) / block_size);
    if (nb == 0) return LZ4MI_OK;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    (void)stream;
    // the chain reaches at most 65535 bytes before `start`: stage src[base, start + len) and
    // shift the table's positions by base (int32 wrap keeps the entries exact, as in
    // lz4mi_compress_block_table)
    const int64_t base = std::max<int64_t>(0, (int64_t)start - 65536);
    const uint64_t sbytes = (uint64_t)start + len - base;
    std::vector<uint64_t> d_off(nb);
    uint64_t opos = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t n = std::min<uint64_t>(block_size, (uint64_t)len - (uint64_t)b * block_size);
        d_off[b] = opos;
        opos += round16(lz4mi_compress_bound(n));
    }
    LZ4MI_TRY(g_ctx.in.ensure(sbytes + 64, s));
    LZ4MI_TRY(g_ctx.out.ensure(opos + 64, s));
    LZ4MI_TRY(g_ctx.meta.ensure(16384 * 4 + (size_t)nb * 12 + 64, s));
    std::vector<int32_t> t(16384);
    for (int k = 0; k < 16384; ++k) t[k] = (int32_t)((uint32_t)table[k] - (uint32_t)base);
    int32_t* d_table = g_ctx.meta.as<int32_t>();
    uint64_t* m_off = (uint64_t*)(d_table + 16384);
    uint32_t* m_len = (uint32_t*)(m_off + nb);
    LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.p, src + base, sbytes, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(d_table, t.data(), 16384 * 4, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_off, d_off.data(), 8ull * nb, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(lz4mi_launch_compress_chain(g_ctx.in.as<uint8_t>(), sbytes, (int32_t)(start - base), len, block_size,
                                          d_table, g_ctx.out.as<uint8_t>(), m_off, m_len, nb, s));
    LZ4MI_TRY(hipMemcpyAsync(comp_len, m_len, 4ull * nb, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipMemcpyAsync(t.data(), d_table, 16384 * 4, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    for (uint32_t b = 0; b < nb; ++b)
        if (comp_len[b])
            LZ4MI_TRY(hipMemcpyAsync(out + out_off[b], g_ctx.out.as<uint8_t>() + d_off[b], comp_len[b],
                                     hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    for (int k = 0; k < 16384; ++k) table[k] = (int32_t)((uint32_t)t[k] + (uint32_t)base);
    return LZ4MI_OK;
}

int32_t lz4mi_xxh32_blocks(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                           uint32_t* hashes, uint32_t nblocks, uint32_t flags, void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    const int stdv = (flags & LZ4MI_XXH_STANDARD) ? 1 : 0;
    if (nblocks == 0) return LZ4MI_OK;
    if (flags & LZ4MI_DEVICE_PTRS) {
        LZ4MI_TRY(lz4mi_launch_xxh32(in, off, len, seed, hashes, nblocks, stdv, nullptr, nullptr, pick_stream(stream)));
        return LZ4MI_OK;
    }
    if (!in || !off || !len || !hashes) return LZ4MI_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    hipStream_t s = g_ctx.stream;
    std::vector<uint64_t> d_off(nblocks);
    uint64_t pos = 0;
    for (uint32_t b = 0; b < nblocks; ++b) { d_off[b] = pos; pos += round16(len[b]); }
    LZ4MI_TRY(g_ctx.in.ensure(pos + 64, s));
    LZ4MI_TRY(g_ctx.meta.ensure((size_t)nblocks * 16 + 64, s));
    uint64_t* m_off = g_ctx.meta.as<uint64_t>();
    uint32_t* m_len = (uint32_t*)(m_off + nblocks);
    uint32_t* m_h = m_len + nblocks;
    for (uint32_t b = 0; b < nblocks; ++b)
        LZ4MI_TRY(hipMemcpyAsync(g_ctx.in.as<uint8_t>() + d_off[b], in + off[b], len[b], hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_off, d_off.data(), 8ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(hipMemcpyAsync(m_len, len, 4ull * nblocks, hipMemcpyHostToDevice, s));
    LZ4MI_TRY(lz4mi_launch_xxh32(g_ctx.in.as<uint8_t>(), m_off, m_len, seed, m_h, nblocks, stdv, nullptr, nullptr, s));
    LZ4MI_TRY(hipMemcpyAsync(hashes, m_h, 4ull * nblocks, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    return LZ4MI_OK;
}

int32_t lz4mi_frame_pack(const uint8_t* raw, const uint64_t* raw_off, const uint32_t* raw_len, const uint8_t* comp,
                         const uint64_t* comp_off, const uint32_t* comp_len, uint8_t* frame, const uint64_t* rec_off,
                         uint32_t nblocks, uint32_t flags, void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (!(flags & LZ4MI_DEVICE_PTRS)) return LZ4MI_ERR_ARG;
    if (nblocks == 0) return LZ4MI_OK;
    hipStream_t s = pick_stream(stream);
    if (!(flags & LZ4MI_BLOCK_CHECKSUM)) {
        LZ4MI_TRY(lz4mi_launch_frame_pack(raw, raw_off, raw_len, comp, comp_off, comp_len, frame, rec_off, nblocks,
                                          nullptr, nullptr, nullptr, s));
        return LZ4MI_OK;
    }
    // records carry XXH32 (spec) of their payload after it: the pack kernel writes each
    // payload's position and length, the batched XXH32 kernel hashes the payloads in place
    // and stores each digest after its payload
    StreamCtx* c = stream_ctx(s);
    std::lock_guard<std::mutex> sl(c->mu);
    LZ4MI_TRY(c->frame_meta.ensure((size_t)nblocks * 20 + 64, s));
    uint64_t* pay_off = c->frame_meta.as<uint64_t>();
    uint64_t* sum_off = pay_off + nblocks;
    uint32_t* pay_len = (uint32_t*)(sum_off + nblocks);
    LZ4MI_TRY(lz4mi_launch_frame_pack(raw, raw_off, raw_len, comp, comp_off, comp_len, frame, rec_off, nblocks,
                                      pay_off, sum_off, pay_len, s));
    LZ4MI_TRY(lz4mi_launch_xxh32(frame, pay_off, pay_len, 0, nullptr, nblocks, 1, frame, sum_off, s));
    return LZ4MI_OK;
}

int32_t lz4mi_frame_decompress(const uint8_t* frame, uint64_t len, uint8_t* out, uint64_t out_cap, int64_t* info,
                               uint32_t flags, void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (!(flags & LZ4MI_DEVICE_PTRS) || !info || (flags & LZ4MI_JS_COMPAT)) return LZ4MI_ERR_ARG;
    for (int k = 0; k < 8; ++k) info[k] = 0;
    hipStream_t s = pick_stream(stream);
    const int mode = (flags & LZ4MI_JS_EXACT) ? 2 : 0;
    // the header (<= 19 bytes) first: the content size bounds the number of blocks of the reference's layout
    uint8_t h[19] = {0};
    LZ4MI_TRY(hipMemcpyAsync(h, frame, std::min<uint64_t>(len, 19), hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    // magic and version as the device walk reports them (bufferDecompress.js:59-67)
    if (len < 4 || le32(h) != 0x184D2204u) {
        info[0] = LZ4MI_ERR_MAGIC;
        return LZ4MI_OK;
    }
    info[1] = len > 4 ? h[4] : 0;
    if (((info[1] & 0xC0) >> 6) != 1) {
        info[0] = LZ4MI_ERR_VERSION;
        return LZ4MI_OK;
    }
    const uint64_t size = (len >= 14 && (h[4] & 0x08)) ? (uint64_t)le32(h + 6) | ((uint64_t)le32(h + 10) << 32) : 0;
    info[2] = (int64_t)size;
    // no content size (or 0), or more than the caller's buffer: the host path decodes the frame;
    // checked before any scratch is sized from the header's claim
    if (size == 0 || size > out_cap) return LZ4MI_ERR_ARG;
    const uint32_t id = len > 5 ? (h[5] >> 4) & 7 : 7;
    const uint64_t bmax = id == 4 ? 65536 : id == 5 ? 262144 : id == 6 ? 1048576 : 4194304;
    // every record takes at least its 4-byte size word
    const uint64_t cap_blocks = std::min<uint64_t>(size / bmax, len / 4) + 2;
    if (cap_blocks > 0xFFFFFFF0ull) return LZ4MI_ERR_ARG;
    StreamCtx* c = stream_ctx(s);
    std::lock_guard<std::mutex> sl(c->mu);
    const size_t per = 8 + 4 + 8 + 4 + 4;   // compressed lists (in_off, in_len, out_off, out_cap, idx)
    const size_t per_s = 8 + 4 + 8 + 4;     // stored lists (in_off, len, out_off, idx)
    const size_t meta = cap_blocks * (per + per_s + 4 + 4) + 64 + 64;   // + out_len, status
    LZ4MI_TRY(c->scan.ensure(meta, s));
    uint8_t* m = c->scan.as<uint8_t>();
    int64_t* d_info = (int64_t*)m;
    uint64_t* c_in_off = (uint64_t*)(m + 64);
    uint64_t* c_out_off = c_in_off + cap_blocks;
    uint64_t* s_in_off = c_out_off + cap_blocks;
    uint64_t* s_out_off = s_in_off + cap_blocks;
    uint32_t* c_in_len = (uint32_t*)(s_out_off + cap_blocks);
    uint32_t* c_out_cap = c_in_len + cap_blocks;
    uint32_t* c_idx = c_out_cap + cap_blocks;
    uint32_t* s_len = c_idx + cap_blocks;
    uint32_t* s_idx = s_len + cap_blocks;
    uint32_t* d_out_len = s_idx + cap_blocks;
    int32_t* d_status = (int32_t*)(d_out_len + cap_blocks);
    LZ4MI_TRY(lz4mi_launch_frame_scan(frame, len, (uint32_t)cap_blocks, c_in_off, c_in_len, c_out_off, c_out_cap,
                                      s_in_off, s_len, s_out_off, c_idx, s_idx, d_info, s));
    int64_t hi[8];
    LZ4MI_TRY(hipMemcpyAsync(hi, d_info, sizeof hi, hipMemcpyDeviceToHost, s));
    LZ4MI_TRY(hipStreamSynchronize(s));
    for (int k = 0; k < 8; ++k) info[k] = hi[k];
    if (hi[0]) return LZ4MI_OK;                        // magic / version: info[0] holds the reference's error
    if (hi[2] <= 0 || hi[7]) return LZ4MI_ERR_ARG;     // no content size, or not the reference's layout: host path
    if ((uint64_t)hi[2] > out_cap) return LZ4MI_ERR_ARG;
    const uint32_t nc = (uint32_t)hi[3], ns = (uint32_t)hi[4];
    // stored blocks, then every compressed block in one batch (spec or reference-exact)
    LZ4MI_TRY(lz4mi_launch_frame_stored(frame, len, s_in_off, s_len, s_out_off, out, (uint64_t)hi[2], ns, s));
    if (nc) LZ4MI_TRY(decode_launch(frame, c_in_off, c_in_len, out, c_out_off, c_out_cap, nullptr, 0, d_out_len,
                                    d_status, nc, mode, s, &c->order));
    std::vector<uint32_t> olen(nc), cap(nc), cidx(nc), slen(ns), sidx(ns);
    std::vector<int32_t> stat(nc);
    std::vector<uint64_t> soff(ns), ooff(nc), ioff(nc);
    if (nc) {
        LZ4MI_TRY(hipMemcpyAsync(olen.data(), d_out_len, 4ull * nc, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(stat.data(), d_status, 4ull * nc, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(cap.data(), c_out_cap, 4ull * nc, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(cidx.data(), c_idx, 4ull * nc, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(ooff.data(), c_out_off, 8ull * nc, hipMemcpyDeviceToHost, s));
    }
    if (ns) {
        LZ4MI_TRY(hipMemcpyAsync(slen.data(), s_len, 4ull * ns, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(sidx.data(), s_idx, 4ull * ns, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(soff.data(), s_out_off, 8ull * ns, hipMemcpyDeviceToHost, s));
    }
    LZ4MI_TRY(hipStreamSynchronize(s));
    // blocks that read earlier blocks' output (dependent frames, or an F1 rewrite at a block start):
    // every block before them is final now; decode each alone, in order
    for (uint32_t k = 0; k < nc; ++k) {
        if (stat[k] != LZ4MI_ERR_CROSS_BLOCK) continue;
        LZ4MI_TRY(decode_launch(frame, c_in_off + k, c_in_len + k, out, c_out_off + k, c_out_cap + k, nullptr, 0,
                                d_out_len + k, d_status + k, 1, mode, s, nullptr));
        LZ4MI_TRY(hipMemcpyAsync(&olen[k], d_out_len + k, 4, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipMemcpyAsync(&stat[k], d_status + k, 4, hipMemcpyDeviceToHost, s));
        LZ4MI_TRY(hipStreamSynchronize(s));
    }
    // the reference's first error in block order; every compressed block but the frame's last must fill
    // block_max (the layout the output positions assumed), else the host path decodes the frame
    const uint64_t size_v = (uint64_t)hi[2];
    uint32_t first = UINT32_MAX;
    int32_t first_st = 0;
    uint64_t written = 0;
    for (uint32_t k = 0; k < nc; ++k) {
        // the reference's capacity is the whole result, not the block's slot: a block that overran
        // its slot is not the reference encoder's layout (the host path decodes such a frame)
        if (stat[k] == LZ4MI_ERR_OUTPUT_TOO_SMALL && ooff[k] + cap[k] < size_v) return LZ4MI_ERR_ARG;
        if (stat[k] && cidx[k] < first) { first = cidx[k]; first_st = stat[k]; }
        if (!stat[k]) written = std::max<uint64_t>(written, ooff[k] + olen[k]);
        if (!stat[k] && olen[k] != cap[k] && cidx[k] != nc + ns - 1) return LZ4MI_ERR_ARG;
    }
    for (uint32_t k = 0; k < ns; ++k) {
        if (soff[k] + slen[k] > size_v && sidx[k] < first) { first = sidx[k]; first_st = LZ4MI_ERR_RANGE; }
        written = std::max<uint64_t>(written, std::min<uint64_t>(soff[k] + slen[k], size_v));
    }
    info[0] = first_st;
    info[3] = (int64_t)written;
    return LZ4MI_OK;
}

int32_t lz4mi_frame_index(const uint8_t* frame, uint64_t len, uint64_t* pay_off, uint32_t* size_word,
                          uint32_t cap_blocks, int64_t* info, uint32_t flags, void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (!(flags & LZ4MI_DEVICE_PTRS) || !frame || !info || (cap_blocks && (!pay_off || !size_word)))
        return LZ4MI_ERR_ARG;
    LZ4MI_TRY(lz4mi_launch_frame_index(frame, len, cap_blocks, pay_off, size_word, info, pick_stream(stream)));
    return LZ4MI_OK;
}

int32_t lz4mi_generate_blocks(uint8_t* out, uint32_t kind, uint32_t seed0, uint32_t block_size, uint32_t nblocks,
                              void* stream) {
    DeviceGuard dg;
    if (dg.status()) return dg.status();
    if (kind > 2) return LZ4MI_ERR_ARG;
    LZ4MI_TRY(lz4mi_launch_generate(out, kind, seed0, block_size, nblocks, pick_stream(stream)));
    return LZ4MI_OK;
}

}  // extern "C"
