// lz4mi_decompress_ring.hip — two-pass LZ4 block decoder for batches of
// independent blocks (gfx950).
//
// Replaces decompressBlock (reference src/block/blockDecompress.js:30-275) as
// called per block by the frame decoder (src/buffer/bufferDecompress.js:133-192)
// for independent blocks: LZ4 spec semantics, no dictionary, every block's
// back-references stay inside the block. The single-pass kernel
// (lz4mi_decompress.hip) keeps every other case and re-decodes any block this
// path hands back (status kStatusRedo): errors in the reference's check order,
// clipped matches, references before the block, pathological spans.
//
// Pass 1 — lz4mi_token_map_kernel: one LANE per 1 KiB chunk of compressed
//   input. The lane walks the token chain serially from kWarmMap bytes before
//   its chunk (LZ4 token chains started anywhere merge with the true chain
//   within a few tokens) and writes a bitmap of the token starts it visits
//   inside its chunk: 1 bit per compressed byte. 64 chunks per wave, every lane
//   doing useful serial work, no LDS.
//
// Pass 2 — lz4mi_ring_decode_kernel: one wave per block. The last 64 KiB of the
//   block's output — the whole LZ4 window — lives in an LDS ring, so
//   back-references never leave the CU; HBM sees the compressed bytes once and
//   the output once, as aligned 16-byte stores. Per chunk:
//    1. stage the chunk (+ kPad bytes) in LDS (loaded during the previous chunk);
//    2. take the pass-1 bitmap if it holds the true entry token (the previous
//       chunk's exit), else rebuild it by a serial walk over the staged bytes;
//    3. sequence table: lane l decodes the tokens in bytes [16l, 16l+16);
//       output starts by wave prefix sums;
//    4. output into the ring: at-risk sources (the ring slots this chunk's
//       output will overwrite) are read into registers first, then literal
//       runs, then matches in dependency rounds — a match goes when no
//       earlier, still pending match writes the 16-byte units of its source
//       (an LDS min-map per output unit of the chunk);
//    5. flush the chunk's complete 16-byte units from the ring to HBM.
//   A sequence with multi-byte length fields (long literal runs, long matches)
//   is written straight to HBM by the whole wave and the ring reloaded from
//   its last 64 KiB.
#include "lz4mi_common.h"
#include "lz4mi_decompress.h"

#ifndef LZ4MI_RING_ABLATE
#define LZ4MI_RING_ABLATE 0   // timing-only variants: 1 = sources always ready, 2 = no unit phase
#endif

#ifndef LZ4MI_RING_PROFILE
#define LZ4MI_RING_PROFILE 0   // timing-only variant (tools/ring_prof.py): per-phase wall-clock accumulation
#endif

namespace lz4mi {
namespace ring {

#if LZ4MI_RING_PROFILE
__device__ unsigned long long g_rprof[16];
#define RPROF(i)                             \
    do {                                     \
        const uint64_t t_ = wall_clock64();  \
        rprof[i] += t_ - rprof_t;            \
        rprof_t = t_;                        \
    } while (0)
#define RPROF_COUNT(i, n) (rprof[i] += (n))
#else
#define RPROF(i) ((void)0)
#define RPROF_COUNT(i, n) ((void)0)
#endif

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kC = 1024;                     // compressed bytes per chunk
constexpr int kWords = kC / 64;              // bitmap words per chunk
constexpr int32_t kWarmMap = 384;            // pass 1: walks start this far before their chunk
constexpr int kPad = 320;                    // staged bytes past the chunk: every 1-extension-byte sequence fits
constexpr int kStage = kC + kPad;            // 1344 = 84 x 16
constexpr int kStagePieces = kStage / 16;
constexpr int kMaxSeq = kC / 3 + 4;          // tokens in one chunk
constexpr int32_t kRing = 65536;
constexpr int32_t kRingMask = kRing - 1;
constexpr int32_t kSpanMax = 16384;          // output of one chunk's regular sequences (else redo)

static_assert(kStage % 16 == 0, "stage in 16-byte pieces");

struct MapArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    const uint32_t* out_cap;
    uint32_t min_ratio;           // blocks compressed less than out_cap / in_len >= min_ratio are not mapped
    const uint32_t* chunk_base;   // first chunk index of each block in `bitmap` (kNoMap: block not mapped)
    uint64_t* bitmap;             // kWords words per chunk
    uint32_t nblocks;
};

constexpr uint32_t kNoMap = 0xFFFFFFFFu;   // chunk_base of a block the ring decoder does not take

struct RingArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    const uint32_t* out_cap;
    uint32_t* out_len;
    int32_t* status;
    const uint32_t* chunk_base;
    const uint64_t* bitmap;
    uint32_t min_ratio;          // blocks below this out_cap / in_len ratio go to the single-pass kernel
    uint32_t* stats;             // optional counters (nullptr): [0] rebuilt bitmaps, [1] direct sequences,
                                 // [2] blocks handed back, [3..5] why: malformed token, sequence error, direct error
    uint32_t nblocks;
};

// ------------------------------------------------------------------ pass 1
// 8 bytes of blk at p (zero past len), little-endian.
__device__ __forceinline__ uint64_t ld8(const uint8_t* blk, int32_t p, int32_t len) {
    if (p + 8 <= len) {
        uint64_t v;
        __builtin_memcpy(&v, blk + p, 8);
        return v;
    }
    uint64_t v = 0;
    for (int j = 0; j < 8 && p + j < len; ++j) v |= (uint64_t)blk[p + j] << (8 * j);
    return v;
}

// Sum of a 255-run length field starting at q (q advanced past its last byte).
__device__ __forceinline__ int32_t varint8(const uint8_t* blk, int32_t& q, int32_t len) {
    int32_t sum = 0;
    for (;;) {
        if (q >= len) return sum;
        const uint64_t v = ld8(blk, q, len);
        const uint64_t nff = ~v;   // first byte != 255
        if (nff == 0) {
            sum += 8 * 255;
            q += 8;
            continue;
        }
        const int n = __builtin_ctzll(nff) >> 3;
        sum += 255 * n + (int32_t)((v >> (8 * n)) & 255u);
        q += n + 1;
        return sum;
    }
}

// Position of the token after the one at p; >= len ends the chain (final
// literal-only sequence, or input exhausted / malformed).
__device__ __forceinline__ int32_t next_token_at(const uint8_t* blk, int32_t p, int32_t len) {
    const uint64_t v = ld8(blk, p, len);
    const uint32_t tok = (uint32_t)v & 255u;
    int32_t ll = (int32_t)(tok >> 4);
    int32_t q = p + 1;
    uint32_t sh = 8;
    if (ll == 15) {
        const uint32_t b1 = (uint32_t)(v >> 8) & 255u;
        if (b1 != 255u) {
            ll += (int32_t)b1;
            q += 1;
            sh = 16;
        } else {
            q += 1;
            ll += 255 + varint8(blk, q, len);
            sh = 64;   // fields below are not in v
        }
    }
    q += ll;
    if (q >= len) return len;
    uint32_t w;   // offset (2 bytes) + first extension byte
    const int32_t rel = q - p;
    if (sh != 64 && rel <= 5) w = (uint32_t)(v >> (8 * rel));
    else w = (uint32_t)ld8(blk, q, len);
    q += 2;
    if ((tok & 15u) == 15u) {
        const uint32_t mb = (w >> 16) & 255u;
        if (mb != 255u) q += 1;
        else {
            q += 1;
            (void)varint8(blk, q, len);
        }
    }
    return q;
}

// Device-side plan of the two-pass decode (no host round trip): block b is taken by the
// ring decoder when it is compressed at least min_ratio:1 and its chunks fit the bitmap
// scratch (capacity chunks); chunk_base[b] = its first chunk (exclusive scan over the
// taken blocks) or kNoMap. *needed = the chunks all eligible blocks would take, read back
// lazily by the host to grow the scratch for later calls (host-mapped word).
constexpr int kPlanThreads = 1024;
__global__ __launch_bounds__(kPlanThreads) void lz4mi_ring_plan_kernel(const uint32_t* in_len, const uint32_t* out_cap,
                                                                      uint32_t min_ratio, uint32_t nblocks,
                                                                      uint64_t capacity, uint32_t* chunk_base,
                                                                      uint32_t* needed) {
    __shared__ uint64_t part[kPlanThreads / kWave];
    __shared__ uint64_t carry_s;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    uint64_t carry = 0;
    for (uint32_t t0 = 0; t0 < nblocks; t0 += kPlanThreads) {
        const uint32_t b = t0 + tid;
        uint64_t nch = 0;
        bool elig = false;
        if (b < nblocks) {
            const uint64_t len = in_len[b];
            elig = len * min_ratio <= (uint64_t)out_cap[b];
            nch = elig ? (len + kC - 1) / kC : 0;
        }
        uint64_t x = nch;   // inclusive wave scan
        for (int d = 1; d < kWave; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, kWave);
            if (lane >= d) x += y;
        }
        if (lane == kWave - 1) part[wv] = x;
        __syncthreads();
        uint64_t before = carry;
        for (int w = 0; w < wv; ++w) before += part[w];
        const uint64_t base = before + x - nch;
        if (b < nblocks) chunk_base[b] = (elig && base + nch <= capacity) ? (uint32_t)base : kNoMap;
        if (tid == kPlanThreads - 1) carry_s = before + x;
        __syncthreads();
        carry = carry_s;
        __syncthreads();
    }
    if (tid == 0) *needed = carry > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)carry;
}

// One workgroup per block, one lane per 1 KiB chunk (looping over the block's chunks).
__global__ __launch_bounds__(64) void lz4mi_token_map_kernel(MapArgs a) {
    const uint32_t b = blockIdx.x;
    if (b >= a.nblocks || a.chunk_base[b] == kNoMap) return;
    const int32_t len = (int32_t)a.in_len[b];
    const int32_t nch = (len + kC - 1) / kC;
    const uint8_t* blk = a.in + a.in_off[b];
    for (int32_t k = (int32_t)threadIdx.x; k < nch; k += 64) {
    uint64_t* bm = a.bitmap + ((uint64_t)a.chunk_base[b] + (uint64_t)k) * kWords;
    const int32_t base = k * kC;
    const int32_t end = base + kC < len ? base + kC : len;
    int32_t p = base > kWarmMap ? base - kWarmMap : 0;
    if (k == 0) p = 0;
    while (p < base) p = next_token_at(blk, p, len);
    uint64_t word = 0;
    int wi = 0;
    while (p < end) {
        const int32_t r = p - base;
        const int w = r >> 6;
        while (wi < w) {
            bm[wi++] = word;
            word = 0;
        }
        word |= 1ull << (r & 63);
        p = next_token_at(blk, p, len);
    }
    while (wi < kWords) {
        bm[wi++] = word;
        word = 0;
    }
    }
}

// ------------------------------------------------------------------ pass 2
constexpr int kThreads = 256;                // one workgroup (4 waves) per block
constexpr int kWavesPerBlock = kThreads / kWave;
constexpr int kMirror = 32;                  // ring[kRing, +32) mirrors ring[0, 32)
constexpr int kStgPad = 16;                  // staged bytes sit at stg[kStgPad + i]: reads may start 15 bytes early
constexpr int kMaxUnits = kSpanMax / 16 + 2;
constexpr int kRows = (kMaxSeq + kThreads - 1) / kThreads;   // sequence rows of the table

struct RingShared {
    uint8_t ring[kRing + kMirror];            // output position x at ring[x & 0xFFFF]
    uint8_t stg[kStgPad + kStage + 32];       // chunk bytes [base, base + kStage)
    uint32_t t_out[kMaxSeq + 1];              // output start of each sequence (block-relative); [nseq] = step end
    uint2 t_info[kMaxSeq];                    // {literal stage index | ll << 16, offset | ml << 16}
    uint16_t t_nxt[kMaxSeq];                  // stage index of the token after each sequence
    uint16_t t_pos[kMaxSeq];                  // stage index of each sequence's token
    uint16_t owner[kMaxUnits];                // per output unit of the step: sequence holding its first new byte
    uint16_t vis[64];                         // pass-1 token bits of the chunk (16 per segment)
    uint16_t vis2[64];                        // bitmap rebuild: walked bits
    uint32_t red[8][kWavesPerBlock];          // per-wave partials of workgroup reductions
    uint64_t done[kWavesPerBlock];            // units of the current batch that are written
    int32_t sync;
};
static_assert(sizeof(RingShared) <= 80 * 1024, "two blocks per CU");

// Bytes [idx, idx + 16) of an LDS byte array (base 16-aligned) from five
// naturally aligned dword reads: a misaligned b64/b128 LDS access replays at
// ~64 LDS cycles CU-wide (tools/probe/lds_unaligned.hip), aligned dwords do not.
__device__ __forceinline__ uint4 lds16(const uint8_t* base, int32_t idx) {
    const uint32_t* w = (const uint32_t*)(base + (idx & ~3));
    const uint32_t sh = (uint32_t)idx & 3u;
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
    return make_uint4(funnel(d0, d1, sh), funnel(d1, d2, sh), funnel(d2, d3, sh), funnel(d3, d4, sh));
}
__device__ __forceinline__ uint4 ring16(const RingShared& S, int32_t pos) { return lds16(S.ring, pos & kRingMask); }
__device__ __forceinline__ uint4 stg16(const RingShared& S, int32_t i) { return lds16(S.stg + kStgPad, i); }

// dword mask of bytes [lo, hi) (clamped to the dword)
__device__ __forceinline__ uint32_t bmask(int32_t lo, int32_t hi) {
    lo = lo < 0 ? 0 : lo > 4 ? 4 : lo;
    hi = hi < 0 ? 0 : hi > 4 ? 4 : hi;
    const uint32_t mh = hi >= 4 ? 0xFFFFFFFFu : (1u << (8 * hi)) - 1u;
    const uint32_t ml = lo >= 4 ? 0xFFFFFFFFu : (1u << (8 * lo)) - 1u;
    return mh & ~ml;
}
// V bytes [o, o + n) := val bytes [o, o + n)
__device__ __forceinline__ void merge(uint4& V, uint4 val, int32_t o, int32_t n) {
    const int32_t e = o + n;
    uint32_t m;
    m = bmask(o, e);
    V.x = (V.x & ~m) | (val.x & m);
    m = bmask(o - 4, e - 4);
    V.y = (V.y & ~m) | (val.y & m);
    m = bmask(o - 8, e - 8);
    V.z = (V.z & ~m) | (val.z & m);
    m = bmask(o - 12, e - 12);
    V.w = (V.w & ~m) | (val.w & m);
}

// V bytes [0, b) from a, [b, 16) from c (b in 0..16)
__device__ __forceinline__ uint4 cut16(uint4 a, uint4 c, int32_t b) {
    const uint64_t m0 = b >= 8 ? ~0ull : (1ull << (8 * b)) - 1ull;
    const uint64_t m1 = b >= 16 ? ~0ull : b <= 8 ? 0ull : (1ull << (8 * (b - 8))) - 1ull;
    const uint32_t mx = (uint32_t)m0, my = (uint32_t)(m0 >> 32), mz = (uint32_t)m1, mw = (uint32_t)(m1 >> 32);
    return make_uint4((a.x & mx) | (c.x & ~mx), (a.y & my) | (c.y & ~my), (a.z & mz) | (c.z & ~mz),
                      (a.w & mw) | (c.w & ~mw));
}

__device__ __forceinline__ void st_w(uint8_t* p, uint4 v, uint32_t w) {
    if (w == 16) {
        __builtin_memcpy(p, &v, 16);
    } else if (w == 8) {
        __builtin_memcpy(p, &v, 8);
    } else if (w == 4) {
        __builtin_memcpy(p, &v.x, 4);
    } else if (w == 2) {
        const uint16_t t = (uint16_t)v.x;
        __builtin_memcpy(p, &t, 2);
    } else {
        *p = (uint8_t)v.x;
    }
}

__device__ __forceinline__ uint4 shr_bytes(uint4 v, uint32_t n) {
    unsigned __int128 x;
    __builtin_memcpy(&x, &v, 16);
    x = n >= 16 ? 0 : x >> (8 * n);
    __builtin_memcpy(&v, &x, 16);
    return v;
}
__device__ __forceinline__ uint4 shl_bytes(uint4 v, uint32_t n) {
    unsigned __int128 x;
    __builtin_memcpy(&x, &v, 16);
    x = n >= 16 ? 0 : x << (8 * n);
    __builtin_memcpy(&v, &x, 16);
    return v;
}

// bytes [0, k) of a followed by bytes [0, 16 - k) of b
__device__ __forceinline__ uint4 splice(uint4 a, uint4 b, int32_t k) {
    unsigned __int128 x, y;
    __builtin_memcpy(&x, &a, 16);
    __builtin_memcpy(&y, &b, 16);
    const unsigned __int128 m = (((unsigned __int128)1) << (8 * k)) - 1;
    x = (x & m) | (y << (8 * k));
    __builtin_memcpy(&a, &x, 16);
    return a;
}

// 16 bytes of a period per < 16 held in A[0, per), starting at phase r.
__device__ __forceinline__ uint4 expand_period(uint4 A, int32_t r, int32_t per) {
    uint32_t o[4] = {0, 0, 0, 0};
    int32_t idx = r;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t dw = idx < 4 ? A.x : idx < 8 ? A.y : idx < 12 ? A.z : A.w;
        o[j >> 2] |= ((dw >> ((idx & 3) * 8)) & 255u) << ((j & 3) * 8);
        idx = idx + 1 == per ? 0 : idx + 1;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Pieces of a run of n bytes: 16-byte pieces (the last overlapping its
// predecessor) or, below 16 bytes, two overlapping 8/4/2/1-byte pieces.
__device__ __forceinline__ int run_pieces(int32_t n) {
    return n >= 16 ? (n + 15) >> 4 : (n <= 0 ? 0 : ((n & (n - 1)) == 0 ? 1 : 2));
}
__device__ __forceinline__ void piece_at(int32_t n, int p, int32_t& d, uint32_t& w) {
    if (n >= 16) {
        w = 16;
        d = 16 * p < n - 16 ? 16 * p : n - 16;
    } else {
        w = n >= 8 ? 8u : n >= 4 ? 4u : n >= 2 ? 2u : 1u;
        d = p ? n - (int32_t)w : 0;
    }
}

// ---- workgroup reductions (all 256 threads call; slot s of S.red must not be
// in use by an earlier reduction still being read)
__device__ __forceinline__ uint32_t wg_excl_scan(RingShared& S, int slot, uint32_t v, int tid, uint32_t& total) {
    const int lane = tid & (kWave - 1), w = tid / kWave;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == kWave - 1) S.red[slot][w] = incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) {
        const uint32_t x = S.red[slot][i];
        before += i < w ? x : 0u;
        tot += x;
    }
    total = tot;
    return before + incl - v;
}
// minimum of two values over the workgroup (one barrier)
__device__ __forceinline__ void wg_min2(RingShared& S, int slot, uint32_t& a, uint32_t& b, int tid) {
    const int lane = tid & (kWave - 1), w = tid / kWave;
    const uint32_t ma = wave_min(a), mb = wave_min(b);
    if (lane == 0) {
        S.red[slot][w] = ma;
        S.red[slot + 1][w] = mb;
    }
    __syncthreads();
    uint32_t ra = 0xFFFFFFFFu, rb = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) {
        ra = min(ra, S.red[slot][i]);
        rb = min(rb, S.red[slot + 1][i]);
    }
    a = ra;
    b = rb;
}

// Output [lo, hi) from the ring to dst, exactly (lo a multiple of 16).
__device__ void flush_exact(const RingShared& S, uint8_t* dst, int32_t lo, int32_t hi, int tid) {
    const int32_t full = hi & ~15;
    for (int32_t u = lo + 16 * tid; u < full; u += 16 * kThreads) {
        uint4 v;
        __builtin_memcpy(&v, S.ring + (u & kRingMask), 16);
        __builtin_memcpy(dst + u, &v, 16);
    }
    if (full < hi && full >= lo && tid == 0) {
        const int32_t n = hi - full;
        uint4 v;
        __builtin_memcpy(&v, S.ring + (full & kRingMask), 16);
        const uint32_t w = n >= 8 ? 8u : n >= 4 ? 4u : n >= 2 ? 2u : 1u;
        st_w(dst + full, v, w);
        st_w(dst + full + n - (int32_t)w, shr_bytes(v, (uint32_t)(n - (int32_t)w)), w);
    }
}

// ring <- out[lo, hi) (bytes past hi may be anything): aligned units from global.
__device__ void ring_reload(RingShared& S, const uint8_t* dst, int32_t lo, int32_t hi, int32_t cap, int tid) {
    const int32_t u0 = lo & ~15;
    for (int32_t u = u0 + 16 * tid; u < hi; u += 16 * kThreads) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (u + 16 <= cap) {
            const u32x4_t t = *(const u32x4_t*)(dst + u);
            v = make_uint4(t.x, t.y, t.z, t.w);
        } else {
            unsigned __int128 x = 0;
            for (int j = 0; j < 16 && u + j < cap; ++j) x |= (unsigned __int128)*(dst + u + j) << (8 * j);
            __builtin_memcpy(&v, &x, 16);
        }
        __builtin_memcpy(S.ring + (u & kRingMask), &v, 16);
    }
    __syncthreads();
    if (tid < kMirror / 4) {
        uint32_t t;
        __builtin_memcpy(&t, S.ring + 4 * tid, 4);
        __builtin_memcpy(S.ring + kRing + 4 * tid, &t, 4);
    }
    __syncthreads();
}

// Wave-wide 255-run varint at block-relative q (q advanced past its last byte).
__device__ int32_t wave_varint(const uint8_t* blk, int32_t len, int lane, int32_t& q) {
    int32_t sum = 0;
    for (;;) {
        const int32_t p = q + 16 * lane;
        int first = 16;
        uint32_t lastb = 0;
        for (int j = 0; j < 16; ++j) {
            const int32_t r = p + j;
            const uint32_t bb = (r < len) ? blk[r] : 0u;
            if (bb != 255u && first == 16) {
                first = j;
                lastb = bb;
            }
        }
        const uint64_t mask = __ballot(first < 16);
        if (mask) {
            const uint32_t fl = (uint32_t)__builtin_ctzll(mask);
            const int32_t fi = (int32_t)lane_val((uint32_t)first, fl);
            const uint32_t fb = lane_val(lastb, fl);
            const int32_t cnt = (int32_t)fl * 16 + fi;
            sum += 255 * cnt + (int32_t)fb;
            q += cnt + 1;
            return sum;
        }
        sum += 255 * 16 * kWave;
        q += 16 * kWave;
    }
}

// Straight global -> global copy of n bytes (literal run of a direct sequence).
__device__ void direct_copy(uint8_t* dst, const uint8_t* src, int32_t n, int tid) {
    constexpr int kD = 8;
    if (n < 16) {
        if (tid == 0)
            for (int32_t j = 0; j < n; ++j) dst[j] = src[j];
        return;
    }
    const int32_t np = (n + 15) >> 4;
    for (int32_t p0 = 0; p0 < np; p0 += kThreads * kD) {
        uint4 v0, v1, v2, v3, v4, v5, v6, v7;
        int32_t d[kD];
#pragma unroll
        for (int j = 0; j < kD; ++j) {
            const int32_t p = p0 + tid + kThreads * j;
            d[j] = 16 * p < n - 16 ? 16 * p : n - 16;   // past the end: the last piece again
        }
        __builtin_memcpy(&v0, src + d[0], 16);
        __builtin_memcpy(&v1, src + d[1], 16);
        __builtin_memcpy(&v2, src + d[2], 16);
        __builtin_memcpy(&v3, src + d[3], 16);
        __builtin_memcpy(&v4, src + d[4], 16);
        __builtin_memcpy(&v5, src + d[5], 16);
        __builtin_memcpy(&v6, src + d[6], 16);
        __builtin_memcpy(&v7, src + d[7], 16);
        __builtin_memcpy(dst + d[0], &v0, 16);
        __builtin_memcpy(dst + d[1], &v1, 16);
        __builtin_memcpy(dst + d[2], &v2, 16);
        __builtin_memcpy(dst + d[3], &v3, 16);
        __builtin_memcpy(dst + d[4], &v4, 16);
        __builtin_memcpy(dst + d[5], &v5, 16);
        __builtin_memcpy(dst + d[6], &v6, 16);
        __builtin_memcpy(dst + d[7], &v7, 16);
    }
}

// Match of a direct sequence: out[ms, ms + n) = out[ms - off + i] read from
// global memory (everything below ms was stored and waited for). Periods under
// 16 bytes via an LDS phase table (pat: 256 bytes of scratch).
__device__ void direct_match(uint8_t* pat, uint8_t* dst, int32_t ms, int32_t off, int32_t n, int tid) {
    const int32_t src = ms - off;
    const int32_t per = off < n ? off : 0;
    if (per && per < 16) {
        __syncthreads();
        for (int idx = tid; idx < 16 * per; idx += kThreads) {
            const int r = idx >> 4, j = idx & 15;
            pat[idx] = *(dst + src + (r + j) % per);
        }
        __syncthreads();
    }
    const int np = run_pieces(n);
    constexpr int kD = 4;
    for (int p0 = 0; p0 < np; p0 += kThreads * kD) {
        uint4 v[kD];
        int32_t dd[kD];
        uint32_t ww[kD];
#pragma unroll
        for (int j = 0; j < kD; ++j) {
            const int p = p0 + tid + kThreads * j;
            piece_at(n, p < np ? p : np - 1, dd[j], ww[j]);
            const int32_t d = dd[j];
            if (per == 0) {
                const u32x4_t t = *(const u32x4_t*)(dst + src + d);
                v[j] = make_uint4(t.x, t.y, t.z, t.w);
            } else if (per < 16) {
                __builtin_memcpy(&v[j], pat + 16 * (d % per), 16);
            } else {
                const int32_t r = d % per;
                const u32x4_t t = *(const u32x4_t*)(dst + src + r);
                v[j] = make_uint4(t.x, t.y, t.z, t.w);
                if (r + 16 > per) {   // the window wraps: bytes [per - r, 16) restart at the period's start
                    const u32x4_t t2 = *(const u32x4_t*)(dst + src);
                    v[j] = splice(v[j], make_uint4(t2.x, t2.y, t2.z, t2.w), per - r);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kD; ++j) {
            const int p = p0 + tid + kThreads * j;
            if (p < np) st_w(dst + ms + dd[j], v[j], ww[j]);
        }
    }
    if (per && per < 16) __syncthreads();
}

// 16 compressed bytes at block-relative r0 (zero past len).
__device__ __forceinline__ uint4 stage_piece(const uint8_t* blk, int32_t len, int32_t r0) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + 16 <= len) {
        __builtin_memcpy(&v, blk + r0, 16);
    } else if (r0 < len) {
        unsigned __int128 x = 0;
        for (int j = 0; j < 16 && r0 + j < len; ++j) x |= (unsigned __int128)blk[r0 + j] << (8 * j);
        __builtin_memcpy(&v, &x, 16);
    }
    return v;
}

struct Tok {   // one decoded token of the staged chunk
    int32_t lit, ll, off, ml, nxt;   // stage-relative literal start / next token
    uint32_t kind;                   // 0 regular, 1 final (literal-only), 2 direct (multi-byte length field), 3 malformed
};

// Decode the token at stage index p (p < kC). rem = block bytes from the chunk base.
__device__ __forceinline__ Tok decode_tok(const RingShared& S, int32_t p, int32_t rem) {
    Tok t{0, 0, 0, 0, 0, 0u};
    const uint4 w = stg16(S, p);
    const uint32_t tok = w.x & 255u, b1 = (w.x >> 8) & 255u;
    const uint32_t x1 = (tok >> 4) == 15 ? 1u : 0u;
    if (x1 && b1 == 255u) { t.kind = 2; return t; }
    t.ll = x1 ? 15 + (int32_t)b1 : (int32_t)(tok >> 4);
    t.lit = p + 1 + (int32_t)x1;
    const int32_t q = t.lit + t.ll;
    if (x1 && p + 1 >= rem) { t.kind = 3; return t; }
    if (q >= rem) { t.kind = q == rem ? 1u : 3u; t.nxt = q; return t; }
    const int32_t d = q - p;   // offset and first match-length byte: in w when d <= 13
    uint32_t f;
    if (d <= 13) {
        const uint32_t lo = d < 4 ? w.x : d < 8 ? w.y : d < 12 ? w.z : w.w;
        const uint32_t hi = d < 4 ? w.y : d < 8 ? w.z : w.w;
        f = funnel(lo, hi, (uint32_t)d & 3u);
    } else {
        f = stg16(S, q).x;
    }
    t.off = (int32_t)(f & 0xFFFFu);
    const uint32_t x2 = (tok & 15u) == 15u ? 1u : 0u;
    const uint32_t mb = (f >> 16) & 255u;
    if (x2 && mb == 255u) { t.kind = 2; return t; }
    t.ml = (x2 ? 15 + (int32_t)mb : (int32_t)(tok & 15u)) + 4;
    t.nxt = q + 2 + (int32_t)x2;
    if (t.nxt > rem) t.kind = 3;
    return t;
}

struct Step {   // the current chunk's regular sequences and their output
    int32_t A, B, A0;   // output [A, B); A0 = A rounded down to 16
    uint32_t nseq;
};

// Units of the current batch that are written (bit r of batch-relative unit r).
struct Done {
    uint64_t w[kWavesPerBlock];
    __device__ __forceinline__ bool has(int32_t u) const { return (w[u >> 6] >> (u & 63)) & 1ull; }
};

// Unit U (a multiple of 16 in [A0, B)) of the step's output, assembled from
// its segments (the general path: any number of segments, short periods).
// A segment whose source bytes lie in this batch's units [bU0, U) must wait
// until those units are written (`done`); far sources that the batch's own
// stores may have overwritten in the ring (re-passes only) are read from HBM.
__device__ __noinline__ uint4 make_unit(const RingShared& S, const Step& st, int32_t U, int32_t bU0, const Done done,
                                        bool repass, const uint8_t* dst, bool& deferred) {
    uint4 V = make_uint4(0, 0, 0, 0);
    deferred = false;
    const int32_t end = U + 16 < st.B ? U + 16 : st.B;
    int32_t pos = U;
    auto ready = [&](int32_t s, int32_t e) -> bool {   // bytes [s, e) of earlier output are complete
        if (LZ4MI_RING_ABLATE & 1) return true;
        const int32_t lo = s > bU0 ? s : bU0;
        if (e <= lo || e <= st.A) return true;
        const int32_t u0 = (lo - bU0) >> 4, u1 = (e - 1 - bU0) >> 4;
        const int32_t me = (U - bU0) >> 4;
        for (int32_t u = u0; u <= u1; ++u)
            if (u != me && !done.has(u)) return false;
        return true;
    };
    auto hist16 = [&](int32_t p) -> uint4 {   // 16 bytes of earlier output from p
        if (repass && p < bU0 + 16 * kThreads - kRing + 16) {
            wait_vmem();   // those bytes' stores are complete in HBM
            uint4 v = make_uint4(0, 0, 0, 0);
            unsigned __int128 x = 0;
            for (int j = 0; j < 16; ++j)
                if (p + j >= 0) x |= (unsigned __int128)*(dst + p + j) << (8 * j);
            __builtin_memcpy(&v, &x, 16);
            return v;
        }
        return ring16(S, p);
    };
    if (pos < st.A) {   // bytes of the previous step in the unit's head
        const int32_t n = (st.A < end ? st.A : end) - pos;
        merge(V, ring16(S, U), 0, n);
        pos += n;
    }
    if (pos >= end) return V;
    uint32_t k = S.owner[(U - st.A0) >> 4];
    bool broken = false;   // an earlier segment of this unit is deferred: V holds no valid bytes past it
    while (pos < end) {
        const int32_t t0 = (int32_t)S.t_out[k];
        const uint2 inf = S.t_info[k];
        const int32_t ll = (int32_t)(inf.x >> 16), ml = (int32_t)(inf.y >> 16);
        const int32_t ms = t0 + ll, me = ms + ml;
        const int32_t o = pos - U;
        if (pos < ms) {   // literal bytes
            const int32_t n = (ms < end ? ms : end) - pos;
            const int32_t sp = (int32_t)(inf.x & 0xFFFFu) + (pos - t0);
            merge(V, stg16(S, sp - o), o, n);
            pos += n;
        } else if (pos < me) {   // match bytes
            const int32_t off = (int32_t)(inf.y & 0xFFFFu);
            const int32_t n = (me < end ? me : end) - pos;
            if (off >= 16) {   // the source lies before this unit
                if (ready(pos - off, pos - off + n)) merge(V, hist16(U - off), o, n);
                else deferred = true;
            } else {           // period off < 16: expand the period out[ms - off, ms)
                const int32_t ps = ms - off;
                if (broken || !ready(ps, ms < U ? ms : U)) {
                    deferred = true;
                } else {
                    uint4 P = hist16(ps);
                    if (ms > U) {   // part of the period is this unit's earlier bytes (in V)
                        const int32_t d = ps - U;   // may be negative
                        const uint4 Vs = d >= 0 ? shr_bytes(V, (uint32_t)d) : shl_bytes(V, (uint32_t)(-d));
                        merge(P, Vs, d >= 0 ? 0 : -d, 16 - (d >= 0 ? 0 : -d));
                    }
                    int32_t r = (U - ms) % off;
                    if (r < 0) r += off;
                    merge(V, expand_period(P, r, off), o, n);
                }
            }
            if (deferred) broken = true;
            pos += n;
        } else {
            ++k;
        }
    }
    return V;
}

// One contiguous part of the output from position p: [p, end) comes from the
// 16-byte window `val` aligned to the unit start U (val byte j <-> output U + j).
// ok = false: a period under 16 bytes (the general path handles it).
struct Part {
    int32_t end;
    int32_t rs, re;   // its source range when it is a match (rs == re: literal / earlier step)
    bool ok;
};
__device__ __forceinline__ Part part_at(const RingShared& S, const Step& st, uint32_t& k, int32_t p, int32_t U,
                                        uint4& val) {
    Part P{0, 0, 0, true};
    if (p < st.A) {   // bytes of the previous step
        val = ring16(S, U);
        P.end = st.A;
        return P;
    }
    int32_t t0 = (int32_t)S.t_out[k];
    uint2 inf = S.t_info[k];
    int32_t ms = t0 + (int32_t)(inf.x >> 16), me = ms + (int32_t)(inf.y >> 16);
    while (p >= me) {   // (zero-length parts end where the next sequence starts)
        ++k;
        t0 = (int32_t)S.t_out[k];
        inf = S.t_info[k];
        ms = t0 + (int32_t)(inf.x >> 16);
        me = ms + (int32_t)(inf.y >> 16);
    }
    if (p < ms) {
        val = stg16(S, (int32_t)(inf.x & 0xFFFFu) + (U - t0));
        P.end = ms;
        return P;
    }
    const int32_t off = (int32_t)(inf.y & 0xFFFFu);
    P.end = me;
    if (off < 16) {
        P.ok = false;
        return P;
    }
    val = ring16(S, U - off);
    P.rs = p - off;
    P.re = (me < U + 16 ? me : U + 16) - off;
    return P;
}

// Fast path: a unit of at most three contiguous parts, no short period.
__device__ __forceinline__ uint4 fast_unit(const RingShared& S, const Step& st, int32_t r, int32_t U, int32_t bU0,
                                           const Done& done, bool repass, bool& slow, bool& deferred) {
    const int32_t uend = U + 16 < st.B ? U + 16 : st.B;
    uint32_t kk = S.owner[r];
    uint4 v1, v2, v3;
    const Part p1 = part_at(S, st, kk, U, U, v1);
    slow = !p1.ok;
    Part p2{0, 0, 0, true}, p3{0, 0, 0, true};
    if (!slow && p1.end < uend) {
        p2 = part_at(S, st, kk, p1.end, U, v2);
        slow = !p2.ok;
        if (!slow && p2.end < uend) {
            p3 = part_at(S, st, kk, p2.end, U, v3);
            slow = !p3.ok || p3.end < uend;
            v2 = cut16(v2, v3, p2.end - U);
        }
        v1 = cut16(v1, v2, p1.end - U);
    }
    const int32_t lim = bU0 > st.A ? bU0 : st.A;
    auto waits = [&](int32_t rs, int32_t re) -> bool {
        if (re <= rs || (LZ4MI_RING_ABLATE & 1)) return false;
        if (repass && rs < bU0 + 16 * kThreads - kRing + 16) slow = true;   // maybe overwritten: general path
        if (re <= lim) return false;
        const int32_t u0 = ((rs > lim ? rs : lim) - bU0) >> 4, u1 = (re - 1 - bU0) >> 4;
        return !(done.has(u0) && done.has(u1));
    };
    deferred = false;
    if (!slow) deferred = waits(p1.rs, p1.re) || waits(p2.rs, p2.re) || waits(p3.rs, p3.re);
    return v1;
}

__global__ __launch_bounds__(kThreads, 2) void lz4mi_ring_decode_kernel(RingArgs a) {
    __shared__ __attribute__((aligned(16))) RingShared S;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1), wv = tid / kWave;
    const uint32_t b = blockIdx.x;
    if (b >= a.nblocks) return;
    const uint8_t* blk = a.in + a.in_off[b];
    const int32_t len = (int32_t)a.in_len[b];
    if ((uint64_t)len * a.min_ratio > (uint64_t)a.out_cap[b] || a.chunk_base[b] == kNoMap) {   // single-pass kernel's block
        if (tid == 0) a.status[b] = kStatusRedo;
        return;
    }
    uint8_t* dst = a.out + a.out_off[b];
    const int32_t cap = a.out_cap[b] > 0x7FFFFFFFu ? 0x7FFFFFFF : (int32_t)a.out_cap[b];
    const uint16_t* bm = (const uint16_t*)(a.bitmap + (uint64_t)a.chunk_base[b] * kWords);

    int32_t ent = 0;   // next token (block-relative compressed position)
    int32_t O = 0;     // output bytes produced; everything below O & ~15 is in HBM
    int32_t status = 0;
    uint32_t n_rebuild = 0, n_direct = 0, redo_why = 0;
#define RSTAT(i) (redo_why = (i))

    // the chunk's staged bytes (threads < kStagePieces) and pass-1 bits (threads < 64), loaded ahead
    int32_t pf_k = 0;
    uint4 pf = tid < kStagePieces ? stage_piece(blk, len, 16 * tid) : make_uint4(0, 0, 0, 0);
    uint32_t pfm = (tid < 64 && len > 0) ? bm[tid] : 0u;
#if LZ4MI_RING_PROFILE
    uint64_t rprof[16] = {0};
    uint64_t rprof_t = wall_clock64();
#endif

    while (ent < len) {
        RPROF_COUNT(15, 1);
        const int32_t k = ent / kC;
        const int32_t base = k * kC;
        const int32_t rem = len - base;
        if (pf_k != k) {
            if (tid < kStagePieces) pf = stage_piece(blk, len, base + 16 * tid);
            if (tid < 64) pfm = bm[(size_t)k * (kWords * 4) + tid];
            pf_k = k;
        }
        if (tid < kStagePieces) __builtin_memcpy(S.stg + kStgPad + 16 * tid, &pf, 16);
        if (tid < 64) S.vis[tid] = (uint16_t)pfm;
        __syncthreads();
        RPROF(0);

        // ---- the chunk's token bits from the true entry on
        const int32_t rel = ent - base;
        if (!((S.vis[rel >> 4] >> (rel & 15)) & 1u)) {
            // pass 1's walk was off the true chain at the entry: walk the true
            // chain until it lands on a token of pass 1's walk (from there on the
            // two are the same chain)
            ++n_rebuild;
            if (tid < 64) S.vis2[tid] = 0;
            __syncthreads();
            if (tid == 0) {
                int32_t p = rel;
                while (p < kC && p < rem) {
                    if ((S.vis[p >> 4] >> (p & 15)) & 1u) break;
                    S.vis2[p >> 4] |= (uint16_t)(1u << (p & 15));
                    const Tok t = decode_tok(S, p, rem);
                    if (t.kind != 0) {   // the table stops at this token anyway
                        p = kC;
                        break;
                    }
                    p = t.nxt;
                }
                S.sync = p;
            }
            __syncthreads();
            if (tid < 64) {
                const int32_t ps = S.sync, s0 = 16 * tid;
                uint32_t keep = S.vis[tid];
                if (s0 + 16 <= ps) keep = 0;
                else if (s0 < ps) keep &= ~((1u << (ps - s0)) - 1u);
                S.vis[tid] = (uint16_t)(keep | S.vis2[tid]);
            }
            __syncthreads();
        }
        const int32_t p0 = 4 * tid;   // this thread's 4 bytes of the chunk
        uint32_t nib = (S.vis[tid >> 2] >> (4 * (tid & 3))) & 15u;
        if (p0 + 4 <= rel) nib = 0;
        else if (p0 < rel) nib &= ~((1u << (rel - p0)) - 1u);
        RPROF(1);

        // ---- sequence table
        const uint32_t cnt = __popc(nib);
        uint32_t ntok;
        const uint32_t sbase = wg_excl_scan(S, 0, cnt, tid, ntok);
        uint32_t stop_key = 0xFFFFFFFFu;   // (index << 2 | kind) of the first sequence that is not a plain one
        {
            uint32_t m = nib, kk = sbase;
            for (uint32_t i = 0; i < cnt; ++i, ++kk) {
                const int32_t p = p0 + __builtin_ctz(m);
                m &= m - 1;
                const Tok t = decode_tok(S, p, rem);
                if (t.kind >= 2 && stop_key == 0xFFFFFFFFu) stop_key = (kk << 2) | t.kind;
                if (kk < (uint32_t)kMaxSeq) {
                    S.t_info[kk] = make_uint2((uint32_t)t.lit | ((uint32_t)t.ll << 16),
                                              (uint32_t)t.off | ((uint32_t)t.ml << 16));
                    S.t_nxt[kk] = (uint16_t)(t.kind == 1 ? kC + kPad : t.nxt);
                    S.t_pos[kk] = (uint16_t)p;
                }
            }
        }
        uint32_t unused = 0xFFFFFFFFu;
        wg_min2(S, 1, stop_key, unused, tid);
        const uint32_t wstop = stop_key == 0xFFFFFFFFu ? 0xFFFFFFFFu : stop_key >> 2;
        const uint32_t wkind = stop_key == 0xFFFFFFFFu ? 0u : stop_key & 3u;
        if (wkind == 3u || ntok > (uint32_t)kMaxSeq) { status = kStatusRedo; RSTAT(3); break; }
        uint32_t nseq = wstop < ntok ? wstop : ntok;   // plain sequences of this step

        // output starts; a step writes at most kSpanMax bytes: the table is cut
        // before the first sequence that would end past that
        uint32_t cut = 0xFFFFFFFFu, bad_at = 0xFFFFFFFFu;
        uint32_t row_base = 0;
        for (int row = 0; row < kRows && (uint32_t)(kThreads * row) < nseq; ++row) {
            const uint32_t kk = kThreads * row + tid;
            uint32_t len_k = 0;
            uint2 inf = make_uint2(0, 0);
            if (kk < nseq) {
                inf = S.t_info[kk];
                len_k = (inf.x >> 16) + (inf.y >> 16);
            }
            uint32_t rtot;
            const uint32_t rel_os = row_base + wg_excl_scan(S, 3 + row, len_k, tid, rtot);
            const uint32_t os = (uint32_t)O + rel_os;
            if (kk < nseq) {
                const int32_t ll = (int32_t)(inf.x >> 16), ml = (int32_t)(inf.y >> 16);
                const int32_t off = (int32_t)(inf.y & 0xFFFFu);
                bool bad = (int64_t)os + ll + ml > cap;                       // output too small / clipped match
                if (ml && (off == 0 || off > (int32_t)os + ll)) bad = true;   // offset 0 / before the block
                if (bad && kk < bad_at) bad_at = kk;
                if (rel_os + len_k > (uint32_t)kSpanMax && kk < cut) cut = kk;
                S.t_out[kk] = os;
            }
            row_base += rtot;
        }
        wg_min2(S, 5, cut, bad_at, tid);   // (its barrier also publishes t_out)
        const bool trimmed = cut < nseq;   // (cut >= 1: one sequence writes at most 542 bytes)
        if (trimmed) nseq = cut;
        if (bad_at < nseq) { status = kStatusRedo; RSTAT(4); break; }
        const int32_t span = trimmed ? (int32_t)S.t_out[nseq] - O : (int32_t)row_base;
        const int32_t exit_rel = nseq ? (int32_t)S.t_nxt[nseq - 1] : -1;
        const bool has_direct = wstop != 0xFFFFFFFFu && !trimmed;
        const int32_t p_dir = has_direct ? (int32_t)S.t_pos[wstop] : 0;
        __syncthreads();
        if (tid == 0) S.t_out[nseq] = (uint32_t)(O + span);

        // next chunk's bytes: loaded while this chunk's output is written
        const int32_t next_ent = has_direct ? -1 : (exit_rel >= kC + kPad ? len : base + exit_rel);
        if (next_ent >= 0 && next_ent < len) {
            const int32_t nk = next_ent / kC;
            if (nk != k) {
                if (tid < kStagePieces) pf = stage_piece(blk, len, nk * kC + 16 * tid);
                if (tid < 64) pfm = bm[(size_t)nk * (kWords * 4) + tid];
                pf_k = nk;
            }
        }
        __syncthreads();
        RPROF(2);

        // ---- owner map: unit -> sequence holding its first byte of this step
        const Step st{O, O + span, O & ~15, nseq};
        const int32_t nunits = (st.B - st.A0 + 15) >> 4;
        for (int row = 0; row < kRows; ++row) {
            const uint32_t kk = kThreads * row + tid;
            if (kk >= nseq) break;
            const int32_t t0 = (int32_t)S.t_out[kk], t1 = (int32_t)S.t_out[kk + 1];
            int32_t r0 = (t0 - st.A0 + 15) >> 4;   // units whose first byte of this step lies in [t0, t1)
            if (kk == 0) r0 = 0;
            const int32_t r1 = (t1 - st.A0 + 15) >> 4;
            for (int32_t r = r0; r < r1; ++r) S.owner[r] = (uint16_t)kk;
        }
        __syncthreads();
        RPROF(3);

        // ---- output units, kThreads per batch, in position order
        for (int32_t bu = 0; bu < ((LZ4MI_RING_ABLATE & 2) ? 0 : nunits); bu += kThreads) {
            const int32_t r = bu + tid;
            const int32_t U = st.A0 + 16 * r;
            const int32_t bU0 = st.A0 + 16 * bu;
            const bool mine = r < nunits;
            Done done{{0ull, 0ull, 0ull, 0ull}};
            bool deferred = false, slow = false;
            uint4 V = make_uint4(0, 0, 0, 0);
            if (mine) V = fast_unit(S, st, r, U, bU0, done, false, slow, deferred);
            if (__ballot(slow))
                if (slow) V = make_unit(S, st, U, bU0, done, false, dst, deferred);
            RPROF_COUNT(12, __popcll(__ballot(slow)));
            RPROF_COUNT(13, __popcll(__ballot(deferred)));
            bool pending = mine;   // not stored yet
            for (;;) {
                // (1) every unit of the batch has read its sources (a unit's store overwrites the
                // ring slot of the output 64 KiB before it, which an earlier unit in another wave
                // may still read) and the units still waiting are known
                const uint64_t mdone = __ballot(!(pending && deferred));
                if (lane == 0) S.done[wv] = mdone;
                __syncthreads();
                bool all = true;
#pragma unroll
                for (int i = 0; i < kWavesPerBlock; ++i) {
                    done.w[i] = S.done[i];
                    all = all && done.w[i] == ~0ull;
                }
                if (pending && !deferred) {
                    __builtin_memcpy(S.ring + (U & kRingMask), &V, 16);
                    if ((U & kRingMask) < kMirror) __builtin_memcpy(S.ring + kRing + (U & kRingMask), &V, 16);
                    if (U + 16 <= st.B) __builtin_memcpy(dst + U, &V, 16);
                    pending = false;
                }
                // (2) the stores are visible to every wave (and S.done may be rewritten)
                __syncthreads();
                if (all) break;
                // units waiting for units of this batch: again, now that those are written
                RPROF_COUNT(14, 1);
                if (pending) {
                    V = fast_unit(S, st, r, U, bU0, done, true, slow, deferred);
                    if (slow) V = make_unit(S, st, U, bU0, done, true, dst, deferred);
                }
            }
        }
        O = st.B;
        RPROF(4);

        if (!has_direct) {
            ent = next_ent >= len || next_ent < 0 ? len : next_ent;
            continue;
        }

        // ---- direct sequence (multi-byte length fields): straight to HBM
        ++n_direct;
        flush_exact(S, dst, O & ~15, O, tid);   // the unit the sequence starts in
        wait_vmem();                              // everything below the sequence is complete in HBM
        __syncthreads();
        int32_t q = base + p_dir;                 // (every wave parses the fields itself)
        const uint32_t tok = blk[q++];
        int32_t ll = (int32_t)(tok >> 4);
        if (ll == 15) {
            if (q >= len) { status = kStatusRedo; RSTAT(5); break; }
            const uint32_t b1 = blk[q];
            if (b1 != 255u) {
                ll += (int32_t)b1;
                ++q;
            } else {
                ll += wave_varint(blk, len, lane, q);
            }
        }
        const int32_t lit = q;
        q += ll;
        const int32_t T = O;
        if (q > len || (int64_t)T + ll > cap) { status = kStatusRedo; RSTAT(5); break; }
        int32_t off = 0, ml = 0;
        if (q < len) {
            if (q + 2 > len) { status = kStatusRedo; RSTAT(5); break; }
            off = (int32_t)((uint32_t)blk[q] | ((uint32_t)blk[q + 1] << 8));
            q += 2;
            ml = (int32_t)(tok & 15u);
            if (ml == 15) {
                if (q >= len) { status = kStatusRedo; RSTAT(5); break; }
                const uint32_t mb = blk[q];
                if (mb != 255u) {
                    ml += (int32_t)mb;
                    ++q;
                } else {
                    ml += wave_varint(blk, len, lane, q);
                }
            }
            ml += 4;
            if (q > len || off == 0 || off > T + ll || (int64_t)T + ll + ml > cap) {
                status = kStatusRedo;
                RSTAT(5);
                break;
            }
        }
        direct_copy(dst + T, blk + lit, ll, tid);
        if (ml) {
            wait_vmem();   // the literals are read back as the match source
            __syncthreads();
            direct_match((uint8_t*)S.owner, dst, T + ll, off, ml, tid);
        }
        wait_vmem();
        __syncthreads();
        const int32_t E = T + ll + ml;
        ring_reload(S, dst, E - kRing > T ? E - kRing : T, E, cap, tid);
        O = E;
        ent = q;
        pf_k = -1;
        RPROF(5);
    }

    if (status == 0) flush_exact(S, dst, O & ~15, O, tid);   // the last partial unit
#if LZ4MI_RING_PROFILE
    if (tid == 0)
        for (int i = 0; i < 16; ++i) atomicAdd(&g_rprof[i], (unsigned long long)rprof[i]);
#endif
    if (a.stats && tid == 0) {
        if (n_rebuild) atomicAdd(&a.stats[0], n_rebuild);
        if (n_direct) atomicAdd(&a.stats[1], n_direct);
        if (status) atomicAdd(&a.stats[2], 1u);
        if (redo_why) atomicAdd(&a.stats[redo_why], 1u);
    }
    if (tid == 0) {
        a.status[b] = status;
        a.out_len[b] = status ? 0u : (uint32_t)O;
    }
}

}  // namespace ring
}  // namespace lz4mi

#if LZ4MI_RING_PROFILE
// Per-phase wall-clock ticks (100 MHz) summed over all blocks since the last call; resets.
extern "C" int lz4mi_debug_ring_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lz4mi::ring::g_rprof), sizeof(unsigned long long) * 16) != hipSuccess)
        return -1;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(lz4mi::ring::g_rprof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

extern "C" hipError_t lz4mi_launch_ring_plan(const uint32_t* in_len, const uint32_t* out_cap, uint32_t min_ratio,
                                             uint32_t nblocks, uint64_t capacity_chunks, uint32_t* chunk_base,
                                             uint32_t* needed, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(lz4mi::ring::lz4mi_ring_plan_kernel, dim3(1), dim3(lz4mi::ring::kPlanThreads), 0, stream,
                       in_len, out_cap, min_ratio, nblocks, capacity_chunks, chunk_base, needed);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_token_map(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                             const uint32_t* out_cap, uint32_t min_ratio, const uint32_t* chunk_base,
                                             uint64_t* bitmap, uint32_t nblocks, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    lz4mi::ring::MapArgs a{in, in_off, in_len, out_cap, min_ratio, chunk_base, bitmap, nblocks};
    hipLaunchKernelGGL(lz4mi::ring::lz4mi_token_map_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_ring_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                               uint32_t* out_len, int32_t* status, const uint32_t* chunk_base,
                                               const uint64_t* bitmap, uint32_t min_ratio, uint32_t* stats,
                                               uint32_t nblocks, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    lz4mi::ring::RingArgs a{in, in_off, in_len, out, out_off, out_cap, out_len, status, chunk_base, bitmap, min_ratio,
                            stats, nblocks};
    hipLaunchKernelGGL(lz4mi::ring::lz4mi_ring_decode_kernel, dim3(nblocks), dim3(lz4mi::ring::kThreads), 0, stream, a);
    return hipGetLastError();
}
