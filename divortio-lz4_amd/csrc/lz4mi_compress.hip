// lz4mi_compress.hip — LZ4 block encoder for MI355X (gfx950), byte-identical
// to the reference encoder compressBlock (src/block/blockCompress.js:31-233).
//
// The reference parse is a single greedy chain: hash the 4 bytes at i
// (Math.imul(seq, 2654435761) >>> 18), read-and-replace the 16384-entry table
// slot, verify distance (< 65536) and content, skip ahead by (miss++ >> 6) on a
// miss, extend forward only, emit, continue at the match end. Every decision
// depends on the previous one, so each block is one wave walking that chain
// exactly; the wave's 64 lanes make each step wide (speculative probe batches,
// 128-byte window compares, emission) instead of making the chain parallel.
// Two kernels:
//   lz4mi_compress_gts_kernel    independent blocks, one wave per block, 16 per CU
//                                (global 15-bit tables + LDS epoch codes);
//   lz4mi_compress_chain_kernel  dependent blocks / one block with the caller's
//                                table (LZ4.compressRaw): one wave, the table, the
//                                source window and the output ring in LDS.
#include "lz4mi_common.h"

#include <cstdlib>

#ifndef LZ4MI_CTIMELINE
#define LZ4MI_CTIMELINE 0   // diagnostic build (tools/timeline.py --what compress): per-block start / end, HW_ID
#endif

#ifndef LZ4MI_CPROFILE
#define LZ4MI_CPROFILE 0   // timing-only variant (tools/): per-phase wall-clock of the batch encoder
#endif

namespace lz4mi {

#if LZ4MI_CPROFILE
__device__ unsigned long long g_cprof[16];
#define CPROF(i)                             \
    do {                                     \
        const uint64_t t_ = wall_clock64();  \
        cprof[i] += t_ - cprof_t;            \
        cprof_t = t_;                        \
    } while (0)
#define CPROF_COUNT(i, n) (cprof[i] += (n))
#else
#define CPROF(i) ((void)0)
#define CPROF_COUNT(i, n) ((void)0)
#endif

struct CompJob {
    const uint8_t* src;   // positions are absolute from here
    uint64_t src_total;   // readable bytes from src
    int32_t start, len;   // block = src[start, start+len)
    uint8_t* dst;         // output positions are absolute from here
    uint64_t dst_total;   // writable bytes from dst (writes past it are dropped)
    int32_t dst_pos;      // first output position
    int32_t* table;       // optional caller table (in/out); null = fresh table
};

struct CompArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    uint32_t* out_len;
    uint32_t nblocks;
};

constexpr uint32_t kP1 = 2654435761u;


__device__ __forceinline__ uint32_t src_byte(const CompJob& j, int64_t p) {
    return (p >= 0 && (uint64_t)p < j.src_total) ? (uint32_t)j.src[p] : 0u;
}

// Lanes 8g .. 8g+7 get v of lane g (g < 8): one LDS permute (eight v_readlane instead were slower:
// SGPR spills, round 4).
__device__ __forceinline__ int32_t group_val(int32_t v, int g) { return __shfl(v, g, kWave); }

// Lane l gets v of lane 8 (l & 7) + f, f = the first set bit of byte (l & 7) of mm (0 when
// the byte is 0; `ft` is that lane's own f): one LDS permute.
__device__ __forceinline__ uint32_t first_val(uint32_t v, uint64_t mm, int lane, int ft) {
    (void)mm;
    return __shfl(v, 8 * (lane & 7) + ft, kWave);
}

// Value of v in lane l, l uniform (a ballot's ctz, a lane count): v_readlane
// instead of the LDS permute __shfl compiles to (on the chain's critical path).
__device__ __forceinline__ uint32_t lane_val(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int32_t lane_val(int32_t v, int l) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, l); }

__device__ __forceinline__ uint32_t ld_u32(const CompJob& j, int64_t p) {
    if (p >= 0 && (uint64_t)p + 4 <= j.src_total) {
        uint32_t v;
        __builtin_memcpy(&v, j.src + p, 4);
        return v;
    }
    return src_byte(j, p) | (src_byte(j, p + 1) << 8) | (src_byte(j, p + 2) << 16) | (src_byte(j, p + 3) << 24);
}

// ---- source ring of the dependent-block chain (lz4mi_compress_chain): the last
// 64 KiB of the parse plus up to 32 KiB ahead of it, in LDS, so a probe's window,
// the candidate's bytes and the literal copies are LDS reads instead of global
// round trips (the chain is one wave's serial walk: its latency is the speed).
// Byte p (absolute) lives at g_ring[p mod kRingBytes] while p in [lo, hi).
constexpr uint32_t kRingBytes = 88 * 1024;
constexpr int64_t kRingStep = 16 * 1024;     // refill granularity (16-byte aligned pieces)
constexpr int64_t kRingAhead = 4096;         // refill when fewer bytes than this are ahead of the parse
static_assert(kRingBytes - 65536 >= kRingStep + kRingAhead, "a refill never evicts a byte a probe can reach");
__shared__ uint8_t g_ring[kRingBytes];

struct Ring {
    int64_t lo, hi;
};

// Source readers: global (the batch kernels) or through the chain's ring.
struct SrcG {
    __device__ static __forceinline__ uint32_t byte(const CompJob& j, const Ring*, int64_t p) { return src_byte(j, p); }
    __device__ static __forceinline__ uint32_t u32(const CompJob& j, const Ring*, int64_t p) { return ld_u32(j, p); }
};
struct SrcR {
    __device__ static __forceinline__ uint32_t byte(const CompJob& j, const Ring* r, int64_t p) {
        if (p >= r->lo && p < r->hi) return g_ring[(uint32_t)p % kRingBytes];
        return src_byte(j, p);
    }
    __device__ static __forceinline__ uint32_t u32(const CompJob& j, const Ring* r, int64_t p) {
        if (p >= r->lo && p + 4 <= r->hi) {
            const uint32_t q = (uint32_t)p % kRingBytes;
            if (q <= kRingBytes - 4) return *(const uint32_t*)&g_ring[q];   // unaligned LDS dword (unaligned mode)
            return g_ring[q] | (g_ring[(q + 1) % kRingBytes] << 8) | (g_ring[(q + 2) % kRingBytes] << 16) |
                   ((uint32_t)g_ring[(q + 3) % kRingBytes] << 24);
        }
        return ld_u32(j, p);
    }
};

// Bring at least kRingAhead bytes ahead of position i into the ring (whole wave).
__device__ void ring_advance(const CompJob& j, Ring& r, int lane, int64_t i) {
    while ((uint64_t)r.hi < j.src_total && r.hi - i < kRingAhead + 256) {
        const int64_t n = (int64_t)j.src_total - r.hi < kRingStep ? (int64_t)j.src_total - r.hi : kRingStep;
        for (int64_t k = 16 * lane; k < n; k += 16 * kWave) {
            const int64_t p = r.hi + k;
            const uint32_t q = (uint32_t)p % kRingBytes;
            if (k + 16 <= n) {
                uint4 v;
                __builtin_memcpy(&v, j.src + p, 16);
                *(uint4*)&g_ring[q] = v;
            } else {
                for (int64_t t = 0; k + t < n; ++t) g_ring[q + t] = j.src[p + t];
            }
        }
        __syncthreads();
        r.hi += n;
        if (r.hi - r.lo > (int64_t)kRingBytes) r.lo = r.hi - kRingBytes;
    }
}

// First differing byte of src[a + t] vs src[b + t], t in [0, lim) (lim if none).
__device__ int64_t match_extent(const CompJob& j, int lane, int64_t a, int64_t b, int64_t lim) {
    int64_t base = 0;
    while (base < lim) {
        if (base >= 4 * kWave && base + 16 * kWave * 2 <= lim) {
            // past the first 256 bytes (most matches end there): 2 KiB per step, two
            // 16-byte loads per lane and side in flight (long matches of repetitive data;
            // four in flight: 4 % faster there, 1 % slower on tiles216 from register pressure)
            uint4 x[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int64_t o = base + 16 * (lane + kWave * u);
                uint4 va, vb;
                __builtin_memcpy(&va, j.src + a + o, 16);
                __builtin_memcpy(&vb, j.src + b + o, 16);
                x[u] = make_uint4(va.x ^ vb.x, va.y ^ vb.y, va.z ^ vb.z, va.w ^ vb.w);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint64_t m = __ballot((x[u].x | x[u].y | x[u].z | x[u].w) != 0);
                if (m) {
                    const int fl = __builtin_ctzll(m);
                    const uint32_t w0 = lane_val(x[u].x, fl), w1 = lane_val(x[u].y, fl);
                    const uint32_t w2 = lane_val(x[u].z, fl), w3 = lane_val(x[u].w, fl);
                    const int k = w0 ? 0 : w1 ? 4 : w2 ? 8 : 12;
                    const uint32_t wf = w0 ? w0 : w1 ? w1 : w2 ? w2 : w3;
                    const int64_t f = base + 16 * (fl + kWave * u) + k + (__builtin_ctz(wf) >> 3);
                    return f < lim ? f : lim;
                }
            }
            base += 16 * kWave * 2;
            continue;
        }
        const uint32_t x = ld_u32(j, a + base + 4 * lane) ^ ld_u32(j, b + base + 4 * lane);
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const int fl = __builtin_ctzll(m);
            const uint32_t xf = lane_val(x, fl);
            const int64_t f = base + 4 * fl + (__builtin_ctz(xf) >> 3);
            return f < lim ? f : lim;
        }
        base += 4 * kWave;
    }
    return lim;
}

// A register whose load has been waited for: redefine it opaquely so the compiler's
// wait insertion stops tracking it. Without this, the window bytes carried into the
// next probe are waited for with vmcnt(0), which also waits for every store the
// previous sequence's emission issued after them: a store round trip per sequence on
// the chain (the loads themselves completed long before).
__device__ __forceinline__ void settle32(uint32_t& v) { asm volatile("" : "+v"(v)); }

// ---------------------------------------------------------------------------
// Batch encoder (fresh table per block): the same parse, 4 blocks per CU.
//
// Table: a block's positions fit 22 bits, but a candidate only matters while
// it is < 65536 bytes back, so each entry keeps the position's low 16 bits plus
// a 2-bit code of its 32 KiB epoch (epoch mod 4): epochs g-2..g decode
// uniquely, code (g+1) mod 4 means empty/stale, and entering epoch g relabels
// the fields still carrying code g mod 4 (4 epochs old) as stale. 36 KiB
// instead of 64 KiB; exact (the distance check still runs on the decoded position).
//
// Probing: up to 64 consecutive probes of the miss chain (positions i + the
// prefix sum of the skip steps c >> 6) are evaluated at once, one per lane:
// hash, table read, candidate verification. Every probe up to and including
// the first hit happens in the reference, in order, each inserting its own
// position; a batch is cut before the first lane whose hash repeats an
// earlier lane's (found by writing lane ids into the table and reading them
// back), so the batch's inserts never interact and the result is the serial one.
//
// Output goes to an LDS ring (4 KiB; 2 KiB in the batch encoder) flushed in 16-byte
// units; literal runs longer than the ring takes are copied global -> global directly. No vector-memory store precedes the
// next probe's loads except at ring flushes.
constexpr int kCodeWords = 16384 / 16;
#define RING_SZ(F) ((int64_t)sizeof((F).ring))   // the output ring's size in the caller's shared struct
#define RING_MASK(F) (RING_SZ(F) - 1)
constexpr int32_t kDirectLit = 2048;   // longer literal runs bypass the ring


struct FastOut {
    uint8_t* dst;
    int64_t op, flushed;   // flushed is 16-aligned except after the final flush
};


// ring [flushed, floor16(op)) -> dst
template <class SH>
__device__ __forceinline__ void ring_flush(SH& F, FastOut& o, int lane) {
    const int64_t upto = o.op & ~(int64_t)15;
    for (int64_t p = o.flushed + 16 * lane; p < upto; p += 16 * kWave) {
        uint4 v;
        __builtin_memcpy(&v, F.ring + (p & RING_MASK(F)), 16);
        __builtin_memcpy(o.dst + p, &v, 16);
    }
    if (upto > o.flushed) o.flushed = upto;
}

template <class SH>
__device__ __forceinline__ void ring_reserve(SH& F, FastOut& o, int lane, int64_t n) {
    if (o.op + n - o.flushed > RING_SZ(F)) ring_flush(F, o, lane);
}

// n bytes of value v (n <= RING_SZ(F) - 16 per call)
template <class SH>
__device__ void ring_fill(SH& F, FastOut& o, int lane, int64_t n, uint32_t v) {
    while (n > 0) {
        const int64_t k = n < RING_SZ(F) - 16 ? n : RING_SZ(F) - 16;
        ring_reserve(F, o, lane, k);
        for (int64_t t = lane; t < k; t += kWave) F.ring[(o.op + t) & RING_MASK(F)] = (uint8_t)v;
        o.op += k;
        n -= k;
    }
}

template <class SH>
__device__ __forceinline__ void ring_put(SH& F, FastOut& o, int lane, uint32_t v) {
    ring_reserve(F, o, lane, 1);
    if (lane == 0) F.ring[o.op & RING_MASK(F)] = (uint8_t)v;
    o.op += 1;
}

// 255-run tail of a length field
template <class SH>
__device__ __forceinline__ void ring_len_ext(SH& F, FastOut& o, int lane, int64_t ext) {
    const int64_t nff = ext / 255;
    if (nff) ring_fill(F, o, lane, nff, 255);
    ring_put(F, o, lane, (uint32_t)(ext - 255 * nff));
}

// src[pos, pos+n) -> output at op
template <class SH, class SRC = SrcG>
__device__ void ring_copy(SH& F, FastOut& o, const CompJob& j, int lane, int64_t pos, int64_t n,
                          const Ring* rg = nullptr) {
    // a run through the ring must fit beside the <= 15 bytes a flush leaves pending: the
    // batch encoder's 2 KiB ring takes at most 2032 (2034..2048 wrapped onto those bytes)
    constexpr int64_t kViaRing = RING_SZ(F) - 16 < kDirectLit ? RING_SZ(F) - 16 : kDirectLit;
    if (n > kViaRing) {
        // head into the ring up to a 16-byte boundary, flush, bulk direct, tail into the ring
        const int64_t h = (16 - (o.op & 15)) & 15;
        ring_reserve(F, o, lane, 16);
        if (lane < h) F.ring[(o.op + lane) & RING_MASK(F)] = (uint8_t)SRC::byte(j, rg, pos + lane);
        o.op += h; pos += h; n -= h;
        ring_flush(F, o, lane);
        const int64_t m = n & ~(int64_t)15;
        const bool inb = (uint64_t)(pos + m) <= j.src_total;
        for (int64_t t0 = 0; t0 < m; t0 += 16 * kWave * 4) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t t = t0 + 16 * (lane + kWave * u);
                if (t < m) {
                    if (inb) {
                        __builtin_memcpy(&v[u], j.src + pos + t, 16);
                    } else {
                        uint32_t w[4];
                        for (int q = 0; q < 4; ++q) w[q] = ld_u32(j, pos + t + 4 * q);
                        v[u] = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t t = t0 + 16 * (lane + kWave * u);
                if (t < m) __builtin_memcpy(o.dst + o.op + t, &v[u], 16);
            }
        }
        o.op += m; pos += m; n -= m;
        o.flushed = o.op;
    }
    ring_reserve(F, o, lane, n);
    for (int64_t t = lane; t < n; t += kWave) F.ring[(o.op + t) & RING_MASK(F)] = (uint8_t)SRC::byte(j, rg, pos + t);
    o.op += n;
}

// token + literal length + literals
template <class SH, class SRC = SrcG>
__device__ void fast_literals(SH& F, FastOut& o, const CompJob& j, int lane, int64_t anchor, int64_t lit,
                              uint32_t mnib, const Ring* rg = nullptr) {
    ring_put(F, o, lane, (lit >= 15 ? 0xF0u : (uint32_t)lit << 4) | mnib);
    if (lit >= 15) ring_len_ext(F, o, lane, lit - 15);
    if (lit) ring_copy<SH, SRC>(F, o, j, lane, anchor, lit, rg);
}



// The miss-chain distance covered by the skip steps (c + t) >> 6, t < k: the sum of floor(u / 64)
// over u in [c, c + k), k < 64, in 32-bit arithmetic (floor(u / 64) is c >> 6, then at most once
// more plus one).
__device__ __forceinline__ int32_t skip_span(uint32_t c, uint32_t k) {
    const uint32_t qa = c >> 6, b = c + k, e = (qa + 1) << 6;
    return (int32_t)(k * qa + (b > e ? b - e : 0u));
}

// The general case of emit_seq (15+ literals or a match length field of 2+ extra bytes),
// out of line with the output state passed by value and returned: inlining it at every
// emission site costs the batch encoders their registers, and a FastOut passed by reference
// to a call lives in scratch memory (every emission then reads it back with a vmcnt(0) wait).
template <class SH, class SRC = SrcG>
__device__ __noinline__ FastOut emit_general(SH& F, FastOut o, const CompJob& j, int lane, int32_t anchor, int32_t pm,
                                             uint32_t off, int32_t mcode, const Ring* rg) {
    const int32_t lit = pm - anchor;
    const uint32_t mnib = mcode >= 15 ? 15u : (uint32_t)mcode;
    fast_literals<SH, SRC>(F, o, j, lane, anchor, lit, mnib, rg);
    ring_put(F, o, lane, off & 255);
    ring_put(F, o, lane, (off >> 8) & 255);
    if (mcode >= 15) ring_len_ext(F, o, lane, mcode - 15);
    return o;
}

// The final literal run (out of line, as emit_general).
template <class SH, class SRC = SrcG>
__device__ __noinline__ FastOut emit_tail(SH& F, FastOut o, const CompJob& j, int lane, int64_t anchor, int64_t lit,
                                          const Ring* rg) {
    fast_literals<SH, SRC>(F, o, j, lane, anchor, lit, 0, rg);
    return o;
}

// One sequence's bytes: token, literal length, literals, offset, match length.
// Common case (at most 14 literals, match length field of at most one extra
// byte) written by one ds_write_b8 per lane.
template <class SH, class SRC = SrcG>
__device__ __forceinline__ void emit_seq(SH& F, FastOut& o, const CompJob& j, int lane, int32_t anchor,
                                         int32_t pm, uint32_t off, int32_t mcode, const Ring* rg = nullptr,
                                         bool has_pre = false, uint32_t pre = 0) {
    const int32_t lit = pm - anchor;
    const uint32_t mnib = mcode >= 15 ? 15u : (uint32_t)mcode;
    if (lit < 15 && mcode < 15 + 255) {
        const int32_t total = 1 + lit + 2 + (mcode >= 15 ? 1 : 0);
        ring_reserve(F, o, lane, total);
        if (lane < total) {
            uint32_t v;
            if (lane == 0) v = ((uint32_t)lit << 4) | mnib;
            else if (lane <= lit) v = has_pre ? pre : SRC::byte(j, rg, anchor + lane - 1);   // pre: loaded earlier
            else if (lane == lit + 1) v = off & 255;
            else if (lane == lit + 2) v = (off >> 8) & 255;
            else v = (uint32_t)(mcode - 15);
            F.ring[(o.op + lane) & RING_MASK(F)] = (uint8_t)v;
        }
        o.op += total;
        return;
    }
    o = emit_general<SH, SRC>(F, o, j, lane, anchor, pm, off, mcode, rg);
}


// A batch's common-case sequences into the ring (lanes k < npend: sequence k at ring offset
// start, `total` bytes in all; sequence 0 alone has literals, lit0 < 15, whose byte l - 1 lane
// l holds in litv; every match length field at most one extra byte).
template <class SH>
__device__ __forceinline__ void ring_seqs(SH& F, FastOut& o, int lane, int npend, int32_t lit0, int32_t mcode,
                                          uint32_t off, uint32_t start, int32_t total, uint32_t litv) {
    const bool mine = lane < npend;
    const int32_t lit = lane == 0 ? lit0 : 0;
    ring_reserve(F, o, lane, total);
    // each sequence's own lane writes its token, offset and length byte; lanes 1 .. lit0 the
    // literal bytes of sequence 0 (which starts the batch)
    const uint32_t base = (uint32_t)o.op, msk = (uint32_t)RING_MASK(F);
    if (mine) {
        const uint32_t a = base + start, b = a + 1u + (uint32_t)lit;
        F.ring[a & msk] = (uint8_t)(((uint32_t)lit << 4) | (mcode >= 15 ? 15u : (uint32_t)mcode));
        F.ring[b & msk] = (uint8_t)off;
        F.ring[(b + 1u) & msk] = (uint8_t)(off >> 8);
        if (mcode >= 15) F.ring[(b + 2u) & msk] = (uint8_t)(mcode - 15);
    }
    if (lane >= 1 && lane <= lit0) F.ring[(base + (uint32_t)lane) & msk] = (uint8_t)litv;
    o.op += total;
}


// ---------------------------------------------------------------------------
// Batch encoder tables: one per block in global scratch, each entry the probed
// position's low 15 bits (32 KiB per block) plus a 2-bit code of its 32 KiB epoch in
// LDS (4 KiB per block). Epochs g-2..g decode uniquely; entering epoch g relabels the
// codes 4 epochs old as stale. A 15-bit entry + its code -> the position it stands
// for (-1: empty/stale).
__device__ __forceinline__ int32_t gt16_decode(uint32_t lo, uint32_t cd, int32_t g) {
    if (cd == (uint32_t)((g + 1) & 3)) return -1;
    const int32_t ge = g - (int32_t)((g - (int32_t)cd) & 3);
    return ge < 0 ? -1 : ((ge << 15) | (int32_t)(lo & 0x7FFFu));
}
template <class SH>
__device__ __forceinline__ uint32_t gt_code_of(const SH& F, uint32_t h) {
    return (F.code[h >> 4] >> ((h & 15) * 2)) & 3u;
}
template <class SH>
__device__ void gt_scrub_epoch(SH& F, int lane, int32_t g) {
    const uint32_t X = (uint32_t)(g & 3) * 0x55555555u, Y = (uint32_t)((g + 1) & 3) * 0x55555555u;
    for (int w = lane; w < kCodeWords; w += kWave) {
        const uint32_t v = F.code[w], x = v ^ X;
        const uint32_t eq = ~(x | (x >> 1)) & 0x55555555u;
        const uint32_t fm = eq | (eq << 1);
        F.code[w] = (v & ~fm) | (Y & fm);
    }
}


// ---------------------------------------------------------------------------
// Speculative hit chains (round 3, default). After a hit of step S (match end -
// probe position) the next probe is at the match end, and on mid-ratio data the
// next match often has the same step again (tiles216: 94 % of matches are 64
// bytes and followed directly by a hit). One probe per step costs two dependent
// global round trips per sequence (table, then the candidate's bytes); here one
// batch probes up to kSpecK positions i, i + S, i + 2S, ... at once, assuming each
// is a hit of step S:
//   round 1: the K table reads (a probe whose hash repeats an earlier probe of the
//            batch takes that probe's position instead: it inserts first);
//   round 2: per probe, 128 bytes at the probe and at its candidate (8 lanes x 16
//            bytes; the first differing byte is the match length when < 128), and
//            the 4 bytes at each probe position of the next batch (prefetch);
// then the probes are accepted in order while each is a hit whose end is the next
// probe's position. Every accepted probe and the first rejected one (the probe at
// the end of the last accepted match, which does happen) are exactly the serial
// parse's probes: they insert their positions (the last of equal hashes wins), and
// the parse continues from there -- the next batch, or the miss chain on a miss.
// Round trips per sequence: 2 / (accepted probes per batch); tiles216 3.8 (CPU model
// of the serial parse, K = 8). Table reads after the previous batch's stores need no
// wait: one wave's load of an address it stored to observes the store (program order).
constexpr int kSpecK = 8;     // probes per speculative batch (8 lanes each for the windows)
constexpr int kSpecW = 128;   // window bytes per probe

// 16 source bytes at p (zero past the end).
__device__ __forceinline__ uint4 ld16(const CompJob& j, int64_t p) {
    uint4 v;
    if (p >= 0 && (uint64_t)p + 16 <= j.src_total) {
        __builtin_memcpy(&v, j.src + p, 16);
        return v;
    }
    return make_uint4(ld_u32(j, p), ld_u32(j, p + 4), ld_u32(j, p + 8), ld_u32(j, p + 12));
}

// The batch encoder's loads (zero outside the block). 32-bit offsets from the block's scalar
// base instead were slower (77.9 vs 74.9 ms, round 4).
__device__ __forceinline__ uint4 ld16o(const CompJob& j, uint32_t lim, int32_t p) {
    (void)lim;
    return ld16(j, p);
}
__device__ __forceinline__ uint32_t ld_u32o(const CompJob& j, uint32_t lim, int32_t p) {
    (void)lim;
    return ld_u32(j, p);
}

// Index of the first nonzero byte of x (16 if none).
__device__ __forceinline__ uint32_t first_nz16(uint4 x) {
    return x.x ? (__builtin_ctz(x.x) >> 3)
               : x.y ? 4 + (__builtin_ctz(x.y) >> 3)
                     : x.z ? 8 + (__builtin_ctz(x.z) >> 3) : x.w ? 12 + (__builtin_ctz(x.w) >> 3) : 16u;
}

constexpr int32_t kWinBytes = 2048;   // source window in LDS: the probes' 4-byte reads

struct GtsShared {
    uint8_t ring[2048];                  // output ring (half the batch encoder's: the window takes the rest)
    uint8_t slot[1024];                  // miss batches: lane ids keyed by hash & 1023
    uint32_t code[kCodeWords];           // 2-bit epoch code per table entry
    uint32_t win[kWinBytes / 4 + 4];     // source bytes [wb, wb + kWinBytes)
};
// Small batches (<= kLdsTableMaxBlocks): the 15-bit table in LDS too (41 KB per block, 3 blocks
// per CU, the batch one resident round): 1 block 26.7 -> 25.5 ms, 16: 32.4 -> 31.2, 256: 34.5
// -> 32.9, 768: 42.4 -> 37.7 (profiles/r05f2/ldst_small.log); at 4096 blocks it needs 5.3 rounds
// (200 vs 70 ms, profiles/r05n)
struct GtsSharedL : GtsShared {
    uint16_t tab[16384];
};
constexpr uint32_t kLdsTableMaxBlocks = 768;
__device__ __forceinline__ uint16_t* gts_table(GtsShared&, int32_t* T) { return (uint16_t*)T; }
__device__ __forceinline__ uint16_t* gts_table(GtsSharedL& F, int32_t*) { return F.tab; }

template <class SH>
__device__ int64_t compress_block_gts(const CompJob& j, SH& F, int32_t* T, int lane) {
    const int32_t n = j.len;
    const uint32_t n32 = (uint32_t)j.src_total;   // (= n: the block is the whole source)
    const int32_t mflimit = n - 12, matchlimit = n - 5;
    FastOut o{j.dst, 0, 0};
    int32_t i = 0, anchor = 0;
    uint32_t c = 67;
    int32_t S = 0;                       // step of the last hit (0: in a miss chain): the speculated probe distance
    const int kmax = kSpecK;
    // accepted sequences not emitted yet (lanes 0 .. npend-1: probe, candidate, match end),
    // emitted while the next batch's table reads are in flight
    int npend = 0;
    int32_t pd_p = 0, pd_c = 0, pd_e = 0;
    int32_t wb = -(1 << 30);             // F.win holds source [wb, wb + kWinBytes)
    uint16_t* T16 = gts_table(F, T);
    int32_t g = 0;
    for (int k = lane; k < 16384 / 8; k += kWave) ((uint4*)T16)[k] = make_uint4(0, 0, 0, 0);
    for (int k = lane; k < kCodeWords; k += kWave) F.code[k] = 0x55555555u;   // code 1: stale in epoch 0
    wait_vmem();
#if LZ4MI_CPROFILE
    uint64_t cprof[16] = {0};
    uint64_t cprof_t = wall_clock64();
#endif
    // Only the first pending sequence can have literals (the others are back-to-back hits).
    // Its 1..14 literal bytes (lane l: byte l - 1) are loaded and waited for before the
    // emission, so no load is pending inside it but the next batch's table reads: the inline
    // emission never waits for memory (longer runs go through emit_general, out of line).
    auto load_lit = [&]() -> uint32_t {
        uint32_t litv = 0;
        const int32_t lit0 = lane_val(pd_p, 0) - anchor;
        if (lit0 <= 0 || lit0 >= 15) return 0u;                // (uniform: most batches have no literals)
        const bool ld = lane >= 1 && lane <= lit0;
        const int32_t ow = anchor - wb;
        if (ow >= 0 && ow + lit0 + 4 <= kWinBytes) {          // from the window
            const int32_t q = ow + lane - 1;
            if (ld) litv = (F.win[q >> 2] >> (8 * (q & 3))) & 255u;
        } else if (__ballot(ld)) {
            if (ld) litv = src_byte(j, anchor + lane - 1);
            wait_vmem();
        }
        settle32(litv);
        return litv;
    };
    auto emit_pending = [&](uint32_t litv) {
        for (int k = 0; k < npend; ++k) {
            const int32_t pm = lane_val(pd_p, k), cm = lane_val(pd_c, k), e = lane_val(pd_e, k);
            emit_seq(F, o, j, lane, anchor, pm, (uint32_t)(pm - cm), e - pm - 4, nullptr, true, litv);
            anchor = e;
        }
        npend = 0;
    };
    // All pending sequences in one ring write when each is the common case (sequence 0 has
    // < 15 literals, every match length field at most one extra byte): lane k < npend has
    // size_k = token + literals + offset + extension bytes at ring offset start_k; output
    // lane t finds its sequence among the <= 8 starts. Else one sequence at a time.
    auto emit_batch = [&](uint32_t litv) {
        const int32_t lit0 = lane_val(pd_p, 0) - anchor;
        const int32_t mcode = pd_e - pd_p - 4;
        const bool mine = lane < npend;
        if (lit0 >= 15 || __ballot(mine && mcode >= 15 + 255)) {
            emit_pending(litv);
            return;
        }
        const int32_t lit = lane == 0 ? lit0 : 0;
        const uint32_t size = mine ? 3u + (uint32_t)lit + (mcode >= 15 ? 1u : 0u) : 0u;
        uint32_t incl = size;                                   // inclusive scan over lanes 0..7 (row 0)
        incl += dpp<kRowShr1>(0u, incl);
        incl += dpp<kRowShr2>(0u, incl);
        incl += dpp<kRowShr4>(0u, incl);
        const uint32_t start = incl - size;
        const int32_t total = (int32_t)lane_val(incl, npend - 1);
        ring_seqs(F, o, lane, npend, lit0, mcode, (uint32_t)(pd_p - pd_c), start, total, litv);
        anchor = lane_val(pd_e, npend - 1);
        npend = 0;
    };
    auto insert = [&](bool ins, uint32_t h, int32_t p) {   // distinct hashes among inserting lanes
        if (ins) {
            T16[h] = (uint16_t)(p & 0x7FFF);
            const uint32_t sh = (h & 15) * 2;                  // two hashes may share a code word: LDS atomics
            atomicAnd(&F.code[h >> 4], ~(3u << sh));
            atomicOr(&F.code[h >> 4], (uint32_t)(g & 3) << sh);
        }
    };
    // 4 source bytes at x for the lanes that `need` them: from the window, else memory
    auto seq_at = [&](int32_t x, bool need) -> uint32_t {
        const int32_t ow = x - wb;
        const bool inw = ow >= 0 && ow + 4 <= kWinBytes;
        uint32_t v = 0;
        {   // every lane reads (a clamped index where it needs nothing): no exec-mask branch
            const int32_t oc = need && inw ? ow : 0;
            v = funnel(F.win[oc >> 2], F.win[(oc >> 2) + 1], (uint32_t)(oc & 3));
            if (!(need && inw)) v = 0;
        }
        if (__ballot(need && !inw)) {   // (waited for here, not where the paths join: that wait would
            if (need && !inw) v = ld_u32o(j, n32, x);   // also cover the previous batch's table stores)
            wait_vmem();
        }
        settle32(v);
        return v;
    };
    // window refill at base b: loads issued now (with a round trip's other loads), written after its wait
    uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
    auto refill_issue = [&](int32_t b) {
        r0 = ld16o(j, n32, b + 16 * lane);
        r1 = ld16o(j, n32, b + 1024 + 16 * lane);
    };
    auto refill_write = [&](int32_t b) {
        settle32(r0.x); settle32(r0.y); settle32(r0.z); settle32(r0.w);
        settle32(r1.x); settle32(r1.y); settle32(r1.z); settle32(r1.w);
        *(uint4*)&F.win[4 * lane] = r0;
        *(uint4*)&F.win[256 + 4 * lane] = r1;
        wb = b;
    };
    while (i < mflimit) {
        while ((i >> 15) > g) gt_scrub_epoch(F, lane, ++g);
        __builtin_amdgcn_s_setprio(3);
        if (c == 67 && S > 0) {
            // ================= hit batch: probes at i + kS, k < K, each assumed a hit of step S
            int K;
            {
                const int32_t lim = min(mflimit - 1, ((g + 1) << 15) - 1) - i;   // same epoch, before mflimit
                // (a division only near an epoch or block end: it is ~30 instructions on the chain)
                K = lim >= (kmax - 1) * S ? kmax : 1 + lim / S;
            }
            const bool act = lane < K;
            const int32_t p = i + lane * S;
            const uint32_t seq = seq_at(p, act);
            const uint32_t h = (seq * kP1) >> 18;
            int32_t cand = -1;
            bool dup = false;
            // the latest earlier probe of the batch with this hash: row_shr:d (lanes 0..7 share row 0)
#define LZ4MI_DUP(d)                                                   \
            {                                                          \
                const uint32_t hd = dpp<0x110 + d>(0xFFFFFFFFu, h);    \
                if (!dup && lane >= d && hd == h) {                    \
                    cand = p - d * S;                                  \
                    dup = true;                                        \
                }                                                      \
            }
            // repeated hashes are rare: a lane-id slot keyed by hash & 1023 finds whether the batch
            // has any (two lanes of one hash always collide; a collision of two hashes only sends
            // the batch through the exact checks below)
            bool anydup = false;
            if (K > 1) {
                volatile uint8_t* vs = F.slot;
                if (act) vs[h & 1023] = (uint8_t)lane;
                __builtin_amdgcn_wave_barrier();
                anydup = __ballot(act && vs[h & 1023] != (uint8_t)lane) != 0;
            }
            if (anydup) { LZ4MI_DUP(1) LZ4MI_DUP(2) LZ4MI_DUP(3) LZ4MI_DUP(4) LZ4MI_DUP(5) LZ4MI_DUP(6) LZ4MI_DUP(7) }
#undef LZ4MI_DUP
            static_assert(kSpecK == 8, "LZ4MI_DUP / LZ4MI_LATER cover distances 1..7");
            const uint32_t litv = npend ? load_lit() : 0u;
            CPROF(0);
            CPROF_COUNT(8, 1);
            uint32_t tlo = 0, tcd = 0;
            if (act && !dup) {
                tlo = T16[h];
                tcd = gt_code_of(F, h);
            }
            if (npend) {                                        // off the chain, while the reads are in flight
                __builtin_amdgcn_s_setprio(0);
                emit_batch(litv);
                __builtin_amdgcn_s_setprio(3);
            }
            // (the read's value is opaque until here: otherwise the compiler consumes it, and
            // waits for it, right after the load, before the emission)
            asm volatile("" : "+v"(tlo) :: "memory");
            CPROF(1);
            if (act && !dup) cand = gt16_decode(tlo, tcd, g);
            if (cand >= 0 && (p - cand < 1 || p - cand > 65535)) cand = -1;
            // ---- windows: lanes 8k .. 8k+7 hold 128 bytes at probe k and at its candidate
            const int gk = lane >> 3, gt = lane & 7;
            const int32_t gc = group_val(cand, gk);
            uint4 xa = make_uint4(0, 0, 0, 0), xb = xa;
            if (i + (K - 1) * S + kSpecW <= (int32_t)n32) {
                // every window of the batch lies in the block (all but the last batches): both loads
                // for every lane, from clamped addresses where the lane has no probe or candidate
                // (its bytes are not used), no per-lane bounds branches (tiles216 -0.6..1.2 %, mix
                // -2 %; table reads for every lane too: +2 %, profiles/r05z)
                const int32_t pa = gk < K ? i + gk * S : i, pb = gc >= 0 ? gc : i;
                __builtin_memcpy(&xa, j.src + pa + 16 * gt, 16);
                __builtin_memcpy(&xb, j.src + pb + 16 * gt, 16);
            } else if (gk < K) {
                xa = ld16o(j, n32, i + gk * S + 16 * gt);
                if (gc >= 0) xb = ld16o(j, n32, gc + 16 * gt);
            }
            const bool rf = (uint32_t)(i - wb) > 768u;          // the next batches' probes: window ahead
            if (rf) refill_issue(i);
            wait_vmem();
            if (rf) refill_write(i);
            CPROF(2);
            const uint32_t lm = (gk < K && gc >= 0) ? first_nz16(make_uint4(xa.x ^ xb.x, xa.y ^ xb.y, xa.z ^ xb.z, xa.w ^ xb.w))
                                                    : 0u;
            const uint64_t mm = __ballot(lm < 16);
            // lane k < K: bytes equal at probe k (m, 128 = the whole window)
            const uint32_t gm = (uint32_t)(mm >> (8 * (lane & 7))) & 0xFFu;
            const int ft = gm ? __builtin_ctz(gm) : 0;
            const uint32_t lmv = first_val(lm, mm, lane, ft);
            const int32_t m = gm ? 16 * ft + (int32_t)lmv : kSpecW;
            const bool hit = act && cand >= 0 && m >= 4;
            const bool lng = hit && m >= kSpecW && p + kSpecW < matchlimit;
            const int32_t e = p + (m < matchlimit - p ? m : matchlimit - p);
            const bool ok = hit && !lng && lane + 1 < K && e == p + S;
            const int J = __builtin_ctzll(__ballot(act && !ok));   // the first probe that ends the batch
            CPROF_COUNT(9, J);
            // probes 0 .. J happened: each inserts its position (the last of equal hashes)
            bool later = false;
#define LZ4MI_LATER(d)                                                 \
            {                                                          \
                const uint32_t hd = dpp<0x100 + d>(0xFFFFFFFFu, h);    \
                if (lane + d <= J && hd == h) later = true;            \
            }
            if (J > 0 && anydup) { LZ4MI_LATER(1) LZ4MI_LATER(2) LZ4MI_LATER(3) LZ4MI_LATER(4) LZ4MI_LATER(5) LZ4MI_LATER(6) LZ4MI_LATER(7) }
#undef LZ4MI_LATER
            insert(lane <= J && !later, h, p);
            const int32_t pJ = lane_val(p, J), cJ = lane_val(cand, J);
            const bool hitJ = (__ballot(hit) >> J) & 1ull;
            pd_p = p;
            pd_c = cand;
            pd_e = e;
            CPROF(3);
            if (hitJ) {
                CPROF_COUNT(9, 1);
                int32_t eJ = lane_val(e, J);
                if ((__ballot(lng) >> J) & 1ull)
                    eJ = pJ + kSpecW + (int32_t)match_extent(j, lane, pJ + kSpecW, cJ + kSpecW, matchlimit - (pJ + kSpecW));
                if (lane == J) pd_e = eJ;
                npend = J + 1;
                S = eJ - pJ;
                i = eJ;
                CPROF(4);
                continue;
            }
            // probe J missed (and inserted itself): the accepted hits go out, the miss chain
            // goes on at the next position
            npend = J;
            if (npend) emit_pending(load_lit());
            i = pJ + 1;                                         // (c = 67: step 1)
            c = 68;
            S = 0;
            CPROF(4);
            continue;
        }
        // ================= miss batch: the next 64 probes of the miss chain, starting at i
        if (npend) emit_pending(load_lit());
        CPROF_COUNT(10, 1);
        const int32_t pm_ = i + skip_span(c, (uint32_t)lane);
        const uint32_t step = (c + lane) >> 6;
        bool mact = pm_ < mflimit && (pm_ >> 15) == g;          // probes of the next epoch: the next batch
        const uint32_t mseq = seq_at(pm_, mact);
        const uint32_t mh = (mseq * kP1) >> 18;
        int nb = __popcll(__ballot(mact));
        {   // cut the batch before the first lane whose hash repeats an earlier lane's: a lane-id
            // map keyed by hash & 1023 flags the lanes that lost their slot; every true repeat
            // group has such a lane, whose hash is then compared with all lanes' (exact)
            volatile uint8_t* vs = F.slot;
            if (mact) vs[mh & 1023] = (uint8_t)lane;
            __builtin_amdgcn_wave_barrier();
            const bool lost = mact && vs[mh & 1023] != (uint8_t)lane;
            for (uint64_t fm = __ballot(lost); fm; fm &= fm - 1) {
                const uint32_t hf = lane_val(mh, __builtin_ctzll(fm));
                const uint64_t same = __ballot(mact && mh == hf);
                const uint64_t rest = same & (same - 1);       // all but the group's first lane
                if (rest) {
                    const int d = __builtin_ctzll(rest);
                    if (d < nb) nb = d;
                }
            }
            mact = mact && lane < nb;
        }
        CPROF(5);
        int32_t mc = -1;
        if (mact) {
            mc = gt16_decode(T16[mh], gt_code_of(F, mh), g);
            if (mc < 0 || pm_ - mc < 1 || pm_ - mc > 65535) mc = -1;
        }
        const uint32_t vw = mc >= 0 ? ld_u32o(j, n32, mc) : 0u;
        const int32_t inext = lane_val(pm_ + (int32_t)step, nb - 1);   // where a batch without a hit goes on
        const bool rf = (uint32_t)(i - wb) > 512u;              // the window for what follows either way
        if (rf) refill_issue(i);
        const uint64_t hm = __ballot(mc >= 0 && vw == mseq);
        if (rf) refill_write(i);
        const int nprobe = hm ? __builtin_ctzll(hm) + 1 : nb;
        insert(lane < nprobe, mh, pm_);                         // the probes that happen
        CPROF(6);
        if (!hm) {
            i = inext;
            c += nb;
            continue;
        }
        CPROF_COUNT(11, 1);
        const int mi = nprobe - 1;
        const int32_t pm = lane_val(pm_, mi), cm = lane_val(mc, mi);
        c = 67;
        const int32_t e1 = pm + 4 + (int32_t)match_extent(j, lane, pm + 4, cm + 4, matchlimit - (pm + 4));
        pd_p = pm;
        pd_c = cm;
        pd_e = e1;
        npend = 1;
        S = e1 - pm;
        i = e1;
        CPROF(7);
    }
#if LZ4MI_CPROFILE
    if (lane == 0)
        for (int k = 0; k < 12; ++k) atomicAdd(&g_cprof[k], (unsigned long long)cprof[k]);
#endif
    if (npend) emit_pending(load_lit());
    o = emit_tail(F, o, j, lane, anchor, n - anchor, nullptr);
    ring_flush(F, o, lane);
    for (int64_t t = o.flushed + lane; t < o.op; t += kWave) j.dst[t] = F.ring[t & RING_MASK(F)];
    return o.op;
}

#if LZ4MI_CTIMELINE
constexpr uint32_t kCtlMax = 16384;
__device__ unsigned long long g_ctl[2 * kCtlMax];   // per block: start, end (s_memrealtime, 100 MHz)
__device__ unsigned int g_ctl_id[2 * kCtlMax];      // per block: HW_ID, XCC_ID
#endif

template <class SH>
__global__ __launch_bounds__(64, 4) void lz4mi_compress_gts_kernel(CompArgs a, int32_t* tables) {
    __shared__ SH F;
    const uint32_t b = blockIdx.x;
    if (b >= a.nblocks) return;
#if LZ4MI_CTIMELINE
    const uint64_t tl_t0 = wall_clock64();
#endif
    CompJob j;
    j.src = a.in + a.in_off[b];
    j.src_total = a.in_len[b];
    j.start = 0;
    j.len = (int32_t)a.in_len[b];
    j.dst = a.out + a.out_off[b];
    j.dst_total = (uint64_t)a.in_len[b] + a.in_len[b] / 255u + 16u;
    j.dst_pos = 0;
    j.table = nullptr;
    const int64_t r = compress_block_gts(j, F, tables + (size_t)b * 16384, threadIdx.x);
    if (threadIdx.x == 0) a.out_len[b] = (uint32_t)r;
#if LZ4MI_CTIMELINE
    wait_vmem();
    const uint64_t tl_t1 = wall_clock64();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0 && b < kCtlMax) {
        g_ctl[2 * b] = tl_t0;
        g_ctl[2 * b + 1] = tl_t1;
        g_ctl_id[2 * b] = hw;
        g_ctl_id[2 * b + 1] = xcc;
    }
#endif
}


// ---------------------------------------------------------------------------
// Dependent blocks (the reference's LZ4.compress default, bufferCompress.js:182-236): the
// blocks of one frame in order with one hash table carried from block to block (the
// caller's Int32Array(16384), in and out: values = absolute position + 1, <= 0 empty), each
// block's output in its own slot. One wave walks the whole chain, so everything it touches
// is in LDS: the table (64 KiB, int32 as the reference's), the last 64 KiB of source plus up
// to 24 KiB ahead (the ring above), the output ring; the probes of a miss chain go as one
// 64-wide batch as in compress_block_gts. A sequence costs LDS round trips only (the batch
// encoder's two dependent global round trips per sequence, the old single-wave table kernel's
// one probe per step, are what made dependent frames 0.027 GB/s).
struct ChainShared {
    uint8_t ring[4096];   // output ring
    uint8_t slot[1024];   // batch duplicate-hash detection: lane ids keyed by hash & 1023
};
__shared__ int32_t g_ctab[16384];


// The dependent-block chain with compress_block_gts's batching (round 3): hit batches of up to
// kSpecK probes of one step, miss batches starting at the probe itself with the exact duplicate
// cut, one ring write per batch of sequences. Everything it reads is in LDS: the table (int32,
// the reference's values), the source ring (windows and probe bytes: aligned dword reads), the
// output ring; one wave walks the frame, so a batch's cost is its instruction latency.
__device__ __forceinline__ uint32_t ring_dw(uint32_t wi) { return ((const uint32_t*)g_ring)[wi]; }

// 16 source bytes at p: from the ring while it holds them, else global memory.
__device__ __forceinline__ uint4 rr16(const CompJob& j, const Ring& r, int64_t p) {
    if (p >= r.lo && p + 16 <= r.hi) {
        constexpr uint32_t W = kRingBytes / 4;
        const uint32_t q = (uint32_t)(p % kRingBytes), w0 = q >> 2, sh = q & 3;
        uint32_t d[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t x = w0 + k;
            d[k] = ring_dw(x >= W ? x - W : x);
        }
        return make_uint4(funnel(d[0], d[1], sh), funnel(d[1], d[2], sh), funnel(d[2], d[3], sh), funnel(d[3], d[4], sh));
    }
    return ld16(j, p);
}
__device__ __forceinline__ uint32_t rr32(const CompJob& j, const Ring& r, int64_t p) {
    if (p >= r.lo && p + 4 <= r.hi) {
        constexpr uint32_t W = kRingBytes / 4;
        const uint32_t q = (uint32_t)(p % kRingBytes), w0 = q >> 2;
        const uint32_t w1 = w0 + 1 >= W ? 0u : w0 + 1;
        return funnel(ring_dw(w0), ring_dw(w1), q & 3);
    }
    return ld_u32(j, p);
}

// match_extent with its first 256 bytes read from the ring (one step of 4 bytes per lane).
__device__ int64_t match_extent_ring(const CompJob& j, const Ring& r, int lane, int64_t a, int64_t b, int64_t lim) {
    const uint32_t x = rr32(j, r, a + 4 * lane) ^ rr32(j, r, b + 4 * lane);
    const uint64_t m = __ballot(x != 0);
    if (m) {
        const int fl = __builtin_ctzll(m);
        const int64_t f = 4 * fl + (__builtin_ctz(lane_val(x, fl)) >> 3);
        return f < lim ? f : lim;
    }
    if (lim <= 4 * kWave) return lim;
    return 4 * kWave + match_extent(j, lane, a + 4 * kWave, b + 4 * kWave, lim - 4 * kWave);
}

__device__ int64_t compress_block_chain2(const CompJob& j, ChainShared& F, int lane, Ring& r) {
    int32_t* T = g_ctab;
    const int32_t start = j.start, end = j.start + j.len;
    const int32_t mflimit = end - 12, matchlimit = end - 5;
    FastOut o{j.dst, 0, 0};
    int32_t i = start, anchor = start;
    uint32_t c = 67;
    int32_t S = 0;
    const int kmax = kSpecK;
    int npend = 0;
    int32_t pd_p = 0, pd_c = 0, pd_e = 0;
    auto emit_pending = [&](uint32_t litv) {
        for (int k = 0; k < npend; ++k) {
            const int32_t pm = lane_val(pd_p, k), cm = lane_val(pd_c, k), e = lane_val(pd_e, k);
            emit_seq<ChainShared, SrcR>(F, o, j, lane, anchor, pm, (uint32_t)(pm - cm), e - pm - 4, &r, true, litv);
            anchor = e;
        }
        npend = 0;
    };
    auto load_lit = [&]() -> uint32_t {
        const int32_t lit0 = lane_val(pd_p, 0) - anchor;
        const bool ld = lit0 > 0 && lit0 < 15 && lane >= 1 && lane <= lit0;
        return ld ? SrcR::byte(j, &r, anchor + lane - 1) : 0u;
    };
    auto emit_batch = [&](uint32_t litv) {   // as compress_block_gts's
        const int32_t lit0 = lane_val(pd_p, 0) - anchor;
        const int32_t mcode = pd_e - pd_p - 4;
        const bool mine = lane < npend;
        if (lit0 >= 15 || __ballot(mine && mcode >= 15 + 255)) {
            emit_pending(litv);
            return;
        }
        const int32_t lit = lane == 0 ? lit0 : 0;
        const uint32_t size = mine ? 3u + (uint32_t)lit + (mcode >= 15 ? 1u : 0u) : 0u;
        uint32_t incl = size;
        incl += dpp<kRowShr1>(0u, incl);
        incl += dpp<kRowShr2>(0u, incl);
        incl += dpp<kRowShr4>(0u, incl);
        const uint32_t st = incl - size;
        const int32_t total = (int32_t)lane_val(incl, npend - 1);
        ring_seqs(F, o, lane, npend, lit0, mcode, (uint32_t)(pd_p - pd_c), st, total, litv);
        anchor = lane_val(pd_e, npend - 1);
        npend = 0;
    };
    while (i < mflimit) {
        if (r.hi - i < kRingAhead) ring_advance(j, r, lane, i);
        if (c == 67 && S > 0) {
            // ================= hit batch
            int K = __popcll(__ballot(lane < kmax && lane * S <= mflimit - 1 - i));
            const bool act = lane < K;
            const int32_t p = i + lane * S;
            const uint32_t seq = act ? rr32(j, r, p) : 0u;
            const uint32_t h = (seq * kP1) >> 18;
            int32_t cand = -1;
            bool dup = false;
#define LZ4MI_DUP(d)                                                   \
            {                                                          \
                const uint32_t hd = dpp<0x110 + d>(0xFFFFFFFFu, h);    \
                if (!dup && lane >= d && hd == h) {                    \
                    cand = p - d * S;                                  \
                    dup = true;                                        \
                }                                                      \
            }
            if (K > 1) { LZ4MI_DUP(1) LZ4MI_DUP(2) LZ4MI_DUP(3) LZ4MI_DUP(4) LZ4MI_DUP(5) LZ4MI_DUP(6) LZ4MI_DUP(7) }
#undef LZ4MI_DUP
            if (act && !dup) {
                const int32_t old = T[h];
                cand = old - 1;
                if (old <= 0) cand = -1;
            }
            if (cand >= 0 && (cand == p || (uint32_t)(p - cand) > 65535u)) cand = -1;
            if (npend) emit_batch(load_lit());
            const int gk = lane >> 3, gt = lane & 7;
            const int32_t gc = group_val(cand, gk);
            uint4 xa = make_uint4(0, 0, 0, 0), xb = xa;
            if (gk < K) {
                xa = rr16(j, r, (int64_t)i + gk * S + 16 * gt);
                if (gc >= 0) xb = rr16(j, r, (int64_t)gc + 16 * gt);
            }
            const uint32_t lm = (gk < K && gc >= 0) ? first_nz16(make_uint4(xa.x ^ xb.x, xa.y ^ xb.y, xa.z ^ xb.z, xa.w ^ xb.w))
                                                    : 0u;
            const uint64_t mm = __ballot(lm < 16);
            const uint32_t gm = (uint32_t)(mm >> (8 * (lane & 7))) & 0xFFu;
            const int ft = gm ? __builtin_ctz(gm) : 0;
            const uint32_t lmv = first_val(lm, mm, lane, ft);
            const int32_t m = gm ? 16 * ft + (int32_t)lmv : kSpecW;
            const bool hit = act && cand >= 0 && m >= 4;
            const bool lng = hit && m >= kSpecW && p + kSpecW < matchlimit;
            const int32_t e = p + (m < matchlimit - p ? m : matchlimit - p);
            const bool ok = hit && !lng && lane + 1 < K && e == p + S;
            const int J = __builtin_ctzll(__ballot(act && !ok));
            bool later = false;
#define LZ4MI_LATER(d)                                                 \
            {                                                          \
                const uint32_t hd = dpp<0x100 + d>(0xFFFFFFFFu, h);    \
                if (lane + d <= J && hd == h) later = true;            \
            }
            if (J > 0) { LZ4MI_LATER(1) LZ4MI_LATER(2) LZ4MI_LATER(3) LZ4MI_LATER(4) LZ4MI_LATER(5) LZ4MI_LATER(6) LZ4MI_LATER(7) }
#undef LZ4MI_LATER
            __builtin_amdgcn_wave_barrier();
            if (lane <= J && !later) T[h] = p + 1;
            __builtin_amdgcn_wave_barrier();
            const int32_t pJ = lane_val(p, J), cJ = lane_val(cand, J);
            const bool hitJ = (__ballot(hit) >> J) & 1ull;
            pd_p = p;
            pd_c = cand;
            pd_e = e;
            if (hitJ) {
                int32_t eJ = lane_val(e, J);
                if ((__ballot(lng) >> J) & 1ull)
                    eJ = pJ + kSpecW + (int32_t)match_extent_ring(j, r, lane, pJ + kSpecW, cJ + kSpecW, matchlimit - (pJ + kSpecW));
                if (lane == J) pd_e = eJ;
                npend = J + 1;
                S = eJ - pJ;
                i = eJ;
                continue;
            }
            npend = J;
            if (npend) emit_batch(load_lit());
            i = pJ + 1;
            c = 68;
            S = 0;
            continue;
        }
        // ================= miss batch
        if (npend) emit_batch(load_lit());
        const int32_t pm_ = i + skip_span(c, (uint32_t)lane);
        const uint32_t step = (c + lane) >> 6;
        bool mact = pm_ < mflimit;
        const uint32_t mseq = mact ? SrcR::u32(j, &r, pm_) : 0u;
        const uint32_t mh = (mseq * kP1) >> 18;
        int nb = __popcll(__ballot(mact));
        {
            volatile uint8_t* vs = F.slot;
            if (mact) vs[mh & 1023] = (uint8_t)lane;
            __builtin_amdgcn_wave_barrier();
            const bool lost = mact && vs[mh & 1023] != (uint8_t)lane;
            for (uint64_t fm = __ballot(lost); fm; fm &= fm - 1) {
                const uint32_t hf = lane_val(mh, __builtin_ctzll(fm));
                const uint64_t same = __ballot(mact && mh == hf);
                const uint64_t rest = same & (same - 1);
                if (rest) {
                    const int d = __builtin_ctzll(rest);
                    if (d < nb) nb = d;
                }
            }
            mact = mact && lane < nb;
        }
        int32_t mc = -1;
        if (mact) {
            const int32_t ov = T[mh];
            mc = ov - 1;
            if (ov <= 0 || mc == pm_ || (uint32_t)(pm_ - mc) > 65535u) mc = -1;
        }
        const uint32_t vw = mc >= 0 ? SrcR::u32(j, &r, mc) : 0u;
        const uint64_t hm = __ballot(mc >= 0 && vw == mseq);
        const int nprobe = hm ? __builtin_ctzll(hm) + 1 : nb;
        __builtin_amdgcn_wave_barrier();
        if (lane < nprobe) T[mh] = pm_ + 1;
        __builtin_amdgcn_wave_barrier();
        if (!hm) {
            i = lane_val(pm_ + (int32_t)step, nb - 1);
            c += nb;
            continue;
        }
        const int mi = nprobe - 1;
        const int32_t pm = lane_val(pm_, mi), cm = lane_val(mc, mi);
        c = 67;
        const int32_t e1 = pm + 4 + (int32_t)match_extent_ring(j, r, lane, pm + 4, cm + 4, matchlimit - (pm + 4));
        pd_p = pm;
        pd_c = cm;
        pd_e = e1;
        npend = 1;
        S = e1 - pm;
        i = e1;
    }
    if (npend) emit_batch(load_lit());
    o = emit_tail<ChainShared, SrcR>(F, o, j, lane, anchor, end - anchor, &r);
    ring_flush(F, o, lane);
    for (int64_t t = o.flushed + lane; t < o.op; t += kWave) j.dst[t] = F.ring[t & RING_MASK(F)];
    return o.op;
}

struct ChainArgs {
    const uint8_t* src;
    uint64_t src_total;
    int32_t start, len, bsize;
    int32_t* table;
    uint8_t* out;
    const uint64_t* out_off;
    uint32_t* comp_len;
    uint32_t nblocks;
};

__global__ __launch_bounds__(64) void lz4mi_compress_chain_kernel(ChainArgs a) {
    __shared__ ChainShared F;
    const int lane = threadIdx.x;
    for (int k = lane; k < 16384; k += kWave) g_ctab[k] = a.table[k];
    __syncthreads();
    int64_t lo = (int64_t)a.start - 65536;
    lo = lo < 0 ? 0 : (lo & ~(int64_t)15);
    Ring r{lo, lo};
    for (uint32_t b = 0; b < a.nblocks; ++b) {
        const int64_t s0 = (int64_t)a.start + (int64_t)b * a.bsize;
        const int64_t rest = (int64_t)a.start + a.len - s0;
        const int32_t n = (int32_t)(rest < a.bsize ? rest : a.bsize);
        CompJob j{a.src, a.src_total, (int32_t)s0, n, a.out + a.out_off[b],
                  (uint64_t)n + (uint64_t)n / 255u + 16u, 0, nullptr};
        const int64_t w = compress_block_chain2(j, F, lane, r);
        if (lane == 0) a.comp_len[b] = (uint32_t)w;
    }
    __syncthreads();
    for (int k = lane; k < 16384; k += kWave) a.table[k] = g_ctab[k];
}

}  // namespace lz4mi

#if LZ4MI_CTIMELINE
// The last batch-encoder launch's per-block timeline (as lz4mi_debug_timeline for the decoder).
extern "C" int lz4mi_debug_ctimeline(unsigned long long* t, unsigned int* id, unsigned int n) {
    if (n > lz4mi::kCtlMax) n = lz4mi::kCtlMax;
    if (hipMemcpyFromSymbol(t, HIP_SYMBOL(lz4mi::g_ctl), sizeof(unsigned long long) * 2 * n) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(id, HIP_SYMBOL(lz4mi::g_ctl_id), sizeof(unsigned int) * 2 * n) == hipSuccess ? 0 : -1;
}
#endif

#if LZ4MI_CPROFILE
extern "C" int lz4mi_debug_cprof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lz4mi::g_cprof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(lz4mi::g_cprof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

extern "C" hipError_t lz4mi_launch_compress(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                            uint8_t* out, const uint64_t* out_off, uint32_t* out_len,
                                            uint32_t nblocks, int32_t* tables, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    lz4mi::CompArgs a{};
    a.in = in; a.in_off = in_off; a.in_len = in_len; a.out = out; a.out_off = out_off; a.out_len = out_len;
    a.nblocks = nblocks;
    // speculative hit-chain batch encoder, 16 blocks per CU; `tables` = per-block scratch
    if (nblocks <= lz4mi::kLdsTableMaxBlocks)   // one resident round at 3 blocks per CU: the table in LDS
        hipLaunchKernelGGL(lz4mi::lz4mi_compress_gts_kernel<lz4mi::GtsSharedL>, dim3(nblocks), dim3(64), 0, stream,
                           a, tables);
    else
        hipLaunchKernelGGL(lz4mi::lz4mi_compress_gts_kernel<lz4mi::GtsShared>, dim3(nblocks), dim3(64), 0, stream,
                           a, tables);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_compress_chain(const uint8_t* src, uint64_t src_total, int32_t start, int32_t len,
                                                  int32_t bsize, int32_t* table, uint8_t* out, const uint64_t* out_off,
                                                  uint32_t* comp_len, uint32_t nblocks, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    lz4mi::ChainArgs a{src, src_total, start, len, bsize, table, out, out_off, comp_len, nblocks};
    hipLaunchKernelGGL(lz4mi::lz4mi_compress_chain_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}
