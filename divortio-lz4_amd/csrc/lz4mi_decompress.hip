// lz4mi_decompress.hip — LZ4 raw-block decoder for MI355X (gfx950).
//
// Replaces decompressBlock (reference src/block/blockDecompress.js:30-275) for
// batches of independent blocks. Semantics follow the reference exactly for
// spec-valid input (positions absolute in `out`, dictionary below out[0],
// clipped match writes, the four error strings); LZ4MI_JS_COMPAT selects the
// serial kernel (lz4mi_decompress_serial.hip), which also reproduces the
// reference's double-copy-tail rewrite.
//
// One wave64 per block, all 4096 blocks of a batch resident at once
// (< 10 KiB LDS, <= 128 VGPRs -> 16 waves per CU). Per 1 KiB chunk of the
// compressed stream:
//  1. Stage it (+64 B lookahead) in LDS.
//  2. next(p) of every position, branch-free (length fields of one extension
//     byte; longer ones through a ballot-gated exact loop) into an LDS table.
//  3. Speculative walks: lane l walks next() from 256 bytes before its 16-byte
//     segment and records the tokens it visits in the segment; LZ4 token
//     chains resynchronise within a few steps, so walks are almost always on
//     the true chain. Certification left to right by ballot: the first lane
//     whose left neighbour's exit is not on its walk re-walks from it (its
//     neighbour is settled). The result is the exact serial parse. Walks
//     start 256 bytes back: inside long literal runs a walk can take a while
//     to fall onto the true chain, and every unsettled lane costs a pass.
//  4. Sequence table in LDS (literal source, lengths, offset, output start by
//     wave prefix sums) and errors in the reference's order.
//  5. Output, sequence-parallel (lane l takes sequence 64i+l), every run
//     written with exact-width unaligned 16/8/4/2/1-byte pieces (the last
//     16-byte piece of a run overlaps its predecessor instead of spilling),
//     so lanes never touch each other's bytes:
//       round 1: all literal runs (from LDS) and every match whose source
//                lies entirely in output finished by earlier chunks;
//       round r: after the previous round's stores are complete, every
//                pending match whose source range meets no pending match.
//     The earliest pending match is always ready, so the rounds terminate;
//     on typical data two or three suffice. Matches are read straight from
//     the output (L2, bypassing L1); an overlapping match (offset < length)
//     is read through its period: a 16-byte window that wraps is merged from
//     two loads, periods under 16 bytes are expanded in registers. Runs
//     longer than 128 bytes are written by the whole wave.
//  6. A sequence whose parse leaves the staged window (long literal runs or
//     length varints: incompressible or highly repetitive data) is parsed from
//     global memory with wave-wide 255-run scans and written by the whole
//     wave, literal run first, then (after it is stored) the match run.
#include "../../include/lz4mi.h"
#include "lz4mi_common.h"
#include "lz4mi_decompress.h"

#ifndef LZ4MI_LL_ADAPT
#define LZ4MI_LL_ADAPT 127   // long literal runs: s_sleep argument after every 4 KiB step while blocks with a
                             // compression ratio above 2 run on the same XCD (0: no pacing; A/B switch)
#endif
#ifndef LZ4MI_ORDER
#define LZ4MI_ORDER 1   // batches dispatched latency-bound blocks first, most compressed bytes first; 2: the
                        // latency-bound blocks first in index order; 0: index order (A/B switch)
#endif
#ifndef LZ4MI_ABLATE
#define LZ4MI_ABLATE 0   // timing-only variants (tools/): 1 = no output, 2 = parse only, 3 = next table only,
                         // 4 = output loads without stores, 5 = output stores without loads, 6 = round 1 only
#endif

#ifndef LZ4MI_TIMELINE
#define LZ4MI_TIMELINE 0   // diagnostic build (tools/timeline.py): every block's start / end time, CU, XCD
#endif

#ifndef LZ4MI_PROFILE
#define LZ4MI_PROFILE 0  // timing-only variant (tools/): per-phase wall-clock accumulation
#endif

namespace lz4mi {

// One 16-byte output piece (any alignment: gfx950 runs in unaligned mode), default cache
// policy: the written lines stay in L2 for the history reads that follow (nontemporal
// stores, which skip L2, made tiles216 2x slower: 40.6 vs 20.5 ms).
__device__ __forceinline__ void out16(uint8_t* p, const uint4& v) { __builtin_memcpy(p, &v, 16); }
// 16 bytes read / written once (streamed: nontemporal, so they do not evict the history lines
// the matches read back from L2)
typedef uint32_t u32x4_nt __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ uint4 ld16_nt(const uint8_t* p) {
    const u32x4_nt t = __builtin_nontemporal_load((const u32x4_nt*)p);
    return make_uint4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ void st16_nt(uint8_t* p, const uint4& v) {
    const u32x4_nt t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, (u32x4_nt*)p);
}

#if LZ4MI_LL_ADAPT
__device__ unsigned int g_lat_active[8 * 32];   // per XCD (one 128-byte line each): latency-bound blocks running
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}
#endif

#if LZ4MI_TIMELINE
constexpr uint32_t kTlMax = 16384;
__device__ unsigned long long g_tl[2 * kTlMax];   // per block: start, end (s_memrealtime, 100 MHz)
__device__ unsigned int g_tl_id[2 * kTlMax];      // per block: HW_ID (wave, SIMD, CU, SH, SE), XCC_ID
#endif

#if LZ4MI_PROFILE
__device__ unsigned long long g_prof[24];
#define PROF(i)                              \
    do {                                     \
        const uint64_t t_ = wall_clock64();  \
        prof[i] += t_ - prof_t;              \
        prof_t = t_;                         \
    } while (0)
#define PROF_COUNT(i, n) (prof[i] += (n))
#else
#define PROF(i) ((void)0)
#define PROF_COUNT(i, n) ((void)0)
#endif

constexpr int kChunk = 1024;                  // compressed bytes parsed per step
constexpr int kPad = 64;                      // lookahead for sequences straddling the chunk end
constexpr int kLim = kChunk + kPad;           // chunk-relative bytes a regular sequence may touch
constexpr int kStageWords = (kLim + 28) / 4;  // + slack for 16-byte literal loads at the window end
constexpr int kMaxSeq = kChunk / 3 + 3;       // tokens starting in the chunk: every non-final sequence is >= 3 bytes
constexpr uint32_t kWarm = 512;               // speculative walks start this far before their segment
constexpr int kMaxVarint = 250;               // longer length varints go to the cut path (ml < 65536)
constexpr int32_t LZ4MI_ERR_RANGE_STATUS = LZ4MI_ERR_RANGE;   // (include/lz4mi.h)
constexpr uint32_t kEnd = 0x40000000u;        // chain ends (last sequence of the block)
constexpr uint32_t kStop = 0x40000001u;       // sequence cannot be parsed inside the window
constexpr int kWaveB = 2;                     // ... (whole-wave runs: streaming copies)
constexpr int kWaveB2 = 1;                    // ... (whole-wave periodic runs: two windows per piece)
constexpr int kLaneBytes = 256;               // longer runs are written by the whole wave (128: tiles216 +1.8 %)
constexpr int kPeriodBulk = 1024;             // longer periodic runs are generated from an LDS copy of the pattern
constexpr int32_t kLongLit = 4096;            // literal runs at least this long: long_literals()
constexpr uint64_t kXRatioMax = 32;           // XP: blocks of higher ratio are decoded by one wave
constexpr int kSegRestarts = 16;              // XP: a guess's walk starts over at most this often
constexpr uint32_t kSegWarm = 3072;           // XP: a segment's warm-up parse (tiles216: 99 % of wrong
                                              // starts join the token chain within 860 bytes)

struct DecShared {
    union {
        uint4 t_seq[kMaxSeq];     // per sequence: {output start (block-relative), literal source (chunk-
                                  //  relative) | literal length << 16, match offset | match length << 16
                                  //  (0: final literal-only sequence), source remapped by remap_src}
        struct {
            uint16_t nxt2[kChunk];   // parse: token 2 steps after p
            uint16_t nxt4[kChunk];   // parse: token 4 steps after p (warm-up walks)
        };
    };
    union {
        uint16_t nxt[kLim];       // parse: next-token table
        uint32_t pme[kLim / 2];   // output: ends of the pending matches
    };
    uint32_t pms[kMaxSeq];        // output: starts of the pending matches
    uint32_t stage[kStageWords];
};
static_assert(kLim / 2 >= kMaxSeq, "pending list must fit in the next-token table");
static_assert(kStageWords * 4 > kLim, "the table build reads s[q + 2] for offsets ending at kLim");
static_assert(offsetof(DecShared, stage) % 16 == 0 && offsetof(DecShared, pme) % 16 == 0, "16-byte aligned rows");

// LDS a whole-wave periodic run may copy its pattern into, by phase of the
// chunk: round 1 (the pending list is not built yet), rounds 2+ (the staged
// literals are all written), the cut sequence (all of it; with the F1 check on,
// all but the sequence tables the check reads afterwards).
struct PatBuf {
    uint32_t* w;
    int32_t bytes;
};
__device__ __forceinline__ PatBuf no_pat() { return PatBuf{nullptr, 0}; }   // literal runs
__device__ __forceinline__ PatBuf pat_round1(DecShared& S) { return PatBuf{S.pms, (int32_t)sizeof(S.pms)}; }
__device__ __forceinline__ PatBuf pat_rounds(DecShared& S) { return PatBuf{S.stage, (int32_t)sizeof(S.stage)}; }
__device__ __forceinline__ PatBuf pat_all(DecShared& S) { return PatBuf{(uint32_t*)&S, (int32_t)sizeof(DecShared)}; }
__device__ __forceinline__ PatBuf pat_cut(DecShared& S) {
    return PatBuf{S.pme, (int32_t)(sizeof(DecShared) - offsetof(DecShared, pme))};
}
static_assert(offsetof(DecShared, pms) == offsetof(DecShared, pme) + sizeof(uint32_t) * (kLim / 2) &&
              offsetof(DecShared, stage) == offsetof(DecShared, pms) + sizeof(uint32_t) * kMaxSeq,
              "the cut pattern buffer spans pme, pms and the stage");

struct Ctx {
    const uint8_t* blk;   // compressed block
    uint8_t* dst;         // output start of the block (out + out_off)
    int64_t out_off;      // absolute position of dst in `out`
    int32_t in_len;
    int32_t cap;          // writable bytes from dst
    const uint8_t* dict;
    int32_t dict_len;
    int isolate;
    int32_t ip;           // chunk start (block-relative compressed position)
    int64_t O;            // output start of the current table (block-relative)
};

// 16 bytes of base[0, len) at r0, zero past len (r0 < len).
__device__ __forceinline__ uint4 load16_tail(const uint8_t* base, int64_t r0, int64_t len) {
    uint4 v = make_uint4(0, 0, 0, 0);
    unsigned __int128 x = 0;
    if (len >= 16) {   // the last 16 bytes, shifted down
        __builtin_memcpy(&x, base + len - 16, 16);
        x >>= 8 * (uint32_t)(r0 - (len - 16));
    } else {
#pragma unroll 1
        for (int j = 0; r0 + j < len; ++j) x |= (unsigned __int128)base[r0 + j] << (8 * j);
    }
    __builtin_memcpy(&v, &x, 16);
    return v;
}

// Bytes [idx, idx + 16) of the staged chunk from five naturally aligned dword
// reads: a misaligned b64/b128 LDS access replays at ~64 LDS cycles, CU-wide
// (tools/probe/lds_unaligned.hip), aligned dwords do not.
__device__ __forceinline__ uint4 stage16(const uint32_t* stage, int32_t idx) {
    const uint32_t* w = stage + (idx >> 2);
    const uint32_t sh = (uint32_t)idx & 3u;
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
    return make_uint4(funnel(d0, d1, sh), funnel(d1, d2, sh), funnel(d2, d3, sh), funnel(d3, d4, sh));
}

// 16 compressed bytes at block-relative r0 (zero past the block end).
__device__ __forceinline__ uint4 stage_piece(const Ctx& c, int64_t r0) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + 16 <= c.in_len) __builtin_memcpy(&v, c.blk + r0, 16);
    else if (r0 < c.in_len) v = load16_tail(c.blk, r0, c.in_len);
    return v;
}

// ---------------------------------------------------------------- parsing
// Position of the token after the one at p (chunk-relative), or kEnd / kStop.
// Exact for any field lengths.
__device__ __forceinline__ uint32_t next_token(const uint8_t* s, uint32_t p, uint32_t rem) {
    if (p >= (uint32_t)kLim) return kStop;
    uint32_t tok = s[p];
    uint32_t q = p + 1;
    uint32_t ll = tok >> 4;
    if (ll == 15) {
        uint32_t b;
        do {
            if (q >= (uint32_t)kLim) return kStop;
            b = s[q++];
            ll += b;
        } while (b == 255);
    }
    q += ll;
    if (q >= rem) return q <= (uint32_t)kLim ? kEnd : kStop;   // literal-only final sequence
    if (q + 2 > (uint32_t)kLim) return kStop;
    q += 2;
    if ((tok & 15) == 15) {
        uint32_t b, n = 0;
        do {
            if (q >= (uint32_t)kLim || ++n > (uint32_t)kMaxVarint) return kStop;
            b = s[q++];
        } while (b == 255);
    }
    return q >= rem ? kEnd : q;
}

// Same, branch-free, for length fields of at most one extension byte each;
// `slow` is set when a field is longer (the caller then uses next_token).
__device__ __forceinline__ uint32_t next_fast(const uint8_t* s, uint32_t p, uint32_t rem, bool& slow) {
    const uint32_t t = s[p], b1 = s[p + 1];
    const uint32_t x1 = (t >> 4) == 15 ? 1u : 0u;
    const uint32_t ll = x1 ? 15u + b1 : t >> 4;
    const uint32_t q = p + 1 + x1 + ll;                        // offset position
    const uint32_t mb = s[q + 2 < (uint32_t)kLim ? q + 2 : 0u];
    const uint32_t x2 = (t & 15) == 15 ? 1u : 0u;
    const uint32_t n = q + 2 + x2;
    uint32_t v = n > (uint32_t)kLim ? kStop : (n >= rem ? kEnd : n);
    if (q >= rem) v = q <= (uint32_t)kLim ? kEnd : kStop;       // literal-only final sequence
    if (x1 && p + 1 >= (uint32_t)kLim) v = kStop;
    slow = (x1 && b1 == 255) || (x2 && mb == 255 && q < rem);
    return v;
}

// The fast next-token table: positions 4w .. 4w+3 (w = lane + 64 r) from the stage
// dwords w and w+1, next = p + 1 + [literal ext] + literals + 2 + [match ext], i.e. every
// length field taken to be at most one extension byte. Valid while no field or next()
// can reach the block's end (rem > kFastRem). A literal field of 2+ bytes (ext byte 255)
// stops the chain there (0xFFFF); a match field of 2+ bytes is caught on the true tokens
// (table build) and the chunk re-parsed with the exact table. Values past the window stay
// raw (<= 1297): every walk ends at them, and a tail past kLim is a cut.
constexpr uint32_t kFastRem = kLim + 300;
__device__ __forceinline__ uint32_t next4_half(uint32_t t, uint32_t b1, uint32_t p) {
    const uint32_t hi = t >> 4;
    const uint32_t x1 = hi == 15 ? 1u : 0u;
    const uint32_t ll = x1 ? 15u + b1 : hi;
    const uint32_t x2 = (t & 15) == 15 ? 1u : 0u;
    const uint32_t n = p + 3 + x1 + x2 + ll;
    return (x1 && b1 == 255) ? 0xFFFFu : n;
}
// The lane index as a value the compiler cannot hoist out of the chunk loop: per-lane
// constants derived from it (p + 1, p + 2, ... of every row) would otherwise be computed
// once and kept in (spilled) registers, their reloads scratch loads that wait, in order,
// for every store still in flight.
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ void next_table_fast(const uint32_t* stage, uint16_t* nxt, int lane) {
    static_assert(kChunk % (4 * kWave) == 0, "whole dword rows per lane");
    lane = opaque(lane);
    uint32_t d0[kChunk / (4 * kWave)], d1[kChunk / (4 * kWave)];
#pragma unroll
    for (int r = 0; r < kChunk / (4 * kWave); ++r) {
        const uint32_t w = lane + kWave * r;
        d0[r] = stage[w];
        d1[r] = stage[w + 1];
    }
#pragma unroll
    for (int r = 0; r < kChunk / (4 * kWave); ++r) {
        const uint32_t w = lane + kWave * r, p = 4 * w;
        const uint32_t a = d0[r], b = d1[r];
        const uint32_t n0 = next4_half(a & 255, (a >> 8) & 255, p);
        const uint32_t n1 = next4_half((a >> 8) & 255, (a >> 16) & 255, p + 1);
        const uint32_t n2 = next4_half((a >> 16) & 255, a >> 24, p + 2);
        const uint32_t n3 = next4_half(a >> 24, b & 255, p + 3);
        *(uint2*)(nxt + p) = make_uint2(n0 | (n1 << 16), n2 | (n3 << 16));
    }
}

// out[p] = in[in[p]] (or in[p] when that is past the chunk): 4 positions per lane, the
// 16 gathers of a lane issued together.
__device__ __forceinline__ void jump_table(const uint16_t* in, uint16_t* out, int lane) {
    constexpr int R = kChunk / (4 * kWave);
    lane = opaque(lane);
    uint2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = *(const uint2*)(in + 4 * (lane + kWave * r));
    uint32_t y[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t a[4] = {v[r].x & 0xFFFFu, v[r].x >> 16, v[r].y & 0xFFFFu, v[r].y >> 16};
#pragma unroll
        for (int j = 0; j < 4; ++j) y[r][j] = a[j] < (uint32_t)kChunk ? in[a[j]] : a[j];
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        *(uint2*)(out + 4 * (lane + kWave * r)) = make_uint2(y[r][0] | (y[r][1] << 16), y[r][2] | (y[r][3] << 16));
}

// Registers loaded by global loads that an explicit wait_vmem() has already
// covered: redefine them opaquely so the compiler's wait insertion no longer
// tracks them (it would otherwise wait for every later store before their use).
__device__ __forceinline__ void settle(uint4& v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

__device__ __forceinline__ uint16_t enc_next(uint32_t v) {
    return (uint16_t)(v == kEnd ? 0xFFFEu : v == kStop ? 0xFFFFu : v);
}

__device__ __forceinline__ uint32_t next_of(const uint16_t* nxt, uint32_t p) {
    uint32_t v = nxt[p];
    return v >= 0xFFFEu ? (v == 0xFFFEu ? kEnd : kStop) : v;
}

struct SeqInfo {
    int32_t out, lit, ll, off, ml, rsrc;
};
__device__ __forceinline__ SeqInfo seq_of(uint4 v) {
    return SeqInfo{(int32_t)v.x, (int32_t)(v.y & 0xFFFF), (int32_t)(v.y >> 16), (int32_t)(v.z & 0xFFFF),
                   (int32_t)(v.z >> 16), (int32_t)v.w};
}
// one ds_read_b128: everything of sequence k
__device__ __forceinline__ SeqInfo seq_info(const DecShared& S, uint32_t k) { return seq_of(S.t_seq[k]); }

// History (earlier output of this wave) is read with plain loads: the CU's L1 sees
// the wave's own completed stores (every read of output follows an s_waitcnt on
// the stores that wrote it), and L2 keeps the lines. Nontemporal loads (used
// until round 2) cost tiles216 17 % (19.15 vs 15.87 ms, one process, same box).
__device__ __forceinline__ uint32_t hist_u8(const uint8_t* p) { return *p; }

// Byte of earlier output at block-relative position pos (dictionary below out[0]).
__device__ __forceinline__ uint32_t hist_byte(const Ctx& c, int64_t pos) {
    int64_t abs = c.out_off + pos;
    if (abs >= 0) return hist_u8(c.dst + pos);
    return c.dict ? c.dict[c.dict_len + abs] : 0u;
}

// ------------------------------------------------------------------ runs
// A run: n output bytes at y and where they come from.
enum : uint32_t {
    R_NONE = 0,
    R_LDS = 1,    // literal bytes in the staged chunk (src = stage byte index)
    R_COMP = 2,   // literal bytes in the compressed block in global memory (src = block position)
    R_HIST = 3,   // match: earlier output (src = its block-relative position), read through `period`
    R_BYTES = 4,  // match read byte by byte (dictionary, or within 16 bytes of a buffer edge)
};

struct Run {
    int32_t y, n, src, period;   // period = match offset when the match overlaps itself, else 0
    uint32_t kind;
};

__device__ __forceinline__ Run no_run() { return Run{0, 0, 0, 0, R_NONE}; }

// lane l's value (l wave-uniform): v_readlane, not an LDS permute
__device__ __forceinline__ int32_t lane_of(int32_t v, int l) { return (int32_t)__builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t lane_of(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l); }

__device__ __forceinline__ Run shfl_run(const Run& R, int l) {
    return Run{lane_of(R.y, l), lane_of(R.n, l), lane_of(R.src, l), lane_of(R.period, l), lane_of(R.kind, l)};
}

// The match run of a sequence whose match starts at ms; n = 0 when nothing is
// written (no match, or entirely past the capacity: the reference clips).
__device__ __forceinline__ Run match_run(const Ctx& c, int32_t ms, int32_t off, int32_t ml) {
    Run M{ms, 0, ms - off, off < ml ? off : 0, R_HIST};
    if (ml == 0 || ms >= c.cap) return M;
    M.n = (ms + ml > c.cap ? c.cap : ms + ml) - ms;
    // byte-wise: a dictionary source, a periodic source within 16 bytes of the
    // buffer start (its two-window pieces would read below it), or an output end
    // within 16 bytes (a plain source's 16-byte pieces stay inside [src, src + n))
    if (c.out_off + M.src < 0 || (M.period && c.out_off + M.src < 16) || ms + 16 > c.cap) M.kind = R_BYTES;
    return M;
}
// One past the last output byte a match run reads.
__device__ __forceinline__ int32_t match_src_end(const Run& M) { return M.period ? M.y : M.src + M.n; }

__device__ __forceinline__ int run_pieces(int32_t n) {
    return n >= 16 ? (n + 15) >> 4 : (n <= 0 ? 0 : ((n & (n - 1)) == 0 ? 1 : 2));
}

// One store of a run: w bytes at y. mode 1 = window a, 2 = bytes [0, k) from
// window a and the rest from window b (a period that wraps), 3 = period
// `period` < w expanded from the 16 bytes at a starting at phase k,
// 4 = byte-wise (a = run offset, b = source start).
struct Piece {
    int32_t y, a, b, k, period;
    uint32_t w, mode, kind;
};

__device__ __forceinline__ Piece plan_piece(const Run& R, int p) {
    Piece P{0, 0, 0, 16, 0, 16u, 0u, R.kind};
    if (R.kind == R_NONE || p >= run_pieces(R.n)) return P;
    int32_t d;
    if (R.n >= 16) {
        P.w = 16;
        d = 16 * p < R.n - 16 ? 16 * p : R.n - 16;
    } else {
        P.w = R.n >= 8 ? 8u : R.n >= 4 ? 4u : R.n >= 2 ? 2u : 1u;
        d = p ? R.n - (int32_t)P.w : 0;
    }
    P.y = R.y + d;
    P.period = R.period;
    if (R.kind == R_BYTES) {
        P.mode = 4;
        P.a = d;
        P.b = R.src;
    } else if (R.period == 0) {
        P.mode = 1;
        P.a = R.src + d;
    } else {
        const int32_t per = R.period, r = d % per;
        if (per < (int32_t)P.w) {
            P.mode = 3;
            P.a = R.src;
            P.k = r;
        } else if (r + (int32_t)P.w <= per) {
            P.mode = 1;
            P.a = R.src + r;
        } else {
            P.mode = 2;
            P.a = R.src + r;
            P.b = R.src + r - per;    // >= src - 15: match_run keeps 16 bytes of margin
            P.k = per - r;
        }
    }
    return P;
}

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store_w(uint8_t* p, uint4 v, uint32_t w) {
    if (w == 16) {
        __builtin_memcpy(p, &v, 16);
    } else if (w == 8) {
        __builtin_memcpy(p, &v, 8);
    } else if (w == 4) {
        __builtin_memcpy(p, &v.x, 4);
    } else if (w == 2) {
        uint16_t t = (uint16_t)v.x;
        __builtin_memcpy(p, &t, 2);
    } else {
        *p = (uint8_t)v.x;
    }
}

// bytes [0, k) from a, the rest from b
__device__ __forceinline__ uint32_t pick(uint32_t a, uint32_t b, int32_t k) {
    if (k >= 4) return a;
    if (k <= 0) return b;
    uint32_t m = (1u << (8 * k)) - 1u;
    return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint4 pick4(uint4 a, uint4 b, int32_t k) {
    return make_uint4(pick(a.x, b.x, k), pick(a.y, b.y, k - 4), pick(a.z, b.z, k - 8), pick(a.w, b.w, k - 12));
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

__device__ __forceinline__ void bytes_piece(const Ctx& c, int32_t y, int32_t a, int32_t src, uint32_t w, int32_t per) {
    uint32_t o[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < w; ++j) {
        const int32_t d = a + (int32_t)j;
        const uint32_t v = hist_byte(c, (int64_t)src + (per ? d % per : d));
        o[j >> 2] |= v << ((j & 3) * 8);
    }
    store_w(c.dst + y, make_uint4(o[0], o[1], o[2], o[3]), w);
}

// A pipeline slot: one store of w bytes at y; mode 1 = window at a, 2 = bytes
// [0, k) from the window at a, the rest from the window at a - per (a period
// that wraps), 3 = period per < 16 expanded from the window at a from phase k.
// Windows are always 16 bytes (match_run / the staging slack keep them in bounds).
struct Slot {
    int32_t y, a, k, per;
    uint32_t wm;     // width | mode << 8
};

__device__ __forceinline__ Slot no_slot() { return Slot{0, 0, 0, 0, 0u}; }

// Slot of piece p of run R (R is not R_BYTES; wrapping periods only when TWO).
__device__ __forceinline__ Slot slot_of(const Run& R, int p) {
    const Piece P = plan_piece(R, p);
    return Slot{P.y, P.a, P.k, P.period, P.mode ? (P.w | (P.mode << 8)) : 0u};
}
template <uint32_t KIND>
__device__ __forceinline__ uint4 load16(const Ctx& c, const DecShared& S, int32_t a) {
    uint4 v;
    if (KIND == R_LDS) {
        v = stage16(S.stage, a);
    } else if (KIND == R_COMP) {
        __builtin_memcpy(&v, c.blk + a, 16);
    } else {
        const u32x4_t t = *(const u32x4_t*)(c.dst + a);
        v = make_uint4(t.x, t.y, t.z, t.w);
    }
    return v;
}

template <uint32_t KIND, bool TWO, int NB>
__device__ __forceinline__ void load_slots(const Ctx& c, const DecShared& S, const Slot (&s)[NB], uint4 (&A)[NB],
                                           uint4 (&B)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        if (LZ4MI_ABLATE == 5) { A[j] = make_uint4(0, 0, 0, 0); B[j] = A[j]; continue; }
        if (s[j].wm >> 8) A[j] = load16<KIND>(c, S, s[j].a);
        if (TWO && (s[j].wm >> 8) == 2) B[j] = load16<KIND>(c, S, s[j].a - s[j].per);
    }
}

template <bool TWO, int NB>
__device__ __forceinline__ void store_slots(const Ctx& c, DecShared& S, const Slot (&s)[NB], const uint4 (&A0)[NB],
                                            const uint4 (&B0)[NB]) {
    uint4 A[NB], B[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        A[j] = A0[j];          // (consumed on every path: see lane_store)
        settle(A[j]);
        if (TWO) {
            B[j] = B0[j];
            settle(B[j]);
        }
        const uint32_t mode = s[j].wm >> 8;
        if (!mode) continue;
        uint4 v = A[j];
        if (TWO && mode == 2) v = pick4(A[j], B[j], s[j].k);
        else if (mode == 3) v = expand_period(A[j], s[j].k, s[j].per);
        if (LZ4MI_ABLATE == 4) {      // timing only: loads kept alive, no stores
            if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) S.pms[0] = 1;
            continue;
        }
        const uint32_t w = s[j].wm & 255u;
        if (w == 16) out16(c.dst + s[j].y, v);
        else store_w(c.dst + s[j].y, v, w);
    }
}

template <int NB>
__device__ __forceinline__ bool any_slot(const Slot (&s)[NB]) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) m |= s[j].wm;
    return m != 0;
}

// Software-pipelined copy: the loads of stage n+1 are issued before the stores
// of stage n, so no load waits behind a store it does not depend on (gfx9
// counts loads and stores in one in-order vmcnt). Gen::fill(Slot (&)[NB])
// hands out this lane's next pieces (sources already complete).
template <uint32_t KIND, bool TWO, int NB, class Gen>
__device__ __forceinline__ void pipe(const Ctx& c, DecShared& S, Gen& g) {
    // (every issued load is consumed by a store before the function returns: a load left
    // in flight at the exit would make the next write of its registers wait for vmcnt(0),
    // i.e. for every store in flight)
    Slot s0[NB], s1[NB];
    uint4 a0[NB], b0[NB], a1[NB], b1[NB];
    g.fill(s0);
    if (!__ballot(any_slot<NB>(s0))) return;
    load_slots<KIND, TWO, NB>(c, S, s0, a0, b0);
    for (;;) {
        g.fill(s1);
        if (!__ballot(any_slot<NB>(s1))) {
            store_slots<TWO, NB>(c, S, s0, a0, b0);
            return;
        }
        load_slots<KIND, TWO, NB>(c, S, s1, a1, b1);
        store_slots<TWO, NB>(c, S, s0, a0, b0);
        g.fill(s0);
        if (!__ballot(any_slot<NB>(s0))) {
            store_slots<TWO, NB>(c, S, s1, a1, b1);
            return;
        }
        load_slots<KIND, TWO, NB>(c, S, s0, a0, b0);
        store_slots<TWO, NB>(c, S, s1, a1, b1);
    }
}

// Pieces of the whole wave over one run: piece p0 + lane + 64 j.
template <int NB>
struct WaveGen {
    Run R;
    int np, p0, lane;
    __device__ __forceinline__ void fill(Slot (&s)[NB]) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int p = p0 + lane + kWave * j;
            s[j] = p < np ? slot_of(R, p) : no_slot();
        }
        p0 += kWave * NB;
    }
};

// SeqInfo::rsrc (t_seq .w) of a sequence whose match source was mapped to finished output:
// the source + kMemoBase when the whole match was mapped (remap_src follows it in one step for
// later rows), + kSplitBase when only its part after a literal prefix was (0: not mapped).
constexpr int32_t kMemoBase = 0x40000000, kSplitBase = 0x20000000;

// A match source [rs, re) inside this table's output, mapped back through the
// sequences that wrote it (out[y] = out[y - off] inside a match): 1 = it now
// lies in output finished by earlier chunks, 2 = in sequence j's literal run
// (*lds = its stage index), 0 = it straddles sequences / the table start.
// 3 (with `split`): it starts in sequence j's literal run and goes on into j's match:
// its first *nlit bytes are literal bytes at stage index *lds, the rest maps on to
// [rs, re) (finished output) — tiles216's usual reason for a later round (72 % of them).
// S.nxt doubles as an output -> sequence map during round 1: entry b is the
// sequence holding output O + (b << sh) (built by the kernel before round 1).
__device__ __forceinline__ int remap_src(const Ctx& c, const DecShared& S, uint32_t nseq, uint32_t sh, int32_t& rs,
                                         int32_t& re, int32_t& lds, int32_t& nlit, bool split) {
    nlit = 0;
    for (int d = 0; d < 8; ++d) {
        if (re <= (int32_t)c.O) return nlit ? 3 : 1;
        if (rs < (int32_t)c.O) return 0;
        uint32_t lo = S.nxt[(uint32_t)(rs - (int32_t)c.O) >> sh];   // last sequence starting at or before rs
        SeqInfo q = seq_info(S, lo);
        int32_t nx = lo + 1 < nseq ? (int32_t)S.t_seq[lo + 1].x : INT32_MAX;   // (read together with q)
        while (nx <= rs) {
            ++lo;
            q = seq_info(S, lo);
            nx = lo + 1 < nseq ? (int32_t)S.t_seq[lo + 1].x : INT32_MAX;
        }
        const int32_t t0 = q.out;
        const int32_t ms = t0 + q.ll;
        if (re <= ms) {
            if (nlit) return 0;   // (one split at most)
            lds = q.lit + (rs - t0);
            return 2;
        }
        if (rs < ms) {
            if (!split || nlit || ms - rs > 255 || re > ms + q.ml) return 0;
            lds = q.lit + (rs - t0);
            nlit = ms - rs;
            rs = ms;
        }
        if (re > ms + q.ml) return 0;
        if (q.rsrc >= kMemoBase - 65536 && q.rsrc < kMemoBase + (1 << 27)) {
            // sequence lo's match was itself mapped (by an earlier row) to finished output:
            // follow that mapping in one step instead of hop by hop
            const int32_t base = q.rsrc - kMemoBase - ms;
            rs += base;
            re += base;
            continue;
        }
        rs -= q.off;
        re -= q.off;
    }
    return 0;
}

// One 16-byte piece of a match copy: y, source, width.
struct LSlot {
    int32_t y, a;
    uint32_t w;   // 0 = none
};

template <int NB>
__device__ __forceinline__ void lane_store(const Ctx& c, DecShared& S, const LSlot (&s)[NB], const uint4 (&A0)[NB]) {
    uint4 A[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        // consumed on every path (a counted wait here): a load whose register is left
        // pending on the paths that skip its store would make the next chunk's first write
        // of that register wait for vmcnt(0) — for every store in flight
        A[j] = A0[j];
        settle(A[j]);
        if (!s[j].w) continue;
        if (LZ4MI_ABLATE == 4) {
            if ((A[j].x ^ A[j].y) == 0x9E3779B9u) S.pms[0] = 1;
            continue;
        }
        out16(c.dst + s[j].y, A[j]);
    }
}

// Piece-parallel copy of a set of ready matches (sources complete, non-periodic,
// 16 <= n <= kLaneBytes): every match is cut into 16-byte pieces (the last one
// overlaps its predecessor) and the pieces of all matches are dealt to the lanes
// in order, 64 per row, so one store instruction writes ~64 pieces of ~15
// consecutive matches (4-5 adjacent lanes per match) instead of one piece of
// each of 64 matches 64+ bytes apart, and no lane idles behind a longer match of
// another lane. A match list (rank -> {y, src, n, first piece}) and a bitmap of
// first pieces live in the pending-list LDS (free while a round writes); a lane
// finds its piece's match as the number of first pieces at or below it.
struct PEnt {
    int32_t y, src, n, p0;
};
constexpr int kPieceRows = 32;                 // bitmap rows: 2 sequence rows x 64 matches x <= 16 pieces
constexpr int kPieceBatch = 8;                 // piece rows whose loads are in flight together
static_assert(2 * kWave * (kLaneBytes / 16) <= kPieceRows * kWave, "bitmap holds two sequence rows");
static_assert(2 * kWave * sizeof(PEnt) + kPieceRows * 8 <= sizeof(uint32_t) * (kLim / 2 + kMaxSeq),
              "match list and bitmap fit the pending list");

struct PieceGen {
    const PEnt* L;
    const uint64_t* bm;
    uint32_t P;        // pieces
    uint32_t t;        // next row
    int32_t rb;        // ranks before row t, minus one
    int lane;
    template <int NB>
    __device__ __forceinline__ void fill(LSlot (&s)[NB]) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const uint32_t row = t + j;
            const uint32_t p = 64u * row + (uint32_t)lane;
            s[j] = LSlot{0, 0, 0u};
            if (64u * row < P) {
                const uint64_t w = bm[row];
                const int32_t below = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(w >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)w, 0u));
                const int32_t r = rb + below + (int32_t)((w >> lane) & 1u);
                rb += __popcll(w);
                if (p < P) {
                    const PEnt e = L[r];
                    const int32_t d0 = 16 * ((int32_t)p - e.p0);
                    const int32_t d = d0 < e.n - 16 ? d0 : e.n - 16;
                    s[j] = LSlot{e.y + d, e.src + d, 16u};
                }
            }
        }
        t += NB;
    }
};

// The matches of sequences 64 i + lane for every bit i of `ready` (sources: SeqInfo::rsrc
// where `rbits` says so), two sequence rows per batch.
__device__ __forceinline__ void piece_pipe(const Ctx& c, DecShared& S, uint32_t ready, uint32_t rbits, int lane,
                                           uint32_t nseq, uint32_t nlit_pack) {
    PEnt* L = reinterpret_cast<PEnt*>(S.pme);
    uint64_t* bm = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(S.pme) + 2 * kWave * sizeof(PEnt));
    for (uint32_t i0 = 0; 64u * i0 < nseq; i0 += 2) {
        if (__ballot(((ready >> i0) & 3u) != 0) == 0) continue;
        if (lane < kPieceRows) bm[lane] = 0;
        __syncthreads();
        uint32_t P = 0, R = 0;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t i = i0 + h;
            const bool rd = (ready >> i) & 1u;
            int32_t y = 0, src = 0, n = 0;
            if (rd) {
                const uint32_t k = 64u * i + (uint32_t)lane;
                const SeqInfo q = seq_info(S, k);
                const int32_t ms = q.out + q.ll;
                const int32_t nl = i < 4 ? (int32_t)((nlit_pack >> (8 * i)) & 255u) : 0;   // split prefix
                y = ms + nl;
                n = (ms + q.ml > c.cap ? c.cap : ms + q.ml) - y;
                src = (rbits >> i) & 1u ? q.rsrc - (nl ? kSplitBase : kMemoBase) : ms - q.off;
            }
            const uint32_t np = rd ? (uint32_t)(n + 15) >> 4 : 0u;
            const uint32_t incl = wave_incl_scan(np, lane);
            const uint64_t bal = __ballot(rd);
            const uint32_t r = R + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            const uint32_t p0 = P + incl - np;
            if (rd) {
                L[r] = PEnt{y, src, n, (int32_t)p0};
                atomicOr((unsigned long long*)&bm[p0 >> 6], 1ull << (p0 & 63u));
            }
            P += lane_of(incl, kWave - 1);
            R += (uint32_t)__popcll(bal);
        }
        __syncthreads();
        PieceGen g{L, bm, P, 0u, -1, lane};
        // kPieceBatch rows at a time, all loads before all stores: every slot loads (an empty
        // one the block's first 16 bytes), so the loads are straight-line code and each store
        // waits only for its own load (counted vmcnt), not for every store in flight
        while (64u * g.t < P) {
            LSlot sl[kPieceBatch];
            uint4 v[kPieceBatch];
            g.template fill<kPieceBatch>(sl);
#pragma unroll
            for (int j = 0; j < kPieceBatch; ++j) {
                const u32x4_t t = *(const u32x4_t*)(c.dst + (sl[j].w ? sl[j].a : 0));
                v[j] = make_uint4(t.x, t.y, t.z, t.w);
            }
            lane_store<kPieceBatch>(c, S, sl, v);
        }
        __syncthreads();   // the next batch rewrites the list
    }
}

// A lane's match run the pipeline does not take (periodic, or byte-wise near a
// buffer edge / in the dictionary): piece by piece.
__device__ __forceinline__ void lane_slow_run(const Ctx& c, const DecShared& S, const Run& R) {
    const int np = run_pieces(R.n);
    for (int p = 0; p < np; ++p) {
        const Piece P = plan_piece(R, p);
        if (P.mode == 4) {
            bytes_piece(c, P.y, P.a, P.b, P.w, P.period);
            continue;
        }
        const uint4 A = load16<R_HIST>(c, S, P.a);
        uint4 v = A;
        if (P.mode == 2) v = pick4(A, load16<R_HIST>(c, S, P.b), P.k);
        else if (P.mode == 3) v = expand_period(A, P.k, P.period);
        store_w(c.dst + P.y, v, P.w);
    }
}

// Long periodic run (match offset < length): the pattern plus 20 bytes of its
// repetition are copied into LDS, then every 16-byte piece at output distance d
// is five aligned dword reads at phase d mod period (no history re-reads through
// the fabric, one output stream per lane). A period longer than the buffer is
// done in slices of phases, one LDS fill and one pass over the run per slice,
// each pass writing the pieces whose phase falls in its slice.
__device__ __forceinline__ void periodic_run(const Ctx& c, const DecShared& S, int lane, const Run& R, PatBuf B) {
    const int32_t per = R.period;
    const uint8_t* src = c.dst + R.src;
    const int32_t W = B.bytes - 48;   // phases per slice (the fill covers W + 20 bytes, rounded to 16)
    const int32_t dl = R.n - 16;      // the last piece (overlaps its predecessor when n % 16)
    for (int32_t s0 = 0; s0 < per; s0 += W) {
        const int32_t e0 = per - s0 <= W ? per : s0 + W;   // this slice's phases [s0, e0)
        __syncthreads();
        for (int k = lane; 16 * k < e0 - s0 + 20; k += kWave) {
            const int32_t q = s0 + 16 * k;
            uint4 v;
            if (q + 16 <= per) {
                v = load16<R_HIST>(c, S, R.src + q);
            } else {
                unsigned __int128 x = 0;
#pragma unroll 1
                for (int j = 0; j < 16; ++j) x |= (unsigned __int128)src[(q + j) % per] << (8 * j);
                __builtin_memcpy(&v, &x, 16);
            }
            B.w[4 * k] = v.x;
            B.w[4 * k + 1] = v.y;
            B.w[4 * k + 2] = v.z;
            B.w[4 * k + 3] = v.w;
        }
        __syncthreads();
        // every piece whose phase falls in this slice; the phase is carried from piece to piece
        // pieces on the absolute 16-byte grid (whole-line stores), the unaligned head piece
        // written once more by lane 0 (same bytes), the last piece overlapping its predecessor
        const int32_t a0 = (int32_t)((0u - (uint32_t)(uintptr_t)(c.dst + R.y)) & 15u);
        if (lane == 0 && a0) {
            const int32_t ph = 0 - s0;
            if ((uint32_t)ph < (uint32_t)(e0 - s0)) out16(c.dst + R.y, stage16(B.w, ph));
        }
        const int32_t np = (R.n - a0 + 15) >> 4;
        const int32_t step = (16 * kWave) % per;
        int32_t r = (a0 + 16 * lane) % per;
#pragma unroll 2
        for (int32_t p = lane; p < np; p += kWave) {
            const int32_t d0 = a0 + 16 * p;
            const bool last = d0 > dl;
            const int32_t d = last ? dl : d0;
            const int32_t ph = (last ? d % per : r) - s0;
            if ((uint32_t)ph < (uint32_t)(e0 - s0) && LZ4MI_ABLATE != 4) {
                out16(c.dst + R.y + d, stage16(B.w, ph));
            }
            r += step;
            if (r >= per) r -= per;
        }
    }
    __syncthreads();
}


// A long literal run (incompressible data: one run per block) copied global ->
// global with 4 16-byte pieces per lane in flight (4 KiB per wave), enough to
// keep HBM busy with one wave per block; the last piece overlaps its predecessor.
// Paced (LZ4MI_LL_ADAPT) while latency-bound blocks run on the same XCD: at full rate
// these copies fill the CU's vector-memory queues, and the blocks of short matches beside
// them, whose every chunk waits on a few dependent history reads, slow down by ~25 % for
// as long as the copies run (the per-block timeline, DESIGN §4.1 "Round 5"); spread out,
// the copies finish later but inside those blocks' own lifetime.
__device__ __forceinline__ void long_literals(uint8_t* dst, const uint8_t* src, int32_t n, int lane) {
    const int32_t np = (n + 15) >> 4;
    auto at = [&](int32_t p) { return 16 * p < n - 16 ? 16 * p : n - 16; };   // past the end: the last piece again
#if LZ4MI_LL_ADAPT
    const unsigned int* lat = &g_lat_active[32 * xcc_id()];
#endif
    for (int32_t p0 = lane; p0 < np; p0 += kWave * 4) {
#if LZ4MI_LL_ADAPT
        // (issued before the step's loads: its wait is not behind theirs)
        const uint32_t busy = __hip_atomic_load(lat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        const int32_t d0 = at(p0), d1 = at(p0 + kWave), d2 = at(p0 + 2 * kWave), d3 = at(p0 + 3 * kWave);
        uint4 v0, v1, v2, v3;
        // streamed once, never re-read soon: nontemporal, so they do not evict the history lines
        // other blocks' matches read back from L2
        v0 = ld16_nt(src + d0);
        v1 = ld16_nt(src + d1);
        v2 = ld16_nt(src + d2);
        v3 = ld16_nt(src + d3);
        st16_nt(dst + d0, v0);
        st16_nt(dst + d1, v1);
        st16_nt(dst + d2, v2);
        st16_nt(dst + d3, v3);
#if LZ4MI_LL_ADAPT
        if (busy) __builtin_amdgcn_s_sleep(LZ4MI_LL_ADAPT);
#endif
    }
}

// The whole wave writes one run (uniform R).
__device__ __forceinline__ void wave_run(const Ctx& c, DecShared& S, int lane, const Run& R, PatBuf B) {
    if (R.kind == R_NONE || R.n <= 0) return;
    // (a byte-wise periodic run whose source is inside the buffer qualifies too:
    // periodic_run reads only [src, src + period))
    const bool in_buf = R.kind == R_HIST || (R.kind == R_BYTES && c.out_off + R.src >= 0);
    if (in_buf && R.period && R.n > kPeriodBulk &&
        B.bytes > 0 && (R.period + 48 <= B.bytes || (R.n >= 4 * R.period && B.bytes >= 1024))) {
        periodic_run(c, S, lane, R, B);
        return;
    }
    const int np = run_pieces(R.n);
    if (R.kind == R_BYTES) {
        for (int p = lane; p < np; p += kWave) {
            const Piece P = plan_piece(R, p);
            bytes_piece(c, P.y, P.a, P.b, P.w, P.period);
        }
        return;
    }
    if (R.period) {
        WaveGen<kWaveB2> g{R, np, 0, lane};
        pipe<R_HIST, true, kWaveB2>(c, S, g);
        return;
    }
    WaveGen<kWaveB> g{R, np, 0, lane};
    if (R.kind == R_LDS) pipe<R_LDS, false, kWaveB>(c, S, g);
    else if (R.kind == R_COMP && R.n >= kLongLit) long_literals(c.dst + R.y, c.blk + R.src, R.n, lane);
    else if (R.kind == R_COMP) pipe<R_COMP, false, kWaveB>(c, S, g);
    else pipe<R_HIST, false, kWaveB>(c, S, g);
}

// A literal run of 1..15 bytes (v: its stage bytes) in 8/4/2/1-byte pieces by the bits of n
// (no per-width branches).
__device__ __forceinline__ void short_literals(const Ctx& c, int32_t y, int32_t n, const uint4& v) {
    if (LZ4MI_ABLATE == 4) return;
    uint8_t* d = c.dst + y;
    uint64_t lo = v.x | ((uint64_t)v.y << 32);
    const uint64_t hi = v.z | ((uint64_t)v.w << 32);
    int32_t o = 0;
    if (n & 8) { __builtin_memcpy(d, &lo, 8); lo = hi; o = 8; }
    if (n & 4) { const uint32_t t = (uint32_t)lo; __builtin_memcpy(d + o, &t, 4); lo >>= 32; o += 4; }
    if (n & 2) { const uint16_t t = (uint16_t)lo; __builtin_memcpy(d + o, &t, 2); lo >>= 16; o += 2; }
    if (n & 1) d[o] = (uint8_t)lo;
}

// Each lane copies its own short literal runs (LDS -> output; no vector-memory loads).
__device__ __forceinline__ void lane_literals(const Ctx& c, const DecShared& S, const Run& L) {
    const int32_t n = L.kind == R_NONE ? 0 : L.n;
    const int np = n >= 16 ? (n + 15) >> 4 : 0;
    for (int q = 0; __ballot(q < np) != 0; q += 2) {       // runs of >= 16 bytes: 16-byte pieces
        const int32_t d0 = 16 * q < n - 16 ? 16 * q : n - 16, d1 = 16 * (q + 1) < n - 16 ? 16 * (q + 1) : n - 16;
        const uint4 v0 = stage16(S.stage, L.src + d0);
        const uint4 v1 = stage16(S.stage, L.src + d1);
        if (LZ4MI_ABLATE == 4) continue;
        if (q < np) out16(c.dst + L.y + d0, v0);
        if (q + 1 < np) out16(c.dst + L.y + d1, v1);
    }
    if (__ballot(n > 0 && n < 16)) {                       // shorter runs: one stage read
        if (n > 0 && n < 16) short_literals(c, L.y, n, stage16(S.stage, L.src));
    }
}

// Wave-wide 255-run varint starting at block-relative q: returns the sum and
// advances q past the terminating byte. Bytes past the block end read as 0.
__device__ __forceinline__ int64_t wave_varint(const Ctx& c, int lane, int64_t& q) {
    int64_t sum = 0;
    for (;;) {
        int64_t p = q + 16 * lane;
        int first = 16;
        uint32_t lastb = 0;
        for (int j = 0; j < 16; ++j) {
            int64_t r = p + j;
            uint32_t b = (r < c.in_len) ? c.blk[r] : 0u;
            if (b != 255u && first == 16) { first = j; lastb = b; }
        }
        uint64_t mask = __ballot(first < 16);
        if (mask) {
            int fl = __builtin_ctzll(mask);
            int fi = lane_of(first, fl);
            uint32_t fb = lane_of(lastb, fl);
            int64_t cnt = (int64_t)fl * 16 + fi;
            sum += 255 * cnt + fb;
            q += cnt + 1;
            return sum;
        }
        sum += 255 * 16 * kWave;
        q += 16 * kWave;
    }
}

// Error of a sequence per the reference's check order (0 = none):
// 1 Output Buffer Too Small, 2 Malformed Input, 3 Invalid Offset 0,
// 4 Dictionary Offset Out of Bounds, 5 reaches into another block's output.
__device__ __forceinline__ uint32_t seq_error(const Ctx& c, int64_t out_start, int64_t lit, int64_t ll, uint32_t off,
                                              int64_t ml) {
    if (out_start + ll > c.cap) return 1;
    if (lit + ll > c.in_len) return 2;
    if (ml == 0) return 0;                                // final literal-only sequence
    if (off == 0) return 3;
    int64_t ms_abs = c.out_off + out_start + ll;
    if ((int64_t)off > ms_abs + c.dict_len) return 4;
    if (c.isolate && (int64_t)off > out_start + ll) return 5;
    return 0;
}

__device__ __forceinline__ int32_t err_status(uint32_t e) { return e == 5 ? -9 : -(int32_t)e; }
// An exported segment (XP, rel) knows only its relative output positions: checks 2 and 3 here,
// 1, 4 and 5 after the parse (lz4mi_xcheck_kernel), in the same order per sequence.
template <bool XP>
__device__ __forceinline__ uint32_t seq_err(const Ctx& c, bool rel, int64_t out_start, int64_t lit, int64_t ll,
                                            uint32_t off, int64_t ml) {
    if (XP && rel) {
        if (lit + ll > c.in_len) return 2;
        if (ml == 0) return 0;
        return off == 0 ? 3u : 0u;
    }
    return seq_error(c, out_start, lit, ll, off, ml);
}

// Would the reference's double-copy-tail rewrite (src/block/blockDecompress.js:219-250,
// offset >= 8, length < 8, source in the output) change a byte of
// this match's finished output? out[p] = out[p - off] for p in [ms + ml - 8, ms).
// Reads bytes of this wave's completed output (after wait_vmem).
// 0 = no change, 1 = changes (re-decode serially), 2 = the rewrite reads bytes
// before the block's start: another block's output in a batch (reported as
// LZ4MI_ERR_CROSS_BLOCK there, like any back-reference out of the block).
__device__ __forceinline__ uint32_t f1_changes(const Ctx& c, int32_t ms, int32_t off, int32_t ml) {
    if (ml == 0 || ml >= 8 || off < 8 || c.out_off + ms - off < 0) return 0;
    const int32_t p0 = ms + ml - 8;
    if (p0 - off < 0) return c.isolate ? 2u : 1u;
    for (int32_t p = p0; p < ms && p < c.cap; ++p)
        if (hist_u8(c.dst + p) != hist_u8(c.dst + p - off)) return 1;
    return 0;
}

// Reference-exact fix-up of one chunk (LZ4MI_JS_EXACT) whose matches include a
// double-copy-tail rewrite that changes bytes (f1_changes == 1): the chunk was written
// with spec semantics; replay its matches in order with the reference's semantics.
// Literal bytes never change. Everything before the first rewritten position `lo` is
// already final, so a match is copied again only if its source reaches past `lo`
// (periodic copy: its source bytes before its start are final when it runs), and every
// rewrite is applied (blockDecompress.js:219-250: out[p] = out[p - off] for
// p in [ms + ml - 8, ms), after the copy). Later chunks then read the fixed output.
__device__ void f1_fixup(const Ctx c, const DecShared& S, int lane, uint32_t nseq, bool cut, int64_t cut_ms,
                         int32_t coff, int32_t cml) {
    int64_t lo = INT64_MAX;
    const uint32_t n = nseq + (cut ? 1u : 0u);
    for (uint32_t k = 0; k < n; ++k) {
        int64_t ms;
        int32_t off, ml;
        if (k < nseq) {
            const SeqInfo q = seq_info(S, k);
            ms = (int64_t)q.out + q.ll;
            off = q.off;
            ml = q.ml;
        } else {
            ms = cut_ms;
            off = coff;
            ml = cml;
        }
        if (ml == 0) continue;
        const bool internal = c.out_off + ms - off >= 0;   // the reference's non-dictionary branch
        if (ms - off + ml > lo) {
            if (internal) {
                for (int32_t t = lane; t < ml; t += kWave) {
                    const int64_t d = ms + t;
                    const int64_t s = ms - off + (off < ml ? t % off : t);
                    const uint32_t v = hist_u8(c.dst + s);
                    if (d < c.cap) c.dst[d] = (uint8_t)v;
                }
            } else if (lane == 0) {   // spills from the dictionary into the output: in order, byte by byte
                for (int32_t t = 0; t < ml; ++t) {
                    const uint32_t v = hist_byte(c, ms - off + t);
                    if (ms + t < c.cap) c.dst[ms + t] = (uint8_t)v;
                }
            }
            wait_vmem();
        }
        if (internal && off >= 8 && ml < 8) {
            const int64_t p = ms + ml - 8 + lane;
            const bool mine = lane < 8 - ml && c.out_off + p >= 0 && p < c.cap;
            const uint32_t v = mine ? (c.out_off + p - off >= 0 ? hist_u8(c.dst + p - off) : 0u) : 0u;
            if (mine) c.dst[p] = (uint8_t)v;
            const int64_t p0 = ms + ml - 8;
            if (p0 < lo) lo = p0;
            wait_vmem();
        }
    }
}

template <bool XP>
__device__ __forceinline__ void decompress_block(const DecArgs& a) {
    __shared__ DecShared S;
    const int lane = threadIdx.x;
    const uint32_t nseg = XP ? a.xsegs : 1u;   // XP: waves per block (one per segment)
    if (blockIdx.x >= a.nblocks * nseg) return;
    const uint32_t wblk = XP ? blockIdx.x / nseg : blockIdx.x;   // (XP: block-major, segments of a block on
    const uint32_t sg = XP ? blockIdx.x - wblk * nseg : 0u;       //  consecutive CUs, every XCD)
    const uint32_t b = a.order ? uniform(a.order[wblk]) : wblk;
    if (!XP && a.redo && !uniform(a.redo[b])) return;   // (small batches, reference mode: the blocks to redo)
#if LZ4MI_TIMELINE
    const uint64_t tl_t0 = wall_clock64();
#endif

    // the block's scalars in SGPRs (readfirstlane): as VGPRs the compiler would keep
    // per-lane copies of values derived from them and spill those to scratch
    const uint64_t in_off = uniform64(a.in_off[b]), out_off = uniform64(a.out_off[b]);
    const uint32_t out_cap = uniform(a.out_cap[b]);
    Ctx c;
    c.blk = a.in + in_off;
    const uint32_t word = uniform(a.in_len[b]);
    c.in_len = (int32_t)(a.frame_words ? word & 0x7FFFFFFFu : word);
    c.out_off = (int64_t)out_off;
    c.dst = a.out + out_off;
    c.cap = out_cap > 0x7FFFFFFFu ? 0x7FFFFFFF : (int32_t)out_cap;
    c.dict = a.dict;
    c.dict_len = a.dict ? (int32_t)a.dict_len : 0;
    c.isolate = a.isolate;
    c.ip = 0;
    c.O = 0;
    int32_t status = 0;
    if (a.frame_words && (word & 0x80000000u)) {
        // a frame's stored block (bufferDecompress.js:173-180): its bytes, in this launch, paced
        // like any long literal run; larger than the slot: the reference's RangeError
        const int32_t n = c.in_len;
        if ((uint32_t)n > out_cap) {
            status = LZ4MI_ERR_RANGE_STATUS;
        } else if (n >= 16) {
            long_literals(c.dst, c.blk, n, lane);
        } else if (lane < n) {
            c.dst[lane] = c.blk[lane];
        }
        if (lane == 0) {
            a.status[b] = status;
            a.out_len[b] = status ? 0u : (uint32_t)n;
        }
        return;
    }
    // small-batch export (XP, lz4mi_expand.hip): segment sg of the block, parsed only
    // (a block of long runs -- output over 32x its compressed size: repetitive data, one periodic
    // match -- decodes faster in one wave, as in the batch kernel: 1.1 ms for 4 MiB at any batch
    // size, against 0.77 ms alone / 1.57 ms for 16 through the pointers, profiles/r06c)
    const bool xp = XP && (uint32_t)c.in_len <= a.x_in_max && out_cap <= a.x_out_max &&
                    (uint64_t)out_cap < (uint64_t)c.in_len * kXRatioMax &&
                    !(a.x_flat1 && (uint64_t)c.in_len * 16 >= (uint64_t)out_cap * 15);
    // past the export limits (or ratio >= 32): one wave decodes the block as usual -- segment
    // b mod 256, i.e. workgroup 257 b (mod 256 CUs: a CU of its own for every block, where
    // segment 0 would put the blocks of a batch on one CU)
    if (XP && !xp && (a.xphase != 0 || sg != wblk % nseg)) return;
    uint4* xs = nullptr;
    SegRec* xr = nullptr;
    uint32_t seg_lo = 0, seg_hi = 0;    // the segment: tokens in [seg_lo, seg_hi)
    if (XP && xp) {
        const SegGeom G = seg_geom((uint32_t)c.in_len);   // S segments of ~kSegTarget bytes
        if (sg >= G.S) return;
        seg_lo = sg * G.L;
        seg_hi = sg + 1 == G.S ? (uint32_t)c.in_len : min((uint32_t)c.in_len, seg_lo + G.L);
        xs = a.xseq + (size_t)wblk * a.xseq_stride + (size_t)sg * G.stride;
        xr = a.xrec + (size_t)wblk * nseg + sg;
    }
    if (XP && a.xphase != 0 && !xp) return;
    // export state (uniform): the entry found, done, the speculation failed, entry / exit tokens,
    // sequences exported, their output bytes, the first parse error; x_OG: output position of
    // the entry in this wave's running count; pass 1: the exact re-parse from x_entry
    bool x_started = false, x_done = false, x_fail = false;
    uint32_t x_G = 0, x_X = 0, nx = 0, x_olen = 0, x_err = 0xFFFFFFFFu, x_entry = 0;
    int64_t x_OG = 0;
    int x_pass = 0, x_restart = 0;
    if (XP && xp && a.xphase == 2) {
        // phase 2: every segment whose guess disagrees with the previous one's exit, re-parsed
        // from that exit at once (lz4mi_xverify_kernel's `from`), a guess again -- the check then
        // runs again: a wrong guess does not make the later guesses wrong, and the segments
        // before a wrong one are mostly right (text, ~10 % of ~190 segments: chained one after
        // another in phase 1, 2.1 ms for a block)
        const uint32_t from = uniform(xr->from);
        if (from == kNoBase) return;
        x_pass = 2;
        x_entry = from;
    }
    if (XP && xp && a.xphase == 1) {
        // phase 1: segments from the first wrong entry on, in order: re-parse from the previous
        // segment's final exit unless the speculative entry equals it
        const uint32_t sstar = a.xfirst[wblk];
        if (sg < sstar) return;
        uint32_t fp = 0;
        if (sg == sstar) {
            fp = xr[-1].exit;                    // final: accepted by lz4mi_xverify_kernel
        } else {
            if (lane == 0) {
                const uint32_t* f = &xr[-1].fin;
                while ((fp = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
                    __builtin_amdgcn_s_sleep(8);
            }
            fp = lane_of(fp, 0) - 1u;
        }
        uint32_t fin = 0;
        bool reparse = false;
        if (fp == kFinErr) {                     // after the block's first error: nothing here
            fin = kFinErr;
            if (lane == 0) { xr->cnt = 0; xr->olen = 0; xr->err = 0xFFFFFFFFu; }
        } else if (fp >= seg_hi) {               // the chain passes over the segment
            fin = fp;
            if (lane == 0) { xr->entry = xr->exit = fp; xr->cnt = 0; xr->olen = 0; xr->err = 0xFFFFFFFFu; }
        } else if (sg != sstar && !xr->fail && xr->entry == fp) {
            fin = xr->err != 0xFFFFFFFFu ? kFinErr : xr->exit;
        } else {
            reparse = true;
        }
        if (!reparse) {
            if (lane == 0) __hip_atomic_store(&xr->fin, fin + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        x_pass = 1;
        x_entry = fp;
    }
#if LZ4MI_LL_ADAPT
    const bool lat_bound = (uint64_t)c.in_len * 2 < (uint64_t)out_cap;   // ratio > 2: a chain of short copies
    unsigned int* lat = &g_lat_active[32 * xcc_id()];
    if (lat_bound && lane == 0) atomicAdd(lat, 1u);
#endif
    uint4 pf0 = make_uint4(0, 0, 0, 0), pf1 = pf0;   // the next chunk's staged bytes, loaded early
    bool have_pf = false;
    int64_t pf_at = -1;                    // compressed position pf0/pf1 were loaded from
#if LZ4MI_PROFILE
    uint64_t prof[24] = {0};
    uint64_t prof_t = wall_clock64();
#endif

    if (XP && xp) {
        c.O = 0;
        have_pf = false;
        c.ip = x_pass ? (int32_t)x_entry
                      : (seg_lo >= (uint32_t)c.in_len ? c.in_len : (int32_t)(seg_lo - min(seg_lo, kSegWarm)));
        x_started = x_done = x_fail = false;
        x_G = x_X = nx = x_olen = 0;
        x_err = 0xFFFFFFFFu;
        x_OG = 0;
    }
    while (c.ip < c.in_len) {
        if (XP && x_done) break;   // (XP: the segment's exit found)
        PROF_COUNT(10, 1);
        // ---- 1. stage [ip, ip + kLim) (16-byte unaligned loads, issued during
        // the previous chunk's output phase, ahead of its stores) -------------
        // (each branch writes the stage itself: a write after the join would wait for the
        // fresh loads of the first branch on both, i.e. for every store still in flight)
        if (!have_pf || pf_at != c.ip) {
            const uint4 a = stage_piece(c, (int64_t)c.ip + 16 * opaque(lane));
            uint4 b = make_uint4(0, 0, 0, 0);
            if (lane < kStageWords / 4 - kWave) b = stage_piece(c, (int64_t)c.ip + 16 * (kWave + opaque(lane)));
            __builtin_memcpy((uint8_t*)S.stage + 16 * lane, &a, 16);
            if (lane < kStageWords / 4 - kWave) __builtin_memcpy((uint8_t*)S.stage + 16 * (kWave + lane), &b, 16);
        } else {
            __builtin_memcpy((uint8_t*)S.stage + 16 * lane, &pf0, 16);
            if (lane < kStageWords / 4 - kWave) __builtin_memcpy((uint8_t*)S.stage + 16 * (kWave + lane), &pf1, 16);
        }
        have_pf = false;
        __syncthreads();
        const uint8_t* s = (const uint8_t*)S.stage;
        const uint32_t rem = (uint32_t)(c.in_len - c.ip);

        const uint32_t seg0 = 16u * lane, seg1 = seg0 + 16;
        uint32_t vis, tail;
        bool fast_tab = rem > kFastRem;
    parse:
        {
        PROF(0);
        // Wave priorities by phase (the 4 waves of a SIMD are in different phases):
        // output rounds 3 > walks 1 > next-token table 0. The copies' loads and
        // stores go out first and the LDS-bound parse fills the gaps: tiles216 -0.9 %,
        // mix -2.5 %, copy -1.5 % (A/B in one process, profiles/r02j/prio_ab.json).
        __builtin_amdgcn_s_setprio(0);
        // ---- 2. next-token table -----------------------------------------
        // Away from the block's end (fast_tab) four positions per lane from two stage
        // dwords, assuming length fields of at most one extension byte: a token whose
        // literal field runs on (b1 == 255) stops the chain (the cut path parses it), and
        // a match field that runs on (checked on the true tokens in the table build) sends
        // the chunk back here for the exact table. Near the end: the exact table.
        uint16_t* nxt = S.nxt;
        if (fast_tab) {
            next_table_fast(S.stage, nxt, lane);
        } else {   // all positions' fields read at once; the rare longer length fields afterwards
            static_assert(kChunk % kWave == 0, "whole rows per lane");
            uint32_t slm = 0;
#pragma unroll
            for (int i = 0; i < kChunk / kWave; ++i) {
                bool slow;
                const uint32_t v = next_fast(s, lane + kWave * i, rem, slow);
                slm |= (slow ? 1u : 0u) << i;
                nxt[lane + kWave * i] = enc_next(v);
            }
            if (__ballot(slm != 0)) {
                for (uint32_t m = slm; m; m &= m - 1) {
                    const uint32_t p = lane + kWave * __builtin_ctz(m);
                    nxt[p] = enc_next(next_token(s, p, rem));
                }
            }
        }
        __syncthreads();
        // 2- and 4-step jumps (the warm-up walks only need where the chain lands)
        jump_table(nxt, S.nxt2, lane);
        __syncthreads();
        jump_table(S.nxt2, S.nxt4, lane);
        __syncthreads();
#if LZ4MI_ABLATE == 3
        c.ip += kChunk;
        __syncthreads();
        continue;
#endif

        PROF(1);
        __builtin_amdgcn_s_setprio(1);
        // ---- 3. speculative walks + certification -------------------------
        uint32_t x;
        vis = 0;
        {   // warm-up walk; lanes whose warm-up would start before the chunk start at it, a true token
            uint32_t p = seg0 < kWarm ? 0u : seg0 - kWarm;
            for (uint32_t q; (q = S.nxt4[p]) < seg0;) p = q;    // jumps stay short of the segment
            for (uint32_t q; (q = S.nxt2[p]) < seg0;) p = q;
            while (p < seg1) {
                if (p >= seg0) vis |= 1u << (p - seg0);
                p = next_of(nxt, p);
                PROF_COUNT(15, 1);
            }
            x = p;
        }
        uint32_t es = vis ? seg0 + __builtin_ctz(vis) : x;
        uint32_t nE = 0;
        for (int it = 0; it <= kWave; ++it) {
            // lane l - 1's values by DPP wave_shr:1 (a VALU operand, not an LDS permute)
            const uint32_t pes = dpp<kWaveShr1>(0u, es), px = dpp<kWaveShr1>(0u, x);
            nE = lane == 0 ? 0u : (pes >= seg0 ? pes : px);
            bool valid = nE >= seg1 ? (vis == 0 && x == nE) : ((vis >> (nE - seg0)) & 1u) != 0;
            uint64_t bad = __ballot(!valid);
            PROF_COUNT(13, 1);
            if (it == 0) PROF_COUNT(14, __popcll(bad));
            if (bad == 0) break;
            if (lane == __builtin_ctzll(bad)) {   // first inconsistent lane: re-walk from its true entry
                vis = 0;
                uint32_t p = nE;
                while (p < seg1) {
                    vis |= 1u << (p - seg0);
                    p = next_of(nxt, p);
                }
                x = p;
                es = vis ? seg0 + __builtin_ctz(vis) : x;
            }
        }
        if (nE >= seg1) vis = 0;
        else vis &= ~((1u << (nE - seg0)) - 1u);
        tail = lane_of(x, kWave - 1);   // where the chain leaves the chunk
        if (tail > (uint32_t)kLim && tail < kEnd) tail = kStop;   // (fast table: raw positions past the window)
        }
        (void)seg1;
        const uint64_t has = __ballot(vis != 0);
        const int last_lane = 63 - __builtin_clzll(has);
        const uint32_t last_tok = lane_val(seg0 + 31 - __builtin_clz(vis | 1u), (uint32_t)last_lane);
        const bool cut = tail == kStop;
        if (!cut && tail < kEnd && (int64_t)c.ip + tail < c.in_len) {
            // the next chunk's bytes: loaded while this chunk's table is built
            int64_t nip = (int64_t)c.ip + tail;
            pf0 = stage_piece(c, nip + 16 * opaque(lane));
            if (lane < kStageWords / 4 - kWave) pf1 = stage_piece(c, nip + 16 * (kWave + opaque(lane)));
            pf_at = nip;
            have_pf = true;
        }
#if LZ4MI_ABLATE == 2
        c.ip = tail == kEnd ? c.in_len : c.ip + (cut ? kChunk : (int32_t)tail);
        __syncthreads();
        continue;
#endif

        PROF(2);
        // ---- 4. sequence table -----------------------------------------
        // A lane's tokens (those of its segment, in order) four at a time, each group's
        // byte reads issued together (two LDS round trips per group, not per token);
        // output starts by wave prefix sums; errors in the reference's order.
        const uint32_t cnt = __popc(vis) - ((cut && lane == last_lane) ? 1u : 0u);
        const uint32_t incl = wave_incl_scan(cnt, lane);
        const uint32_t base = incl - cnt;
        const uint32_t nseq = lane_of(incl, kWave - 1);
        uint32_t run = 0;
        bool rerun = false;   // a true token's match length runs on past one byte (fast table)
        {
            uint32_t m = vis;
            for (uint32_t g = 0; __ballot(g < cnt) != 0; g += 4) {
                uint32_t p[4], tok[4], b1[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    p[j] = g + j < cnt ? seg0 + __builtin_ctz(m) : seg0;
                    if (g + j < cnt) m &= m - 1;
                    tok[j] = s[p[j]];
                    b1[j] = s[p[j] + 1];
                }
                uint32_t q[4], lit[4], ll[4], o0[4], o1[4], mb[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t x1 = (tok[j] >> 4) == 15 ? 1u : 0u;
                    ll[j] = x1 ? 15u + b1[j] : tok[j] >> 4;
                    lit[j] = p[j] + 1 + x1;
                    q[j] = lit[j] + ll[j];
                    // offset bytes inside the window (q + 2 <= kLim: a sequence may end on its last byte,
                    // as next_token accepts; s[q + 2] is still staged) -- past it only a long literal run
                    // (slow below)
                    const uint32_t qa = q[j] + 2 <= (uint32_t)kLim ? q[j] : 0u;
                    o0[j] = s[qa];
                    o1[j] = s[qa + 1];
                    mb[j] = s[qa + 2];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (g + j >= cnt) continue;
                    uint32_t llj = ll[j], litj = lit[j], qj = q[j], off = 0, ml = 0;
                    if ((tok[j] >> 4) == 15 && b1[j] == 255) {   // literal length field of 2+ bytes
                        uint32_t r = p[j] + 1, bb;
                        llj = 15;
                        do { bb = s[r++]; llj += bb; } while (bb == 255);
                        litj = r;
                        qj = r + llj;
                        if (qj < rem) { o0[j] = s[qj]; o1[j] = s[qj + 1]; mb[j] = s[qj + 2]; }
                    }
                    if (qj < rem) {
                        off = o0[j] | (o1[j] << 8);
                        ml = tok[j] & 15;
                        if (ml == 15) {
                            if (mb[j] != 255) {
                                ml += mb[j];
                            } else {
                                rerun |= fast_tab;
                                uint32_t r = qj + 2, bb;
                                do { bb = s[r++]; ml += bb; } while (bb == 255 && r < (uint32_t)kLim);
                            }
                        }
                        ml += 4;
                    }
                    const uint32_t k = base + g + j;
                    S.t_seq[k] = make_uint4(run, litj | (llj << 16), off | (ml << 16), 0u);
                    run += llj + ml;
                }
            }
        }
        if (__ballot(rerun)) {   // the fast table assumed a one-byte match length field
            fast_tab = false;
            wait_vmem();          // (no load in flight into the parse: its registers are free)
            settle(pf0);
            settle(pf1);
            __syncthreads();
            goto parse;
        }
        const uint32_t lincl = wave_incl_scan(run, lane);
        const uint32_t lbase = lincl - run;
        const int64_t total = lane_of(lincl, kWave - 1);
        uint32_t first_err = 0xFFFFFFFFu;
        for (uint32_t g = 0; __ballot(g < cnt) != 0; g += 4) {
            SeqInfo q[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = seq_info(S, base + (g + j < cnt ? g + j : 0u));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (g + j >= cnt) continue;
                const uint32_t k = base + g + j;
                const int64_t os = c.O + lbase + (uint32_t)q[j].out;
                S.t_seq[k].x = (uint32_t)os;
                const uint32_t e = seq_err<XP>(c, xp, os, (int64_t)c.ip + q[j].lit, q[j].ll, q[j].off, q[j].ml);
                if (e && first_err == 0xFFFFFFFFu) first_err = (k << 3) | e;
            }
        }
        first_err = wave_min(first_err);
        __syncthreads();
        if (first_err != 0xFFFFFFFFu && !(XP && xp)) { status = err_status(first_err & 7); break; }

        PROF(3);
        // ---- 6. the sequence the window could not hold: parse it from memory
        int64_t cq = 0, cll = 0, cml = 0, clit = 0;
        uint32_t coff = 0;
        if (cut) {
            // token and literal length from the staged bytes while they last
            constexpr uint32_t kStaged = 16 * (kStageWords / 4);
            uint32_t r = last_tok;
            const uint32_t tok = s[r++];
            cll = tok >> 4;
            bool more = cll == 15;
            while (more && r < kStaged) {
                const uint32_t b = s[r++];
                cll += b;
                more = b == 255;
            }
            int64_t q = (int64_t)c.ip + r;
            if (more) cll += wave_varint(c, lane, q);
            clit = q;
            q += cll;
            if (q < c.in_len) {
                // offset and match length: one 16-byte load covers them unless the length runs on
                uint32_t w[4];
                if (q + 16 <= c.in_len) {
                    __builtin_memcpy(w, c.blk + q, 16);
                } else {
                    const uint4 t = load16_tail(c.blk, q, c.in_len);
                    w[0] = t.x;
                    w[1] = t.y;
                    w[2] = t.z;
                    w[3] = t.w;
                }
                coff = w[0] & 0xFFFFu;
                q += 2;
                cml = tok & 15;
                if (cml == 15) {
                    bool run = true;
                    for (int t = 2; t < 16 && run; ++t) {
                        const uint32_t wd = t < 4 ? w[0] : t < 8 ? w[1] : t < 12 ? w[2] : w[3];
                        const uint32_t b = (wd >> (8 * (t & 3))) & 255u;
                        cml += b;
                        ++q;
                        run = b == 255;
                    }
                    if (run) cml += wave_varint(c, lane, q);
                }
                cml += 4;
            }
            cq = q;
        }
        const int64_t tab_hi = c.O + total;
        if (XP && xp) {
            // export the sequences whose tokens lie in [seg_lo, seg_hi); the first one found is
            // the segment's entry, the first at or past seg_hi its exit
            const uint32_t ipc = (uint32_t)c.ip;
            const uint32_t ntot = nseq + (cut ? 1u : 0u);   // the cut sequence is number nseq
            const uint32_t ecut = cut ? seq_err<XP>(c, true, tab_hi, clit, cll, coff, cml) : 0u;
            const uint32_t ferr = first_err != 0xFFFFFFFFu ? first_err : (ecut ? ((nseq << 3) | ecut) : 0xFFFFFFFFu);
            const uint32_t fk = ferr == 0xFFFFFFFFu ? ntot : (ferr >> 3);
            auto x_tok = [&](uint32_t k) -> uint32_t {   // token position (block-relative)
                if (k >= nseq) return ipc + last_tok;
                const SeqInfo q = seq_info(S, k);
                return ipc + (uint32_t)q.lit - 1u - (q.ll >= 15 ? (uint32_t)(q.ll - 15) / 255u + 1u : 0u);
            };
            auto x_out = [&](uint32_t k) -> int64_t { return k >= nseq ? tab_hi : (int64_t)S.t_seq[k].x; };
            uint32_t k0 = ntot, k1 = ntot;
            for (uint32_t r = 0; 64u * r < ntot; ++r) {
                const uint32_t k = 64u * r + lane;
                const uint32_t t = k < ntot ? x_tok(k) : 0xFFFFFFFFu;
                const uint64_t m0 = __ballot(k < ntot && t >= seg_lo), m1 = __ballot(k < ntot && t >= seg_hi);
                if (k0 == ntot && m0) k0 = 64u * r + (uint32_t)__builtin_ctzll(m0);
                if (k1 == ntot && m1) k1 = 64u * r + (uint32_t)__builtin_ctzll(m1);
            }
            bool restart = false;
            if (!x_started && fk < k0) {
                // an error before the segment: a wrong walk, or an earlier segment's error (which
                // that segment's parse reports) -- never this segment's. A guess starts over one
                // byte past the impossible token (text: an offset of 0 read from the wrong bytes
                // failed 22 of a 4 MiB block's 255 guesses, which then waited for re-parses)
                if (x_pass == 0 && x_restart < kSegRestarts) {
                    restart = true;
                    ++x_restart;
                } else {
                    x_fail = x_done = true;
                }
            } else {
                if (!x_started && k0 < ntot) {
                    x_started = true;
                    x_G = x_tok(k0);
                    x_OG = x_out(k0);
                }
                if (x_started) {
                    const uint32_t ke = fk < k1 ? fk + 1 : k1;   // with the failing one (checks 1, 4, 5)
                    for (uint32_t k = k0 + lane; k < ke; k += kWave) {
                        uint4 e;
                        if (k < nseq) {
                            const SeqInfo q = seq_info(S, k);
                            e = make_uint4((uint32_t)(x_out(k) - x_OG), ipc + (uint32_t)q.lit, (uint32_t)q.ll,
                                           q.ml ? (uint32_t)q.off : 0u);
                        } else {
                            e = make_uint4((uint32_t)(tab_hi - x_OG), (uint32_t)clit, (uint32_t)cll, cml ? coff : 0u);
                        }
                        xs[nx + (k - k0)] = e;
                    }
                    if (fk < k1) {
                        x_err = ((nx + (fk - k0)) << 3) | (ferr & 7u);
                        x_done = true;
                    } else if (k1 < ntot) {
                        x_done = true;
                        x_X = x_tok(k1);
                        x_olen = (uint32_t)(x_out(k1) - x_OG);
                    }
                    nx += ke - k0;
                }
            }
            if (restart) {
                c.ip = (int32_t)(x_tok(fk) + 1u);
                c.O = 0;
            } else if (!x_done) {   // on to the next chunk
                if (cut) {
                    c.O = tab_hi + cll + cml;
                    c.ip = (int32_t)(cq < c.in_len ? cq : c.in_len);
                } else {
                    c.O = tab_hi;
                    c.ip = tail >= kEnd ? c.in_len : c.ip + (int32_t)tail;
                }
                if ((uint32_t)c.ip >= seg_hi && c.ip < c.in_len) {   // the chain leaps the segment's end
                    if (!x_started) {
                        x_started = true;
                        x_G = (uint32_t)c.ip;
                        x_OG = c.O;
                    }
                    x_done = true;
                    x_X = (uint32_t)c.ip;
                    x_olen = (uint32_t)(c.O - x_OG);
                }
            }
            __syncthreads();
            continue;
        }
        if (cut) {   // the next chunk's bytes: their loads go out before this chunk's stores
            int64_t nip = cq < c.in_len ? cq : c.in_len;
            if (nip < c.in_len) {
                    pf0 = stage_piece(c, nip + 16 * opaque(lane));
                if (lane < kStageWords / 4 - kWave) pf1 = stage_piece(c, nip + 16 * (kWave + opaque(lane)));
                    pf_at = nip;
                have_pf = true;
            }
        }

#if LZ4MI_ABLATE == 0 || LZ4MI_ABLATE >= 4
        PROF(4);
        __builtin_amdgcn_s_setprio(3);
        // ---- 5. output rounds ---------------------------------------------
        // The previous chunk's stores (read back as history below) and the next
        // chunk's loads are complete: the stores had the whole parse to drain.
        wait_vmem();
        settle(pf0);    // (so the next chunk's stage does not wait for this chunk's stores)
        settle(pf1);
        PROF(21);
        // output -> sequence map for remap_src, in the (now idle) next-token table
        // output -> sequence map granule: 32 bytes for long sequences (tiles216: 16 B costs 1.8 %),
        // 16 for short ones (text: 32 B costs 6 %, more sequences per granule to step over)
        uint32_t msh = total >= 32u * nseq ? 5u : 4u;
        while ((total >> msh) >= kLim) ++msh;
        for (uint32_t k = lane; k < nseq; k += kWave) {
            const uint32_t t0 = S.t_seq[k].x - (uint32_t)c.O;
            const uint32_t t1 = (k + 1 < nseq ? S.t_seq[k + 1].x : (uint32_t)(c.O + total)) - (uint32_t)c.O;
            for (uint32_t b = (t0 + (1u << msh) - 1) >> msh; (b << msh) < t1; ++b) S.nxt[b] = (uint16_t)k;
        }
        __syncthreads();
        PROF(22);
        uint32_t pend = 0;    // bit i: the match of sequence 64i+lane is still to be written
        uint32_t ready = 0;   // bit i: ... is written by this lane in this round
        uint32_t rbits = 0;   // bit i: ... reads a remapped source (SeqInfo::rsrc)
        uint32_t nlit_pack = 0;   // byte i (rows < 4): literal prefix of a split match (remap_src 3)
        for (uint32_t i = 0; 64 * i < nseq; ++i) {            // round 1
            const uint32_t k = 64 * i + lane;
            Run M = no_run(), ML = no_run();
            SeqInfo q = seq_info(S, k < nseq ? k : 0u);
            if (k >= nseq) q.ll = 0;
            {   // the literal runs first (their registers are free before the remap)
                const Run L = q.ll ? Run{q.out, q.ll, q.lit, 0, R_LDS} : no_run();
                const bool longL = L.n > kLaneBytes;
                lane_literals(c, S, longL ? no_run() : L);
                for (uint64_t lm = __ballot(longL); lm; lm &= lm - 1) wave_run(c, S, lane, shfl_run(L, __builtin_ctzll(lm)), no_pat());
            }
            PROF(23);
            if (k < nseq) {
                const int32_t t0 = q.out;
                M = match_run(c, t0 + q.ll, q.off, q.ml);
                if (M.n == 0) {
                    M.kind = R_NONE;
                } else if (match_src_end(M) > (int32_t)c.O) {
                    // the source is output of this table: map it back through the
                    // sequences that wrote it, else wait for a later round
                    int32_t rs = M.src, re = match_src_end(M), li = 0, nl = 0;
                    const int r = (M.kind == R_HIST && M.period == 0)
                                      ? remap_src(c, S, nseq, msh, rs, re, li, nl, i < 4)
                                      : 0;
                    if (r == 3) {   // literal prefix from the stage, the rest from finished output
                        ML = Run{M.y, nl, li, 0, R_LDS};
                        M.y += nl;
                        M.n -= nl;
                        nlit_pack |= (uint32_t)nl << (8 * i);
                    }
                    if (r == 1 || r == 3) {
                        M.src = rs;
                        if (c.out_off + rs < 16) M.kind = R_BYTES;
                        S.t_seq[k].w = (uint32_t)(rs + (r == 3 ? kSplitBase : kMemoBase));
                        rbits |= 1u << i;
                    } else if (r == 2) {
                        ML = Run{M.y, M.n, li, 0, R_LDS};
                        M.kind = R_NONE;
                    } else {
                        pend |= 1u << i;
                        M.kind = R_NONE;
                    }
                }
            }
            const bool longM = M.kind != R_NONE && M.n > kLaneBytes;
            const bool longML = ML.n > kLaneBytes;
            const bool fastM = M.kind == R_HIST && M.period == 0 && M.n >= 16;
            if (M.kind != R_NONE && !longM && fastM) ready |= 1u << i;
            PROF(16);
            lane_literals(c, S, longML ? no_run() : ML);
            PROF(17);
            for (uint64_t lm = __ballot(longML); lm; lm &= lm - 1) wave_run(c, S, lane, shfl_run(ML, __builtin_ctzll(lm)), no_pat());
            if (M.kind != R_NONE && !longM && !fastM) lane_slow_run(c, S, M);
            for (uint64_t mm = __ballot(longM); mm; mm &= mm - 1) wave_run(c, S, lane, shfl_run(M, __builtin_ctzll(mm)), pat_round1(S));
            PROF(18);
        }
        piece_pipe(c, S, ready, rbits, lane, nseq, nlit_pack);
        PROF(19);
        for (; LZ4MI_ABLATE != 6;) {                           // rounds 2, 3, ...
            uint32_t np = 0;
            for (uint32_t i = 0; 64 * i < nseq; ++i) {
                const bool pk = (pend >> i) & 1u;
                const uint64_t bal = __ballot(pk);
                if (pk) {
                    const uint32_t k = 64 * i + lane;
                    const uint32_t idx = np + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    const SeqInfo q = seq_info(S, k);
                    const int32_t ms = q.out + q.ll;
                    S.pms[idx] = (uint32_t)ms;
                    S.pme[idx] = (uint32_t)(ms + q.ml > c.cap ? c.cap : ms + q.ml);
                }
                np += (uint32_t)__popcll(bal);
            }
            if (np == 0) break;
            PROF_COUNT(11, 1);
            __syncthreads();
            wait_vmem();      // the previous round's stores are complete
            PROF(20);
            ready = 0;
            for (uint32_t i = 0; 64 * i < nseq; ++i) {
                if (__ballot((pend >> i) & 1u) == 0) continue;
                Run M = no_run();
                if ((pend >> i) & 1u) {
                    const uint32_t k = 64 * i + lane;
                    const SeqInfo q = seq_info(S, k);
                    M = match_run(c, q.out + q.ll, q.off, q.ml);
                    // first pending match ending past the source start: ready if it starts at or past the source end
                    const int32_t rs = M.src, re = match_src_end(M);
                    uint32_t lo = 0, hi = np;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if ((int32_t)S.pme[mid] > rs) hi = mid;
                        else lo = mid + 1;
                    }
                    if (lo >= np || (int32_t)S.pms[lo] >= re) pend &= ~(1u << i);
                    else M.kind = R_NONE;
                }
                const bool longM = M.kind != R_NONE && M.n > kLaneBytes;
                const bool fastM = M.kind == R_HIST && M.period == 0 && M.n >= 16;
                if (M.kind != R_NONE && !longM && fastM) ready |= 1u << i;
                if (M.kind != R_NONE && !longM && !fastM) lane_slow_run(c, S, M);
                for (uint64_t mm = __ballot(longM); mm; mm &= mm - 1) wave_run(c, S, lane, shfl_run(M, __builtin_ctzll(mm)), pat_rounds(S));
            }
            piece_pipe(c, S, ready, 0u, lane, nseq, 0u);
            __syncthreads();
        }
        PROF(6);
        if (cut) {
            PROF_COUNT(12, 1);
            const uint32_t e = seq_error(c, tab_hi, clit, cll, coff, cml);
            if (e) { status = err_status(e); break; }
            wave_run(c, S, lane, Run{(int32_t)tab_hi, (int32_t)cll, (int32_t)clit, 0, cll ? (uint32_t)R_COMP : (uint32_t)R_NONE}, no_pat());
        }
#else
        if (cut) {
            const uint32_t e = seq_error(c, tab_hi, clit, cll, coff, cml);
            if (e) { status = err_status(e); break; }
        }
#endif
        PROF(7);
        if (a.f1check) {
            // candidates first, from the sequence table alone (offset >= 8, length < 8): a chunk
            // without one -- every tiles216 chunk -- neither drains its stores here nor reads
            // them back, so they keep draining beside the next chunk's parse as in spec mode
            bool cand = false;
            for (uint32_t k = lane; k < nseq; k += kWave) {
                const SeqInfo q = seq_info(S, k);
                cand |= q.ml != 0 && q.ml < 8 && q.off >= 8;
            }
            if (__ballot(cand)) {
                wait_vmem();    // this chunk's stores are complete before they are read back
                uint32_t dv = 0;
                for (uint32_t k = lane; k < nseq; k += kWave) {
                    const SeqInfo q = seq_info(S, k);
                    dv |= f1_changes(c, q.out + q.ll, q.off, q.ml);
                }
                if (__ballot(dv & 2u)) { status = -9; break; }
                if (__ballot(dv)) f1_fixup(c, S, lane, nseq, false, 0, 0, 0);
            }
        }
#if LZ4MI_ABLATE == 0 || LZ4MI_ABLATE >= 4
        // the cut sequence's match, after the table's F1 replay (it reads the replayed
        // bytes, as the reference's copy does); the tables are idle now: all of LDS
        // can hold a periodic pattern
        if (cut) {
            const Run M = match_run(c, (int32_t)(tab_hi + cll), (int32_t)coff, (int32_t)cml);
            if (M.n > 0) {
                wait_vmem();    // everything below the match is read back as history
                wave_run(c, S, lane, M, pat_all(S));
            }
            if (a.f1check && cml != 0 && cml < 8 && coff >= 8) {    // its own tail rewrite, after its copy as in the reference
                wait_vmem();
                const uint32_t dv = lane == 0 ? f1_changes(c, (int32_t)(tab_hi + cll), (int32_t)coff, (int32_t)cml) : 0u;
                if (__ballot(dv & 2u)) { status = -9; break; }
                if (__ballot(dv)) f1_fixup(c, S, lane, 0, true, (int64_t)(tab_hi + cll), (int32_t)coff, (int32_t)cml);
            }
        }
#endif
        c.O = tab_hi;
        if (cut) {
            c.O += cll + cml;
            c.ip = (int32_t)(cq < c.in_len ? cq : c.in_len);
        } else if (tail >= kEnd) {
            c.ip = c.in_len;
        } else {
            c.ip += (int32_t)tail;
        }
        __syncthreads();
        PROF(8);
    }
    if (XP && xp) {
        if (!x_done) {   // the block's end
            if (!x_started) {
                x_G = (uint32_t)c.in_len;
                x_OG = c.O;
            }
            x_X = (uint32_t)c.in_len;
            x_olen = (uint32_t)(c.O - x_OG);
        }
        if (lane == 0) {
            xr->entry = x_G;
            xr->exit = x_X;
            xr->cnt = nx;
            xr->olen = x_olen;
            xr->err = x_err;
            xr->fail = (x_fail || (a.xforce && sg > 0 && (a.xforce == 2 ? x_pass != 1 : x_pass == 0))) ? 1u : 0u;
            if (x_pass == 1)   // the exact re-parse of phase 1: final
                __hip_atomic_store(&xr->fin, (x_err != 0xFFFFFFFFu ? kFinErr : x_X) + 1u, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
#if LZ4MI_LL_ADAPT
        if (lat_bound && lane == 0) atomicSub(lat, 1u);
#endif
        return;   // status and length: lz4mi_xcheck_kernel
    }
#if LZ4MI_PROFILE
    if (lane == 0)
        for (int i = 0; i < 24; ++i) atomicAdd(&g_prof[i], (unsigned long long)prof[i]);
#endif
    if (lane == 0) {
        a.status[b] = status;
        a.out_len[b] = status ? 0u : (uint32_t)c.O;
        if (XP) a.xcnt[b] = kNotExported;   // (XP: a block past the export limits)
    }
#if LZ4MI_LL_ADAPT
    if (lat_bound && lane == 0) atomicSub(lat, 1u);
#endif
#if LZ4MI_TIMELINE
    wait_vmem();
    const uint64_t tl_t1 = wall_clock64();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0 && b < kTlMax) {
        g_tl[2 * b] = tl_t0;
        g_tl[2 * b + 1] = tl_t1;
        g_tl_id[2 * b] = hw;
        g_tl_id[2 * b + 1] = xcc;
    }
#endif
}

__global__ __launch_bounds__(64, 4) void lz4mi_decompress_kernel(DecArgs a) { decompress_block<false>(a); }
// small batches: a wave per segment of each block, sequences exported (lz4mi_expand.hip)
__global__ __launch_bounds__(64, 4) void lz4mi_decompress_x_kernel(DecArgs a) { decompress_block<true>(a); }

// After phase 0 and after phase 2 of an exported small batch, per block: the segments in order
// from segment 0 (whose entry is the block's first token): each whose speculative entry equals
// the previous one's exit is final (fin), and one the chain passes over is empty; xfirst[b] = the
// first segment that is neither (xsegs: none), where phase 1 starts; and every later segment's
// re-parse entry for phase 2 (`from`).
__global__ __launch_bounds__(64) void lz4mi_xverify_kernel(DecArgs a) {
    static_assert(kSegMax == 4 * 64, "four records per lane");
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (a.xcnt[b] == kNotExported) return;
    const uint32_t nseg = a.xsegs, in_len = a.in_len[b];
    const SegGeom G = seg_geom(in_len);
    SegRec* R = a.xrec + (size_t)b * nseg;
    // the records, four per lane (segment 64 q + lane), in one round trip; then the walk in registers
    uint32_t entry[4], exit[4], err[4], fail[4], hi_l[4], my_fin[4], kind[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        const bool in = sg < G.S;
        entry[q] = in ? R[sg].entry : 0u;
        exit[q] = in ? R[sg].exit : 0u;
        err[q] = in ? R[sg].err : 0xFFFFFFFFu;
        fail[q] = in ? R[sg].fail : 0u;
        hi_l[q] = sg + 1 >= G.S ? in_len : min(in_len, sg * G.L + G.L);
        my_fin[q] = 0;
        kind[q] = 0;                   // 0 as parsed, 1 empty (after an error / passed over)
    }
    // the previous segment's exit and error, per lane
    uint32_t pex[4], per[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        pex[q] = __shfl_up(exit[q], 1);
        per[q] = __shfl_up(err[q], 1);
        if (lane == 0) {
            pex[q] = q ? __builtin_amdgcn_readlane(exit[q > 0 ? q - 1 : 0], 63) : 0u;
            per[q] = q ? __builtin_amdgcn_readlane(err[q > 0 ? q - 1 : 0], 63) : 0xFFFFFFFFu;
        }
    }
    // the usual case at once: segment 0, and every one after it whose guess the previous one's
    // exit confirms (no error before it, no segment passed over) -- final up to s0, the first
    // that is not (the walk below, one segment at a time, goes on from there)
    uint32_t s0 = G.S;
#pragma unroll
    for (int q = 3; q >= 0; --q) {
        const uint32_t sg = 64u * q + lane;
        const bool ok = sg < G.S && (sg == 0 || (!fail[q] && entry[q] == pex[q] && per[q] == 0xFFFFFFFFu &&
                                                 pex[q] < hi_l[q]));
        const uint64_t bad = __ballot(sg < G.S && !ok);
        if (bad) s0 = 64u * q + (uint32_t)__builtin_ctzll(bad);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (64u * q + lane < s0) my_fin[q] = err[q] != 0xFFFFFFFFu ? kFinErr : exit[q];
    uint32_t first = G.S, prev = 0;    // prev: the previous segment's final exit (kFinErr: an error)
    if (s0 > 0 && s0 < G.S) {
        const uint32_t t = s0 - 1;
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if ((t >> 6) == (uint32_t)q) v = __builtin_amdgcn_readlane(my_fin[q], t & 63);
        prev = v;
    }
    bool stop = s0 >= G.S;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (stop || 64u * q + 63 < s0) continue;
        for (uint32_t l = 64u * q < s0 ? s0 - 64u * q : 0u; l < 64 && !stop; ++l) {
            const uint32_t sg = 64u * q + l;
            if (sg >= G.S) {
                stop = true;
                break;
            }
            const uint32_t hi = __builtin_amdgcn_readlane(hi_l[q], l);
            const uint32_t en = __builtin_amdgcn_readlane(entry[q], l), ex = __builtin_amdgcn_readlane(exit[q], l);
            const uint32_t er = __builtin_amdgcn_readlane(err[q], l), fl = __builtin_amdgcn_readlane(fail[q], l);
            uint32_t fin, k = 0;
            if (sg > 0 && prev == kFinErr) {
                fin = kFinErr;
                k = 1;
            } else if (sg > 0 && prev >= hi) {
                fin = prev;
                k = 1;
            } else if (sg == 0 || (!fl && en == prev)) {
                fin = er != 0xFFFFFFFFu ? kFinErr : ex;
            } else {
                first = sg;
                stop = true;
                break;
            }
            if (lane == l) {
                my_fin[q] = fin;
                kind[q] = k;
            }
            prev = fin;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        if (sg < first) {
            if (kind[q]) {   // nothing here: after the block's first error, or the chain passes over it
                if (my_fin[q] != kFinErr) R[sg].entry = R[sg].exit = my_fin[q];
                R[sg].cnt = 0;
                R[sg].olen = 0;
                R[sg].err = 0xFFFFFFFFu;
            }
            R[sg].fin = my_fin[q] + 1u;
        }
    }
    if (lane == 0) a.xfirst_w[b] = first;
    // the re-parse of phase 2: from the previous segment's exit where a segment at or past the
    // first unchecked one disagrees with it (and that one met no error, its guess did not fail,
    // and it does not pass over this one)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        const bool redo = sg < G.S && sg >= first && sg > 0 && (fail[q] || entry[q] != pex[q]) &&
                          per[q] == 0xFFFFFFFFu && pex[q] >= sg * G.L && pex[q] < hi_l[q];   // (a failed guess: exit 0)
        if (sg < G.S) R[sg].from = redo ? pex[q] : kNoBase;
    }
}

// Dispatch order of a batch (LZ4MI_ORDER). Every block is one wave and a batch of up to
// 16 blocks per CU is resident at once, so a block's decode time is its chain latency under
// the contention of the waves beside it; and workgroups land on CUs by index (round-robin
// over the XCDs and their CUs: w, w + 256, ... share a CU, observed, used for speed only), in
// age order within a SIMD, whose oldest wave wins VALU arbitration. Measured per block
// (tools/timeline.py): tiles216 blocks in the youngest wave slot take 7 % longer than in the
// oldest, and blocks with more compressed bytes longer still, so the launch ends with the
// young heavy blocks; in the 50/50 random/tiles216 mix, CUs that drew more tiles216 blocks
// finish last. The order: blocks with a compression ratio above 2 (latency-bound chains of
// short matches) first, most compressed bytes first, then the rest in index order -- the
// heavy blocks get the oldest slots and every CU the same share of chains. A stable key
// sort (LDS bitonic) in one workgroup; batches of more than kOrderMax blocks keep their order.
constexpr uint32_t kOrderMax = 8192;
__global__ __launch_bounds__(1024) void lz4mi_block_order_kernel(const uint32_t* in_len, const uint32_t* out_cap,
                                                                 uint32_t n, uint32_t* order) {
    __shared__ uint64_t key[kOrderMax];
    const uint32_t t = threadIdx.x;
    uint32_t m = 2;
    while (m < n) m <<= 1;
    for (uint32_t i = t; i < m; i += 1024) {
        uint64_t k = ~0ull;
        if (i < n) {
            const uint32_t il = in_len[i], oc = out_cap[i];   // (a stored frame block: bit 31, not latency-bound)
            const bool lat = (uint64_t)il * 2 < (uint64_t)oc;
            const uint32_t work = LZ4MI_ORDER == 2 ? 0u : (il > 0x7FFFFFFFu ? 0x7FFFFFFFu : il);   // 2: classes only
            const uint32_t hi = lat ? 0x7FFFFFFFu - work : 0x80000000u;
            k = ((uint64_t)hi << 32) | i;
        }
        key[i] = k;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= m; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t i = t; i < (m >> 1); i += 1024) {
                const uint32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const uint64_t x = key[lo], y = key[hi];
                if ((x > y) == asc) {
                    key[lo] = y;
                    key[hi] = x;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = t; i < n; i += 1024) order[i] = (uint32_t)key[i];
}

}  // namespace lz4mi

#if LZ4MI_PROFILE
// Per-phase wall-clock ticks (100 MHz) summed over all waves since the last call; resets.
extern "C" int lz4mi_debug_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lz4mi::g_prof), sizeof(unsigned long long) * 24) != hipSuccess) return -1;
    unsigned long long z[24] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(lz4mi::g_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

#if LZ4MI_TIMELINE
// The last launch's per-block timeline (n <= kTlMax blocks): t[2b] start, t[2b+1] end, id[2b] HW_ID, id[2b+1] XCC_ID.
extern "C" int lz4mi_debug_timeline(unsigned long long* t, unsigned int* id, unsigned int n) {
    if (n > lz4mi::kTlMax) n = lz4mi::kTlMax;
    if (hipMemcpyFromSymbol(t, HIP_SYMBOL(lz4mi::g_tl), sizeof(unsigned long long) * 2 * n) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(id, HIP_SYMBOL(lz4mi::g_tl_id), sizeof(unsigned int) * 2 * n) == hipSuccess ? 0 : -1;
}
#endif

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                              const uint8_t* dict, uint32_t dict_len, uint32_t* out_len,
                                              int32_t* status, uint32_t nblocks, int mode, uint32_t* order,
                                              hipStream_t stream) {
    // mode 0: LZ4 spec; 1: reference-exact serial kernel; 2: spec kernel with the in-chunk
    // reference-exact fix-up of every chunk a double-copy-tail rewrite changes (f1_fixup).
    // order: nblocks words of scratch for the dispatch order (nullptr: index order)
    // mode bit 2 (4): in_len holds frame size words (LZ4MI_FRAME_WORDS)
    const int fw = (mode & 4) ? 1 : 0;
    mode &= 3;
    lz4mi::DecArgs a{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                     nblocks > 1 ? 1 : 0, mode == 2 ? 1 : 0};
    a.frame_words = fw;
    if (nblocks == 0) return hipSuccess;
    if (mode == 1) return lz4mi_launch_decompress_serial(a, stream);
    if (LZ4MI_ORDER && order && nblocks > 1 && nblocks <= lz4mi::kOrderMax) {
        hipLaunchKernelGGL(lz4mi::lz4mi_block_order_kernel, dim3(1), dim3(1024), 0, stream, in_len, out_cap, nblocks,
                           order);
        a.order = order;
    }
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_expand(const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*, const uint64_t*,
                                          const uint32_t*,
                                          const uint8_t*, uint32_t, uint32_t*, int32_t*, const uint4*, const uint32_t*,
                                          lz4mi::SegRec*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*, int,
                                          uint32_t**, uint32_t, hipStream_t);

// A small batch in LZ4 spec or reference mode (lz4mi_expand.hip): each block within the export
// limits (x_in_max compressed, x_out_max output bytes, ratio < 32) is parsed by up to kSegMax
// waves, one per ~kSegTarget bytes of its compressed block (seg_geom), which export its
// sequences instead of writing them; the whole GPU then computes the output by pointer jumping.
// Other blocks are decoded by the same launch as usual. `xs` scratch (lz4mi_small_scratch_bytes):
// the blocks' sequence entries, their counts, first wrong segments and segment records,
// nblocks * x_out_max pointers, and the output kernels' flags.
using lz4mi::kSegMax;
static size_t small_meta_bytes(uint32_t nblocks) {   // counts, first wrong segments, segment records
    return ((size_t)nblocks * 8 + (size_t)nblocks * kSegMax * sizeof(lz4mi::SegRec) + 255) / 256 * 256;
}
extern "C" size_t lz4mi_small_scratch_bytes(uint32_t nblocks, uint32_t x_in_max, uint32_t x_out_max) {
    const size_t seqs = (size_t)nblocks * lz4mi::seg_block_capacity(x_in_max) * 16;
    return (seqs + 255) / 256 * 256 + small_meta_bytes(nblocks) + (size_t)nblocks * x_out_max * 4 +
           128 + ((size_t)nblocks + 63) / 64 * 512 + (size_t)nblocks * (x_out_max / 16) + 256;
}
extern "C" hipError_t lz4mi_launch_decompress_small(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                                    uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                                    const uint8_t* dict, uint32_t dict_len, uint32_t* out_len,
                                                    int32_t* status, uint32_t nblocks, uint32_t x_in_max,
                                                    uint32_t x_out_max, void* xs, int force_reparse, int f1,
                                                    hipStream_t stream) {
    using lz4mi::SegRec;
    if (nblocks == 0) return hipSuccess;
    const uint32_t stride = lz4mi::seg_block_capacity(x_in_max);
    uint8_t* p = (uint8_t*)xs;
    uint4* xseq = (uint4*)p;
    p += ((size_t)nblocks * stride * 16 + 255) / 256 * 256;
    uint32_t* xcnt = (uint32_t*)p;
    uint32_t* xfirst = xcnt + nblocks;
    SegRec* xrec = (SegRec*)(xfirst + nblocks);
    hipError_t e = hipMemsetAsync(p, 0, small_meta_bytes(nblocks), stream);   // exported; records not final
    if (e != hipSuccess) return e;
    p += small_meta_bytes(nblocks);
    uint32_t* ptr = (uint32_t*)p;
    p += (size_t)nblocks * x_out_max * 4;
    uint32_t* aux = (uint32_t*)p;   // jump rounds: round flags, check results, per-thread done bytes
    // (f1check: a block past the export limits is decoded by its segment-0 wave in the caller's mode)
    lz4mi::DecArgs a{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                     nblocks > 1 ? 1 : 0, f1};
    a.xseq = xseq;
    a.xcnt = xcnt;
    a.xrec = xrec;
    a.xseq_stride = stride;
    a.xsegs = kSegMax;
    a.x_in_max = x_in_max;
    a.x_out_max = x_out_max;
    a.xfirst = xfirst;
    a.xfirst_w = xfirst;
    a.xforce = force_reparse;
    // from 64 blocks on, nearly incompressible blocks (compressed >= 15/16 of the output: random data) go to one
    // wave each too: 4 MiB of literal pointers cost more than a wave's copy once there are many such blocks
    // (random 64 / 192 blocks 1.76 / 4.79 -> 0.92 / 1.19 ms, the 50/50 mix 192 blocks 6.16 -> 4.83; below 64 a
    // mix loses: the paced one-wave copies become the critical path -- 32 blocks 1.43 -> 1.62; round 6, profiles/r06fl)
    a.x_flat1 = nblocks >= 64 ? 1 : 0;
    // phase 0: every segment speculatively; the check; phase 1: the segments from the first
    // wrong entry on (an empty launch when there is none). A phase-1 wave waits only for its
    // predecessor, whose workgroup index is lower (dispatched first): the wait always ends.
    const dim3 grid(nblocks * kSegMax);
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_x_kernel, grid, dim3(64), 0, stream, a);
    hipLaunchKernelGGL(lz4mi::lz4mi_xverify_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    // phase 2: the segments whose guesses disagree, re-parsed at once, then the check again;
    // phase 1 chains what is left (a second phase-2 pass: ~11 us of empty launches per call
    // once the guesses restart past impossible tokens)
    a.xphase = 2;
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_x_kernel, grid, dim3(64), 0, stream, a);
    hipLaunchKernelGGL(lz4mi::lz4mi_xverify_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    a.xphase = 1;
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_x_kernel, grid, dim3(64), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    uint32_t* redo = nullptr;
    e = lz4mi_launch_expand(in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, xseq, xcnt, xrec,
                            kSegMax, stride, ptr, x_out_max, aux, f1, &redo, nblocks, stream);
    if (e != hipSuccess || !f1) return e;
    // reference mode (LZ4MI_JS_EXACT): the double-copy-tail rewrites were applied to the pointers
    // (lz4mi_xf1ptr_kernel); a block with a rewrite reading before the block is decoded again by the
    // batch kernel (LZ4MI_ERR_CROSS_BLOCK when batched); the launch is empty when there is none
    lz4mi::DecArgs r{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                     nblocks > 1 ? 1 : 0, 1};
    r.redo = redo;
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_kernel, dim3(nblocks), dim3(64), 0, stream, r);
    return hipGetLastError();
}
