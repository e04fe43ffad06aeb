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
// (~9.9 KiB LDS, <= 128 VGPRs -> 16 waves per CU). Per 1 KiB chunk of the
// compressed stream:
//  1. Stage it (+64 B lookahead) in LDS.
//  2. next(p) of every position, branch-free (length fields of one extension
//     byte; longer ones through a ballot-gated exact loop) into an LDS table.
//  3. Speculative walks: lane l walks next() from 64 bytes before its 16-byte
//     segment and records the tokens it visits in the segment; LZ4 token
//     chains resynchronise within a few steps, so walks are almost always on
//     the true chain. Certification left to right by ballot: the first lane
//     whose left neighbour's exit is not on its walk re-walks from it. The
//     result is the exact serial parse.
//  4. Sequence table in LDS (literal source, lengths, offset, output start by
//     wave prefix sums), errors in the reference's order, an output->sequence
//     bucket map, and for every match its final source resolved once (through
//     earlier sequences of the chunk down to a literal or to output finished
//     by an earlier chunk).
//  5. Output in 16-byte units aligned in the output address space, sequence-
//     parallel: lane l takes sequence 64i+l and writes every unit whose first
//     byte lies in it (a unit running into the next sequence takes its second
//     source window from that sequence's entry), all loads in flight before
//     the stores, 1 KiB per wave store instruction. Long sequences go to the
//     whole wave; earlier output is read back from L2 (bypassing L1).
//  6. A sequence whose parse leaves the staged window (long literal runs or
//     length varints: incompressible or highly repetitive data) is parsed from
//     global memory with wave-wide 255-run scans and produced by the whole wave
//     as a bulk literal copy and a bulk (possibly periodic) match copy.
#include "lz4mi_common.h"
#include "lz4mi_decompress.h"

#ifndef LZ4MI_ABLATE
#define LZ4MI_ABLATE 0   // timing-only variant (tools/): 1 = parse + table only, no output
#endif

namespace lz4mi {

constexpr int kChunk = 1024;                  // compressed bytes parsed per step
constexpr int kPad = 64;                      // lookahead for sequences straddling the chunk end
constexpr int kLim = kChunk + kPad;           // chunk-relative bytes a regular sequence may touch
constexpr int kStageWords = (kLim + 28) / 4;  // + 3-byte shift + 20-byte load window
constexpr int kMaxSeq = kChunk / 3 + 4;       // every non-final sequence is >= 3 bytes
constexpr int kBuckets = 1024;                // output -> sequence map granularity
constexpr int kMaxVarint = 250;               // longer length varints go to the cut path (ml < 65536)
constexpr uint32_t kEnd = 0x40000000u;        // chain ends (last sequence of the block)
constexpr uint32_t kStop = 0x40000001u;       // sequence cannot be parsed inside the window
constexpr int kU = 2;                         // output units per lane in flight
constexpr int kLaneUnits = 8;                 // sequences with more units are produced by the whole wave

struct DecShared {
    uint32_t stage[kStageWords];
    uint32_t t_out[kMaxSeq + 1];  // output start of each sequence (block-relative); [nseq] = table end
    uint2 t_info[kMaxSeq + 1];    // {literal source (chunk-relative) | literal length << 16,
                                  //  match offset | match length << 16 (0: final literal-only sequence)}
    uint32_t t_src[kMaxSeq + 1];  // final source of each match (pack_src)
    uint16_t u2s[kLim];           // next-token table during the parse, then the bucket map
    uint32_t unit[kWave * 4];     // per-lane 16-byte assembly slot / phase table
};

struct Ctx {
    const uint8_t* blk;   // compressed block
    uint8_t* dst;         // output start of the block (out + out_off)
    int64_t out_off;      // absolute position of dst in `out`
    int32_t in_len;
    int32_t cap;          // writable bytes from dst
    const uint8_t* dict;
    int32_t dict_len;
    int isolate;
    int32_t mis;          // dst address mod 16 (units are aligned in the address space)
    int32_t ip;           // chunk start (block-relative compressed position)
    uint32_t sh;          // staging shift
    int64_t O;            // output start of the current table (block-relative)
    uint32_t nseq;
    uint32_t shift;       // bucket = (y - O) >> shift
    uint32_t nbk;
};

// ---------------------------------------------------------------- parsing
// Position of the token after the one at p (chunk-relative), or kEnd / kStop.
// Exact for any field lengths.
__device__ uint32_t next_token(const uint8_t* s, uint32_t p, uint32_t rem) {
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

__device__ __forceinline__ uint32_t next_of(const uint16_t* nxt, uint32_t p) {
    uint32_t v = nxt[p];
    return v >= 0xFFFEu ? (v == 0xFFFEu ? kEnd : kStop) : v;
}

struct SeqInfo {
    int32_t lit, ll, off, ml;
};
__device__ __forceinline__ SeqInfo seq_info(const DecShared& S, uint32_t k) {
    uint2 v = S.t_info[k];
    return SeqInfo{(int32_t)(v.x & 0xFFFF), (int32_t)(v.x >> 16), (int32_t)(v.y & 0xFFFF), (int32_t)(v.y >> 16)};
}

// Last sequence whose output start is <= y (y inside the table's output).
__device__ __forceinline__ uint32_t seq_at(const Ctx& c, const DecShared& S, int32_t y) {
    uint32_t b = (uint32_t)(y - (int32_t)c.O) >> c.shift;
    if (b >= c.nbk) b = c.nbk - 1;
    uint32_t s = S.u2s[b];
    while (s + 1 < c.nseq && (int32_t)S.t_out[s + 1] <= y) ++s;
    return s;
}

// ------------------------------------------------------------ byte access
__device__ __forceinline__ uint32_t stage_byte(const DecShared& S, uint32_t idx) {
    return ((const uint8_t*)S.stage)[idx];
}

// Byte of earlier output at block-relative position pos (dictionary below out[0]).
__device__ __forceinline__ uint32_t hist_byte(const Ctx& c, int64_t pos) {
    int64_t abs = c.out_off + pos;
    if (abs >= 0) return ld_nt_u8(c.dst + pos);
    return c.dict ? c.dict[c.dict_len + abs] : 0u;
}

// ------------------------------------------------------ source resolution
enum : uint32_t { K_HIST = 0, K_COMP = 1, K_GCOMP = 2, K_SLOW = 3 };

// A contiguous source run: K_HIST = earlier output (block-relative position,
// read back from L2), K_COMP = staged stream (LDS byte index), K_GCOMP =
// compressed stream in global memory (block-relative position).
struct Src {
    int32_t pos;
    int32_t m;
    uint32_t kind;
};

__device__ __forceinline__ uint32_t pack_src(uint32_t kind, int32_t pos) {
    return (kind << 30) | ((uint32_t)pos & 0x3FFFFFFFu);
}
__device__ __forceinline__ uint32_t src_kind(uint32_t v) { return v >> 30; }
__device__ __forceinline__ int32_t src_pos(uint32_t v) { return ((int32_t)(v << 2)) >> 2; }

// Can a 20-byte window be read at pos? (16 bytes + alignment slack)
__device__ __forceinline__ bool window_ok(const Ctx& c, uint32_t kind, int32_t pos) {
    if (kind == K_COMP) return pos >= 0;
    if (kind == K_HIST) return c.out_off + pos >= 4 && pos + 20 <= c.cap;
    return pos >= 4 && pos + 20 <= c.in_len;
}

// Final source of the output run [y, y+m) of the current table, following
// back-references through earlier sequences (periodic matches map straight
// below their start); m shrinks to where the source stays contiguous.
__device__ Src resolve(const Ctx& c, const DecShared& S, int32_t y, int32_t m) {
    for (int d = 0; d < 16; ++d) {
        if (y < (int32_t)c.O) {
            if (m > (int32_t)c.O - y) m = (int32_t)c.O - y;
            return Src{y, m, window_ok(c, K_HIST, y) ? K_HIST : K_SLOW};
        }
        uint32_t s = seq_at(c, S, y);
        int32_t t0 = (int32_t)S.t_out[s];
        int32_t rel = y - t0;
        SeqInfo q = seq_info(S, s);
        if (rel < q.ll) {
            if (m > q.ll - rel) m = q.ll - rel;
            return Src{(int32_t)c.sh + q.lit + rel, m, K_COMP};
        }
        int32_t mrel = rel - q.ll;
        if (m > q.ml - mrel) m = q.ml - mrel;
        int32_t r = mrel < q.off ? mrel : mrel % q.off;
        if (m > q.off - r) m = q.off - r;
        y = t0 + q.ll - q.off + r;
    }
    return Src{y, m, K_SLOW};
}

// Source of the output run starting at y (at most `want` bytes) inside a
// sequence (output start t0, fields q, packed match source sv).
__device__ __forceinline__ Src seq_piece(const Ctx& c, int32_t t0, const SeqInfo& q, uint32_t sv, int32_t y,
                                         int32_t want) {
    const int32_t rel = y - t0;
    if (rel < q.ll) return Src{(int32_t)c.sh + q.lit + rel, min(want, q.ll - rel), K_COMP};
    const int32_t d = rel - q.ll;
    uint32_t kind = src_kind(sv);
    int32_t pos = src_pos(sv), m;
    if (q.off >= q.ml) {
        pos += d;
        m = q.ml - d;
    } else {
        int32_t r = d < q.off ? d : d % q.off;
        pos += r;
        m = min(q.off - r, q.ml - d);
    }
    if (kind == K_HIST && pos + 20 > c.cap) kind = K_SLOW;
    return Src{pos, min(m, want), kind};
}

// Same, locating the sequence through the bucket map.
__device__ __forceinline__ Src table_src(const Ctx& c, const DecShared& S, int32_t y, int32_t want) {
    uint32_t s = seq_at(c, S, y);
    return seq_piece(c, (int32_t)S.t_out[s], seq_info(S, s), S.t_src[s], y, want);
}

// Bulk mapping (the one sequence a chunk could not hold): out[y] is source
// byte base + phase, phase = y - lo, or (y - lo) mod period for a periodic match.
struct Bulk {
    uint32_t kind;
    int32_t base, lo, period;
};

__device__ __forceinline__ Src bulk_src(const Ctx& c, const Bulk& B, int32_t y, int32_t want) {
    int32_t d = y - B.lo;
    int32_t r = B.period ? d % B.period : d;
    int32_t m = B.period ? min(want, B.period - r) : want;
    int32_t pos = B.base + r;
    return Src{pos, m, window_ok(c, B.kind, pos) ? B.kind : K_SLOW};
}

__device__ __forceinline__ uint4 funnel4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4, uint32_t b) {
    return make_uint4(funnel(d0, d1, b), funnel(d1, d2, b), funnel(d2, d3, b), funnel(d3, d4, b));
}

// 16 source bytes of a run. One code path for all kinds: a generic pointer
// into the staged stream (LDS) or global memory, read as 5 aligned dwords
// (non-temporal: output history is read from L2, never from a stale L1).
__device__ __forceinline__ uint4 fetch16(const Ctx& c, const DecShared& S, const Src& r) {
    const uint8_t* base = r.kind == K_COMP ? (const uint8_t*)S.stage : (r.kind == K_HIST ? (const uint8_t*)c.dst : c.blk);
    uintptr_t a = (uintptr_t)(base + r.pos), a0 = a & ~(uintptr_t)3;
    const uint32_t* q = (const uint32_t*)a0;
    return funnel4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1), __builtin_nontemporal_load(q + 2),
                   __builtin_nontemporal_load(q + 3), __builtin_nontemporal_load(q + 4), (uint32_t)(a - a0));
}

// bytes [0, k) from a, the rest from b
__device__ __forceinline__ uint32_t pick(uint32_t a, uint32_t b, int32_t k) {
    if (k >= 4) return a;
    if (k <= 0) return b;
    uint32_t m = (1u << (8 * k)) - 1u;
    return (a & m) | (b & ~m);
}

// Unit alignment: units are 16-byte aligned in the address space of dst.
__device__ __forceinline__ int32_t fl16(int32_t y, int32_t mis) { return ((y + mis) & ~15) - mis; }
__device__ __forceinline__ int32_t cl16(int32_t y, int32_t mis) { return ((y + mis + 15) & ~15) - mis; }

// Byte-wise unit (unit edges, runs that split more than once, dictionary
// reads): resolved run by run, assembled in the lane's LDS slot.
__device__ void unit_bytes(const Ctx& c, DecShared& S, int lane, int32_t y, int32_t n, bool bulk, const Bulk& B) {
    uint8_t* ub = (uint8_t*)&S.unit[lane * 4];
    int32_t k = 0;
    while (k < n) {
        int32_t yc = y + k, m = n - k;
        uint32_t kind;
        int64_t sp;
        if (bulk) {
            int32_t d = yc - B.lo;
            int32_t r = B.period ? d % B.period : d;
            if (B.period && B.period - r < m) m = B.period - r;
            kind = B.kind;
            sp = (int64_t)B.base + r;
        } else {
            for (;;) {
                if (yc < (int32_t)c.O) {
                    if (m > (int32_t)c.O - yc) m = (int32_t)c.O - yc;
                    kind = K_HIST;
                    sp = yc;
                    break;
                }
                uint32_t s = seq_at(c, S, yc);
                int32_t t0 = (int32_t)S.t_out[s];
                int32_t rel = yc - t0;
                SeqInfo q = seq_info(S, s);
                if (rel < q.ll) {
                    if (m > q.ll - rel) m = q.ll - rel;
                    kind = K_COMP;
                    sp = (int64_t)c.sh + q.lit + rel;
                    break;
                }
                int32_t mrel = rel - q.ll;
                if (m > q.ml - mrel) m = q.ml - mrel;
                int32_t r = mrel < q.off ? mrel : mrel % q.off;
                if (m > q.off - r) m = q.off - r;
                yc = t0 + q.ll - q.off + r;
            }
        }
        for (int32_t j = 0; j < m; ++j) {
            uint32_t v;
            if (kind == K_HIST) v = hist_byte(c, sp + j);
            else if (kind == K_COMP) v = stage_byte(S, (uint32_t)(sp + j));
            else v = (sp + j < c.in_len) ? c.blk[sp + j] : 0u;
            ub[k + j] = (uint8_t)v;
        }
        k += m;
    }
    if (n == 16) {
        *(uint4*)(c.dst + y) = *(const uint4*)&S.unit[lane * 4];
    } else {
        for (int32_t j = 0; j < n; ++j) c.dst[y + j] = ub[j];
    }
}

template <int N>
__device__ __forceinline__ int32_t pick_slot(const int32_t (&a)[N], int j) {
    int32_t v = a[0];
#pragma unroll
    for (int i = 1; i < N; ++i) v = j == i ? a[i] : v;
    return v;
}

// Units prepared by the producers below: md 1 = one window, 2 = two windows
// (bytes [0, A.m) from A, the rest from R), 3 = byte-wise.
struct UnitBatch {
    Src A[kU], R[kU];
    int32_t y[kU], n[kU];
    uint32_t md[kU];
};

__device__ __forceinline__ void plan_two(const Ctx& c, UnitBatch& U, int j) {
    U.R[j].pos -= U.A[j].m;     // R's bytes land at unit offset A.m
    if (U.R[j].kind != K_SLOW && U.A[j].m + U.R[j].m == 16 && window_ok(c, U.R[j].kind, U.R[j].pos)) U.md[j] = 2;
}

// Load, merge and store a batch: every load is in flight before the first store.
__device__ __forceinline__ void emit_units(const Ctx& c, DecShared& S, int lane, const UnitBatch& U, bool bulk,
                                           const Bulk& B) {
    uint4 va[kU], vb[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        if (U.md[j] == 1 || U.md[j] == 2) va[j] = fetch16(c, S, U.A[j]);
        if (U.md[j] == 2) vb[j] = fetch16(c, S, U.R[j]);
    }
    uint32_t slow = 0;
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        if (U.md[j] == 1) {
            *(uint4*)(c.dst + U.y[j]) = va[j];
        } else if (U.md[j] == 2) {
            int32_t k = U.A[j].m;
            *(uint4*)(c.dst + U.y[j]) = make_uint4(pick(va[j].x, vb[j].x, k), pick(va[j].y, vb[j].y, k - 4),
                                                   pick(va[j].z, vb[j].z, k - 8), pick(va[j].w, vb[j].w, k - 12));
        }
        slow |= (U.md[j] == 3 ? 1u : 0u) << j;
    }
    if (__ballot(slow != 0)) {
        while (slow) {       // one call site for the byte-wise path
            int j = __builtin_ctz(slow);
            slow &= slow - 1;
            unit_bytes(c, S, lane, pick_slot(U.y, j), pick_slot(U.n, j), bulk, B);
        }
    }
}

// Whole-wave production of out[lo, hi): units spread over the lanes, each
// unit's sources found through the table (or the Bulk mapping).
__device__ void produce_units(const Ctx& c, DecShared& S, int lane, int32_t lo, int32_t hi, bool bulk, Bulk B) {
    if (lo >= hi) return;
    const int32_t y0 = fl16(lo, c.mis);
    const uint32_t nunits = (uint32_t)(cl16(hi, c.mis) - y0) >> 4;
    for (uint32_t u0 = lane; u0 < nunits; u0 += kWave * kU) {
        UnitBatch U;
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            uint32_t u = u0 + kWave * j;
            int32_t ua = y0 + 16 * (int32_t)u;
            U.y[j] = ua < lo ? lo : ua;
            U.n[j] = (ua + 16 > hi ? hi : ua + 16) - U.y[j];
            U.md[j] = u < nunits ? 3u : 0u;
            if (u < nunits && U.n[j] == 16) {
                U.A[j] = bulk ? bulk_src(c, B, U.y[j], 16) : table_src(c, S, U.y[j], 16);
                if (U.A[j].kind != K_SLOW) {
                    if (U.A[j].m == 16) {
                        U.md[j] = 1;
                    } else {
                        int32_t y2 = U.y[j] + U.A[j].m, w = 16 - U.A[j].m;
                        U.R[j] = bulk ? bulk_src(c, B, y2, w) : table_src(c, S, y2, w);
                        plan_two(c, U, j);
                    }
                }
            }
        }
        emit_units(c, S, lane, U, bulk, B);
    }
}

// Sequence-parallel production of the table: lane l takes sequence 64i+l and
// writes the units whose first byte lies in it (sequence 0 also the partial
// unit holding lo), at most kLaneUnits; longer sequences are flagged in
// `longbits` (bit i) for the whole wave. All fields come from the sequence's
// entry and the next one: no per-unit lookups.
__device__ void produce_seqs(const Ctx& c, DecShared& S, int lane, int32_t lo, int32_t hi, uint32_t& longbits) {
    const Bulk none{0, 0, 0, 0};
    for (uint32_t i = 0; 64 * i < c.nseq; ++i) {
        const uint32_t k = 64 * i + lane;
        int32_t first = 0, nu = 0, t0 = 0, t1 = 0;
        SeqInfo q{0, 0, 0, 0}, qn{0, 0, 0, 0};
        uint32_t sv = 0, svn = 0;
        if (k < c.nseq) {
            t0 = (int32_t)S.t_out[k];
            t1 = (int32_t)S.t_out[k + 1];
            q = seq_info(S, k);
            sv = S.t_src[k];
            qn = seq_info(S, k + 1);
            svn = S.t_src[k + 1];
            first = k == 0 ? fl16(lo, c.mis) : cl16(t0, c.mis);
            const int32_t t1c = t1 < hi ? t1 : hi;
            nu = t1c > first ? (t1c - first + 15) >> 4 : 0;
            if (nu > kLaneUnits) {
                longbits |= 1u << i;
                nu = 0;
            }
        }
        for (int32_t j0 = 0; __ballot(j0 < nu) != 0; j0 += kU) {
            UnitBatch U;
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int32_t u = first + 16 * (j0 + j);
                U.md[j] = 0;
                U.y[j] = u < lo ? lo : u;
                U.n[j] = (u + 16 < hi ? u + 16 : hi) - U.y[j];
                if (j0 + j < nu) {
                    U.md[j] = 3;
                    if (U.n[j] == 16) {
                        U.A[j] = seq_piece(c, t0, q, sv, U.y[j], 16);
                        if (U.A[j].kind != K_SLOW) {
                            if (U.A[j].m == 16) {
                                U.md[j] = 1;
                            } else {
                                const int32_t y2 = U.y[j] + U.A[j].m, w = 16 - U.A[j].m;
                                U.R[j] = y2 < t1 ? seq_piece(c, t0, q, sv, y2, w) : seq_piece(c, t1, qn, svn, y2, w);
                                plan_two(c, U, j);
                            }
                        }
                    }
                }
            }
            emit_units(c, S, lane, U, false, none);
        }
    }
}

// Periodic match with offset < 16 (long runs of a short pattern): the content
// of a unit depends only on its phase; build the `off` phases once in LDS.
__device__ __noinline__ void produce_short_period(const Ctx& c, DecShared& S, int lane, int32_t ms, int32_t hi,
                                                  int32_t off) {
    if (ms >= hi) return;
    uint8_t* pat = (uint8_t*)S.unit;
    const int32_t sb = ms - off;
    __syncthreads();
    for (int idx = lane; idx < 16 * off; idx += kWave) {
        int r = idx >> 4, j = idx & 15;
        pat[idx] = (uint8_t)hist_byte(c, sb + (r + j) % off);
    }
    __syncthreads();
    const int32_t y0 = fl16(ms, c.mis);
    const uint32_t nunits = (uint32_t)(cl16(hi, c.mis) - y0) >> 4;
    for (uint32_t u = lane; u < nunits; u += kWave) {
        int32_t ua = y0 + 16 * (int32_t)u;
        int32_t y = ua < ms ? ms : ua;
        int32_t n = (ua + 16 > hi ? hi : ua + 16) - y;
        int32_t r = (y - ms) % off;
        if (n == 16) {
            *(uint4*)(c.dst + y) = *(const uint4*)(pat + 16 * r);
        } else {
            for (int32_t j = 0; j < n; ++j) c.dst[y + j] = pat[16 * r + j];
        }
    }
    __syncthreads();
}

// Wave-wide 255-run varint starting at block-relative q: returns the sum and
// advances q past the terminating byte. Bytes past the block end read as 0.
__device__ __noinline__ int64_t wave_varint(const Ctx& c, int lane, int64_t& q) {
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
            int fi = __shfl(first, fl, kWave);
            uint32_t fb = __shfl(lastb, fl, kWave);
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

__global__ __launch_bounds__(64, 4) void lz4mi_decompress_kernel(DecArgs a) {
    __shared__ DecShared S;
    const int lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    if (b >= a.nblocks) return;

    Ctx c;
    c.blk = a.in + a.in_off[b];
    c.in_len = (int32_t)a.in_len[b];
    c.out_off = (int64_t)a.out_off[b];
    c.dst = a.out + a.out_off[b];
    c.cap = a.out_cap[b] > 0x7FFFFFFFu ? 0x7FFFFFFF : (int32_t)a.out_cap[b];
    c.dict = a.dict;
    c.dict_len = a.dict ? (int32_t)a.dict_len : 0;
    c.isolate = a.isolate;
    c.mis = (int32_t)((uintptr_t)c.dst & 15);
    c.ip = 0;
    c.O = 0;
    int32_t status = 0;

    while (c.ip < c.in_len) {
        // ---- 1. stage [ip, ip + kLim) ------------------------------------
        {
            const uintptr_t A = (uintptr_t)(c.blk + c.ip), A0 = A & ~(uintptr_t)3;
            c.sh = (uint32_t)(A - A0);
            const int64_t rel0 = (int64_t)A0 - (int64_t)(uintptr_t)c.blk;
            const bool inside = rel0 >= 0 && rel0 + 4 * kStageWords <= c.in_len;
            for (int k = lane; k < kStageWords; k += kWave) {
                const int64_t rel = rel0 + 4 * k;
                uint32_t v;
                if (inside) {
                    v = *(const uint32_t*)(A0 + 4 * (uintptr_t)k);
                } else {
                    v = 0;
                    for (int j = 0; j < 4; ++j) {
                        int64_t r = rel + j;
                        if (r >= 0 && r < c.in_len) v |= (uint32_t)c.blk[r] << (8 * j);
                    }
                }
                S.stage[k] = v;
            }
        }
        __syncthreads();
        const uint8_t* s = (const uint8_t*)S.stage + c.sh;
        const uint32_t rem = (uint32_t)(c.in_len - c.ip);

        // ---- 2. next-token table -----------------------------------------
        uint16_t* nxt = S.u2s;   // the bucket map is built after the parse
        for (uint32_t p = lane; p < (uint32_t)kLim; p += kWave) {
            bool slow;
            uint32_t v = next_fast(s, p, rem, slow);
            if (__ballot(slow)) {
                if (slow) v = next_token(s, p, rem);
            }
            nxt[p] = (uint16_t)(v == kEnd ? 0xFFFEu : v == kStop ? 0xFFFFu : v);
        }
        __syncthreads();

        // ---- 3. speculative walks + certification -------------------------
        const uint32_t seg0 = 16u * lane, seg1 = seg0 + 16;
        uint32_t vis = 0, x;
        {   // 64-byte warm-up; lanes 0-3 start at the chunk start, a true token
            uint32_t p = seg0 < 64 ? 0u : seg0 - 64;
            while (p < seg1) {
                if (p >= seg0) vis |= 1u << (p - seg0);
                p = next_of(nxt, p);
            }
            x = p;
        }
        uint32_t es = vis ? seg0 + __builtin_ctz(vis) : x;
        uint32_t nE = 0;
        for (int it = 0; it <= kWave; ++it) {
            uint32_t pes = __shfl_up(es, 1, kWave), px = __shfl_up(x, 1, kWave);
            nE = lane == 0 ? 0u : (pes >= seg0 ? pes : px);
            bool valid = nE >= seg1 ? (vis == 0 && x == nE) : ((vis >> (nE - seg0)) & 1u) != 0;
            uint64_t bad = __ballot(!valid);
            if (bad == 0) break;
            if (lane == __builtin_ctzll(bad)) {     // first inconsistent lane: re-walk from its true entry
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
        const uint32_t tail = uniform(__shfl(x, kWave - 1, kWave));   // where the chain leaves the chunk
        const uint64_t has = __ballot(vis != 0);
        const int last_lane = 63 - __builtin_clzll(has);
        const uint32_t last_tok = uniform(__shfl(seg0 + 31 - __builtin_clz(vis | 1u), last_lane, kWave));
        const bool cut = tail == kStop;

        // ---- 4. sequence table -----------------------------------------
        const uint32_t cnt = __popc(vis) - ((cut && lane == last_lane) ? 1u : 0u);
        const uint32_t incl = wave_incl_scan(cnt, lane);
        const uint32_t base = incl - cnt;
        const uint32_t nseq = uniform(__shfl(incl, kWave - 1, kWave));
        uint32_t run = 0;
        {
            uint32_t m = vis, k = base;
            for (uint32_t i = 0; i < cnt; ++i) {
                const uint32_t p = seg0 + __builtin_ctz(m);
                m &= m - 1;
                const uint32_t tok = s[p], b1 = s[p + 1];
                uint32_t q = p + 1, ll = tok >> 4;
                if (ll == 15) {
                    if (b1 != 255) { ll += b1; ++q; }
                    else { uint32_t bb; do { bb = s[q++]; ll += bb; } while (bb == 255); }
                }
                const uint32_t lit = q;
                q += ll;
                uint32_t off = 0, ml = 0;
                if (q < rem) {
                    off = (uint32_t)s[q] | ((uint32_t)s[q + 1] << 8);
                    ml = tok & 15;
                    if (ml == 15) {
                        uint32_t bb = s[q + 2];
                        if (bb != 255) ml += bb;
                        else { uint32_t r = q + 2; do { bb = s[r++]; ml += bb; } while (bb == 255); }
                    }
                    ml += 4;
                }
                S.t_info[k] = make_uint2(lit | (ll << 16), off | (ml << 16));
                S.t_out[k] = run;
                run += ll + ml;
                ++k;
            }
        }
        const uint32_t lincl = wave_incl_scan(run, lane);
        const uint32_t lbase = lincl - run;
        const int64_t total = uniform(__shfl(lincl, kWave - 1, kWave));
        uint32_t shift = 4;
        while ((total >> shift) >= kBuckets) ++shift;
        c.shift = shift;
        c.nbk = (uint32_t)((total + (1 << shift) - 1) >> shift);
        if (c.nbk == 0) c.nbk = 1;
        c.nseq = nseq;
        uint32_t first_err = 0xFFFFFFFFu;
        for (uint32_t k = base; k < base + cnt; ++k) {
            const int64_t loc = (int64_t)lbase + S.t_out[k];
            const int64_t os = c.O + loc;
            S.t_out[k] = (uint32_t)os;
            const SeqInfo q = seq_info(S, k);
            const uint32_t e = seq_error(c, os, (int64_t)c.ip + q.lit, q.ll, q.off, q.ml);
            if (e && first_err == 0xFFFFFFFFu) first_err = (k << 3) | e;
            const int64_t B = 1ll << shift;
            int64_t fb = (loc + B - 1) >> shift, lb = (loc + q.ll + q.ml + B - 1) >> shift;
            if (lb > (int64_t)c.nbk) lb = c.nbk;
            for (int64_t bq = fb; bq < lb; ++bq) S.u2s[bq] = (uint16_t)k;
        }
        if (lane == 0) {           // sentinel entry: the table's end
            S.t_out[nseq] = (uint32_t)(c.O + total);
            S.t_info[nseq] = make_uint2(0, 0);
            S.t_src[nseq] = pack_src(K_SLOW, 0);
        }
        first_err = wave_min(first_err);
        __syncthreads();
        if (first_err != 0xFFFFFFFFu) { status = err_status(first_err & 7); break; }

        // each match's final source, resolved once (sequence-parallel)
        for (uint32_t k = lane; k < nseq; k += kWave) {
            const SeqInfo q = seq_info(S, k);
            uint32_t sv = pack_src(K_SLOW, 0);
            const bool per = q.off < q.ml;
            if (q.ml && (!per || q.off >= 16)) {     // shorter periods go byte-wise
                const int32_t want = per ? q.off : q.ml;
                const Src r = resolve(c, S, (int32_t)S.t_out[k] + q.ll - q.off, want);
                if (r.kind != K_SLOW && r.m == want && r.pos < (1 << 29) && r.pos >= -(1 << 29))
                    sv = pack_src(r.kind, r.pos);
            }
            S.t_src[k] = sv;
        }
        __syncthreads();

        // ---- 6. the sequence the window could not hold: parse it from memory
        int64_t cq = 0, cll = 0, cml = 0, clit = 0;
        uint32_t coff = 0;
        if (cut) {
            int64_t q = (int64_t)c.ip + last_tok;
            const uint32_t tok = q < c.in_len ? c.blk[q] : 0u;
            ++q;
            cll = tok >> 4;
            if (cll == 15) cll += wave_varint(c, lane, q);
            clit = q;
            q += cll;
            if (q < c.in_len) {
                coff = (uint32_t)c.blk[q] | ((uint32_t)(q + 1 < c.in_len ? c.blk[q + 1] : 0) << 8);
                q += 2;
                cml = tok & 15;
                if (cml == 15) cml += wave_varint(c, lane, q);
                cml += 4;
            }
            cq = q;
        }
        const int64_t tab_hi = c.O + total;
        const int64_t tab_end = tab_hi < (int64_t)c.cap ? tab_hi : (int64_t)c.cap;

        // ---- 5. produce: table sequences lane-parallel, then (whole wave)
        // the long ones, the cut sequence's literal run and, once everything
        // below it is stored, its match run
        uint32_t longbits = 0;
#if LZ4MI_ABLATE != 1
        if (nseq && c.O < tab_end) produce_seqs(c, S, lane, (int32_t)c.O, (int32_t)tab_end, longbits);
#endif
        uint64_t longlanes = __ballot(longbits != 0);
        uint32_t lbits = 0;
        int llane = 0;
        int job = 0;     // 0 long table sequences, 1 cut literal, 2 cut match
        while (job < 3) {
            int64_t lo = 0, hi = 0;
            const bool bulk = job > 0;
            Bulk B{0, 0, 0, 0};
            if (job == 0) {
                if (lbits == 0) {
                    if (longlanes == 0) { job = 1; continue; }
                    llane = __builtin_ctzll(longlanes);
                    longlanes &= longlanes - 1;
                    lbits = uniform(__shfl(longbits, llane, kWave));
                }
                const uint32_t k = 64 * __builtin_ctz(lbits) + llane;
                lbits &= lbits - 1;
                const int32_t t0 = (int32_t)S.t_out[k], t1 = (int32_t)S.t_out[k + 1];
                lo = k == 0 ? c.O : cl16(t0, c.mis);
                hi = t1 < tab_end ? cl16(t1, c.mis) : tab_end;
                if (hi > tab_end) hi = tab_end;
            } else if (job == 1) {
                job = 2;
                if (!cut) break;
                const uint32_t e = seq_error(c, tab_hi, clit, cll, coff, cml);
                if (e) { status = err_status(e); break; }
                lo = tab_hi;
                hi = tab_hi + cll;
                B = Bulk{K_GCOMP, (int32_t)clit, (int32_t)lo, 0};
            } else {
                job = 3;
                lo = tab_hi + cll;
                hi = lo + cml;
                if (cml == 0 || lo >= c.cap) break;
                wait_vmem();    // everything below the match is read back as history
                if ((int64_t)coff < cml && coff < 16) {
                    produce_short_period(c, S, lane, (int32_t)lo, (int32_t)(hi < c.cap ? hi : c.cap), (int32_t)coff);
                    break;
                }
                B = Bulk{K_HIST, (int32_t)(lo - coff), (int32_t)lo, (int64_t)coff < cml ? (int32_t)coff : 0};
            }
            if (hi > c.cap) hi = c.cap;
            if (lo < hi) produce_units(c, S, lane, (int32_t)lo, (int32_t)hi, bulk, B);
        }
        if (status) break;
        c.O = tab_hi;
        if (cut) {
            c.O += cll + cml;
            c.ip = (int32_t)(cq < c.in_len ? cq : c.in_len);
        } else if (tail >= kEnd) {
            c.ip = c.in_len;
        } else {
            c.ip += (int32_t)tail;
        }
        wait_vmem();        // this chunk's stores are complete before the next chunk reads them back
        __syncthreads();
    }
    if (lane == 0) {
        a.status[b] = status;
        a.out_len[b] = status ? 0u : (uint32_t)c.O;
    }
}

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                              const uint8_t* dict, uint32_t dict_len, uint32_t* out_len,
                                              int32_t* status, uint32_t nblocks, int js_compat, hipStream_t stream) {
    lz4mi::DecArgs a{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                     nblocks > 1 ? 1 : 0};
    if (nblocks == 0) return hipSuccess;
    if (js_compat) return lz4mi_launch_decompress_serial(a, stream);
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    return hipGetLastError();
}
