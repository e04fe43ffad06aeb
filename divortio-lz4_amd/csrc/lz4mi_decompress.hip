// lz4mi_decompress.hip — LZ4 raw-block decoder for MI355X (gfx950).
//
// Replaces decompressBlock (reference src/block/blockDecompress.js:30-275) for
// batches of independent blocks. Semantics follow the reference exactly for
// spec-valid input (positions absolute in `out`, dictionary below out[0],
// clipped match writes, the four error strings); LZ4MI_JS_COMPAT selects the
// serial kernel at the bottom, which also reproduces the reference's
// double-copy-tail rewrite.
//
// Design (one wave64 per block, all blocks resident at once):
//  1. Stage 1 KiB (+64 B lookahead) of the compressed stream in LDS.
//  2. Parse it wave-parallel: lane l owns byte positions [16l, 16l+16) and
//     walks the token chain speculatively from its segment start (LZ4 token
//     chains resynchronise within a few sequences), recording the positions it
//     visits as a 16-bit mask. Fix-up rounds hand each lane the true entry
//     point from its left neighbour; a lane whose walk did not pass through it
//     re-walks. The fixpoint is the exact serial parse.
//  3. Build the chunk's sequence table in LDS (literal source, lengths,
//     offset, output start by wave prefix sums) and check the reference's
//     errors in sequence order.
//  4. Produce the chunk's output in 16-byte units aligned to the output
//     address, one unit per lane per step (1 KiB coalesced stores per wave
//     instruction). Each unit resolves its source through the table: literal
//     bytes come from the staged stream, back-references are followed through
//     earlier sequences of the same chunk (periodic matches map straight below
//     their start) until they land in a literal or in output finished by an
//     earlier chunk (read back from L2, bypassing L1).
//  5. A sequence whose parse leaves the staged window (long literal runs,
//     long length varints: incompressible or highly repetitive blocks) is
//     parsed from global memory with wave-wide 255-run scans and produced by
//     the same unit loop.
#include "lz4mi_common.h"

namespace lz4mi {

constexpr int kChunk = 1024;                 // compressed bytes parsed per step
constexpr int kPad = 64;                     // lookahead for sequences straddling the chunk end
constexpr int kLim = kChunk + kPad;          // chunk-relative bytes a regular sequence may touch
constexpr int kStageWords = (kLim + 8) / 4;  // staged dwords (covers a 0..3 byte shift)
constexpr int kMaxSeq = kChunk / 3 + 4;      // every non-final sequence is >= 3 bytes
constexpr uint32_t kEnd = 0x40000000u;       // chain ends (last sequence of the block)
constexpr uint32_t kStop = 0x40000001u;      // sequence cannot be parsed inside the window

struct DecArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint32_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    const uint32_t* out_cap;
    const uint8_t* dict;
    uint32_t dict_len;
    uint32_t* out_len;
    int32_t* status;
    uint32_t nblocks;
    int isolate;          // batched blocks: a back-reference before the block start is reported, not followed
};

struct DecShared {
    uint32_t stage[kStageWords];
    uint32_t t_out[kMaxSeq];   // output start of the sequence (block-relative)
    uint32_t t_lit[kMaxSeq];   // literal source (block-relative position in the compressed block)
    uint32_t t_ll[kMaxSeq];    // literal length
    uint32_t t_off[kMaxSeq];   // match offset
    uint32_t t_ml[kMaxSeq];    // match length (0: final literal-only sequence)
    uint32_t unit[kWave * 4];  // per-lane 16-byte assembly slot (slow path)
};

// Position of the token after the one at p (chunk-relative), or kEnd / kStop.
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
    if (q >= rem) return kEnd;                 // literal-only final sequence
    if (q + 2 > (uint32_t)kLim) return kStop;
    q += 2;
    if ((tok & 15) == 15) {
        uint32_t b;
        do {
            if (q >= (uint32_t)kLim) return kStop;
            b = s[q++];
        } while (b == 255);
    }
    return q >= rem ? kEnd : q;
}

__device__ __forceinline__ void walk(const uint8_t* s, uint32_t E, uint32_t seg0, uint32_t rem, uint32_t& vis,
                                     uint32_t& x) {
    uint32_t v = 0, p = E;
    while (p < seg0 + 16) {
        v |= 1u << (p - seg0);
        p = next_token(s, p, rem);
    }
    vis = v;
    x = p;
}

// Last sequence index whose output start is <= y (the table is sorted).
__device__ __forceinline__ uint32_t find_seq(const DecShared& S, uint32_t nseq, int64_t y) {
    uint32_t lo = 0, hi = nseq - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if ((int64_t)S.t_out[mid] <= y) lo = mid; else hi = mid - 1;
    }
    return lo;
}

struct BlockCtx {
    const uint8_t* blk;     // compressed block
    uint8_t* dst;           // output start of the block (out + out_off)
    int64_t out_off;        // absolute position of dst in `out`
    int64_t in_len;
    int64_t cap;            // writable bytes from dst
    const uint8_t* dict;
    int64_t dict_len;
    int64_t ip;             // chunk start (block-relative compressed position)
    uint32_t sh;            // staging shift
    int64_t O;              // output start of the current table (block-relative)
    uint32_t nseq;
    int isolate;
};

__device__ __forceinline__ uint8_t comp_byte(const BlockCtx& c, const DecShared& S, int64_t pos) {
    int64_t r = pos - c.ip;
    if (r >= 0 && r < kLim) return ((const uint8_t*)S.stage)[c.sh + r];
    return (pos >= 0 && pos < c.in_len) ? c.blk[pos] : 0;
}

// 16 bytes of compressed stream at block-relative `pos` (caller guarantees they exist).
__device__ __forceinline__ bool comp16(const BlockCtx& c, const DecShared& S, int64_t pos, uint32_t v[4]) {
    int64_t r = pos - c.ip;
    if (r >= 0 && r + 16 <= kLim) {
        uint32_t idx = c.sh + (uint32_t)r, w = idx >> 2, b = idx & 3;
        uint32_t d0 = S.stage[w], d1 = S.stage[w + 1], d2 = S.stage[w + 2], d3 = S.stage[w + 3], d4 = S.stage[w + 4];
        v[0] = funnel(d0, d1, b); v[1] = funnel(d1, d2, b); v[2] = funnel(d2, d3, b); v[3] = funnel(d3, d4, b);
        return true;
    }
    if (pos >= 4 && pos + 20 <= c.in_len) {
        uintptr_t a = (uintptr_t)(c.blk + pos), a0 = a & ~(uintptr_t)3;
        uint32_t b = (uint32_t)(a - a0);
        const uint32_t* p = (const uint32_t*)a0;
        uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = b ? p[4] : 0u;
        v[0] = funnel(d0, d1, b); v[1] = funnel(d1, d2, b); v[2] = funnel(d2, d3, b); v[3] = funnel(d3, d4, b);
        return true;
    }
    return false;
}

// 16 bytes of earlier output at block-relative `src` (absolute position >= 0).
__device__ __forceinline__ void hist16(const BlockCtx& c, int64_t src, uint32_t v[4]) {
    uintptr_t a = (uintptr_t)(c.dst + src), a0 = a & ~(uintptr_t)3;
    uint32_t b = (uint32_t)(a - a0);
    const uint32_t* p = (const uint32_t*)a0;
    uint32_t d0 = ld_nt_u32(p), d1 = ld_nt_u32(p + 1), d2 = ld_nt_u32(p + 2), d3 = ld_nt_u32(p + 3);
    uint32_t d4 = b ? ld_nt_u32(p + 4) : 0u;
    v[0] = funnel(d0, d1, b); v[1] = funnel(d1, d2, b); v[2] = funnel(d2, d3, b); v[3] = funnel(d3, d4, b);
}

// Fast path: the 16 bytes at y come from one contiguous final source.
__device__ __forceinline__ bool unit_fast(const BlockCtx& c, const DecShared& S, int64_t y, uint32_t v[4]) {
    int64_t yc = y;
    for (int depth = 0; depth < 8; ++depth) {
        if (yc + 16 <= c.O) {
            int64_t abs = c.out_off + yc;
            if (abs < 4 || yc + 20 > c.cap) return false;
            hist16(c, yc, v);
            return true;
        }
        if (yc < c.O) return false;
        uint32_t s = find_seq(S, c.nseq, yc);
        int64_t rel = yc - (int64_t)S.t_out[s];
        int64_t ll = S.t_ll[s];
        if (rel + 16 <= ll) return comp16(c, S, (int64_t)S.t_lit[s] + rel, v);
        if (rel < ll) return false;
        int64_t mrel = rel - ll, off = S.t_off[s];
        if (mrel + 16 > (int64_t)S.t_ml[s]) return false;
        int64_t r = mrel < off ? mrel : mrel % off;
        if (r + 16 > off) return false;
        yc = (int64_t)S.t_out[s] + ll - off + r;
    }
    return false;
}

// General path: resolve the unit run by run and assemble it byte-wise in LDS.
__device__ void unit_slow(const BlockCtx& c, DecShared& S, int lane, int64_t y, uint32_t n) {
    uint8_t* ub = (uint8_t*)&S.unit[lane * 4];
    uint32_t k = 0;
    while (k < n) {
        int64_t yc = y + k;
        int64_t m = n - k;
        int kind;          // 0 history, 1 dictionary, 2 compressed stream
        int64_t sp;
        for (;;) {
            if (yc < c.O) {
                if (c.O - yc < m) m = c.O - yc;
                int64_t abs = c.out_off + yc;
                if (abs < 0) {
                    if (-abs < m) m = -abs;
                    kind = 1; sp = c.dict_len + abs;
                } else {
                    kind = 0; sp = yc;
                }
                break;
            }
            uint32_t s = find_seq(S, c.nseq, yc);
            int64_t rel = yc - (int64_t)S.t_out[s];
            int64_t ll = S.t_ll[s];
            if (rel < ll) {
                if (ll - rel < m) m = ll - rel;
                kind = 2; sp = (int64_t)S.t_lit[s] + rel;
                break;
            }
            int64_t mrel = rel - ll, off = S.t_off[s];
            if ((int64_t)S.t_ml[s] - mrel < m) m = (int64_t)S.t_ml[s] - mrel;
            int64_t r = mrel < off ? mrel : mrel % off;
            if (off - r < m) m = off - r;
            yc = (int64_t)S.t_out[s] + ll - off + r;
        }
        for (int64_t j = 0; j < m; ++j) {
            uint8_t b;
            if (kind == 0) b = ld_nt_u8(c.dst + sp + j);
            else if (kind == 1) b = c.dict[sp + j];
            else b = comp_byte(c, S, sp + j);
            ub[k + j] = b;
        }
        k += (uint32_t)m;
    }
}

// Produce output [c.O, c.O + total) described by the table (clipped to cap).
__device__ void produce(const BlockCtx& c, DecShared& S, int lane, int64_t total) {
    int64_t lo = c.O, hi = c.O + total;
    if (hi > c.cap) hi = c.cap;
    if (lo >= hi) return;
    uintptr_t base = (uintptr_t)c.dst;
    uintptr_t alo = base + lo, ahi = base + hi;
    for (uintptr_t u = (alo & ~(uintptr_t)15) + 16 * (uintptr_t)lane; u < ahi; u += 16 * kWave) {
        uintptr_t ua = u < alo ? alo : u;
        uintptr_t ue = u + 16 > ahi ? ahi : u + 16;
        int64_t y = (int64_t)(ua - base);
        uint32_t n = (uint32_t)(ue - ua);
        uint32_t v[4];
        if (n == 16 && unit_fast(c, S, y, v)) {
            *(uint4*)(c.dst + y) = make_uint4(v[0], v[1], v[2], v[3]);
            continue;
        }
        unit_slow(c, S, lane, y, n);
        if (n == 16) {
            uint4 w = *(const uint4*)&S.unit[lane * 4];
            *(uint4*)(c.dst + y) = w;
        } else {
            const uint8_t* ub = (const uint8_t*)&S.unit[lane * 4];
            for (uint32_t j = 0; j < n; ++j) c.dst[y + j] = ub[j];
        }
    }
}

// Wave-wide 255-run varint starting at block-relative q: returns the sum and
// advances q past the terminating byte. Bytes past the block end read as 0.
__device__ int64_t wave_varint(const BlockCtx& c, int lane, int64_t& q) {
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

__device__ __forceinline__ uint32_t seq_error(const BlockCtx& c, int64_t out_start, int64_t lit, int64_t ll,
                                              uint32_t off, uint32_t ml) {
    if (out_start + ll > c.cap) return 1;                 // Output Buffer Too Small
    if (lit + ll > c.in_len) return 2;                    // Malformed Input
    if (ml == 0) return 0;                                // final literal-only sequence
    if (off == 0) return 3;                               // Invalid Offset 0
    int64_t ms_abs = c.out_off + out_start + ll;
    if ((int64_t)off > ms_abs + c.dict_len) return 4;     // Dictionary Offset Out of Bounds
    if (c.isolate && (int64_t)off > out_start + ll) return 5;   // reaches into another block's output
    return 0;
}

// error code (1..5, see seq_error) -> status
__device__ __forceinline__ int32_t err_status(uint32_t e) {
    return e == 5 ? -9 : -(int32_t)e;
}

__global__ __launch_bounds__(64) void lz4mi_decompress_kernel(DecArgs a) {
    __shared__ DecShared S;
    const int lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    if (b >= a.nblocks) return;

    BlockCtx c;
    c.blk = a.in + a.in_off[b];
    c.in_len = a.in_len[b];
    c.out_off = (int64_t)a.out_off[b];
    c.dst = a.out + a.out_off[b];
    c.cap = a.out_cap[b];
    c.dict = a.dict;
    c.dict_len = a.dict ? a.dict_len : 0;
    c.isolate = a.isolate;
    c.ip = 0;
    c.O = 0;
    int32_t status = 0;

    while (c.ip < c.in_len) {
        // ---- 1. stage [ip, ip + kLim) ------------------------------------
        uintptr_t A = (uintptr_t)(c.blk + c.ip), A0 = A & ~(uintptr_t)3;
        c.sh = (uint32_t)(A - A0);
        for (int k = lane; k < kStageWords; k += kWave) {
            int64_t rel = (int64_t)(A0 + 4 * (uintptr_t)k) - (int64_t)(uintptr_t)c.blk;
            uint32_t v;
            if (rel >= 0 && rel + 4 <= c.in_len) {
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
        __syncthreads();
        const uint8_t* s = (const uint8_t*)S.stage + c.sh;
        int64_t rem64 = c.in_len - c.ip;
        uint32_t rem = rem64 > 0x3FFFFFFF ? 0x3FFFFFFFu : (uint32_t)rem64;

        // ---- 2. speculative parse + fix-up rounds ----------------------
        uint32_t seg0 = 16u * lane, vis, x, E = seg0;
        walk(s, E, seg0, rem, vis, x);
        for (int round = 0; round <= kWave; ++round) {
            uint32_t pE = __shfl_up(E, 1, kWave), pX = __shfl_up(x, 1, kWave);
            uint32_t nE = lane == 0 ? 0u : (pE >= seg0 ? pE : pX);
            bool ch = nE != E;
            if (ch) {
                E = nE;
                if (E >= seg0 + 16) { vis = 0; x = E; }
                else if ((vis >> (E - seg0)) & 1u) vis &= ~((1u << (E - seg0)) - 1u);
                else walk(s, E, seg0, rem, vis, x);
            }
            if (__ballot(ch) == 0) break;
        }
        uint32_t tail = __shfl(x, kWave - 1, kWave);      // where the chain leaves the chunk
        // lane holding the chain's last token (needed for kEnd / kStop)
        uint64_t has = __ballot(vis != 0);
        int last_lane = 63 - __builtin_clzll(has);
        uint32_t last_tok = seg0 + 31 - __builtin_clz(vis | 1u);
        last_tok = __shfl(last_tok, last_lane, kWave);
        bool cut = tail == kStop;
        uint32_t cut_pos = last_tok;

        // ---- 3. sequence table -----------------------------------------
        uint32_t cnt = __popc(vis) - ((cut && lane == last_lane) ? 1u : 0u);
        uint32_t incl = wave_incl_scan(cnt, lane);
        uint32_t base = incl - cnt;
        uint32_t nseq = __shfl(incl, kWave - 1, kWave);
        uint32_t run = 0;
        {
            uint32_t m = vis, k = base;
            for (uint32_t i = 0; i < cnt; ++i) {
                uint32_t p = seg0 + __builtin_ctz(m);
                m &= m - 1;
                uint32_t tok = s[p], q = p + 1, ll = tok >> 4;
                if (ll == 15) { uint32_t bb; do { bb = s[q++]; ll += bb; } while (bb == 255); }
                uint32_t lit = q;
                q += ll;
                uint32_t off = 0, ml = 0;
                if (q < rem) {
                    off = (uint32_t)s[q] | ((uint32_t)s[q + 1] << 8);
                    q += 2;
                    ml = tok & 15;
                    if (ml == 15) { uint32_t bb; do { bb = s[q++]; ml += bb; } while (bb == 255); }
                    ml += 4;
                }
                S.t_lit[k] = (uint32_t)c.ip + lit;
                S.t_ll[k] = ll;
                S.t_off[k] = off;
                S.t_ml[k] = ml;
                S.t_out[k] = run;
                run += ll + ml;
                ++k;
            }
        }
        uint32_t lincl = wave_incl_scan(run, lane);
        uint32_t lbase = lincl - run;
        int64_t total = __shfl(lincl, kWave - 1, kWave);
        uint32_t first_err = 0xFFFFFFFFu;
        for (uint32_t k = base; k < base + cnt; ++k) {
            int64_t os = c.O + lbase + S.t_out[k];
            S.t_out[k] = (uint32_t)os;
            uint32_t e = seq_error(c, os, S.t_lit[k], S.t_ll[k], S.t_off[k], S.t_ml[k]);
            if (e && first_err == 0xFFFFFFFFu) first_err = (k << 3) | e;
        }
        first_err = wave_min(first_err);
        __syncthreads();
        if (first_err != 0xFFFFFFFFu) { status = err_status(first_err & 7); break; }

        // ---- 4. produce the chunk's output -------------------------------
        c.nseq = nseq;
        if (nseq) produce(c, S, lane, total);
        c.O += total;

        // ---- 5. the sequence the window could not hold -------------------
        if (cut) {
            int64_t q = c.ip + cut_pos;
            uint32_t tok = q < c.in_len ? c.blk[q] : 0u;
            ++q;
            int64_t ll = tok >> 4;
            if (ll == 15) ll += wave_varint(c, lane, q);
            int64_t lit = q;
            q += ll;
            uint32_t off = 0, ml = 0;
            if (q < c.in_len) {
                off = (uint32_t)(q < c.in_len ? c.blk[q] : 0) | ((uint32_t)(q + 1 < c.in_len ? c.blk[q + 1] : 0) << 8);
                q += 2;
                int64_t mlv = tok & 15;
                if (mlv == 15) mlv += wave_varint(c, lane, q);
                ml = (uint32_t)(mlv + 4);
            }
            uint32_t e = seq_error(c, c.O, lit, ll, off, ml);
            if (e) { status = err_status(e); break; }
            wait_vmem();    // the regular sequences' stores are read back as history below
            __syncthreads();
            if (lane == 0) {
                S.t_out[0] = (uint32_t)c.O; S.t_lit[0] = (uint32_t)lit; S.t_ll[0] = (uint32_t)ll;
                S.t_off[0] = off; S.t_ml[0] = ml;
            }
            __syncthreads();
            c.nseq = 1;
            produce(c, S, lane, ll + ml);
            c.O += ll + ml;
            c.ip = q;
        } else if (tail >= kEnd) {
            c.ip = c.in_len;
        } else {
            c.ip += tail;
        }
        wait_vmem();        // this chunk's stores are complete before the next chunk reads them back
        __syncthreads();
    }
    if (lane == 0) {
        a.status[b] = status;
        a.out_len[b] = status ? 0u : (uint32_t)c.O;
    }
}

// ---------------------------------------------------------------------------
// Serial decoder, one lane per block: the reference's exact byte order,
// including the double-copy-tail rewrite for offset >= 8, length < 8 matches
// (blockDecompress.js:219-250). Used for LZ4MI_JS_COMPAT.
// Blocks run in order on one lane: the rewrite may touch up to 7 bytes before
// a block's start, and the reference's frame loop decodes blocks in order.
__device__ void decode_block_jscompat(const DecArgs& a, uint32_t b) {
    const uint8_t* in = a.in + a.in_off[b];
    const int64_t iend = a.in_len[b];
    uint8_t* out = a.out;                       // absolute positions
    const int64_t oo = (int64_t)a.out_off[b];
    const int64_t olen = oo + a.out_cap[b];     // the reference's output.length
    const int64_t dlen = a.dict ? a.dict_len : 0;
    int64_t ip = 0, op = oo;
    int32_t st = 0;
    auto inb = [&](int64_t i) -> uint32_t { return (i >= 0 && i < iend) ? in[i] : 0u; };
    while (ip < iend) {
        uint32_t tok = inb(ip++);
        int64_t lit = tok >> 4;
        if (lit == 15) { uint32_t x; do { x = inb(ip++); lit += x; } while (x == 255); }
        if (op + lit > olen) { st = -1; break; }
        if (ip + lit > iend) { st = -2; break; }
        for (int64_t k = 0; k < lit; ++k) out[op + k] = (uint8_t)inb(ip + k);
        op += lit; ip += lit;
        if (ip >= iend) break;
        uint32_t off = inb(ip) | (inb(ip + 1) << 8);
        ip += 2;
        if (off == 0) { st = -3; break; }
        int64_t ml = tok & 15;
        if (ml == 15) { uint32_t x; do { x = inb(ip++); ml += x; } while (x == 255); }
        ml += 4;
        int64_t from = op - off;
        if (from < 0) {
            int64_t nd = -from < ml ? -from : ml;
            int64_t di = dlen + from;
            if (di < 0 || di + nd > dlen) { st = -4; break; }
            for (int64_t k = 0; k < nd; ++k) { if (op < olen) out[op] = a.dict[di + k]; ++op; }
            int64_t rp = op - off;
            for (int64_t k = nd; k < ml; ++k) {
                uint8_t v = (rp >= 0 && rp < olen) ? out[rp] : 0;
                if (op < olen) out[op] = v;
                ++op; ++rp;
            }
            continue;
        }
        int64_t start = op;
        for (int64_t k = 0; k < ml; ++k) {
            int64_t r = op - off;
            uint8_t v = r < olen ? out[r] : 0;
            if (op < olen) out[op] = v;
            ++op;
        }
        if (off >= 8 && ml < 8) {
            for (int64_t p = start + ml - 8; p < start; ++p) {
                int64_t r = p - off;
                uint8_t v = (r >= 0 && r < olen) ? out[r] : 0;
                if (p >= 0 && p < olen) out[p] = v;
            }
        }
    }
    a.status[b] = st;
    a.out_len[b] = st ? 0u : (uint32_t)(op - oo);
}

__global__ __launch_bounds__(64) void lz4mi_decompress_jscompat_kernel(DecArgs a) {
    if (threadIdx.x != 0) return;
    for (uint32_t b = 0; b < a.nblocks; ++b) decode_block_jscompat(a, b);
}

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                              uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                              const uint8_t* dict, uint32_t dict_len, uint32_t* out_len,
                                              int32_t* status, uint32_t nblocks, int js_compat, hipStream_t stream) {
    lz4mi::DecArgs a{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, nblocks,
                     nblocks > 1 ? 1 : 0};
    if (nblocks == 0) return hipSuccess;
    if (js_compat) {
        hipLaunchKernelGGL(lz4mi::lz4mi_decompress_jscompat_kernel, dim3(1), dim3(64), 0, stream, a);
    } else {
        hipLaunchKernelGGL(lz4mi::lz4mi_decompress_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    }
    return hipGetLastError();
}
