// lz4mi_expand.hip — the output of a small batch (few blocks) by pointer jumping.
//
// The batch decoder (lz4mi_decompress.hip) writes a block with one wave: a 4 MiB tiles216
// block alone takes ~8 ms, the latency of that wave's chain, however idle the rest of the
// GPU is. Here a block's output is computed by the whole GPU instead, once its sequence
// table is known (the decoder's parse, run in export mode: DecArgs::xseq):
//
//   expand: every output byte x gets a source pointer: a literal byte -> its position in the
//           compressed block (resolved), a match byte -> x - offset, an earlier output byte
//           (unresolved) or a byte before the block (caller's history / dictionary: resolved);
//   jump:   ptr[x] = ptr[ptr[x]], five times over in one round (kGathers), for every unresolved
//           x, in place; two such rounds, then each pointer left is followed to its end
//           (lz4mi_chase_kernel). A step adds at least the hops the pointer it reads had when
//           the round began (the steps of one round are not synchronised across threads; most
//           reads see pointers already advanced in this round), so a round multiplies a
//           pointer's hops by at least 6 and usually far more (tiles216: chains up to 332
//           matches deep, copy 3 329, text 21 489 -- a byte of an overlapping match points into
//           the period before the match, so every hop lands in an earlier sequence). Five steps
//           per round instead of one step in each of 10 rounds: each pointer is read and written
//           twice instead of 10 times (small batches 12-27 % faster, round 6, profiles/r06j;
//           more rounds instead of the chase: slower, profiles/r06r). Pointers only point
//           backwards and every value on a chain resolves to the same byte, so reading a
//           pointer another thread has just replaced (or not yet) is correct either way;
//   gather: out[x] = the byte the resolved pointer names.
//
// The reference decoder (blockDecompress.js:55-272) copies the same bytes in sequence
// order; the result is identical because every output byte is a copy of exactly one
// literal (or history/dictionary) byte, found by following the matches backwards.
// Memory per block: 4 bytes per output byte (pointers) + 16 bytes per sequence.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4mi_decompress.h"

namespace lz4mi {

constexpr uint32_t kUnres = 0x80000000u;   // ptr < kUnres: an output position still to follow
constexpr uint32_t kLit = 0x80000000u;     // kLit | p: byte p of the compressed block
constexpr uint32_t kHist = 0xC0000000u;    // kHist | (y + 65536): byte y < 0 before the block
constexpr int kXThreads = 256;
constexpr int kXBytes = 16;                // output bytes per thread (a wave: 1 KiB)
#ifndef LZ4MI_JUMP_GATHERS
#define LZ4MI_JUMP_GATHERS 5   // (A/B, profiles/r06j: 1, 2, 3, 4, 5 and 10 steps per round)
#endif
constexpr int kGathers = LZ4MI_JUMP_GATHERS;   // pointer hops per round (each round multiplies a chain's hops by 2^kGathers)
constexpr int kJumpRounds = (10 + kGathers - 1) / kGathers;   // rounds; then lz4mi_chase_kernel follows what is left

struct ExpArgs {
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
    const uint4* xseq;
    const uint32_t* xcnt;
    SegRec* xrec;
    uint32_t nseg;
    uint32_t xseq_stride;     // sequence entries per block (segment s at s * seg_geom(in_len).stride)
    uint32_t* ptr;            // x_out_max pointers per block
    uint32_t x_out_max;
    uint8_t* done;            // per block and 16 output bytes (one thread's): its pointers are all resolved
    uint32_t* flags;          // flags[r]: round r has unresolved pointers to follow
    uint32_t* best;           // per block: min over failing sequences of (index << 3 | check)
    uint32_t ntiles;          // nblocks * x_out_max / kTile
    uint32_t tshift;          // log2(x_out_max / kTile)
};

// The output kernels loop over (block, tile) pairs, a tile = kXThreads * kXBytes output bytes,
// with a grid of at most kXGrid workgroups (one tile each up to 128 blocks of 4 MiB).
constexpr uint32_t kTile = kXThreads * kXBytes;
constexpr uint32_t kXGrid = 1u << 17;   // (2048: 8-10 % slower on tiles216, profiles/r06e)
#define X_TILES(a) for (uint32_t tile_ = blockIdx.x; tile_ < (a).ntiles; tile_ += gridDim.x)
// Tile-major: tile t of every block before tile t + 1 of any, so the waves dispatched first hold the
// early output of every block. Pointers point backwards, so a later tile's rounds (and its chase) read
// pointers the earlier tiles have already advanced. Block-major order (every tile of block 0 first)
// took 34 % longer on tiles216 at 64 and 160 blocks, and 40 % longer on text (round 6, profiles/r06t).
#define X_B(a) (tile_ % ((a).ntiles >> (a).tshift))   // (ntiles >> tshift = the batch's blocks)
#define X_T(a) (tile_ / ((a).ntiles >> (a).tshift))
// This thread's 16 output bytes [x0, x0 + 16) of tile t of block b, and n = the block's
// output length (0: nothing to do here)
__device__ __forceinline__ uint32_t x_span(const ExpArgs& a, uint32_t b, uint32_t t, uint32_t& x0) {
    if (a.status[b] != 0 || a.xcnt[b] == kNotExported) return 0;
    const uint32_t n = min(a.out_len[b], a.out_cap[b]);
    x0 = t * kTile + threadIdx.x * kXBytes;
    return x0 < n ? n : 0u;
}
__device__ __forceinline__ uint8_t* done_flag(const ExpArgs& a, uint32_t b, uint32_t t) {
    return a.done + (size_t)b * (a.x_out_max / kXBytes) + t * kXThreads + threadIdx.x;
}

__device__ __forceinline__ const uint4* seg_entries(const ExpArgs& a, uint32_t b, uint32_t sg, const SegGeom& G) {
    return a.xseq + (size_t)b * a.xseq_stride + (size_t)sg * G.stride;
}

// Per block after the parse (one wave, four segment records per lane): every segment's output
// start and first sequence number (exclusive scans in segment order), the first segment at an
// error (stop) -- the ones after it get kNoBase --, the parse's first error as
// (sequence << 3 | check) into best[b], the output length into out_len[b].
__global__ __launch_bounds__(64) void lz4mi_xbase_kernel(ExpArgs a) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (a.xcnt[b] == kNotExported) return;
    const SegGeom G = seg_geom(a.in_len[b]);
    SegRec* R = a.xrec + (size_t)b * a.nseg;
    uint32_t olen[4], cnt[4], fe[4];
    uint64_t em = 0;
    uint32_t stop = G.S;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        const bool in = sg < G.S;
        const bool e = in && R[sg].fin == kFinErr + 1u;
        olen[q] = in ? R[sg].olen : 0u;
        cnt[q] = in ? R[sg].cnt : 0u;
        fe[q] = e ? 1u : 0u;
        const uint64_t m = __ballot(e);
        if (m && stop == G.S) stop = 64u * q + (uint32_t)__builtin_ctzll(m);
        em |= m;
    }
    uint32_t base = 0, g = 0;   // running totals of the quarters before
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        uint32_t io = olen[q], ic = cnt[q];   // inclusive scans over the quarter's lanes
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t po = __shfl_up(io, d), pc = __shfl_up(ic, d);
            if (lane >= (uint32_t)d) {
                io += po;
                ic += pc;
            }
        }
        if (sg < G.S) {
            R[sg].base = sg <= stop ? base + io - olen[q] : kNoBase;
            R[sg].g0 = g + ic - cnt[q];
        }
        base += __shfl(io, 63);
        g += __shfl(ic, 63);
    }
    // totals of the segments before `stop`, the parse error at `stop`
    uint32_t tb = 0, tg = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sg = 64u * q + lane;
        const bool before = sg < stop;
        uint32_t vo = before ? olen[q] : 0u, vc = before ? cnt[q] : 0u;
        for (int d = 32; d >= 1; d >>= 1) {
            vo += __shfl_xor(vo, d);
            vc += __shfl_xor(vc, d);
        }
        tb += vo;
        tg += vc;
    }
    if (lane == 0) {
        uint32_t perr = 0xFFFFFFFFu;
        if (stop < G.S) {
            const uint32_t er = R[stop].err;
            if (er != 0xFFFFFFFFu) perr = ((tg + (er >> 3)) << 3) | (er & 7u);
        }
        a.best[b] = perr;
        a.out_len[b] = tb;
    }
    (void)fe;
}

// Per (segment, block): the reference's checks that need absolute output positions (1 capacity,
// 4 dictionary bounds, 5 cross-block; the parse did 2 and 3) on the segment's sequences: the
// minimum of (sequence << 3 | check) over the failing ones, with the parse's error, is the
// first check the reference's decoder fails (blockDecompress.js) -> best[b].
__global__ __launch_bounds__(kXThreads) void lz4mi_xcheck_kernel(ExpArgs a, int isolate) {
    const uint32_t sg = blockIdx.x, b = blockIdx.y;
    if (a.xcnt[b] == kNotExported) return;
    const SegGeom G = seg_geom(a.in_len[b]);
    if (sg >= G.S) return;
    const SegRec* R = a.xrec + (size_t)b * a.nseg;
    const uint32_t base = R[sg].base, g0 = R[sg].g0;
    if (base == kNoBase) return;                       // after the block's first error
    const int64_t cap = a.out_cap[b] > 0x7FFFFFFFu ? 0x7FFFFFFF : (int64_t)a.out_cap[b];
    const int64_t out_off = (int64_t)a.out_off[b], dict_len = a.dict ? (int64_t)a.dict_len : 0;
    const uint4* E = seg_entries(a, b, sg, G);
    const uint32_t cnt = R[sg].cnt;
    uint32_t mine = 0xFFFFFFFFu;
    for (uint32_t k = threadIdx.x; k < cnt; k += kXThreads) {
        const uint4 e = E[k];
        const int64_t os = (int64_t)base + e.x, ll = e.z, off = e.w;
        uint32_t code = 0;
        if (os + ll > cap) code = 1;
        else if (off && off > out_off + os + ll + dict_len) code = 4;
        else if (off && isolate && off > os + ll) code = 5;
        if (code) mine = min(mine, ((g0 + k) << 3) | code);
    }
    if (mine != 0xFFFFFFFFu) atomicMin(&a.best[b], mine);
}

// Per block: status and output length from the first failing check (best[b]).
__global__ __launch_bounds__(64) void lz4mi_xstatus_kernel(ExpArgs a) {
    const uint32_t b = blockIdx.x;
    if (threadIdx.x != 0 || a.xcnt[b] == kNotExported) return;
    const uint32_t e = a.best[b];
    if (e != 0xFFFFFFFFu) {
        a.status[b] = (e & 7u) == 5 ? -9 : -(int32_t)(e & 7u);
        a.out_len[b] = 0;
    } else {
        a.status[b] = 0;
    }
}

__global__ __launch_bounds__(kXThreads) void lz4mi_expand_kernel(ExpArgs a) {
  bool unres = false;
  X_TILES(a) {
    uint32_t x0 = 0;
    const uint32_t b = X_B(a);
    const uint32_t n = x_span(a, b, X_T(a), x0);
    if (n) {
        const SegRec* R = a.xrec + (size_t)b * a.nseg;
        const SegGeom G = seg_geom(a.in_len[b]);
        // the segment holding x0 (the first whose end is past it), then its last sequence
        // starting at or before x0
        uint32_t slo = 0, shi = G.S - 1;
        while (slo < shi) {
            const uint32_t mid = (slo + shi) >> 1;
            if (R[mid].base + R[mid].olen > x0) shi = mid;
            else slo = mid + 1;
        }
        uint32_t sg = slo;
        uint32_t base = R[sg].base, send = base + R[sg].olen, cnt = R[sg].cnt;
        const uint4* E = seg_entries(a, b, sg, G);
        uint32_t lo = 0, hi = cnt;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (base + E[mid].x <= x0) lo = mid;
            else hi = mid;
        }
        uint32_t k = lo;
        uint32_t v[kXBytes];
        if (x0 + kXBytes <= send && x0 + kXBytes <= n) {
            // the 16 bytes lie in this segment: they span at most 5 sequences (every sequence but
            // the block's last writes >= 4 bytes), loaded together -- one round trip, not one per
            // sequence boundary the lane crosses (text and copy -3..8 %, round 6)
            // (five named entries, not an array: a select over an array became scratch memory)
            const uint4 sent = make_uint4(send - base, 0u, 0u, 0u);
            const uint4 q0 = E[k];
            const uint4 q1 = k + 1 < cnt ? E[k + 1] : sent;
            const uint4 q2 = k + 2 < cnt ? E[k + 2] : sent;
            const uint4 q3 = k + 3 < cnt ? E[k + 3] : sent;
            const uint4 q4 = k + 4 < cnt ? E[k + 4] : sent;
#pragma unroll
            for (int t = 0; t < kXBytes; ++t) {
                const uint32_t x = x0 + t - base;    // segment-relative
                uint4 e = q0;
                if (x >= q1.x) e = q1;
                if (x >= q2.x) e = q2;
                if (x >= q3.x) e = q3;
                if (x >= q4.x) e = q4;
                if (x - e.x < e.z) {
                    v[t] = kLit | (e.y + (x - e.x));
                } else {
                    const uint32_t ms = base + e.x + e.z, xa = x + base, d = xa - ms;
                    const int32_t y = (int32_t)(d < e.w ? xa : ms + d % e.w) - (int32_t)e.w;
                    v[t] = y >= 0 ? (uint32_t)y : (kHist | (uint32_t)(y + 65536));
                    unres |= y >= 0;
                }
            }
            uint4* P = (uint4*)(a.ptr + (size_t)b * a.x_out_max + x0);
#pragma unroll
            for (int q4 = 0; q4 < kXBytes / 4; ++q4) P[q4] = make_uint4(v[4 * q4], v[4 * q4 + 1], v[4 * q4 + 2], v[4 * q4 + 3]);
            continue;
        }
        // (else: the 16 bytes reach past the segment or the output: one sequence at a time)
        uint4 e = E[k];
        uint32_t nxt = k + 1 < cnt ? base + E[k + 1].x : send;
#pragma unroll
        for (int t = 0; t < kXBytes; ++t) {
            const uint32_t x = x0 + t;
            v[t] = 0;
            if (x >= n) continue;
            while (x >= nxt) {   // the next sequence (in the next non-empty segment)
                if (k + 1 < cnt) {
                    ++k;
                } else {
                    do {
                        ++sg;
                        base = R[sg].base;
                        send = base + R[sg].olen;
                        cnt = R[sg].cnt;
                    } while (send == base);
                    E = seg_entries(a, b, sg, G);
                    k = 0;
                }
                e = E[k];
                nxt = k + 1 < cnt ? base + E[k + 1].x : send;
            }
            const uint32_t ex = base + e.x;
            if (x - ex < e.z) {
                v[t] = kLit | (e.y + (x - ex));
            } else {
                // an overlapping match repeats its first `offset` bytes: point into the period
                // before the match start, so every pointer lands in an earlier sequence (a chain
                // hops at most once per sequence, not once per period)
                const uint32_t ms = ex + e.z, d = x - ms;
                const int32_t y = (int32_t)(d < e.w ? x : ms + d % e.w) - (int32_t)e.w;
                v[t] = y >= 0 ? (uint32_t)y : (kHist | (uint32_t)(y + 65536));
                unres |= y >= 0;
            }
        }
        uint4* P = (uint4*)(a.ptr + (size_t)b * a.x_out_max + x0);
#pragma unroll
        for (int q = 0; q < kXBytes / 4; ++q) P[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  }
    const uint64_t um = __ballot(unres);
    if (um && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(um)) a.flags[0] = 1u;
}

// The jump rounds and the chase work on a wave's KiB of output strided: lane l holds bytes
// l, l + 64, ... l + 960, so each load, gather and store instruction of the wave covers 256
// contiguous bytes (2 cache lines) and the gathers follow runs of consecutive sources -- with
// 16 consecutive bytes per lane an instruction spans 4 KiB (32 lines). done[]: per lane, its
// 16 bytes are resolved (zeroed before the first round).
__device__ __forceinline__ uint32_t x_wave(const ExpArgs& a, uint32_t b, uint32_t t, uint32_t& wbase) {
    if (a.status[b] != 0 || a.xcnt[b] == kNotExported) return 0;
    const uint32_t n = min(a.out_len[b], a.out_cap[b]);
    wbase = t * kTile + (threadIdx.x >> 6) * (64 * kXBytes);
    return wbase < n ? n : 0u;
}

__global__ __launch_bounds__(kXThreads) void lz4mi_jump_kernel(ExpArgs a, int r) {
  if (a.flags[r] == 0) return;
  bool still = false;
  X_TILES(a) {
    uint32_t wbase = 0;
    const uint32_t b = X_B(a), t = X_T(a);
    const uint32_t n = x_wave(a, b, t, wbase);
    if (!n) continue;
    const uint32_t lane = threadIdx.x & 63;
    uint8_t* dn = done_flag(a, b, t);
    bool mine = false;
    if (*dn == 0) {
        uint32_t* P = a.ptr + (size_t)b * a.x_out_max + wbase + lane;
        const uint32_t* Q = a.ptr + (size_t)b * a.x_out_max;
        uint32_t v[kXBytes];
#pragma unroll
        for (int k = 0; k < kXBytes; ++k) v[k] = wbase + lane + 64 * k < n ? P[64 * k] : kLit;
#pragma unroll
        for (int g = 0; g < kGathers; ++g) {
#pragma unroll
            for (int k = 0; k < kXBytes; ++k) v[k] = v[k] < kUnres ? Q[v[k]] : v[k];
        }
#pragma unroll
        for (int k = 0; k < kXBytes; ++k) {
            if (wbase + lane + 64 * k < n) P[64 * k] = v[k];
            mine |= v[k] < kUnres;
        }
        if (!mine) *dn = 1u;
    }
    still |= mine;
  }
    const uint64_t sm = __ballot(still);
    if (sm && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(sm)) a.flags[r + 1] = 1u;
}

// After the jump rounds: every pointer still unresolved is followed to its end (chains the two
// rounds did not finish: at 64 blocks 0.44 ms of a tiles216 decode, 3.1 ms of a text one).
__global__ __launch_bounds__(kXThreads) void lz4mi_chase_kernel(ExpArgs a) {
  if (a.flags[kJumpRounds] == 0) return;
  X_TILES(a) {
    uint32_t wbase = 0;
    const uint32_t b = X_B(a), t = X_T(a);
    const uint32_t n = x_wave(a, b, t, wbase);
    if (!n || *done_flag(a, b, t)) continue;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* Q = a.ptr + (size_t)b * a.x_out_max;
    for (int k = 0; k < kXBytes; ++k) {
        const uint32_t x = wbase + lane + 64 * k;
        if (x >= n) break;
        uint32_t v = Q[x];
        if (v >= kUnres) continue;
        while (v < kUnres) v = Q[v];
        Q[x] = v;
    }
  }
}

// Reference mode (LZ4MI_JS_EXACT) in pointer form (round 6; until then a check after the gather sent every
// block whose output a rewrite would change to the batch kernel's fix-up: one wave, ~8 ms for 4 MiB): the
// reference's tail rewrite for a match at s (offset >= 8, length < 8, blockDecompress.js:219-250) sets
// out[p] = out[p - off] for p in [s + ml - 8, s) after the match is copied. Here those bytes' pointers become
// p - off before the rounds, which is exact: off >= 8 puts p - off below the region, where it is final (a
// later rewrite starts at or after its own match start - 4 >= s, matches write a byte once); no later rewrite
// reaches the region; a read of a region byte before the rewrite can only come from a later byte of the same
// region (the region spans <= 4 bytes before s), which the rewrite overwrites too; and every read after it
// goes through the new pointer. A rewrite reading before the block points into the caller's array (0 before
// it, as the reference reads a missing index); batched, writing before the block, or reading before the
// array with a dictionary, the block goes to the batch kernel (redo[b]: LZ4MI_ERR_CROSS_BLOCK when batched). One workgroup per segment.
__global__ __launch_bounds__(kXThreads) void lz4mi_xf1ptr_kernel(ExpArgs a, int isolate, uint32_t* redo) {
    const uint32_t sg = blockIdx.x, b = blockIdx.y;
    if (a.status[b] != 0 || a.xcnt[b] == kNotExported) return;
    const SegGeom G = seg_geom(a.in_len[b]);
    if (sg >= G.S) return;
    const SegRec* R = a.xrec + (size_t)b * a.nseg;
    const uint32_t base = R[sg].base, send = base + R[sg].olen, cnt = R[sg].cnt;
    const uint4* E = seg_entries(a, b, sg, G);
    const int64_t out_off = (int64_t)a.out_off[b];
    const int64_t n = min(a.out_len[b], a.out_cap[b]);
    uint32_t* P = a.ptr + (size_t)b * a.x_out_max;
    bool any = false, cross = false;
    for (uint32_t k = threadIdx.x; k < cnt; k += kXThreads) {
        const uint4 e = E[k];
        const int64_t ms = (int64_t)base + e.x + e.z, off = e.w;
        const int64_t ml = (k + 1 < cnt ? (int64_t)base + E[k + 1].x : (int64_t)send) - ms;
        if (ml == 0 || ml >= 8 || off < 8 || out_off + ms - off < 0) continue;
        const int64_t p0 = ms + ml - 8;
        if (p0 - off < 0 && (isolate || (p0 < 0 && out_off > 0) || (a.dict && out_off + p0 - off < 0))) {
            // batched: reported as LZ4MI_ERR_CROSS_BLOCK by the redo; a region starting before the block
            // rewrites the caller's bytes before it (the reference's indices are absolute); with a
            // dictionary, a read before the array is the reference's 0, not a dictionary byte
            cross = true;
            continue;
        }
        for (int64_t q = p0 > 0 ? p0 : 0; q < ms && q < n; ++q) {
            // before the block: the caller's bytes in the array, or 0 before the array (the reference's read
            // of a missing index): a history pointer, gathered the same way
            const int64_t y = q - off;
            P[q] = y >= 0 ? (uint32_t)y : (kHist | (uint32_t)(y + 65536));
            any = true;
        }
    }
    if (cross) redo[b] = 1u;
    if (__syncthreads_or(any) && threadIdx.x == 0) a.flags[0] = 1u;
}

__global__ __launch_bounds__(kXThreads) void lz4mi_gather_kernel(ExpArgs a) {
  X_TILES(a) {
    uint32_t x0;
    const uint32_t b = X_B(a);
    const uint32_t n = x_span(a, b, X_T(a), x0);
    if (!n) continue;
    const uint32_t* P = a.ptr + (size_t)b * a.x_out_max + x0;
    const uint8_t* src = a.in + a.in_off[b];
    uint8_t* dst = a.out + a.out_off[b];
    const int64_t out_off = (int64_t)a.out_off[b];
    uint4 w[kXBytes / 4];
#pragma unroll
    for (int q = 0; q < kXBytes / 4; ++q) w[q] = ((const uint4*)P)[q];
    const uint32_t* v = (const uint32_t*)w;
    uint32_t o[kXBytes / 4] = {0, 0, 0, 0};
    // 16 bytes that are one run of consecutive literal bytes (tiles216: runs of ~50 B): one
    // unaligned 16-byte load instead of 16 byte loads (tiles216 192 blocks -11 %, round 6)
    bool run = x0 + kXBytes <= n && (v[0] & kHist) == kLit;
#pragma unroll
    for (int t = 1; t < kXBytes; ++t) run = run && v[t] == v[0] + (uint32_t)t;
    if (run) {
        uint4 r;
        __builtin_memcpy(&r, src + (v[0] & 0x3FFFFFFFu), 16);
        *(uint4*)(dst + x0) = r;
        continue;
    }
#pragma unroll
    for (int t = 0; t < kXBytes; ++t) {
        uint32_t c = 0;
        if ((v[t] & kHist) == kHist) {            // before the block: the caller's bytes or the dictionary
            const int64_t y = (int64_t)(v[t] & 0x3FFFFFFFu) - 65536;
            c = out_off + y >= 0 ? dst[y] : (a.dict ? a.dict[(int64_t)a.dict_len + out_off + y] : 0u);
        } else if (v[t] & kLit) {
            c = src[v[t] & 0x3FFFFFFFu];
        }
        o[t >> 2] |= c << (8 * (t & 3));
    }
    if (x0 + kXBytes <= n) {
        *(uint4*)(dst + x0) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        for (uint32_t t = 0; x0 + t < n; ++t) dst[x0 + t] = (uint8_t)(o[t >> 2] >> (8 * (t & 3)));
    }
  }
}

}  // namespace lz4mi

// The output phase of an exported small batch: the checks with absolute positions, status,
// expand, up to kJumpRounds jump rounds (each returns at once when the previous one left
// nothing to follow; a thread whose 16 bytes are resolved at once too), gather. `aux`: the round
// flags (32 words), nblocks check results, then nblocks * x_out_max / 16 done bytes.
extern "C" hipError_t lz4mi_launch_expand(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                          const uint64_t* out_off, const uint32_t* out_cap, const uint8_t* dict,
                                          uint32_t dict_len, uint32_t* out_len, int32_t* status, const uint4* xseq,
                                          const uint32_t* xcnt, lz4mi::SegRec* xrec, uint32_t nseg,
                                          uint32_t xseq_stride, uint32_t* ptr, uint32_t x_out_max, uint32_t* aux,
                                          int f1, uint32_t** redo_out, uint32_t nblocks, hipStream_t stream) {
    using namespace lz4mi;
    if (nblocks == 0) return hipSuccess;
    uint32_t* flags = aux;
    uint32_t* best = flags + 32;
    uint32_t* redo = best + ((nblocks + 63) & ~63u);
    uint8_t* done = (uint8_t*)(redo + ((nblocks + 63) & ~63u));
    *redo_out = redo;
    ExpArgs a{in, in_off, in_len, out, out_off, out_cap, dict, dict_len, out_len, status, xseq, xcnt, xrec, nseg, xseq_stride,
              ptr, x_out_max, done, flags, best, nblocks * (x_out_max / kTile),
              (uint32_t)__builtin_ctz(x_out_max / kTile)};
    if ((x_out_max & (x_out_max - 1)) || x_out_max < kTile) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(flags, 0, sizeof(uint32_t) * 32, stream);
    if (e == hipSuccess) e = hipMemsetAsync(done, 0, (size_t)nblocks * (x_out_max / kXBytes), stream);
    if (e == hipSuccess && f1) e = hipMemsetAsync(redo, 0, sizeof(uint32_t) * nblocks, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lz4mi_xbase_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(lz4mi_xcheck_kernel, dim3(nseg, nblocks), dim3(kXThreads), 0, stream, a, nblocks > 1 ? 1 : 0);
    hipLaunchKernelGGL(lz4mi_xstatus_kernel, dim3(nblocks), dim3(64), 0, stream, a);
    const dim3 grid(min(a.ntiles, kXGrid));
    hipLaunchKernelGGL(lz4mi_expand_kernel, grid, dim3(kXThreads), 0, stream, a);
    if (f1)
        hipLaunchKernelGGL(lz4mi_xf1ptr_kernel, dim3(nseg, nblocks), dim3(kXThreads), 0, stream, a, nblocks > 1 ? 1 : 0,
                           redo);
    for (int r = 0; r < kJumpRounds; ++r) hipLaunchKernelGGL(lz4mi_jump_kernel, grid, dim3(kXThreads), 0, stream, a, r);
    hipLaunchKernelGGL(lz4mi_chase_kernel, grid, dim3(kXThreads), 0, stream, a);
    hipLaunchKernelGGL(lz4mi_gather_kernel, grid, dim3(kXThreads), 0, stream, a);
    return hipGetLastError();
}
