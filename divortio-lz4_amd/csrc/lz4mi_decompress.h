// lz4mi_decompress.h — arguments shared by the decoder kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4mi {

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
    int isolate;   // batched blocks: a back-reference before the block start is reported, not followed
    int f1check;   // reference-exact (LZ4MI_JS_EXACT): fix up every chunk the reference's F1 rewrite changes
    const uint32_t* order = nullptr;   // workgroup w decodes block order[w] (nullptr: block w)
    int frame_words = 0;               // in_len[b] is a frame size word: bit 31 = stored block (copied)
    // small batches (lz4mi_expand.hip, lz4mi_decompress_x_kernel): a block within the export
    // limits is parsed by xsegs waves, one per segment of its compressed bytes, which export
    // their sequences as {output start in the segment, literal source, literal length, offset}
    // to xseq + (b * xsegs + s) * xseq_stride and their summary to xrec[b * xsegs + s]; a block
    // past the limits is decoded by its segment-0 wave as usual (xcnt[b] = kNotExported)
    uint4* xseq = nullptr;
    uint32_t* xcnt = nullptr;
    struct SegRec* xrec = nullptr;
    uint32_t xseq_stride = 0;          // entries per block (seg_geom: its segments at s * stride)
    uint32_t xsegs = 0;
    uint32_t x_in_max = 0, x_out_max = 0;
    int x_flat1 = 0;                   // nearly incompressible blocks (compressed >= 15/16 of the output) take one wave too
    int xphase = 0;                    // 0: speculative parse; 2: re-parse of the disagreeing ones; 1: in order from the first bad entry
    const uint32_t* xfirst = nullptr;  // phase 1: per block, the first segment whose entry was wrong
    uint32_t* xfirst_w = nullptr;      // (written by lz4mi_xverify_kernel)
    int xforce = 0;                    // test hook: every guess of segments past the first counts as wrong (1: phase 0's, 2: phase 2's too)
    const uint32_t* redo = nullptr;    // batch kernel: decode only the blocks with redo[b] != 0 (nullptr: all)
};
// One segment of an exported block. Its wave parses from a guessed entry (the first token at or
// past the segment start, found by a warm-up parse before it); lz4mi_xverify_kernel accepts the
// segments whose entries equal their predecessors' exits, in order from segment 0 (exact), and
// phase 1 re-parses from the first that does not (and checks the rest again, in order).
struct SegRec {
    uint32_t entry;   // first token at or past the segment start (the chain's end: in_len)
    uint32_t exit;    // first token at or past the segment end
    uint32_t cnt;     // sequences exported (incl. a failing one)
    uint32_t olen;    // their output bytes
    uint32_t err;     // (index in the segment << 3) | check of its first parse error; 0xFFFFFFFF: none
    uint32_t fin;     // final exit + 1 once checked against the previous segment (0: not yet)
    uint32_t base;    // output start of the segment (lz4mi_xbase_kernel; kNoBase: after the block's first error)
    uint32_t fail;    // the speculative parse met an error before the segment: its guess is wrong
    uint32_t g0;      // number of the segment's first sequence in the block (lz4mi_xbase_kernel)
    uint32_t from;    // phase 2: re-parse from this entry (kNoBase: no; lz4mi_xverify_kernel)
    uint32_t pad[2];
};
constexpr uint32_t kNoBase = 0xFFFFFFFFu;
constexpr uint32_t kFinErr = 0xFFFFFFFEu;
constexpr uint32_t kSegMax = 256;            // segments (waves) per exported block, at most
constexpr uint32_t kSegTarget = 8192;        // compressed bytes per segment (a 4 MiB tiles216 block: 64)
// An exported block's segments: S of them, L compressed bytes each (the last takes the rest),
// segment s's sequence entries at s * stride in the block's region (L / 3 sequences of >= 3
// bytes, a failing one, the cut, and the 3 KiB warm-up's margin).
struct SegGeom {
    uint32_t S, L, stride;
};
__host__ __device__ inline SegGeom seg_geom(uint32_t in_len) {
    uint32_t S = (in_len + kSegTarget - 1) / kSegTarget;
    S = S < 1 ? 1 : (S > kSegMax ? kSegMax : S);
    uint32_t L = ((in_len + S - 1) / S + 1023u) & ~1023u;
    if (L < 4096) L = 4096;
    return SegGeom{S, L, L / 3 + 1400};
}
// entries per block: every S * stride above (S * L <= in_len + S * 1024 + 4096) fits
__host__ __device__ constexpr uint32_t seg_block_capacity(uint32_t x_in_max) { return x_in_max / 3 + kSegMax * 1800; }   // fin - 1 of a segment at or after the block's first error
constexpr uint32_t kNotExported = 0xFFFFFFFFu;

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress_serial(const lz4mi::DecArgs& a, hipStream_t stream);
