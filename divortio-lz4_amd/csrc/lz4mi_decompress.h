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
    int redo_only; // decode only the blocks whose status is kStatusRedo (handed back by the ring decoder)
    const uint64_t* bitmap;      // token bitmaps of pass 1 (lz4mi_token_map_kernel): replace the speculative parse
    const uint32_t* chunk_base;  // first bitmap chunk of each block
};

constexpr int32_t kStatusRedo = -11; // internal: the two-pass ring decoder hands the block to the single-pass kernel

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress_serial(const lz4mi::DecArgs& a, hipStream_t stream);

// Two-pass ring decoder (lz4mi_decompress_ring.hip).
extern "C" hipError_t lz4mi_launch_ring_plan(const uint32_t* in_len, const uint32_t* out_cap, uint32_t min_ratio,
                                             uint32_t nblocks, uint64_t capacity_chunks, uint32_t* chunk_base,
                                             uint32_t* needed, hipStream_t stream);
extern "C" hipError_t lz4mi_launch_token_map(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                             const uint32_t* out_cap, uint32_t min_ratio, const uint32_t* chunk_base,
                                             uint64_t* bitmap, uint32_t nblocks, hipStream_t stream);
extern "C" hipError_t lz4mi_launch_ring_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                               uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                               uint32_t* out_len, int32_t* status, const uint32_t* chunk_base,
                                               const uint64_t* bitmap, uint32_t min_ratio, uint32_t* stats,
                                               uint32_t nblocks, hipStream_t stream);
