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
    // small batches (lz4mi_expand.hip): a block within the export limits is parsed only and its
    // sequences exported as {output start, literal source, literal length, offset} to
    // xseq + b * xseq_stride, their count to xcnt[b] (kNotExported: decoded here as usual)
    uint4* xseq = nullptr;
    uint32_t* xcnt = nullptr;
    uint32_t xseq_stride = 0;          // entries per block (>= in_len / 3 + 2 for an exported block)
    uint32_t x_in_max = 0, x_out_max = 0;
};
constexpr uint32_t kNotExported = 0xFFFFFFFFu;

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress_serial(const lz4mi::DecArgs& a, hipStream_t stream);
