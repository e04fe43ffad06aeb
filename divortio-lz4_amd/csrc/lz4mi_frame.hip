// lz4mi_frame.hip — device-side frame block records.
//
// The frame writer's block loop (reference src/buffer/bufferCompress.js:209-239)
// emits, per block, a LE32 size word and the payload: the compressed bytes when
// 0 < compSize < blockSize, else blockSize | 0x80000000 and the raw bytes. With
// independent blocks compressed in one batch on the device, this kernel writes
// those records straight into the frame buffer at caller-computed offsets
// (exclusive prefix sum of 4 + payload), so the frame never visits the host.
// One wave per block; 16-byte unaligned pieces, the last one overlapping.
// With block checksums (FLG bit 0x10) a record is size word + payload + LE32
// XXH32(payload): the kernel then also writes each payload's frame position and
// length (pay_off/pay_len) and its checksum position (sum_off) for the batched
// XXH32 kernel that fills them in.
#include "lz4mi_common.h"

namespace lz4mi {

__global__ __launch_bounds__(64) void lz4mi_frame_pack_kernel(const uint8_t* raw, const uint64_t* raw_off,
                                                              const uint32_t* raw_len, const uint8_t* comp,
                                                              const uint64_t* comp_off, const uint32_t* comp_len,
                                                              uint8_t* frame, const uint64_t* rec_off,
                                                              uint32_t nblocks, uint64_t* pay_off, uint64_t* sum_off,
                                                              uint32_t* pay_len) {
    const uint32_t b = blockIdx.x;
    const int lane = threadIdx.x;
    if (b >= nblocks) return;
    const uint32_t n = raw_len[b], cl = comp_len[b];
    const bool stored = !(cl > 0 && cl < n);
    const uint32_t word = stored ? (n | 0x80000000u) : cl;
    const uint8_t* src = stored ? raw + raw_off[b] : comp + comp_off[b];
    const uint64_t len = stored ? n : cl;
    uint8_t* dst = frame + rec_off[b];
    if (pay_off && lane == 0) {
        pay_off[b] = rec_off[b] + 4;
        sum_off[b] = rec_off[b] + 4 + len;
        pay_len[b] = (uint32_t)len;
    }
    if (lane < 4) dst[lane] = (uint8_t)(word >> (8 * lane));
    dst += 4;
    if (len < 16) {
        if ((uint64_t)lane < len) dst[lane] = src[lane];
        return;
    }
    const uint64_t np = (len + 15) / 16;
    for (uint64_t p0 = 0; p0 < np; p0 += 4 * kWave) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t p = p0 + lane + kWave * u;
            const uint64_t d = 16 * p < len - 16 ? 16 * p : len - 16;
            if (p < np) __builtin_memcpy(&v[u], src + d, 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t p = p0 + lane + kWave * u;
            const uint64_t d = 16 * p < len - 16 ? 16 * p : len - 16;
            if (p < np) __builtin_memcpy(dst + d, &v[u], 16);
        }
    }
}

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_frame_pack(const uint8_t* raw, const uint64_t* raw_off, const uint32_t* raw_len,
                                              const uint8_t* comp, const uint64_t* comp_off, const uint32_t* comp_len,
                                              uint8_t* frame, const uint64_t* rec_off, uint32_t nblocks,
                                              uint64_t* pay_off, uint64_t* sum_off, uint32_t* pay_len,
                                              hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(lz4mi::lz4mi_frame_pack_kernel, dim3(nblocks), dim3(64), 0, stream, raw, raw_off, raw_len,
                       comp, comp_off, comp_len, frame, rec_off, nblocks, pay_off, sum_off, pay_len);
    return hipGetLastError();
}
