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

// ---------------------------------------------------------------------------
// Decode side: the frame's header and block walk on the device (the reference's
// decompressBuffer, src/buffer/bufferDecompress.js:56-92 header, :133-192 block loop).
// One lane walks the size words (each record's position depends on the previous
// size); compressed and stored blocks go to two lists. Output positions assume the
// reference encoder's layout (every block but the last fills block_max bytes; the
// caller checks the decoded lengths, as the JS layer's batch path does).
// info[0] status (0, LZ4MI_ERR_MAGIC -5, LZ4MI_ERR_VERSION -6), [1] FLG, [2] content size,
// [3] compressed blocks, [4] stored blocks, [5] position after the EndMark (content
// checksum), [6] block_max (BD), [7] 1 if the walk ran past the frame or the lists' capacity.
__global__ __launch_bounds__(64) void lz4mi_frame_scan_kernel(const uint8_t* f, uint64_t len, uint32_t cap_blocks,
                                                              uint64_t* c_in_off, uint32_t* c_in_len,
                                                              uint64_t* c_out_off, uint32_t* c_out_cap,
                                                              uint64_t* s_in_off, uint32_t* s_len, uint64_t* s_out_off,
                                                              uint32_t* c_idx, uint32_t* s_idx, int64_t* info) {
    if (threadIdx.x != 0) return;
    auto rd = [&](uint64_t p) -> uint32_t {
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v |= (p + k < len ? (uint32_t)f[p + k] : 0u) << (8 * k);
        return v;
    };
    int64_t st = 0, flg = 0, size = 0, nc = 0, ns = 0, overflow = 0;
    uint64_t pos = 0;
    int64_t bmax = 4194304;
    if (len < 4 || rd(0) != 0x184D2204u) {
        st = -5;
    } else {
        flg = len > 4 ? f[4] : 0;
        if (((flg & 0xC0) >> 6) != 1) {
            st = -6;
        } else {
            const uint32_t bd = len > 5 ? f[5] : 0;
            const uint32_t id = (bd >> 4) & 7;
            bmax = id == 4 ? 65536 : id == 5 ? 262144 : id == 6 ? 1048576 : 4194304;
            pos = 6;
            if (flg & 0x08) {
                size = (int64_t)((uint64_t)rd(pos) | ((uint64_t)rd(pos + 4) << 32));
                pos += 8;
            }
            if (flg & 0x01) pos += 4;
            pos += 1;
            uint64_t op = 0;
            while (pos < len) {
                const uint32_t bs = rd(pos);
                pos += 4;
                if (bs == 0) break;
                const uint32_t n = bs & 0x7FFFFFFFu;
                if (nc + ns >= (int64_t)cap_blocks) { overflow = 1; break; }
                if (bs & 0x80000000u) {
                    s_in_off[ns] = pos;
                    s_len[ns] = n;
                    s_out_off[ns] = op;
                    s_idx[ns] = (uint32_t)(nc + ns);
                    ++ns;
                    op += n;               // the reference advances by the declared size
                } else {
                    c_in_off[nc] = pos;
                    c_in_len[nc] = n;
                    c_out_off[nc] = op;
                    const int64_t left = size - (int64_t)op;
                    c_out_cap[nc] = (uint32_t)(left < 0 ? 0 : (left < bmax ? left : bmax));
                    c_idx[nc] = (uint32_t)(nc + ns);
                    ++nc;
                    op += (uint64_t)bmax;
                }
                pos += n + ((flg & 0x10) ? 4 : 0);
            }
            if (pos > len) overflow = 1;
        }
    }
    info[0] = st; info[1] = flg; info[2] = size; info[3] = nc; info[4] = ns;
    info[5] = (int64_t)pos; info[6] = bmax; info[7] = overflow;
}

// The frame's block index for sharded decoding (lz4mi_frame_index): one lane walks the
// header and the size words like the scan above, and lists every block in frame order:
// payload position and raw size word (stored bit 31 included). info as for the scan,
// with [3] = blocks listed and [4] = 0.
__global__ __launch_bounds__(64) void lz4mi_frame_index_kernel(const uint8_t* f, uint64_t len, uint32_t cap_blocks,
                                                               uint64_t* pay_off, uint32_t* size_word, int64_t* info) {
    if (threadIdx.x != 0) return;
    auto rd = [&](uint64_t p) -> uint32_t {
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v |= (p + k < len ? (uint32_t)f[p + k] : 0u) << (8 * k);
        return v;
    };
    int64_t st = 0, flg = 0, size = 0, nb = 0, overflow = 0;
    uint64_t pos = 0;
    int64_t bmax = 4194304;
    if (len < 4 || rd(0) != 0x184D2204u) {
        st = -5;
    } else {
        flg = len > 4 ? f[4] : 0;
        if (((flg & 0xC0) >> 6) != 1) {
            st = -6;
        } else {
            const uint32_t id = len > 5 ? (f[5] >> 4) & 7 : 7;
            bmax = id == 4 ? 65536 : id == 5 ? 262144 : id == 6 ? 1048576 : 4194304;
            pos = 6;
            if (flg & 0x08) {
                size = (int64_t)((uint64_t)rd(pos) | ((uint64_t)rd(pos + 4) << 32));
                pos += 8;
            }
            if (flg & 0x01) pos += 4;
            pos += 1;
            while (pos < len) {
                const uint32_t bs = rd(pos);
                pos += 4;
                if (bs == 0) break;
                if (nb >= (int64_t)cap_blocks) { overflow = 1; break; }
                pay_off[nb] = pos;
                size_word[nb] = bs;
                ++nb;
                pos += (uint64_t)(bs & 0x7FFFFFFFu) + ((flg & 0x10) ? 4 : 0);
            }
            if (pos > len) overflow = 1;
        }
    }
    info[0] = st; info[1] = flg; info[2] = size; info[3] = nb; info[4] = 0;
    info[5] = (int64_t)pos; info[6] = bmax; info[7] = overflow;
}

// Stored blocks' bytes into the output (one wave per stored block; clipped at `cap`
// like the reference's result.set would throw past it: the caller checks first).
__global__ __launch_bounds__(64) void lz4mi_frame_stored_kernel(const uint8_t* f, uint64_t len, const uint64_t* s_in_off,
                                                                const uint32_t* s_len, const uint64_t* s_out_off,
                                                                uint8_t* out, uint64_t cap, uint32_t ns) {
    const uint32_t b = blockIdx.x;
    const int lane = threadIdx.x;
    if (b >= ns) return;
    const uint64_t src = s_in_off[b], dst = s_out_off[b];
    uint64_t n = s_len[b];
    if (src + n > len) n = src < len ? len - src : 0;      // subarray() clips at the frame end
    if (dst + n > cap) n = dst < cap ? cap - dst : 0;
    if (n < 16) {
        if ((uint64_t)lane < n) out[dst + lane] = f[src + lane];
        return;
    }
    const uint64_t np = (n + 15) / 16;   // 16-byte pieces, the last one overlapping its predecessor
    for (uint64_t p0 = 0; p0 < np; p0 += 4 * kWave) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t p = p0 + lane + kWave * u;
            const uint64_t d = 16 * p < n - 16 ? 16 * p : n - 16;
            if (p < np) __builtin_memcpy(&v[u], f + src + d, 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t p = p0 + lane + kWave * u;
            const uint64_t d = 16 * p < n - 16 ? 16 * p : n - 16;
            if (p < np) __builtin_memcpy(out + dst + d, &v[u], 16);
        }
    }
}

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_frame_scan(const uint8_t* f, uint64_t len, uint32_t cap_blocks, uint64_t* c_in_off,
                                              uint32_t* c_in_len, uint64_t* c_out_off, uint32_t* c_out_cap,
                                              uint64_t* s_in_off, uint32_t* s_len, uint64_t* s_out_off, uint32_t* c_idx,
                                              uint32_t* s_idx, int64_t* info, hipStream_t stream) {
    hipLaunchKernelGGL(lz4mi::lz4mi_frame_scan_kernel, dim3(1), dim3(64), 0, stream, f, len, cap_blocks, c_in_off,
                       c_in_len, c_out_off, c_out_cap, s_in_off, s_len, s_out_off, c_idx, s_idx, info);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_frame_stored(const uint8_t* f, uint64_t len, const uint64_t* s_in_off,
                                                const uint32_t* s_len, const uint64_t* s_out_off, uint8_t* out,
                                                uint64_t cap, uint32_t ns, hipStream_t stream) {
    if (ns == 0) return hipSuccess;
    hipLaunchKernelGGL(lz4mi::lz4mi_frame_stored_kernel, dim3(ns), dim3(64), 0, stream, f, len, s_in_off, s_len,
                       s_out_off, out, cap, ns);
    return hipGetLastError();
}

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

extern "C" hipError_t lz4mi_launch_frame_index(const uint8_t* f, uint64_t len, uint32_t cap_blocks, uint64_t* pay_off,
                                               uint32_t* size_word, int64_t* info, hipStream_t stream) {
    hipLaunchKernelGGL(lz4mi::lz4mi_frame_index_kernel, dim3(1), dim3(64), 0, stream, f, len, cap_blocks, pay_off,
                       size_word, info);
    return hipGetLastError();
}
