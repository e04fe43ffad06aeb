// lz4mi_xxh32.hip — batched XXH32 of independent buffers (gfx950).
//
// Replaces xxHash32 (reference src/xxhash32/xxhash32.js:21-98) for many
// buffers at once (per-block digests, dictionary ids, parity checks). One
// buffer = one quad of lanes: lane j of the quad owns accumulator v(j+1) and
// reads dword j of every 16-byte stripe, so the quad reads each stripe as one
// coalesced 16-byte segment. The four chains are serial by definition, so the
// kernel is latency-bound per buffer and throughput comes from running
// 16 buffers per wave, many waves per CU.
//
// By default the lane convergence follows the reference (xxhash32.js:59-65:
// rotl(rotl(rotl(rotl(v1,1)+v2,7)+v3,12)+v4,18)); `standard` selects the
// XXH32 specification's rotl(v1,1)+rotl(v2,7)+rotl(v3,12)+rotl(v4,18).
#include "lz4mi_common.h"

namespace lz4mi {

constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

__device__ __forceinline__ uint32_t load_le32(const uint8_t* p, bool aligned) {
    if (aligned) return *(const uint32_t*)p;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// hashes[buf] = digest; or (TO_FRAME) the digest stored little-endian at dst + dst_off[buf]
// (frame block checksums written after their payloads). Two instantiations, so the plain
// batch kernel keeps its register allocation.
template <bool TO_FRAME>
__global__ __launch_bounds__(256) void lz4mi_xxh32_kernel(const uint8_t* in, const uint64_t* off, const uint32_t* len,
                                                          uint32_t seed, uint32_t* hashes, uint32_t n, int standard,
                                                          uint8_t* dst, const uint64_t* dst_off) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t buf = gid >> 2;
    const int j = threadIdx.x & 3;
    const bool live = buf < n;
    const uint8_t* p = live ? in + off[buf] : in;
    const uint64_t L = live ? len[buf] : 0;
    const bool aligned = (((uintptr_t)p) & 3) == 0;
    const uint64_t stripes = L >= 16 ? L / 16 : 0;

    uint32_t init[4] = { seed + P1 + P2, seed + P2, seed, seed - P1 };
    uint32_t v = init[j];
    const uint8_t* q = p + 4 * j;
    uint64_t k = 0;
    // software pipeline: the next kDepth stripes' words are in flight while the
    // current kDepth are folded into the accumulator (one load round trip per
    // 2 x kDepth stripes would otherwise stall the serial chain every kDepth steps)
    constexpr int kDepth = 128;
    if (stripes >= 2 * kDepth) {
        uint32_t w[kDepth];
#pragma unroll
        for (int u = 0; u < kDepth; ++u) w[u] = load_le32(q + 16 * u, aligned);
        for (; k + 2 * kDepth <= stripes; k += kDepth) {
            uint32_t nw[kDepth];
#pragma unroll
            for (int u = 0; u < kDepth; ++u) nw[u] = load_le32(q + 16 * (k + kDepth + u), aligned);
#pragma unroll
            for (int u = 0; u < kDepth; ++u) v = rotl(v + w[u] * P2, 13) * P1;
#pragma unroll
            for (int u = 0; u < kDepth; ++u) w[u] = nw[u];
        }
#pragma unroll
        for (int u = 0; u < kDepth; ++u) v = rotl(v + w[u] * P2, 13) * P1;
        k += kDepth;
    }
    for (; k + 8 <= stripes; k += 8) {   // short buffers and the pipeline's remainder
        uint32_t w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = load_le32(q + 16 * (k + u), aligned);
#pragma unroll
        for (int u = 0; u < 8; ++u) v = rotl(v + w[u] * P2, 13) * P1;
    }
    for (; k < stripes; ++k) v = rotl(v + load_le32(q + 16 * k, aligned) * P2, 13) * P1;

    // gather the quad's accumulators into every lane of the quad
    const int lane = threadIdx.x & 63, qb = lane & ~3;
    uint32_t v1 = __shfl(v, qb + 0, 64), v2 = __shfl(v, qb + 1, 64), v3 = __shfl(v, qb + 2, 64),
             v4 = __shfl(v, qb + 3, 64);
    if (!live || j != 0) return;
    uint32_t h;
    if (L >= 16) {
        if (standard) {
            h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        } else {
            h = rotl(v1, 1);
            h = rotl(h + v2, 7);
            h = rotl(h + v3, 12);
            h = rotl(h + v4, 18);
        }
    } else {
        h = seed + P5;
    }
    h += (uint32_t)L;
    uint64_t pos = stripes * 16;
    for (; pos + 4 <= L; pos += 4) h = rotl(h + load_le32(p + pos, false) * P3, 17) * P4;
    for (; pos < L; ++pos) h = rotl(h + p[pos] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    if (TO_FRAME) {
        uint8_t* q8 = dst + dst_off[buf];
        for (int k = 0; k < 4; ++k) q8[k] = (uint8_t)(h >> (8 * k));
    } else {
        hashes[buf] = h;
    }
}

// ---------------------------------------------------------------------------
// Synthetic block generator (identical to oracle/lz4_oracle.c
// orc_generate for kinds 0..2). One wave per block; the serial xorshift32
// stream runs on lane 0 into LDS, the wave writes it out coalesced.
__device__ __forceinline__ uint32_t xs32(uint32_t& x) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return x;
}

__global__ __launch_bounds__(64) void lz4mi_generate_kernel(uint8_t* out, uint32_t kind, uint32_t seed0,
                                                            uint32_t bsize) {
    __shared__ uint32_t tiles[216 * 16];     // 216 tiles x 64 bytes
    __shared__ uint32_t buf[1024];           // 4 KiB staging
    __shared__ uint32_t idx[64];
    const int lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    uint8_t* dst = out + (uint64_t)b * bsize;
    uint32_t x = seed0 + b;
    if (x == 0) x = 1;
    if (kind == 1) {                          // repetitive: b[i] = i % 251
        for (uint32_t i = lane; i < bsize; i += 64) dst[i] = (uint8_t)(i % 251);
        return;
    }
    if (kind == 0) {                          // random: one word per 4 bytes, little-endian
        for (uint32_t base = 0; base < bsize; base += 4096) {
            if (lane == 0) for (int k = 0; k < 1024; ++k) buf[k] = xs32(x);
            __syncthreads();
            uint32_t lim = bsize - base < 4096 ? bsize - base : 4096;
            for (uint32_t i = lane; i < lim; i += 64) dst[base + i] = ((const uint8_t*)buf)[i];
            __syncthreads();
        }
        return;
    }
    // tiles216: 216 random 64-byte tiles (one xorshift per byte), then tiles by r() % 216
    if (lane == 0) {
        uint8_t* t = (uint8_t*)tiles;
        for (int k = 0; k < 216 * 64; ++k) t[k] = (uint8_t)(xs32(x) & 255);
    }
    __syncthreads();
    for (uint32_t base = 0; base < bsize; base += 64 * 64) {
        if (lane == 0) for (int k = 0; k < 64; ++k) idx[k] = xs32(x) % 216;
        __syncthreads();
        // 64 tiles x 64 bytes: lane writes dword `lane % 16` of 4 tiles per step
        for (int s = 0; s < 64; s += 4) {
            int t = s + lane / 16, w = lane & 15;
            uint32_t pos = base + 64 * t + 4 * w;
            uint32_t v = tiles[idx[t] * 16 + w];
            if (pos + 4 <= bsize) {
                *(uint32_t*)(dst + pos) = v;            // bsize is a multiple of 4 in every config
            } else {
                for (uint32_t j = 0; j < 4 && pos + j < bsize; ++j) dst[pos + j] = (uint8_t)(v >> (8 * j));
            }
        }
        __syncthreads();
    }
}

}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_xxh32(const uint8_t* in, const uint64_t* off, const uint32_t* len, uint32_t seed,
                                         uint32_t* hashes, uint32_t n, int standard, uint8_t* dst,
                                         const uint64_t* dst_off, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // one wave (16 buffers) per workgroup: the waves spread over every CU's load path
    uint32_t threads = n * 4;
    if (dst)
        hipLaunchKernelGGL(lz4mi::lz4mi_xxh32_kernel<true>, dim3((threads + 63) / 64), dim3(64), 0, stream, in, off,
                           len, seed, hashes, n, standard, dst, dst_off);
    else
        hipLaunchKernelGGL(lz4mi::lz4mi_xxh32_kernel<false>, dim3((threads + 63) / 64), dim3(64), 0, stream, in, off,
                           len, seed, hashes, n, standard, dst, dst_off);
    return hipGetLastError();
}

extern "C" hipError_t lz4mi_launch_generate(uint8_t* out, uint32_t kind, uint32_t seed0, uint32_t bsize,
                                            uint32_t nblocks, hipStream_t stream) {
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(lz4mi::lz4mi_generate_kernel, dim3(nblocks), dim3(64), 0, stream, out, kind, seed0, bsize);
    return hipGetLastError();
}
