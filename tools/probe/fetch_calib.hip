// Probe: calibrate rocprofv3 FETCH_SIZE for the decoder's read patterns.
// The MI355X guide calibrates FETCH_SIZE only for 16-B/lane coalesced streaming
// reads (FETCH = 1/2 of the bytes). The decoder's history reads are scattered
// 16-byte unaligned loads, one match per lane. Each kernel below reads a known
// number of bytes from a 2 GiB buffer (past the 256 MiB Infinity Cache, cold),
// so FETCH_SIZE / known bytes is the counter's factor for that pattern, and the
// kernel time says whether the fabric moved the bytes read or whole lines.
//   k_stream   16 B/lane coalesced, every byte once             known 2 GiB
//   k_lines    8 lanes per 128-B line, lines in permuted order    known 2 GiB
//   k_half     4 lanes per first 64-B half of each line, permuted  known 1 GiB
//   k_piece    one lane per line, 16 B at an unaligned offset      known 256 MiB
//   k_decoder  one wave per 4 MiB region: 64-byte runs copied from 4-32 KiB
//              back in the region this wave is writing (the decoder's pattern)
// Run: hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
//      rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t kBuf = 1ull << 31;
constexpr uint64_t kLines = kBuf / 128;
constexpr int kRegion = 4 << 20;
constexpr int kRegions = 1024;

__device__ __forceinline__ uint64_t perm(uint64_t i) { return (i * 0x9E3779B1ull) & (kLines - 1); }
__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__global__ __launch_bounds__(256) void k_stream(const uint8_t* b, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < kBuf / 16; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = *(const u32x4*)(b + 16 * i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_lines(const uint8_t* b, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < kLines * 8; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = *(const u32x4*)(b + 128 * perm(i >> 3) + 16 * (i & 7));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_half(const uint8_t* b, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < kLines * 4; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = *(const u32x4*)(b + 128 * perm(i >> 2) + 16 * (i & 3));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_piece(const uint8_t* b, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < kLines; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = ld16(b + 128 * perm(i) + mix((uint32_t)i) % 113);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(64) void k_decoder(uint8_t* b) {
    uint8_t* r = b + (uint64_t)blockIdx.x * kRegion;
    const int l = threadIdx.x;
    for (int o = 36864; o < kRegion; o += 4096) {   // every source >= 4081: inside the region
        const int dst = o + 64 * l;
        const uint32_t h = mix((uint32_t)(blockIdx.x * 4096 + dst));
        const int src = dst - 4096 - (int)(h & 0x7000) - (int)((h >> 16) & 15);
        u32x4 v0 = ld16(r + src), v1 = ld16(r + src + 16), v2 = ld16(r + src + 32), v3 = ld16(r + src + 48);
        __builtin_memcpy(r + dst, &v0, 16);
        __builtin_memcpy(r + dst + 16, &v1, 16);
        __builtin_memcpy(r + dst + 32, &v2, 16);
        __builtin_memcpy(r + dst + 48, &v3, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

int main() {
    uint8_t *buf, *reg;
    uint32_t* sink;
    if (hipMalloc(&buf, kBuf) != hipSuccess || hipMalloc(&reg, (size_t)kRegions * kRegion) != hipSuccess ||
        hipMalloc(&sink, 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, kBuf);
    hipMemset(reg, 2, (size_t)kRegions * kRegion);
    // evict: stream a separate 512 MiB through the Infinity Cache between kernels
    uint8_t* flush;
    hipMalloc(&flush, 512u << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 32;
    const double known[5] = {(double)kBuf, (double)kBuf, kBuf / 2.0, kBuf / 8.0,
                             (double)kRegions * (kRegion - 36864)};
    const char* names[5] = {"k_stream", "k_lines", "k_half", "k_piece", "k_decoder(read bytes)"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int k = 0; k < 5; ++k) {
            hipMemsetAsync(flush, rep + k, 512u << 20);
            hipEventRecord(e0);
            switch (k) {
                case 0: k_stream<<<grid, 256>>>(buf, sink); break;
                case 1: k_lines<<<grid, 256>>>(buf, sink); break;
                case 2: k_half<<<grid, 256>>>(buf, sink); break;
                case 3: k_piece<<<grid, 256>>>(buf, sink); break;
                case 4: k_decoder<<<kRegions, 64>>>(reg); break;
            }
            hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
                printf("kernel %s failed\n", names[k]);
                return 1;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("rep %d %-22s known %.3f GB  %.3f ms  %.0f GB/s of known bytes\n", rep, names[k], known[k] / 1e9,
                   ms, known[k] / 1e6 / ms);
        }
    }
    hipFree(flush);
    hipFree(buf);
    hipFree(reg);
    hipFree(sink);
    return 0;
}
