// Probe: cost of LDS accesses by width and alignment, one wave per CU
// (the ring decoder's access pattern: lane-private addresses, arbitrary byte offsets).
//   hipcc -O3 --offload-arch=gfx950 -o tools/probe/lds_unaligned tools/probe/lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int KIND>
__global__ void k_lds(uint64_t* cyc, uint32_t* sink, int mis, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t L[65536 + 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 65536 / 4; i += blockDim.x) ((uint32_t*)L)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    uint32_t a = (lane * 1000 + mis) & 0xFFFF;   // lane-private, spread over banks
    const uint64_t t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t p = (a + j * 64) & 0xFFF0 | (mis & 15);
            if (KIND == 0) {   // 16-byte read
                uint4 v;
                __builtin_memcpy(&v, L + p, 16);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            } else if (KIND == 1) {   // 16-byte write
                uint4 v = make_uint4(acc, it, j, lane);
                __builtin_memcpy(L + p, &v, 16);
            } else if (KIND == 2) {   // 4-byte read
                uint32_t v;
                __builtin_memcpy(&v, L + p, 4);
                acc += v;
            } else if (KIND == 3) {   // 4-byte write
                uint32_t v = acc + it + j;
                __builtin_memcpy(L + p, &v, 4);
            } else if (KIND == 4) {   // 8-byte read
                uint2 v;
                __builtin_memcpy(&v, L + p, 8);
                acc += v.x ^ v.y;
            } else if (KIND == 5) {   // 16 bytes as 4 x 4-byte reads
                uint32_t v0, v1, v2, v3;
                __builtin_memcpy(&v0, L + p, 4);
                __builtin_memcpy(&v1, L + p + 4, 4);
                __builtin_memcpy(&v2, L + p + 8, 4);
                __builtin_memcpy(&v3, L + p + 12, 4);
                acc += v0 ^ v1 ^ v2 ^ v3;
            } else if (KIND == 6) {   // 16 bytes as 4 x 4-byte writes
                uint32_t v = acc + it;
                __builtin_memcpy(L + p, &v, 4);
                __builtin_memcpy(L + p + 4, &v, 4);
                __builtin_memcpy(L + p + 8, &v, 4);
                __builtin_memcpy(L + p + 12, &v, 4);
            }
        }
        a += 4096 + 7;
    }
    __syncthreads();
    const uint64_t t1 = clock64();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + lane] = acc + L[lane];
}

int main() {
    uint64_t* cyc;
    uint32_t* sink;
    hipMalloc(&cyc, 8 * 1024);
    hipMalloc(&sink, 4 * 64 * 1024);
    const char* names[] = {"read16", "write16", "read4", "write4", "read8", "read16as4x4", "write16as4x4"};
    const int iters = 2000;
    for (int kind = 0; kind < 7; ++kind) {
        for (int mis : {0, 1, 4, 8}) {
            for (int waves : {1, 4}) {
                auto k = kind == 0 ? k_lds<0> : kind == 1 ? k_lds<1> : kind == 2 ? k_lds<2> : kind == 3 ? k_lds<3>
                       : kind == 4 ? k_lds<4> : kind == 5 ? k_lds<5> : k_lds<6>;
                hipLaunchKernelGGL(k, dim3(256), dim3(64 * waves), 0, 0, cyc, sink, mis, iters);
                hipDeviceSynchronize();
                uint64_t h[256];
                hipMemcpy(h, cyc, 8 * 256, hipMemcpyDeviceToHost);
                double avg = 0;
                for (int i = 0; i < 256; ++i) avg += h[i];
                avg /= 256;
                printf("%-13s mis=%2d waves/WG=%d: %6.1f cycles per wave-instruction (per wave)\n", names[kind], mis,
                       waves, avg / (iters * 8.0));
            }
        }
    }
    return 0;
}
