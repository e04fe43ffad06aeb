// Probe: cost of 16-byte scattered stores vs the number of active lanes per
// instruction and the address pattern (decoder output design question).
//   mode 0: all 64 lanes, lane l writes its own 64-byte tile piece by piece (4 instr / 64 tiles)
//   mode 1: 4 lanes per tile (16 tiles per instruction, 4 instr / 64 tiles)
//   mode 2: 16 active lanes per instruction, one tile per lane (16 instr / 64 tiles)
// Every wave writes the same number of tiles (at pseudo-random 64-byte slots of its
// own 4 MiB region, or in order), so bytes written are equal across modes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kTiles = 65536;        // tiles per wave = 4 MiB
template <bool SEQ>
__global__ __launch_bounds__(64) void wr(uint8_t* buf, int mode) {
    uint8_t* r = buf + (size_t)blockIdx.x * (4u << 20);
    const int l = threadIdx.x;
    const uint4 v = make_uint4(l, blockIdx.x, 1, 2);
    auto slot = [](uint32_t t) { return SEQ ? t : (t * 2654435761u) & (kTiles - 1); };   // in order, or a permutation
    if (mode == 0) {
        for (int t0 = 0; t0 < kTiles; t0 += 64) {
            uint8_t* p = r + 64 * (size_t)slot(t0 + l);
#pragma unroll
            for (int j = 0; j < 4; ++j) *(uint4*)(p + 16 * j) = v;
        }
    } else if (mode == 1) {
        for (int t0 = 0; t0 < kTiles; t0 += 16) {
            uint8_t* p = r + 64 * (size_t)slot(t0 + (l >> 2)) + 16 * (l & 3);
            *(uint4*)p = v;
        }
    } else {
        for (int t0 = 0; t0 < kTiles; t0 += 16) {
            if (l < 16) {
                uint8_t* p = r + 64 * (size_t)slot(t0 + l);
#pragma unroll
                for (int j = 0; j < 4; ++j) *(uint4*)(p + 16 * j) = v;
            }
        }
    }
}

int main() {
    const int nb = 4096;
    uint8_t* d;
    if (hipMalloc(&d, (size_t)nb * (4u << 20)) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep)
        for (int seq = 0; seq < 2; ++seq)
            for (int mode = 0; mode < 3; ++mode) {
                hipEventRecord(a);
                if (seq) hipLaunchKernelGGL(wr<true>, dim3(nb), dim3(64), 0, 0, d, mode);
                else hipLaunchKernelGGL(wr<false>, dim3(nb), dim3(64), 0, 0, d, mode);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                printf("%s mode %d: %.2f ms = %.0f GB/s\n", seq ? "in-order" : "scattered", mode, ms,
                       nb * 4194304.0 / ms / 1e6);
            }
    return 0;
}
