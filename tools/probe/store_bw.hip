// Probe: throughput of 16-byte lane stores (global_store_dwordx4) by destination
// alignment, one wave per 4 MiB region, 4096 regions (the decoder's shape).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/store_bw tools/probe/store_bw.hip && /tmp/store_bw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int64_t kRegion = 4 << 20;

// consecutive 1 KiB rows: lane l writes bytes [16l, 16l + 16) of each row, shifted by mis
__global__ __launch_bounds__(64) void rows(uint8_t* dst, int mis) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64) + mis;
    const int l = threadIdx.x;
    const uint4 v = make_uint4(l, 1, 2, 3);
    for (int64_t o = 16 * l; o < kRegion; o += 1024) __builtin_memcpy(r + o, &v, 16);
}

// 64-byte runs: lane l writes 4 pieces at [64l, 64l + 64) of each 4 KiB row
__global__ __launch_bounds__(64) void runs(uint8_t* dst, int mis) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64) + mis;
    const int l = threadIdx.x;
    const uint4 v = make_uint4(l, 1, 2, 3);
    for (int64_t o = 64 * l; o < kRegion; o += 4096) {
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_memcpy(r + o + 16 * j, &v, 16);
    }
}

// 64-byte runs read from 14 KiB back in the same region (copy, like a match)
__global__ __launch_bounds__(64) void copies(uint8_t* dst, int mis, int dist) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64) + mis;
    const int l = threadIdx.x;
    for (int64_t o = 65536 + 64 * l; o < kRegion; o += 4096) {
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_memcpy(&v[j], r + o - dist + 16 * j, 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_memcpy(r + o + 16 * j, &v[j], 16);
    }
}

// copies, software-pipelined by two rows: row i+1's loads are issued before row i's stores
#define LD4(x, p) __builtin_memcpy(&x##0, (p), 16); __builtin_memcpy(&x##1, (p) + 16, 16); \
                  __builtin_memcpy(&x##2, (p) + 32, 16); __builtin_memcpy(&x##3, (p) + 48, 16)
#define ST4(p, x) __builtin_memcpy((p), &x##0, 16); __builtin_memcpy((p) + 16, &x##1, 16); \
                  __builtin_memcpy((p) + 32, &x##2, 16); __builtin_memcpy((p) + 48, &x##3, 16)
__global__ __launch_bounds__(64) void copies_pipe(uint8_t* dst, int mis, int dist) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64) + mis;
    const int l = threadIdx.x;
    uint4 a0, a1, a2, a3, b0, b1, b2, b3;
    int64_t o = 65536 + 64 * l;
    LD4(a, r + o - dist);
    for (; o + 8192 <= kRegion; o += 8192) {
        LD4(b, r + o + 4096 - dist);
        ST4(r + o, a);
        LD4(a, r + o + 8192 - dist);
        ST4(r + o + 4096, b);
    }
}

// plain copy between two buffers (no read-after-write), 64-byte runs per lane
__global__ __launch_bounds__(64) void memcpy_runs(uint8_t* dst, int mis, int dist) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64);
    const uint8_t* q = dst + (int64_t)((blockIdx.x + 2048) % 4096) * (kRegion + 64);
    const int l = threadIdx.x;
    for (int64_t o = 64 * l; o < kRegion; o += 4096) {
        uint4 a0, a1, a2, a3;
        LD4(a, q + o);
        ST4(r + o, a);
    }
}

// copies with each instruction covering 1 KiB contiguous output (lane l: bytes [16l, 16l+16)), pipelined
__global__ __launch_bounds__(64) void copies_rows(uint8_t* dst, int mis, int dist) {
    uint8_t* r = dst + (int64_t)blockIdx.x * (kRegion + 64) + mis;
    const int l = threadIdx.x;
    int64_t o = 65536 + 16 * l;
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) __builtin_memcpy(&v[j], r + o - dist + 1024 * j, 16);
    for (; o < kRegion; o += 4096) {
        uint4 w[4];
        const int64_t n = o + 4096 < kRegion ? o + 4096 : o;
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_memcpy(&w[j], r + n - dist + 1024 * j, 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_memcpy(r + o + 1024 * j, &v[j], 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = w[j];
    }
}

// plain copy, each instruction 1 KiB contiguous, 8 rows (8 KiB) in flight per wave; region size rb
__global__ __launch_bounds__(64) void memcpy_deep(uint8_t* dst, int64_t rb) {
    uint8_t* r = dst + (int64_t)blockIdx.x * rb;
    const uint8_t* q = dst + (int64_t)(gridDim.x + blockIdx.x) * rb;
    const int l = threadIdx.x;
    for (int64_t o = 16 * l; o < rb; o += 8192) {
        uint4 a0, a1, a2, a3, b0, b1, b2, b3;
        __builtin_memcpy(&a0, q + o, 16); __builtin_memcpy(&a1, q + o + 1024, 16);
        __builtin_memcpy(&a2, q + o + 2048, 16); __builtin_memcpy(&a3, q + o + 3072, 16);
        __builtin_memcpy(&b0, q + o + 4096, 16); __builtin_memcpy(&b1, q + o + 5120, 16);
        __builtin_memcpy(&b2, q + o + 6144, 16); __builtin_memcpy(&b3, q + o + 7168, 16);
        __builtin_memcpy(r + o, &a0, 16); __builtin_memcpy(r + o + 1024, &a1, 16);
        __builtin_memcpy(r + o + 2048, &a2, 16); __builtin_memcpy(r + o + 3072, &a3, 16);
        __builtin_memcpy(r + o + 4096, &b0, 16); __builtin_memcpy(r + o + 5120, &b1, 16);
        __builtin_memcpy(r + o + 6144, &b2, 16); __builtin_memcpy(r + o + 7168, &b3, 16);
    }
}

int main() {
    const int nb = 4096;
    uint8_t* d;
    if (hipMalloc(&d, (size_t)nb * (kRegion + 64) + 64) != hipSuccess) return 1;
    hipMemset(d, 0, (size_t)nb * (kRegion + 64) + 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int mis[] = {0, 1};  // (for copies: m = the source distance)
    const char* names[] = {"rows  ", "runs  ", "copies", "c_pipe", "c_rows", "memcpy"};
    const int dists[] = {2048, 8192, 14000, 32768, 60000};
    for (int kind = 0; kind < 6; ++kind) {
        for (int mi = 0; mi < (kind < 2 ? 2 : kind == 5 ? 1 : 5); ++mi) {
            const int m = kind < 2 ? mis[mi] : dists[mi];
            float best = 1e9f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) rows<<<nb, 64>>>(d, m);
                else if (kind == 1) runs<<<nb, 64>>>(d, m);
                else if (kind == 2) copies<<<nb, 64>>>(d, 0, m);
                else if (kind == 3) copies_pipe<<<nb, 64>>>(d, 0, m);
                else if (kind == 4) copies_rows<<<nb, 64>>>(d, 0, m);
                else memcpy_runs<<<nb, 64>>>(d, 0, m);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("%s mis=%2d  %.3f ms  %.1f GB/s stored\n", names[kind], m,
                   best, (double)nb * kRegion / best / 1e6);
        }
    }
    // occupancy sweep of a plain 8 GiB copy: waves (one per region) x region size
    const int64_t total = (int64_t)8 << 30;
    for (int waves : {1024, 2048, 4096, 8192, 16384}) {
        const int64_t rb = total / waves;
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            memcpy_deep<<<waves, 64>>>(d, rb);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("memcpy_deep waves=%5d  %.3f ms  %.1f GB/s copied (x2 traffic)\n", waves, best, total / best / 1e6);
    }
    hipFree(d);
    return 0;
}
