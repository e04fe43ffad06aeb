// Probe: which store cache policy (gfx950 sc0/sc1/nt bits) leaves just-stored
// bytes in the XCD's L2 so a read-back by the same wave hits there instead of
// being fetched from the fabric? Per-kernel FETCH_SIZE / TCC_HIT / TCC_MISS
// (rocprofv3 --pmc, one counter set per pass). 1024 waves x 16 KiB = 2 MiB
// per XCD, inside the 4 MiB L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kBytes = 16384;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int P>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
    if constexpr (P == 0) *(u32x4*)p = v;
    else if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
}

// P = store policy; R = 1: read the region twice without storing (L2 read reuse check);
// R = 2: store only
template <int P, int R>
__global__ __launch_bounds__(64) void l2pol(uint8_t* buf, uint32_t* sink) {
    uint8_t* r = buf + (int64_t)blockIdx.x * (kBytes + 256);
    const int l = threadIdx.x;
    uint32_t acc = 0;
    if (R == 1) {
        for (int o = 16 * l; o < kBytes; o += 1024) {
            const u32x4 v = *(const u32x4*)(r + o);
            acc += v.x;
        }
    } else {
        for (int o = 16 * l; o < kBytes; o += 1024) st16<P>(r + o, u32x4{(uint32_t)o, 1u, 2u, 3u});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (R == 2) return;   // store only: does a store fetch its line?
    for (int o = 16 * l + 7; o + 16 <= kBytes; o += 1024) {
        u32x4 v;
        __builtin_memcpy(&v, r + o, 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int nb = 1024;
    uint8_t* d;
    uint32_t* sink;
    hipMalloc(&d, (size_t)nb * (kBytes + 256) + (64 << 20));
    hipMalloc(&sink, 4);
    uint8_t* flush = d + (size_t)nb * (kBytes + 256);
    for (int rep = 0; rep < 2; ++rep) {
        l2pol<0, 0><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<1, 0><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<2, 0><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<3, 0><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<4, 0><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<0, 1><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<0, 2><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<3, 2><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
        l2pol<4, 2><<<nb, 64>>>(d, sink);
        hipMemsetAsync(flush, rep, 64 << 20);
    }
    hipDeviceSynchronize();
    printf("done\n");
    hipFree(d);
    hipFree(sink);
    return 0;
}
