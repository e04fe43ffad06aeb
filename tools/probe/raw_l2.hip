// Probe: are bytes a wave just stored served from the XCD's L2 when it reads
// them back (write-allocate), or fetched again from the fabric? Compare the
// FETCH_SIZE of the kernels (rocprofv3 --pmc FETCH_SIZE): 1024 waves x 16 KiB
// = 2 MiB per XCD, well inside the 4 MiB L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kBytes = 16384;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int STORE, int LOAD, int SHIFT>
__global__ __launch_bounds__(64) void wr_rd(uint8_t* buf, uint32_t* sink) {
    uint8_t* r = buf + (int64_t)blockIdx.x * (kBytes + 256);
    const int l = threadIdx.x;
    for (int o = 16 * l; o < kBytes; o += 1024) {
        u32x4 v = {(uint32_t)o, 1u, 2u, 3u};
        if (STORE == 0) *(u32x4*)(r + o) = v;
        else __builtin_nontemporal_store(v, (u32x4*)(r + o));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t acc = 0;
    for (int o = 16 * l + SHIFT; o + 16 <= kBytes; o += 1024) {
        u32x4 v;
        if (LOAD == 0) __builtin_memcpy(&v, r + o, 16);
        else v = __builtin_nontemporal_load((const u32x4*)(r + o));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int nb = 1024;
    uint8_t* d;
    uint32_t* sink;
    hipMalloc(&d, (size_t)nb * (kBytes + 256));
    hipMalloc(&sink, 4);
    for (int rep = 0; rep < 2; ++rep) {
        wr_rd<0, 0, 0><<<nb, 64>>>(d, sink);
        wr_rd<1, 0, 0><<<nb, 64>>>(d, sink);
        wr_rd<0, 1, 0><<<nb, 64>>>(d, sink);
        wr_rd<0, 0, 7><<<nb, 64>>>(d, sink);   // unaligned read-back
    }
    hipDeviceSynchronize();
    printf("done\n");
    hipFree(d);
    hipFree(sink);
    return 0;
}
