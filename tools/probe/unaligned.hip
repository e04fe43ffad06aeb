// Probe: do unaligned 16/8/4-byte global and LDS accesses (as emitted for
// align-1 memcpy on gfx950) return/store the right bytes on the device?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t* a, uint8_t* g16, uint8_t* l16, uint8_t* nt16, uint8_t* g8) {
    __shared__ uint8_t L[2048];
    int t = threadIdx.x;
    for (int i = t; i < 2048; i += 64) L[i] = a[i];
    __syncthreads();
    int o = t * 17 + 3;
    uint4 v; __builtin_memcpy(&v, a + o, 16);
    __builtin_memcpy(g16 + t * 19 + 1, &v, 16);
    uint4 x; __builtin_memcpy(&x, L + o, 16);
    __builtin_memcpy(l16 + t * 16, &x, 16);
    u32x4 w = __builtin_nontemporal_load((const u32x4*)(a + o));
    __builtin_memcpy(nt16 + t * 16, &w, 16);
    uint2 y; __builtin_memcpy(&y, a + o + 5, 8);
    __builtin_memcpy(g8 + t * 11 + 3, &y, 8);
}
int main() {
    uint8_t h[4096]; for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 131 + 7);
    uint8_t *a, *b; hipMalloc(&a, 4096); hipMalloc(&b, 4 * 4096);
    hipMemcpy(a, h, 4096, hipMemcpyHostToDevice); hipMemset(b, 0, 4 * 4096);
    k<<<1, 64>>>(a, b, b + 4096, b + 8192, b + 12288);
    uint8_t r[4 * 4096]; hipMemcpy(r, b, sizeof r, hipMemcpyDeviceToHost);
    int bad[4] = {0, 0, 0, 0};
    for (int t = 0; t < 64; ++t) {
        int o = t * 17 + 3;
        for (int j = 0; j < 16; ++j) {
            if (t < 63 && r[t * 19 + 1 + j] != h[o + j]) bad[0]++;
            if (r[4096 + t * 16 + j] != h[o + j]) bad[1]++;
            if (r[8192 + t * 16 + j] != h[o + j]) bad[2]++;
        }
        for (int j = 0; j < 8; ++j) if (t < 63 && r[12288 + t * 11 + 3 + j] != h[o + 5 + j]) bad[3]++;
    }
    printf("unaligned probe: global16 %d lds16 %d nt16 %d global8 %d mismatches\n", bad[0], bad[1], bad[2], bad[3]);
    return bad[0] + bad[1] + bad[2] + bad[3] ? 1 : 0;
}
