// lz4mi_common.h — shared device helpers for the gfx950 LZ4 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4mi {

constexpr int kWave = 64;

// Wave-wide inclusive prefix sum (64 lanes, shuffle-up ladder).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_up(v, d, kWave);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t t = __shfl_xor(v, d, kWave);
        v = t < v ? t : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t t = __shfl_xor(v, d, kWave);
        v = t > v ? t : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Bytes [sh, sh+4) of the little-endian pair (lo, hi), sh in 0..3.
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Wait until every outstanding vector-memory op of this wave has completed
// (stores acknowledged by L2). Also a compiler memory barrier.
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Global loads that bypass the CU's L1 (served from L2): used for every read of
// bytes this wave itself wrote earlier, so a line cached before the write can
// never be observed stale.
__device__ __forceinline__ uint32_t ld_nt_u32(const uint32_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint8_t ld_nt_u8(const uint8_t* p) { return __builtin_nontemporal_load(p); }

}  // namespace lz4mi
