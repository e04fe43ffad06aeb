// lz4mi_common.h — shared device helpers for the gfx950 LZ4 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4mi {

constexpr int kWave = 64;

// Cross-lane steps on DPP (VALU operand modifiers, no LDS round trip): row_shr
// within rows of 16 lanes, then row_bcast:15 / row_bcast:31 across rows.
// `old` is what a lane without a source lane receives.
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, BANK_MASK, false);
}
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;
constexpr int kWaveShr1 = 0x138;   // lane l gets lane l - 1 (GFX9 wave_shr:1; lane 0 gets `old`)

// Wave-wide inclusive prefix sum (64 lanes).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    v += dpp<kRowShr1>(0u, v);
    v += dpp<kRowShr2>(0u, v);
    v += dpp<kRowShr4>(0u, v);
    v += dpp<kRowShr8>(0u, v);
    v += dpp<kRowBcast15, 0xa>(0u, v);
    v += dpp<kRowBcast31, 0xc>(0u, v);
    return v;
}

__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// Wave-wide minimum / maximum (uniform result).
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    const uint32_t F = 0xFFFFFFFFu;
    v = min(v, dpp<kRowShr1>(F, v));
    v = min(v, dpp<kRowShr2>(F, v));
    v = min(v, dpp<kRowShr4>(F, v));
    v = min(v, dpp<kRowShr8>(F, v));
    v = min(v, dpp<kRowBcast15, 0xa>(F, v));
    v = min(v, dpp<kRowBcast31, 0xc>(F, v));
    return lane63(v);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    v = max(v, dpp<kRowShr1>(0u, v));
    v = max(v, dpp<kRowShr2>(0u, v));
    v = max(v, dpp<kRowShr4>(0u, v));
    v = max(v, dpp<kRowShr8>(0u, v));
    v = max(v, dpp<kRowBcast15, 0xa>(0u, v));
    v = max(v, dpp<kRowBcast31, 0xc>(0u, v));
    return lane63(v);
}

// v of lane l (l uniform).
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return (uint64_t)uniform((uint32_t)v) | ((uint64_t)uniform((uint32_t)(v >> 32)) << 32);
}

// Bytes [sh, sh+4) of the little-endian pair (lo, hi), sh in 0..3.
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Wait until every outstanding vector-memory op of this wave has completed
// (stores acknowledged by L2). Also a compiler memory barrier.
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Reads of bytes this wave (or workgroup) wrote earlier in the launch are plain
// loads: the CU's L1 is coherent with the CU's own completed stores (the LLVM
// AMDGPU memory model needs no L1 invalidate for workgroup scope on gfx950), and
// every such read follows an s_waitcnt on the stores that wrote the bytes.

}  // namespace lz4mi
