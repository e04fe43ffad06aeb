// lz4mi_decompress_serial.hip — the reference-exact serial decoder (gfx950).
//
// LZ4MI_JS_COMPAT decodes blocks in order on one lane with the reference's
// exact byte order (src/block/blockDecompress.js:30-275), including the
// double-copy-tail rewrite for offset >= 8, length < 8 matches
// (blockDecompress.js:219-250), which may touch up to 7 bytes
// before a block's start — the reason blocks run in order, as the reference's
// frame loop (src/buffer/bufferDecompress.js:133-192) runs them.
#include "lz4mi_common.h"
#include "lz4mi_decompress.h"

namespace lz4mi {

__device__ void decode_block_jscompat(const DecArgs& a, uint32_t b) {
    const uint8_t* in = a.in + a.in_off[b];
    const int64_t iend = a.in_len[b];
    uint8_t* out = a.out;                       // absolute positions
    const int64_t oo = (int64_t)a.out_off[b];
    const int64_t olen = oo + a.out_cap[b];     // the reference's output.length
    const int64_t dlen = a.dict ? a.dict_len : 0;
    int64_t ip = 0, op = oo;
    int32_t st = 0;
    auto inb = [&](int64_t i) -> uint32_t { return (i >= 0 && i < iend) ? in[i] : 0u; };
    while (ip < iend) {
        uint32_t tok = inb(ip++);
        int64_t lit = tok >> 4;
        if (lit == 15) { uint32_t x; do { x = inb(ip++); lit += x; } while (x == 255); }
        if (op + lit > olen) { st = -1; break; }
        if (ip + lit > iend) { st = -2; break; }
        for (int64_t k = 0; k < lit; ++k) out[op + k] = (uint8_t)inb(ip + k);
        op += lit; ip += lit;
        if (ip >= iend) break;
        uint32_t off = inb(ip) | (inb(ip + 1) << 8);
        ip += 2;
        if (off == 0) { st = -3; break; }
        int64_t ml = tok & 15;
        if (ml == 15) { uint32_t x; do { x = inb(ip++); ml += x; } while (x == 255); }
        ml += 4;
        int64_t from = op - off;
        if (from < 0) {
            int64_t nd = -from < ml ? -from : ml;
            int64_t di = dlen + from;
            if (di < 0 || di + nd > dlen) { st = -4; break; }
            for (int64_t k = 0; k < nd; ++k) { if (op < olen) out[op] = a.dict[di + k]; ++op; }
            int64_t rp = op - off;
            for (int64_t k = nd; k < ml; ++k) {
                uint8_t v = (rp >= 0 && rp < olen) ? out[rp] : 0;
                if (op < olen) out[op] = v;
                ++op; ++rp;
            }
            continue;
        }
        int64_t start = op;
        for (int64_t k = 0; k < ml; ++k) {
            int64_t r = op - off;
            uint8_t v = r < olen ? out[r] : 0;
            if (op < olen) out[op] = v;
            ++op;
        }
        if (off >= 8 && ml < 8) {
            for (int64_t p = start + ml - 8; p < start; ++p) {
                int64_t r = p - off;
                uint8_t v = (r >= 0 && r < olen) ? out[r] : 0;
                if (p >= 0 && p < olen) out[p] = v;
            }
        }
    }
    a.status[b] = st;
    a.out_len[b] = st ? 0u : (uint32_t)(op - oo);
}

__global__ __launch_bounds__(64) void lz4mi_decompress_jscompat_kernel(DecArgs a) {
    if (threadIdx.x != 0) return;
    for (uint32_t b = 0; b < a.nblocks; ++b) decode_block_jscompat(a, b);
}


}  // namespace lz4mi

extern "C" hipError_t lz4mi_launch_decompress_serial(const lz4mi::DecArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(lz4mi::lz4mi_decompress_jscompat_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}
