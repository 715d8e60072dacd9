// mi355x_common.h -- device helpers shared by the gfx950 kernels (wave64, CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define MI_WAVE 64

// Quantized weight blocks exactly as stored by ggml (src/ggml-common.h:144-300). Kernels read
// them with aligned 16-byte loads where the block size allows (Q4_K 144 B, Q5_K 176 B).
struct mi_block_q4_0 { uint16_t d; uint8_t qs[16]; };
struct mi_block_q8_0 { uint16_t d; int8_t qs[32]; };
struct mi_block_q4_K { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; };
struct mi_block_q5_K { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; };
static_assert(sizeof(mi_block_q4_0) == 18, "q4_0");
static_assert(sizeof(mi_block_q8_0) == 34, "q8_0");
static_assert(sizeof(mi_block_q4_K) == 144, "q4_K");
static_assert(sizeof(mi_block_q5_K) == 176, "q5_K");

__device__ __forceinline__ float mi_h2f(uint16_t h) {
    _Float16 v;
    __builtin_memcpy(&v, &h, 2);
    return (float) v;
}

// f32 -> f16 round-to-nearest-even (v_cvt_f16_f32 in the default RNE mode) == F16C _cvtss_sh(x, 0)
__device__ __forceinline__ uint16_t mi_f2h(float f) {
    _Float16 v = (_Float16) f;
    uint16_t h;
    __builtin_memcpy(&h, &v, 2);
    return h;
}

__device__ __forceinline__ float mi_wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, MI_WAVE);
    return v;
}

__device__ __forceinline__ int mi_wave_sum_i(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, MI_WAVE);
    return v;
}

__device__ __forceinline__ float mi_wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, MI_WAVE));
    return v;
}

__device__ __forceinline__ int mi_dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// 6-bit scale / min j of the 12-byte K-quant scale array (src/ggml-quants.c:1357-1364),
// taking the array as three little-endian dwords.
__device__ __forceinline__ void mi_scale_min_k4(int j, uint32_t s0, uint32_t s1, uint32_t s2, int & sc, int & m) {
    auto byte = [&](int i) -> int {
        const uint32_t w = i < 4 ? s0 : (i < 8 ? s1 : s2);
        return (int) ((w >> (8 * (i & 3))) & 0xFF);
    };
    if (j < 4) {
        sc = byte(j) & 63;
        m = byte(j + 4) & 63;
    } else {
        sc = (byte(j + 4) & 0xF) | ((byte(j - 4) >> 6) << 4);
        m = (byte(j + 4) >> 4) | ((byte(j) >> 6) << 4);
    }
}
