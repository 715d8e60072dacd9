// mi355x_common.h -- device helpers shared by the gfx950 kernels (wave64, CDNA4).
#pragma once

// diagnostic builds (make DIAG=1): timing-ablation and stamp kernels, whose results are invalid,
// become reachable through ggml_backend_mi355x_set_tuning; release builds compile them out
#ifndef MI_DIAG
#define MI_DIAG 0
#endif

#include <hip/hip_runtime.h>
#include <stdint.h>

#define MI_WAVE 64

// Phase stamp of a diagnostic build: s_memrealtime (the chip-wide 100 MHz counter) of lane 0 of
// the workgroup's first wave, written with a plain vector store into slot `slot` of the workgroup's
// 8-slot record in `buf` (a buffer of its own, never an output). Compiled out of release builds.
#if MI_DIAG
#define MI_STAMP(buf, slot)                                                                                                \
    do {                                                                                                                   \
        if ((buf) && threadIdx.x == 0)                                                                                     \
            (buf)[((size_t) blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
// the shader clock (s_memtime) at the same point: slot 6 at entry, 5 at exit give the clock the
// workgroup ran at (delta memtime / delta realtime x 100 MHz)
#define MI_STAMP_CLK(buf, slot)                                                                                            \
    do {                                                                                                                   \
        if ((buf) && threadIdx.x == 0)                                                                                     \
            (buf)[((size_t) blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] = __builtin_amdgcn_s_memtime();             \
    } while (0)
#else
#define MI_STAMP(buf, slot) \
    do {                    \
    } while (0)
#define MI_STAMP_CLK(buf, slot) \
    do {                        \
    } while (0)
#endif

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

// Workgroup barrier for LDS hand-offs that leaves global loads in flight: __syncthreads() carries
// a release/acquire fence, for which the compiler waits for every outstanding memory operation
// (vmcnt(0)) -- which drains a register prefetch ring at every barrier. This waits for this
// wave's LDS operations only, then s_barrier; the memory clobber keeps the compiler from moving
// memory accesses across it.
__device__ __forceinline__ void mi_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

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

// ---- DPP wave reductions (gfx9 family: quad_perm, row_half_mirror, row_mirror, row_bcast15/31).
// The total lands in lane 63 and is broadcast with v_readlane into an SGPR, so the result is
// wave-uniform. The whole wave must be active (call from wave-uniform control flow).
#define MI_DPP_QP_1032 0xB1
#define MI_DPP_QP_2301 0x4E
#define MI_DPP_ROW_HALF_MIRROR 0x141
#define MI_DPP_ROW_MIRROR 0x140
#define MI_DPP_ROW_BCAST15 0x142
#define MI_DPP_ROW_BCAST31 0x143

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int mi_dpp(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ double mi_dpp_f64(double v) {  // both halves moved by the same DPP pattern (0.0 where masked)
    const int lo = mi_dpp<CTRL, ROWMASK>(0, __double2loint(v));
    const int hi = mi_dpp<CTRL, ROWMASK>(0, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double mi_wave_sum_u_f64(double v) {  // uniform result (some order)
    v += mi_dpp_f64<MI_DPP_QP_1032>(v);
    v += mi_dpp_f64<MI_DPP_QP_2301>(v);
    v += mi_dpp_f64<MI_DPP_ROW_HALF_MIRROR>(v);
    v += mi_dpp_f64<MI_DPP_ROW_MIRROR>(v);
    v += mi_dpp_f64<MI_DPP_ROW_BCAST15, 0xA>(v);
    v += mi_dpp_f64<MI_DPP_ROW_BCAST31, 0xC>(v);
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63), __builtin_amdgcn_readlane(__double2loint(v), 63));
}

__device__ __forceinline__ float mi_wave_sum_u(float v) {  // uniform result
    auto f = [](int x) { return __int_as_float(x); };
    auto i = [](float x) { return __float_as_int(x); };
    v += f(mi_dpp<MI_DPP_QP_1032>(0, i(v)));
    v += f(mi_dpp<MI_DPP_QP_2301>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_MIRROR>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_BCAST15, 0xA>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_BCAST31, 0xC>(0, i(v)));
    return __int_as_float(__builtin_amdgcn_readlane(i(v), 63));
}

__device__ __forceinline__ uint32_t mi_wave_max_u32_u(uint32_t v) {  // uniform result
    auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_QP_1032>(0, (int) v));
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_QP_2301>(0, (int) v));
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, (int) v));
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_ROW_MIRROR>(0, (int) v));
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_ROW_BCAST15, 0xA>(0, (int) v));
    v = mx(v, (uint32_t) mi_dpp<MI_DPP_ROW_BCAST31, 0xC>(0, (int) v));
    return (uint32_t) __builtin_amdgcn_readlane((int) v, 63);
}

__device__ __forceinline__ uint32_t mi_wave_min_u32_u(uint32_t v) {  // uniform result
    auto mn = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
    constexpr int kId = -1;  // 0xFFFFFFFF: identity of unsigned min for lanes DPP leaves untouched
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_QP_1032>(kId, (int) v));
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_QP_2301>(kId, (int) v));
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(kId, (int) v));
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_ROW_MIRROR>(kId, (int) v));
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_ROW_BCAST15, 0xA>(kId, (int) v));
    v = mn(v, (uint32_t) mi_dpp<MI_DPP_ROW_BCAST31, 0xC>(kId, (int) v));
    return (uint32_t) __builtin_amdgcn_readlane((int) v, 63);
}

// sum over each aligned group of 8 lanes (every lane of the group gets it)
__device__ __forceinline__ int mi_sum8(int v) {
    v += mi_dpp<MI_DPP_QP_1032>(0, v);
    v += mi_dpp<MI_DPP_QP_2301>(0, v);
    v += mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, v);
    return v;
}

// Q8_K quantization of one 256-superblock held four consecutive floats per lane
// (quantize_row_q8_K_reference, src/ggml-quants.c:3370-3407, as the reference's gcc -mfma build
// computes it): the FIRST element of largest |x| keeps its sign, iscale = -127/max,
// q = min(127, RNE(fma(iscale, x, 1.5*2^23)) via the bit trick), d = 1/iscale.
// Writes 4 quants per lane (packed dword), the sums of 32 (one per 8-lane group) and d.
__device__ __forceinline__ void mi_q8K_superblock(const float (&v)[4], int lane, uint32_t & packed, int & sum32, float & d) {
    float best = 0.0f;
    int bidx = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float ax = fabsf(v[i]);
        if (ax > best) { best = ax; bidx = i; }  // first occurrence within the lane
    }
    const uint32_t amax_bits = mi_wave_max_u32_u(__float_as_uint(best));  // |x| >= 0: bit order = value order
    packed = 0;
    sum32 = 0;
    d = 0.0f;
    if (amax_bits == 0) return;  // wave-uniform
    const uint32_t my_idx = __float_as_uint(best) == amax_bits ? (uint32_t) (lane * 4 + bidx) : 0xFFFFFFFFu;
    const uint32_t idx = mi_wave_min_u32_u(my_idx);
    const int owner = (int) (idx >> 2), sel = (int) (idx & 3);
    const float mine = sel == 0 ? v[0] : sel == 1 ? v[1] : sel == 2 ? v[2] : v[3];
    const float vmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), owner));
    const float iscale = -127.f / vmax;
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float t = __builtin_fmaf(iscale, v[i], 12582912.f);
        int q = (__float_as_int(t) & 0x007fffff) - 0x00400000;
        q = q < 127 ? q : 127;
        s += q;
        packed |= ((uint32_t) (q & 0xFF)) << (8 * i);
    }
    sum32 = mi_sum8(s);
    d = 1.0f / iscale;
}

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
