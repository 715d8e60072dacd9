// quantize.hip -- activation quantizers for GGML_OP_MUL_MAT on gfx950.
//
// The reference CPU mul_mat converts every src1 column to the weight type's vec_dot_type
// before the dot products (src/ggml.c:11952-11974). Parity with it is bit-exact only if the
// GPU produces the same int8 quants and scales, so these kernels reproduce the reference x86
// build's exact rounding sequence:
//   Q8_0: AVX2 quantize_row_q8_0 (src/ggml-quants.c:535-618): amax, d = amax/127 -> fp16 RNE,
//         id = 127/amax, q = round-half-even(x*id)           (vmulps + vroundps)
//   Q8_K: quantize_row_q8_K_reference (src/ggml-quants.c:3370-3407) as gcc -mfma compiles it:
//         first max-|x| element (sign kept), iscale = -127/max, q = min(127, RNE(fma(iscale, x,
//         1.5*2^23)) via the bit trick), d = 1/iscale, sums of 16 (we keep sums of 32).
//   F16:  ggml_fp32_to_fp16_row (F16C, RNE)                     (src/ggml.c:365-382)
// All three are HBM-bound streaming kernels: one read of X (4 B/elem) and ~1.1 B/elem written.

#include "mi355x_common.h"
#include "mi355x_kernels.h"

// column c of src1 (c = blockIdx.x in every kernel here: wave-uniform scalar arithmetic, and no
// division at all for a plain 2-D src1)
static __device__ __forceinline__ const float * col_ptr(const mi_src_cols & x, uint32_t c) {
    if (x.ne2 == 1 && x.ne3 == 1) return (const float *) (x.base + (size_t) c * x.nb1);
    const uint32_t ne1 = (uint32_t) x.ne1, ne2 = (uint32_t) x.ne2;
    const uint32_t i1 = c % ne1, i2 = (c / ne1) % ne2, i3 = c / (ne1 * ne2);
    return (const float *) (x.base + (size_t) i1 * x.nb1 + (size_t) i2 * x.nb2 + (size_t) i3 * x.nb3);
}

// f16 GEMM operand layouts: row-major [ncols][K], or K-blocked [K/16][ncols][16] (nblk > 0 =
// ncols) so that the 32 columns x 16 halves of one MFMA K step are 1 KB of contiguous memory
static __device__ __forceinline__ int64_t xh_index(int64_t c, int64_t k, int64_t K, int64_t nblk) {
    return nblk ? ((k >> 4) * nblk + c) * 16 + (k & 15) : c * K + k;
}

size_t mi_act_q8_bytes(int64_t K, int64_t ncols, bool is_q8K) {
    const size_t qs = (size_t) (K * ncols + 255) & ~(size_t) 255;
    const size_t d = ((size_t) (K / (is_q8K ? 256 : 32)) * ncols * sizeof(float) + 255) & ~(size_t) 255;
    const size_t s = is_q8K ? (((size_t) (K / 32) * ncols * sizeof(int16_t) + 255) & ~(size_t) 255) : 0;
    return qs + d + s;
}

mi_act_q8 mi_act_q8_carve(void * base, int64_t K, int64_t ncols, bool is_q8K) {
    char * p = (char *) base;
    mi_act_q8 a;
    a.K = K;
    a.ncols = ncols;
    a.qs = (int8_t *) p;
    p += ((size_t) (K * ncols) + 255) & ~(size_t) 255;
    a.d = (float *) p;
    p += ((size_t) (K / (is_q8K ? 256 : 32)) * ncols * sizeof(float) + 255) & ~(size_t) 255;
    a.s32 = is_q8K ? (int16_t *) p : nullptr;
    return a;
}

// One 32-element block per half-wave, one element per lane; grid (column, group of 8 blocks).
// XH: write f16(d * q) to xh[c*K + k] (the batched-prompt GEMM's operand, mmq.hip) instead of the
// q8 blocks.
template <bool XH>
__global__ __launch_bounds__(256) void k_quantize_q8_0(mi_src_cols x, int64_t K, mi_act_q8 act, uint16_t * xh,
                                                       int64_t xh_blk = 0) {
    const int64_t nb_per_col = K / 32;
    const int64_t b = (int64_t) blockIdx.y * 8 + (threadIdx.x >> 5);
    const int l = threadIdx.x & 31;
    if (b >= nb_per_col) return;  // whole half-waves exit together
    const int64_t c = blockIdx.x;
    const float v = col_ptr(x, c)[b * 32 + l];
    float amax = fabsf(v);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 32));
    const float d = amax / 127.f;
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    const float q = __builtin_rintf(__fmul_rn(v, id));
    if constexpr (XH) {
        xh[xh_index(c, b * 32 + l, K, xh_blk)] = mi_f2h(mi_h2f(mi_f2h(d)) * (float) (int8_t) (int) q);
        return;
    }
    act.qs[c * K + b * 32 + l] = (int8_t) (int) q;
    if (l == 0) act.d[c * nb_per_col + b] = mi_h2f(mi_f2h(d));
}

// One 256-element superblock per wave, four consecutive elements per lane; grid (column, group of
// 4 superblocks) (XH as for q8_0).
template <bool XH>
__global__ __launch_bounds__(256) void k_quantize_q8_K(mi_src_cols x, int64_t K, mi_act_q8 act, uint16_t * xh,
                                                       int64_t xh_blk = 0) {
    const int wave = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t nb_per_col = K / 256;
    const int64_t b = (int64_t) blockIdx.y * 4 + wave;
    if (b >= nb_per_col) return;  // wave-uniform
    const int64_t c = blockIdx.x;
    const float4 v4 = *(const float4 *) (col_ptr(x, c) + b * 256 + lane * 4);
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};

    // first element with the largest |x| (strict '>' scan order), keep its signed value
    float amax = 0.0f, vmax = 0.0f;
    int idx = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float ax = fabsf(v[i]);
        if (ax > amax) { amax = ax; vmax = v[i]; idx = lane * 4 + i; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float oa = __shfl_xor(amax, off, 64);
        const float ov = __shfl_xor(vmax, off, 64);
        const int oi = __shfl_xor(idx, off, 64);
        if (oa > amax || (oa == amax && oi < idx)) { amax = oa; vmax = ov; idx = oi; }
    }
    if constexpr (XH) {
        uint2 o = make_uint2(0, 0);
        if (amax != 0.0f) {
            const float iscale = -127.f / vmax;
            const float d = 1.0f / iscale;
            uint32_t h[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int bits = __float_as_int(__builtin_fmaf(iscale, v[i], 12582912.f));
                int q = (bits & 0x007fffff) - 0x00400000;
                q = q < 127 ? q : 127;
                h[i] = mi_f2h(d * (float) (int8_t) q);
            }
            o = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        }
        *(uint2 *) (xh + xh_index(c, b * 256 + lane * 4, K, xh_blk)) = o;
        return;
    }
    int8_t * qs = act.qs + c * K + b * 256;
    int16_t * s32 = act.s32 + c * (K / 32) + b * 8;
    if (amax == 0.0f) {
        *(uint32_t *) (qs + lane * 4) = 0u;
        if ((lane & 7) == 0) s32[lane >> 3] = 0;
        if (lane == 0) act.d[c * nb_per_col + b] = 0.0f;
        return;
    }
    const float iscale = -127.f / vmax;
    uint32_t packed = 0;
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const float t = __builtin_fmaf(iscale, v[i], 12582912.f);
        const int bits = __float_as_int(t);
        int q = (bits & 0x007fffff) - 0x00400000;
        q = q < 127 ? q : 127;
        sum += q;
        packed |= ((uint32_t) (q & 0xFF)) << (8 * i);
    }
    *(uint32_t *) (qs + lane * 4) = packed;
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    if ((lane & 7) == 0) s32[lane >> 3] = (int16_t) sum;
    if (lane == 0) act.d[c * nb_per_col + b] = 1.0f / iscale;
}

// grid (column, group of 256 elements)
// f32 columns rounded to f16 (the CPU's from_float for vec_dot_type F16), or (SRC_F16) f16 columns
// copied as they are (src1 already of the vec_dot_type: the CPU reads it directly)
template <bool SRC_F16>
__global__ __launch_bounds__(256) void k_convert_f16(mi_src_cols x, int64_t K, uint16_t * out, int64_t xh_blk) {
    const int64_t k = (int64_t) blockIdx.y * 256 + threadIdx.x;
    if (k >= K) return;
    const int64_t c = blockIdx.x;
    if constexpr (SRC_F16) out[xh_index(c, k, K, xh_blk)] = ((const uint16_t *) col_ptr(x, (uint32_t) c))[k];
    else out[xh_index(c, k, K, xh_blk)] = mi_f2h(col_ptr(x, (uint32_t) c)[k]);
}

void mi_quantize_q8_0(const mi_src_cols & x, int64_t K, const mi_act_q8 & act, hipStream_t s) {
    if (act.ncols == 0 || K < 32) return;
    hipLaunchKernelGGL(k_quantize_q8_0<false>, dim3((unsigned) act.ncols, (unsigned) ((K / 32 + 7) / 8)), dim3(256), 0, s, x, K, act,
                       nullptr);
}

void mi_quantize_q8_K(const mi_src_cols & x, int64_t K, const mi_act_q8 & act, hipStream_t s) {
    if (act.ncols == 0 || K < 256) return;
    hipLaunchKernelGGL(k_quantize_q8_K<false>, dim3((unsigned) act.ncols, (unsigned) ((K / 256 + 3) / 4)), dim3(256), 0, s, x, K, act,
                       nullptr);
}

void mi_quantize_expand_f16(const mi_src_cols & x, int64_t K, int64_t ncols, bool is_q8K, uint16_t * xh, hipStream_t s,
                            bool blocked) {
    const int64_t xb = blocked ? ncols : 0;
    if (ncols == 0 || K < 32) return;
    if (is_q8K) {
        hipLaunchKernelGGL(k_quantize_q8_K<true>, dim3((unsigned) ncols, (unsigned) ((K / 256 + 3) / 4)), dim3(256), 0, s, x, K,
                           mi_act_q8{}, xh, xb);
    } else {
        hipLaunchKernelGGL(k_quantize_q8_0<true>, dim3((unsigned) ncols, (unsigned) ((K / 32 + 7) / 8)), dim3(256), 0, s, x, K,
                           mi_act_q8{}, xh, xb);
    }
}

void mi_convert_f16(const mi_src_cols & x, int64_t K, uint16_t * out, hipStream_t s, bool blocked, bool src_f16) {
    const int64_t ncols = x.ne1 * x.ne2 * x.ne3;
    const int64_t xb = blocked ? ncols : 0;
    if (ncols == 0 || K == 0) return;
    if (src_f16) hipLaunchKernelGGL(k_convert_f16<true>, dim3((unsigned) ncols, (unsigned) ((K + 255) / 256)), dim3(256), 0, s, x, K, out, xb);
    else hipLaunchKernelGGL(k_convert_f16<false>, dim3((unsigned) ncols, (unsigned) ((K + 255) / 256)), dim3(256), 0, s, x, K, out, xb);
}

// ---- src1 already of the vec_dot type (Q8_K / Q8_0 rows) -------------------------------------
// The reference CPU mul_mat reads such a src1 as it lies (ggml.c:11952: no conversion when
// src1->type == vec_dot_type); GGML_OP_CPY F32 -> Q8_K / Q8_0 writes it (ggml_compute_forward_dup
// -> from_float = quantize_row_q8_K / quantize_row_q8_0). Reference block layouts:
//   block_q8_K (292 B): float d | int8 qs[256] | int16 bsums[16] (sums of 16 quants)
//   block_q8_0 (34 B):  fp16 d  | int8 qs[32]
static __device__ __forceinline__ const char * col_base(const mi_src_cols & x, uint32_t c) {
    if (x.ne2 == 1 && x.ne3 == 1) return x.base + (size_t) c * x.nb1;
    const uint32_t ne1 = (uint32_t) x.ne1, ne2 = (uint32_t) x.ne2;
    const uint32_t i1 = c % ne1, i2 = (c / ne1) % ne2, i3 = c / (ne1 * ne2);
    return x.base + (size_t) i1 * x.nb1 + (size_t) i2 * x.nb2 + (size_t) i3 * x.nb3;
}

// CPY F32 -> Q8_K: one superblock per wave, grid (column, group of 4 superblocks); the rounding of
// k_quantize_q8_K (quantize_row_q8_K_reference, src/ggml-quants.c:3370-3407). An all-zero
// superblock gets d = 0, zero quants and zero bsums (the reference leaves its bsums untouched;
// every dot product multiplies them by d = 0).
// A16: the source columns are 16-byte aligned (base and nb1..nb3), so a lane reads its 4 values with
// one float4 load; otherwise (a view at an odd float offset) with four scalar loads.
template <bool A16>
__global__ __launch_bounds__(256) void k_quantize_rows_q8_K(mi_src_cols x, int64_t K, mi_src_cols dl) {
    const int wave = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t) blockIdx.y * 4 + wave;
    if (b >= K / 256) return;
    const uint32_t c = blockIdx.x;
    const float * src = (const float *) col_base(x, c) + b * 256 + lane * 4;
    float v[4];
    if constexpr (A16) {
        const float4 v4 = *(const float4 *) src;
        v[0] = v4.x, v[1] = v4.y, v[2] = v4.z, v[3] = v4.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = src[i];
    }
    uint32_t packed;
    int sum32;
    float d;
    mi_q8K_superblock(v, lane, packed, sum32, d);
    (void) sum32;
    char * blk = (char *) col_base(dl, c) + (size_t) b * 292;
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) s += (int) (int8_t) (packed >> (8 * i));
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);  // sum of the 16 quants of lanes 4j..4j+3
    *(uint32_t *) (blk + 4 + lane * 4) = packed;
    if ((lane & 3) == 0) *(int16_t *) (blk + 260 + 2 * (lane >> 2)) = (int16_t) s;
    if (lane == 0) *(float *) blk = d;
}

// CPY F32 -> Q8_0: one block per half-wave (k_quantize_q8_0's rounding, the AVX2 branch of
// quantize_row_q8_0, src/ggml-quants.c:535-618); grid (column, group of 8 blocks). Blocks are
// 2-byte aligned: the quants go out as bytes.
__global__ __launch_bounds__(256) void k_quantize_rows_q8_0(mi_src_cols x, int64_t K, mi_src_cols dl) {
    const int64_t b = (int64_t) blockIdx.y * 8 + (threadIdx.x >> 5);
    const int l = threadIdx.x & 31;
    if (b >= K / 32) return;
    const uint32_t c = blockIdx.x;
    const float v = ((const float *) col_base(x, c))[b * 32 + l];
    float amax = fabsf(v);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 32));
    const float d = amax / 127.f;
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    const float q = __builtin_rintf(__fmul_rn(v, id));
    char * blk = (char *) col_base(dl, c) + (size_t) b * 34;
    blk[2 + l] = (char) (int8_t) (int) q;
    if (l == 0) *(uint16_t *) blk = mi_f2h(d);
}

void mi_quantize_rows_q8(const mi_src_cols & x, int64_t K, bool is_q8K, const mi_src_cols & dst, hipStream_t s) {
    const int64_t ncols = x.ne1 * x.ne2 * x.ne3;
    if (ncols == 0) return;
    if (is_q8K) {
        const bool a16 = (((uintptr_t) x.base) | x.nb1 | x.nb2 | x.nb3) % 16 == 0;
        const dim3 grid((unsigned) ncols, (unsigned) ((K / 256 + 3) / 4));
        if (a16) hipLaunchKernelGGL(k_quantize_rows_q8_K<true>, grid, dim3(256), 0, s, x, K, dst);
        else hipLaunchKernelGGL(k_quantize_rows_q8_K<false>, grid, dim3(256), 0, s, x, K, dst);
    }
    else hipLaunchKernelGGL(k_quantize_rows_q8_0, dim3((unsigned) ncols, (unsigned) ((K / 32 + 7) / 8)), dim3(256), 0, s, x, K, dst);
}

// Q8_K rows -> the kernels' activation layouts. One superblock per wave (four quant bytes per lane),
// grid (column, group of 4 superblocks). MMX: the prefill GEMMs' [K/32][ncols][32] quants, d and the
// f16 halves of the sums of 32 (k_quantize_q8_K_mmx's layout); else the GEMV's q8 SoA (mi_act_q8).
// The sums of 32 are recomputed from the quants (equal to bsums[2j] + bsums[2j+1] whenever d != 0).
template <bool MMX>
__global__ __launch_bounds__(256) void k_q8K_rows_to_act(mi_src_cols xs, int64_t K, mi_act_q8 act, mi_act_mmx mx) {
    const int wave = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t) blockIdx.y * 4 + wave;
    if (b >= K / 256) return;
    const uint32_t c = blockIdx.x;
    const char * blk = col_base(xs, c) + (size_t) b * 292;
    const uint32_t packed = *(const uint32_t *) (blk + 4 + lane * 4);
    const float d = *(const float *) blk;
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) s += (int) (int8_t) (packed >> (8 * i));
    s = s + __shfl_xor(s, 1, 64);
    s = s + __shfl_xor(s, 2, 64);
    s = s + __shfl_xor(s, 4, 64);  // sum of the 32 quants of lanes 8j..8j+7
    if constexpr (MMX) {
        const int64_t ncols = mx.ncols;
        *(uint32_t *) (mx.xq + ((b * 8 + (lane >> 3)) * ncols + c) * 32 + (lane & 7) * 4) = packed;
        if ((lane & 7) == 0) {
            const uint32_t lo = mi_f2h((float) (s & 63)), hi = mi_f2h((float) (s >> 6));
            *(uint32_t *) (mx.xu + (b * ncols + c) * 16 + 2 * (lane >> 3)) = lo | (hi << 16);
        }
        if (lane == 0) mx.xd[b * ncols + c] = d;
    } else {
        *(uint32_t *) (act.qs + (int64_t) c * K + b * 256 + lane * 4) = packed;
        if ((lane & 7) == 0) act.s32[(int64_t) c * (K / 32) + b * 8 + (lane >> 3)] = (int16_t) s;
        if (lane == 0) act.d[(int64_t) c * (K / 256) + b] = d;
    }
}

// Q8_0 rows -> activation layouts: one block per half-wave, one quant per lane; d as f32
template <bool MMX>
__global__ __launch_bounds__(256) void k_q8_0_rows_to_act(mi_src_cols xs, int64_t K, mi_act_q8 act, mi_act_mmx mx) {
    const int64_t b = (int64_t) blockIdx.y * 8 + (threadIdx.x >> 5);
    const int l = threadIdx.x & 31;
    if (b >= K / 32) return;
    const uint32_t c = blockIdx.x;
    const char * blk = col_base(xs, c) + (size_t) b * 34;
    const int8_t q = (int8_t) blk[2 + l];
    const float d = mi_h2f(*(const uint16_t *) blk);
    if constexpr (MMX) {
        mx.xq[(b * mx.ncols + c) * 32 + l] = q;
        if (l == 0) mx.xd[b * mx.ncols + c] = d;
    } else {
        act.qs[(int64_t) c * K + b * 32 + l] = q;
        if (l == 0) act.d[(int64_t) c * (K / 32) + b] = d;
    }
}

void mi_q8_rows_to_act(const mi_src_cols & xs, int64_t K, bool is_q8K, const mi_act_q8 * act, const mi_act_mmx * mx, hipStream_t s) {
    const int64_t ncols = xs.ne1 * xs.ne2 * xs.ne3;
    if (ncols == 0) return;
    const mi_act_q8 a = act ? *act : mi_act_q8{};
    const mi_act_mmx m = mx ? *mx : mi_act_mmx{};
    if (is_q8K) {
        const dim3 grid((unsigned) ncols, (unsigned) ((K / 256 + 3) / 4));
        if (mx) hipLaunchKernelGGL(k_q8K_rows_to_act<true>, grid, dim3(256), 0, s, xs, K, a, m);
        else hipLaunchKernelGGL(k_q8K_rows_to_act<false>, grid, dim3(256), 0, s, xs, K, a, m);
    } else {
        const dim3 grid((unsigned) ncols, (unsigned) ((K / 32 + 7) / 8));
        if (mx) hipLaunchKernelGGL(k_q8_0_rows_to_act<true>, grid, dim3(256), 0, s, xs, K, a, m);
        else hipLaunchKernelGGL(k_q8_0_rows_to_act<false>, grid, dim3(256), 0, s, xs, K, a, m);
    }
}
