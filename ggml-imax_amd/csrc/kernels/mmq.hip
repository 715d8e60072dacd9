// mmq.hip -- batched GGML_OP_MUL_MAT (prompt / prefill regime, many activation columns) on the
// gfx950 matrix cores.
//
// Per workgroup (256 threads = 4 wave64s) a 64 (weight rows n) x 64 (activation columns b)
// output tile; per 256-deep K step:
//   * weights: the 64 rows' blocks are dequantized into LDS as f16 with the reference's
//     dequantize_row_* arithmetic (src/ggml-quants.c:980-998 q4_0, :1074-1088 q8_0,
//     :2181-2218 q4_K, :2464-2507 q5_K; F16 weights are copied as is);
//   * activations: columns already quantized bit-exactly like the CPU path (quantize.hip), staged
//     as f16(d * q) -- for F16 weights the f16-rounded activations of ggml_fp32_to_fp16_row;
//   * each wave runs v_mfma_f32_32x32x16_f16 over its 32x32 sub-tile (f32 accumulation).
// Relative to the CPU path the only extra rounding is the f16 representation of the two
// operands (<= 2^-11 each); the activation quantization itself is identical.
// Rooflines: AI = 2*N*K*B / (weight bytes + 4*K*B + 4*N*B), ~650 flop/B at B=512 -> MFMA-bound
// (f16 dense ~2.5 PF/s).

#include "mi355x_common.h"
#include "mi355x_kernels.h"

namespace {

constexpr int BM = 64;          // weight rows per tile
constexpr int BN = 64;          // activation columns per tile
constexpr int BK = 256;         // K per LDS stage
constexpr int LDA = BK + 8;     // padded f16 row stride (528 B: conflict-free ds_read_b128)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t pack2h(float a, float b) {
    return (uint32_t) mi_f2h(a) | ((uint32_t) mi_f2h(b) << 16);
}

// write 8 f16 (given as f32) to LDS
__device__ __forceinline__ void st8(_Float16 * p, const float (&v)[8]) {
    uint4 u;
    u.x = pack2h(v[0], v[1]);
    u.y = pack2h(v[2], v[3]);
    u.z = pack2h(v[4], v[5]);
    u.w = pack2h(v[6], v[7]);
    *(uint4 *) p = u;
}

// Dequantize 64 consecutive weights (quarter q of the 256-element K step starting at k0) of one
// row into LDS. `row` points at the row start.
template <int TYPE>
__device__ __forceinline__ void dequant64(const uint8_t * row, int64_t k0, int q, _Float16 * out) {
    if constexpr (TYPE == 12 || TYPE == 13) {
        constexpr bool Q5 = TYPE == 13;
        const uint8_t * blk = row + (k0 / 256) * (Q5 ? 176 : 144);
        const uint4 hdr = *(const uint4 *) blk;
        const float d = mi_h2f((uint16_t) (hdr.x & 0xFFFF));
        const float dmin = mi_h2f((uint16_t) (hdr.x >> 16));
        int sc0, m0, sc1, m1;
        mi_scale_min_k4(2 * q, hdr.y, hdr.z, hdr.w, sc0, m0);
        mi_scale_min_k4(2 * q + 1, hdr.y, hdr.z, hdr.w, sc1, m1);
        const float d1 = d * sc0, mm1 = dmin * m0, d2 = d * sc1, mm2 = dmin * m1;
        const uint8_t * qs = blk + (Q5 ? 48 : 16) + 32 * q;
        uint32_t qw[8], hw[8];
        const uint4 a = *(const uint4 *) qs, b = *(const uint4 *) (qs + 16);
        qw[0] = a.x; qw[1] = a.y; qw[2] = a.z; qw[3] = a.w; qw[4] = b.x; qw[5] = b.y; qw[6] = b.z; qw[7] = b.w;
        if constexpr (Q5) {
            const uint4 ha = *(const uint4 *) (blk + 16), hb = *(const uint4 *) (blk + 32);
            hw[0] = ha.x; hw[1] = ha.y; hw[2] = ha.z; hw[3] = ha.w; hw[4] = hb.x; hw[5] = hb.y; hw[6] = hb.z; hw[7] = hb.w;
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {  // 8 bytes -> elements l = 8g..8g+7 (low) and 32+l (high)
            float lo[8], hi[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int l = 8 * g + e;
                const uint32_t byte = (qw[l >> 2] >> (8 * (l & 3))) & 0xFF;
                int vl = byte & 0xF, vh = byte >> 4;
                if constexpr (Q5) {
                    const uint32_t hb8 = (hw[l >> 2] >> (8 * (l & 3))) & 0xFF;
                    vl += (hb8 >> (2 * q)) & 1 ? 16 : 0;
                    vh += (hb8 >> (2 * q + 1)) & 1 ? 16 : 0;
                }
                lo[e] = d1 * (float) vl - mm1;
                hi[e] = d2 * (float) vh - mm2;
            }
            st8(out + 8 * g, lo);
            st8(out + 32 + 8 * g, hi);
        }
    } else if constexpr (TYPE == 2 || TYPE == 8) {
        constexpr bool Q8 = TYPE == 8;
        constexpr int BS = Q8 ? 34 : 18;
#pragma unroll
        for (int bi = 0; bi < 2; bi++) {  // two 32-blocks per quarter
            const uint8_t * blk = row + ((k0 + 64 * q) / 32 + bi) * BS;
            const float d = mi_h2f((uint16_t) (blk[0] | (blk[1] << 8)));
            float v[32];
            if constexpr (Q8) {
#pragma unroll
                for (int e = 0; e < 32; e++) v[e] = (float) (int8_t) blk[2 + e] * d;
            } else {
#pragma unroll
                for (int e = 0; e < 16; e++) {
                    const int byte = blk[2 + e];
                    v[e] = (float) ((byte & 0xF) - 8) * d;
                    v[e + 16] = (float) ((byte >> 4) - 8) * d;
                }
            }
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const float (&vv)[8] = *(const float (*)[8]) (v + 8 * g);
                st8(out + 32 * bi + 8 * g, vv);
            }
        }
    } else {  // F16
        const uint4 * src = (const uint4 *) (row + (k0 + 64 * q) * 2);
#pragma unroll
        for (int g = 0; g < 8; g++) *(uint4 *) (out + 8 * g) = src[g];
    }
}

template <int TYPE>
__global__ __launch_bounds__(256) void k_mmq_f16(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                 mi_act_q8 act, const uint16_t * __restrict__ xh, int64_t ncols,
                                                 float * __restrict__ dst, size_t ycol) {
    __shared__ __attribute__((aligned(16))) _Float16 lw[BM * LDA];
    __shared__ __attribute__((aligned(16))) _Float16 lx[BN * LDA];
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t n0 = (int64_t) blockIdx.x * BM;
    const int64_t b0 = (int64_t) blockIdx.y * BN;
    const int wm = wave & 1, wb = wave >> 1;
    float16v acc = {};

    // staging roles: thread t -> row/column t/4, quarter t%4 (64 elements)
    const int sr = tid >> 2, sq = tid & 3;
    const int64_t wrow = n0 + sr, xcol = b0 + sr;
    constexpr bool QK = TYPE == 12 || TYPE == 13;

    for (int64_t k0 = 0; k0 < K; k0 += BK) {
        // weights -> f16 LDS
        if (wrow < N) {
            dequant64<TYPE>(W + wrow * nb01, k0, sq, lw + sr * LDA + 64 * sq);
        } else {
#pragma unroll
            for (int g = 0; g < 8; g++) *(uint4 *) (lw + sr * LDA + 64 * sq + 8 * g) = make_uint4(0, 0, 0, 0);
        }
        // activations -> f16 LDS
        _Float16 * xo = lx + sr * LDA + 64 * sq;
        if (xcol < ncols) {
            if constexpr (TYPE == 1) {
                const uint4 * src = (const uint4 *) (xh + xcol * K + k0 + 64 * sq);
#pragma unroll
                for (int g = 0; g < 8; g++) *(uint4 *) (xo + 8 * g) = src[g];
            } else {
                const int8_t * qs = act.qs + xcol * K + k0 + 64 * sq;
                const int4 * q4 = (const int4 *) qs;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int4 w = q4[g];
                    const int ww[4] = {w.x, w.y, w.z, w.w};
                    // the 16 quants of this group share one scale (32-block or 256-superblock)
                    const float d = QK ? act.d[xcol * (K / 256) + k0 / 256]
                                       : act.d[xcol * (K / 32) + (k0 + 64 * sq + 16 * g) / 32];
                    float v[16];
#pragma unroll
                    for (int e = 0; e < 16; e++) v[e] = d * (float) (int8_t) (ww[e >> 2] >> (8 * (e & 3)));
                    st8(xo + 16 * g, *(const float (*)[8]) v);
                    st8(xo + 16 * g + 8, *(const float (*)[8]) (v + 8));
                }
            }
        } else {
#pragma unroll
            for (int g = 0; g < 8; g++) *(uint4 *) (xo + 8 * g) = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();

        // 32x32 sub-tile per wave: A = weights (rows n), B = activations (columns b)
        const int r = lane & 31, h = lane >> 5;
        const _Float16 * pa = lw + (wm * 32 + r) * LDA + 8 * h;
        const _Float16 * pb = lx + (wb * 32 + r) * LDA + 8 * h;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 16) {
            const half8 a = *(const half8 *) (pa + kk);
            const half8 b = *(const half8 *) (pb + kk);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }

    // D[n][b]: column b = lane & 31, rows n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    const int64_t b = b0 + wb * 32 + (lane & 31);
    if (b < ncols) {
        float * out = (float *) ((char *) dst + b * ycol);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int64_t n = n0 + wm * 32 + 8 * g + 4 * (lane >> 5);
            if (n + 3 < N) {
                *(float4 *) (out + n) = make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = acc[4 * g + e];
            }
        }
    }
}

} // namespace

bool mi_mmq_supported(int type, int64_t K, size_t nb01, size_t ycol) {
    if (type != 12 && type != 13 && type != 2 && type != 8 && type != 1) return false;
    if (K % BK != 0) return false;
    if (type == 1 && nb01 % 16 != 0) return false;
    return ycol % 16 == 0;
}

void mi_mul_mat_mmq(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_q8 & act, const uint16_t * xh,
                    int64_t ncols, float * dst, size_t ycol, hipStream_t s) {
    const dim3 grid((unsigned) ((N + BM - 1) / BM), (unsigned) ((ncols + BN - 1) / BN));
    const uint8_t * w = (const uint8_t *) W;
    switch (type) {
        case 12: hipLaunchKernelGGL(k_mmq_f16<12>, grid, dim3(256), 0, s, w, nb01, K, N, act, xh, ncols, dst, ycol); break;
        case 13: hipLaunchKernelGGL(k_mmq_f16<13>, grid, dim3(256), 0, s, w, nb01, K, N, act, xh, ncols, dst, ycol); break;
        case 2: hipLaunchKernelGGL(k_mmq_f16<2>, grid, dim3(256), 0, s, w, nb01, K, N, act, xh, ncols, dst, ycol); break;
        case 8: hipLaunchKernelGGL(k_mmq_f16<8>, grid, dim3(256), 0, s, w, nb01, K, N, act, xh, ncols, dst, ycol); break;
        case 1: hipLaunchKernelGGL(k_mmq_f16<1>, grid, dim3(256), 0, s, w, nb01, K, N, act, xh, ncols, dst, ycol); break;
        default: break;
    }
}
