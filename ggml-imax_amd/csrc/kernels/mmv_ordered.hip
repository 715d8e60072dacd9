// mmv_ordered.hip -- F16 x F16 and F32 x F32 mul_mat whose every output is BIT-IDENTICAL to the
// reference CPU's ggml_vec_dot_f16 / ggml_vec_dot_f32 (src/ggml.c:1674-1714, :1567-1608) as the
// reference's x86 build (-mavx -mavx2 -mfma -mf16c, oracle/Makefile) executes them:
//
//   main loop   4 registers x 8 lanes = 32 partial sums; element i + 8r + l goes to sum[r][l]
//               through a fused multiply-add (_mm256_fmadd_ps), in order of i
//   reduce      GGML_F32x8_REDUCE (src/ggml.c:1172-1190): s0+=s2, s1+=s3, s0+=s1, then
//               lanes (k + k+4), then (t0+t1) + (t2+t3)
//   leftovers   K % 32 trailing elements, added in order:
//                 f16: double sum of exact f32 products (src/ggml.c:1704-1707)
//                 f32: float sum; gcc vectorises the loop, so elements in whole 8- and then
//                      4-element chunks are multiplied then added (two roundings) and the last
//                      <= 3 elements are fused (vfmadd231ss) -- read off the built object
//
// On the GPU a quad of lanes plays the 4 AVX registers: lane q of the quad keeps the 8 lane sums
// of register q, loading 16 B (f16) or 32 B (f32) per step, so one wave64 serves 16 dot products.
// These kernels carry GPT-2's f16 projections in decode (few columns) and the attention's KQ and
// KQV products, so GPT-2 logits follow the CPU bit for bit through every dot product.

#include <algorithm>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#include "cpu_order.h"

namespace {

constexpr int kQuadsPerBlock = 64;  // 256 threads

__device__ __forceinline__ float quad_reduce_avx(float (&v)[8]) {
    // sum[0] + sum[2], sum[1] + sum[3] (lane q gets q^2), then (s0+s2) + (s1+s3) (lane q^1)
#pragma unroll
    for (int l = 0; l < 8; l++) v[l] = add_rn(v[l], __shfl_xor(v[l], 2, 64));
#pragma unroll
    for (int l = 0; l < 8; l++) v[l] = add_rn(v[l], __shfl_xor(v[l], 1, 64));
    const float t0 = add_rn(v[0], v[4]), t1 = add_rn(v[1], v[5]);
    const float t2 = add_rn(v[2], v[6]), t3 = add_rn(v[3], v[7]);
    return add_rn(add_rn(t0, t1), add_rn(t2, t3));
}

__device__ __forceinline__ void h8_to_f(const uint4 & h, float (&f)[8]) {
    const uint32_t w[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        f[2 * i] = mi_h2f((uint16_t) (w[i] & 0xffffu));
        f[2 * i + 1] = mi_h2f((uint16_t) (w[i] >> 16));
    }
}

struct ord_geom {
    int64_t K, N;
    int64_t ne11, ne12, ne13;
    int64_t r2, r3;
    size_t nb01, nb02, nb03;
    size_t nb1, nb2, nb3;
    int64_t col_chunks;
};

// 8 halves at p: one 16-byte load, or (ALIGNED false: rows of K % 8 != 0 halves, or a weight row
// stride / base that is not a 16-byte multiple) eight 2-byte loads
template <bool ALIGNED>
__device__ __forceinline__ void ld_h8(const uint16_t * p, float (&f)[8]) {
    if constexpr (ALIGNED) {
        h8_to_f(*(const uint4 *) p, f);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) f[i] = mi_h2f(p[i]);
    }
}

// F16 weights x f16 activation columns (xh: [ncols][K], the CPU's from_float rows).
// One quad per (row, chunk of NC columns).
template <int NC, bool ALIGNED>
__global__ __launch_bounds__(256) void k_mmv_f16_ord(const uint8_t * __restrict__ W, const uint16_t * __restrict__ xh,
                                                     float * __restrict__ dst, ord_geom g) {
    const int q = threadIdx.x & 3;
    const int64_t row = (int64_t) blockIdx.x * kQuadsPerBlock + (threadIdx.x >> 2);
    const bool live = row < g.N;
    const int64_t y = blockIdx.y;
    const int64_t chunk = y % g.col_chunks;
    const int64_t z = y / g.col_chunks;
    const int64_t i12 = z % g.ne12, i13 = z / g.ne12;
    const int64_t i11 = chunk * NC;
    const int64_t i02 = i12 / g.r2, i03 = i13 / g.r3;
    const uint16_t * wrow = (const uint16_t *) (W + i02 * g.nb02 + i03 * g.nb03 + (live ? row : 0) * g.nb01);
    const int64_t col0 = i11 + g.ne11 * (i12 + g.ne12 * i13);
    int nc = (int) (g.ne11 - i11);
    nc = nc > NC ? NC : nc;

    float acc[NC][8];
#pragma unroll
    for (int c = 0; c < NC; c++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[c][l] = 0.0f;

    const int64_t np = g.K & ~(int64_t) 31;
    for (int64_t i = 8 * q; i < np; i += 32) {
        float w[8];
        ld_h8<ALIGNED>(wrow + i, w);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (c < nc) {
                float x[8];
                ld_h8<ALIGNED>(xh + (col0 + c) * g.K + i, x);
#pragma unroll
                for (int l = 0; l < 8; l++) acc[c][l] = __fmaf_rn(w[l], x[l], acc[c][l]);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float r = quad_reduce_avx(acc[c]);
        if (q == 0 && live && c < nc) {
            double s = (double) r;
            for (int64_t i = np; i < g.K; i++) {
                s += (double) mul_rn(mi_h2f(wrow[i]), mi_h2f(xh[(col0 + c) * g.K + i]));
            }
            *(float *) ((char *) dst + (i11 + c) * g.nb1 + i12 * g.nb2 + i13 * g.nb3 + row * sizeof(float)) = (float) s;
        }
    }
}

// F32 x F32, both operands strided (KQ = K^T Q and KQV = V^T softmax of the attention).
// One quad per output element.
__global__ __launch_bounds__(256) void k_mm_f32_ord(const uint8_t * __restrict__ W, mi_src_cols x, float * __restrict__ dst,
                                                    ord_geom g) {
    const int q = threadIdx.x & 3;
    const int64_t row = (int64_t) blockIdx.x * kQuadsPerBlock + (threadIdx.x >> 2);
    const bool live = row < g.N;
    const int64_t y = blockIdx.y;
    const int64_t i11 = y % g.ne11;
    const int64_t z = y / g.ne11;
    const int64_t i12 = z % g.ne12, i13 = z / g.ne12;
    const int64_t i02 = i12 / g.r2, i03 = i13 / g.r3;
    const float * w = (const float *) (W + i02 * g.nb02 + i03 * g.nb03 + (live ? row : 0) * g.nb01);
    const float * xc = (const float *) (x.base + i11 * x.nb1 + i12 * x.nb2 + i13 * x.nb3);

    float acc[8];
#pragma unroll
    for (int l = 0; l < 8; l++) acc[l] = 0.0f;
    const int64_t np = g.K & ~(int64_t) 31;
    for (int64_t i = 8 * q; i < np; i += 32) {
        float wv[8], xv[8];
        // rows of KQ/KQV operands are 4-byte aligned only: scalar loads, contiguous per lane
#pragma unroll
        for (int l = 0; l < 8; l++) {
            wv[l] = w[i + l];
            xv[l] = xc[i + l];
        }
#pragma unroll
        for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(wv[l], xv[l], acc[l]);
    }
    float s = quad_reduce_avx(acc);
    if (q == 0 && live) {
        const int64_t L = g.K - np;
        const int64_t fused_from = (L >= 8 ? (L / 8) * 8 : 0) + (((L >= 8 ? L % 8 : L) >= 4) ? 4 : 0);
        for (int64_t j = 0; j < L; j++) {
            const float a = w[np + j], b = xc[np + j];
            s = j < fused_from ? add_rn(s, mul_rn(a, b)) : __fmaf_rn(a, b, s);
        }
        *(float *) ((char *) dst + i11 * g.nb1 + i12 * g.nb2 + i13 * g.nb3 + row * sizeof(float)) = s;
    }
}

// Stage NC f32 activation columns as f16 in LDS (RNE, as the CPU's ggml_fp32_to_fp16_row,
// src/ggml.c:610-612), optionally through the graph's preceding norm -> mul(g) -> add(b) chain
// (pro), or copy already-converted f16 columns (xh). Ends without a barrier.
template <int NC>
__device__ __forceinline__ void stage_f16_activations(uint16_t * xs, double * shd, int64_t K, int64_t i11, int nc,
                                                      const mi_src_cols & x, const uint16_t * __restrict__ xh,
                                                      const mi_norm_prologue & pro) {
    // stage the activations: 16-byte loads, unrolled so each lane has its loads in flight at once
    constexpr int kJ = 12;  // register path: K <= 64 * kJ
    if (pro.mode && K <= 64 * kJ) {
        // the graph's norm|rms_norm -> mul(g) -> add(b), per column, held in registers by wave 0
        // (no LDS round trips); the other waves wait at the caller's barrier with their weight
        // loads in flight
        const int lane = threadIdx.x & 63;
        if ((threadIdx.x >> 6) != 0) return;
        for (int c = 0; c < nc; c++) {
            const float * xc = (const float *) (x.base + (i11 + c) * x.nb1);
            // unconditional loads at clamped indices + selects (no per-load waits at branch joins)
            const float * gp = pro.g ? pro.g : xc;
            const float * bp = pro.b ? pro.b : xc;
            float v[kJ], gv[kJ], bv[kJ];
#pragma unroll
            for (int j = 0; j < kJ; j++) {
                const int64_t k = (int64_t) j * 64 + lane;
                const bool in = k < K;
                const int64_t kc = in ? k : K - 1;
                const float xv = xc[kc], gl = gp[kc], bl = bp[kc];
                v[j] = in ? xv : 0.0f;
                gv[j] = in && pro.g ? gl : 1.0f;
                bv[j] = in && pro.b ? bl : 0.0f;
            }
            float scale;
            if (pro.mode == 2) {
                const float mean = wave_mean_cpu_order<true, kJ>(v, K);
                scale = 1.0f / sqrtf(add_rn(mean, pro.eps));
            } else {
                const float mean = wave_mean_cpu_order<false, kJ>(v, K);
#pragma unroll
                for (int j = 0; j < kJ; j++) v[j] = sub_rn(v[j], mean);
                const float variance = wave_mean_cpu_order<true, kJ>(v, K);
                scale = 1.0f / sqrtf(add_rn(variance, pro.eps));
            }
#pragma unroll
            for (int j = 0; j < kJ; j++) {
                const int64_t k = (int64_t) j * 64 + lane;
                if (k < K) {
                    float y = mul_rn(v[j], scale);
                    if (pro.g) y = mul_rn(y, gv[j]);
                    if (pro.b) y = add_rn(y, bv[j]);
                    xs[c * K + k] = mi_f2h(y);
                }
            }
        }
    } else if (pro.mode) {
        // the graph's norm|rms_norm -> mul(g) -> add(b) producing this mul_mat's src1, computed per
        // column exactly as k_norm does (ops.hip), then rounded to f16 as the CPU's from_float
        float * xf = (float *) (xs + NC * K);
        for (int c = 0; c < nc; c++) {
            const float * xc = (const float *) (x.base + (i11 + c) * x.nb1);
#pragma unroll 4
            for (int64_t k = threadIdx.x; k < K; k += blockDim.x) xf[k] = xc[k];
            __syncthreads();
            float scale;
            if (pro.mode == 2) {
                const float mean = row_mean_cpu_order<true>(xf, K, shd);
                scale = 1.0f / sqrtf(add_rn(mean, pro.eps));
            } else {
                const float mean = row_mean_cpu_order<false>(xf, K, shd);
                for (int64_t k = threadIdx.x; k < K; k += blockDim.x) xf[k] = sub_rn(xf[k], mean);
                __syncthreads();
                const float variance = row_mean_cpu_order<true>(xf, K, shd);
                scale = 1.0f / sqrtf(add_rn(variance, pro.eps));
            }
            for (int64_t k = threadIdx.x; k < K; k += blockDim.x) {
                float v = mul_rn(xf[k], scale);
                if (pro.g) v = mul_rn(v, pro.g[k]);
                if (pro.b) v = add_rn(v, pro.b[k]);
                xs[c * K + k] = mi_f2h(v);
            }
            __syncthreads();
        }
    } else if (xh) {
        // already converted (f16 [ncols][K] in scratch)
        for (int c = 0; c < nc; c++) {
            const uint4 * src = (const uint4 *) (xh + (i11 + c) * K);
            uint4 * xd = (uint4 *) (xs + c * K);
#pragma unroll 4
            for (int64_t k = threadIdx.x; k < (K >> 3); k += blockDim.x) xd[k] = src[k];
        }
    } else if ((x.nb1 % 16) == 0 && ((uintptr_t) x.base % 16) == 0) {
        const int64_t K4 = K >> 2;  // K % 8 == 0
        for (int c = 0; c < nc; c++) {
            const float4 * xc = (const float4 *) (x.base + (i11 + c) * x.nb1);
            uint2 * xd = (uint2 *) (xs + c * K);
#pragma unroll 8
            for (int64_t k = threadIdx.x; k < K4; k += blockDim.x) {
                const float4 v = xc[k];
                xd[k] = make_uint2((uint32_t) mi_f2h(v.x) | ((uint32_t) mi_f2h(v.y) << 16),
                                   (uint32_t) mi_f2h(v.z) | ((uint32_t) mi_f2h(v.w) << 16));
            }
        }
    } else {
        for (int c = 0; c < nc; c++) {
            const float * xc = (const float *) (x.base + (i11 + c) * x.nb1);
#pragma unroll 8
            for (int64_t k = threadIdx.x; k < K; k += blockDim.x) xs[c * K + k] = mi_f2h(xc[k]);
        }
    }
}

// the epilogue's extra row-range copies (mi_f16_epilogue::copy)
__device__ __forceinline__ void epi_row_copies(const mi_f16_epilogue & e, int64_t row, int64_t col, float v) {
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1) {
            *(float *) (e.copy[k].ptr + col * e.copy[k].col_stride + (row - e.copy[k].row0) * sizeof(float)) = v;
        }
    }
}

// Decode-regime F16 GEMV with the activation conversion and the graph's epilogue fused in:
//   - each workgroup converts its NC f32 activation columns to f16 in LDS (RNE, as the CPU's
//     ggml_fp32_to_fp16_row, src/ggml.c:610-612), so no separate conversion launch;
//   - weights stream through a two-deep register prefetch of kU 16-byte steps per lane, so a
//     quad keeps up to 2*kU loads in flight instead of one per dependent FMA step (kU = 32 when
//     the matrix has too few rows to fill the chip with waves, 8 otherwise);
//   - epilogue (EPI): 1 = + bias[row], 2 = + bias[row] + resid, 3 = gelu(. + bias[row]) via the
//     fp16 table -- the graph's following ADD / ADD / GELU nodes, each rounded as the CPU does.

template <int NC, int EPI, int kU>
__global__ __launch_bounds__(256) void k_mmv_f16_x(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                   mi_src_cols x, const uint16_t * __restrict__ xh, int64_t ncols,
                                                   float * __restrict__ dst, size_t ycol, mi_f16_epilogue e,
                                                   mi_norm_prologue pro) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [NC][K] f16 (+ [K] f32 for the norm prologue)
    __shared__ double shd[9];
    const int q = threadIdx.x & 3;
    const int rpb = blockDim.x >> 2;
    const int64_t row = (int64_t) blockIdx.x * rpb + (threadIdx.x >> 2);
    const bool live = row < N;
    const int64_t i11 = (int64_t) blockIdx.y * NC;
    int nc = (int) (ncols - i11);
    nc = nc > NC ? NC : nc;

    // The weights do not depend on the activations: the first kU steps of the row are requested
    // before the activations are staged (and normalised), so their HBM latency overlaps that work.
    const uint16_t * wrow = (const uint16_t *) (W + (live ? row : 0) * nb01);
    const int64_t nsteps = K >> 5;  // whole 32-element steps
    uint4 cur[kU];
    if (nsteps > 0) {
#pragma unroll
        for (int u = 0; u < kU; u++) cur[u] = *(const uint4 *) (wrow + (u < nsteps ? u : nsteps - 1) * 32 + 8 * q);
    }

    stage_f16_activations<NC>(xs, shd, K, i11, nc, x, xh, pro);
    __syncthreads();

    float acc[NC][8];
#pragma unroll
    for (int c = 0; c < NC; c++)
#pragma unroll
        for (int l = 0; l < 8; l++) acc[c][l] = 0.0f;

    auto step_compute = [&](const uint4 & wv4, int64_t st) {
        float w[8];
        h8_to_f(wv4, w);
        const int64_t i = st * 32 + 8 * q;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (c < nc) {
                float xv[8];
                h8_to_f(*(const uint4 *) (xs + c * K + i), xv);
#pragma unroll
                for (int l = 0; l < 8; l++) acc[c][l] = __fmaf_rn(w[l], xv[l], acc[c][l]);
            }
        }
    };
    if (nsteps > 0) {
        uint4 nxt[kU];
        for (int64_t s0 = 0; s0 < nsteps; s0 += kU) {
            const int64_t s1 = s0 + kU;
            if (s1 < nsteps) {
#pragma unroll
                for (int u = 0; u < kU; u++) nxt[u] = *(const uint4 *) (wrow + (s1 + u < nsteps ? s1 + u : nsteps - 1) * 32 + 8 * q);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                if (s0 + u < nsteps) step_compute(cur[u], s0 + u);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) cur[u] = nxt[u];
        }
    }
    const int64_t np = nsteps * 32;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float r = quad_reduce_avx(acc[c]);
        if (q == 0 && live && c < nc) {
            double sd = (double) r;
            for (int64_t i = np; i < K; i++) sd += (double) mul_rn(mi_h2f(wrow[i]), mi_h2f(xs[c * K + i]));
            float v = (float) sd;
            if (EPI >= 1) v = add_rn(v, e.bias[row]);
            if (EPI == 2) v = add_rn(v, *(const float *) (e.resid + (i11 + c) * e.resid_nb1 + row * sizeof(float)));
            if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
            *(float *) ((char *) dst + (i11 + c) * ycol + row * sizeof(float)) = v;
            epi_row_copies(e, row, i11 + c, v);
        }
    }
}

// Same contract as k_mmv_f16_x, with the 32 partial sums of a dot spread over 16 lanes instead of
// a quad: lane m of a row's 16-lane group owns the two sums of elements i = 2m, 2m+1 (mod 32),
// i.e. AVX register r = m / 4, lanes 2(m % 4) and 2(m % 4) + 1, and loads one dword (two f16) per
// 32-element step. A row's 6 KB (K = 3072) is then 96 dwords per lane, all requested at once
// (kS steps per batch, two batches in flight), so a 768-row matrix keeps the whole matrix in
// flight from 192 waves instead of 48 quads-per-wave waves draining it in dependent rounds. The
// partial sums are combined in GGML_F32x8_REDUCE's order (src/ggml.c:1172-1190) across lanes:
// xor 8 = (s0 += s2, s1 += s3), xor 4 = (s0 += s1), xor 2 = (lane k + lane k+4), then
// (t0 + t1) + (t2 + t3).
template <int NC, int EPI, int kS>
__global__ __launch_bounds__(256) void k_mmv_f16_w16(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                     mi_src_cols x, const uint16_t * __restrict__ xh, int64_t ncols,
                                                     float * __restrict__ dst, size_t ycol, mi_f16_epilogue e,
                                                     mi_norm_prologue pro) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [NC][K] f16 (+ [K] f32 for the norm prologue)
    __shared__ double shd[9];
    const int m = threadIdx.x & 15;
    const int rpb = blockDim.x >> 4;
    const int64_t row = (int64_t) blockIdx.x * rpb + (threadIdx.x >> 4);
    const bool live = row < N;
    const int64_t i11 = (int64_t) blockIdx.y * NC;
    int nc = (int) (ncols - i11);
    nc = nc > NC ? NC : nc;

    const uint32_t * wrow = (const uint32_t *) (W + (live ? row : 0) * nb01);
    const int nsteps = (int) (K >> 5);
    uint32_t cur[kS];
    if (nsteps > 0) {
#pragma unroll
        for (int u = 0; u < kS; u++) cur[u] = wrow[(u < nsteps ? u : nsteps - 1) * 16 + m];
    }

    stage_f16_activations<NC>(xs, shd, K, i11, nc, x, xh, pro);
    __syncthreads();

    float acc[NC][2];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c][0] = acc[c][1] = 0.0f;

    const uint32_t * xs32 = (const uint32_t *) xs;
    auto step_compute = [&](uint32_t wv, int st) {
        const float w0 = mi_h2f((uint16_t) (wv & 0xffffu)), w1 = mi_h2f((uint16_t) (wv >> 16));
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (c < nc) {
                const uint32_t xv = xs32[((size_t) c * K >> 1) + st * 16 + m];
                acc[c][0] = __fmaf_rn(w0, mi_h2f((uint16_t) (xv & 0xffffu)), acc[c][0]);
                acc[c][1] = __fmaf_rn(w1, mi_h2f((uint16_t) (xv >> 16)), acc[c][1]);
            }
        }
    };
    if (nsteps > 0) {
        uint32_t nxt[kS];
        for (int s0 = 0; s0 < nsteps; s0 += kS) {
            const int s1 = s0 + kS;
            if (s1 < nsteps) {
#pragma unroll
                for (int u = 0; u < kS; u++) nxt[u] = wrow[(s1 + u < nsteps ? s1 + u : nsteps - 1) * 16 + m];
            }
#pragma unroll
            for (int u = 0; u < kS; u++) {
                if (s0 + u < nsteps) step_compute(cur[u], s0 + u);
            }
#pragma unroll
            for (int u = 0; u < kS; u++) cur[u] = nxt[u];
        }
    }
    const int64_t np = (int64_t) nsteps * 32;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        float a0 = acc[c][0], a1 = acc[c][1];
        a0 = add_rn(a0, __shfl_xor(a0, 8, 64));
        a1 = add_rn(a1, __shfl_xor(a1, 8, 64));
        a0 = add_rn(a0, __shfl_xor(a0, 4, 64));
        a1 = add_rn(a1, __shfl_xor(a1, 4, 64));
        a0 = add_rn(a0, __shfl_xor(a0, 2, 64));  // lane 0: t0, t1; lane 1: t2, t3
        a1 = add_rn(a1, __shfl_xor(a1, 2, 64));
        float u = add_rn(a0, a1);
        u = add_rn(u, __shfl_xor(u, 1, 64));
        if (m == 0 && live && c < nc) {
            const uint16_t * wr16 = (const uint16_t *) wrow;
            double sd = (double) u;
            for (int64_t i = np; i < K; i++) sd += (double) mul_rn(mi_h2f(wr16[i]), mi_h2f(xs[c * K + i]));
            float v = (float) sd;
            if (EPI >= 1) v = add_rn(v, e.bias[row]);
            if (EPI == 2) v = add_rn(v, *(const float *) (e.resid + (i11 + c) * e.resid_nb1 + row * sizeof(float)));
            if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
            *(float *) ((char *) dst + (i11 + c) * ycol + row * sizeof(float)) = v;
            epi_row_copies(e, row, i11 + c, v);
        }
    }
}

template <int NC, int kS>
void launch_f16_w16(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                    float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s, int threads) {
    const int rpb = threads / 16;
    const dim3 grid((unsigned) ((N + rpb - 1) / rpb), (unsigned) ((ncols + NC - 1) / NC));
    const size_t lds = (size_t) NC * K * sizeof(uint16_t) + (pro.mode ? (size_t) K * sizeof(float) : 0);
    const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
    switch (epi) {
        case 0: hipLaunchKernelGGL((k_mmv_f16_w16<NC, 0, kS>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        case 1: hipLaunchKernelGGL((k_mmv_f16_w16<NC, 1, kS>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        case 2: hipLaunchKernelGGL((k_mmv_f16_w16<NC, 2, kS>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        default: hipLaunchKernelGGL((k_mmv_f16_w16<NC, 3, kS>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
    }
}

template <int NC, int U>
void launch_f16_x_u(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                    float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s, int threads) {
    const int rpb = threads / 4;
    const dim3 grid((unsigned) ((N + rpb - 1) / rpb), (unsigned) ((ncols + NC - 1) / NC));
    const size_t lds = (size_t) NC * K * sizeof(uint16_t) + (pro.mode ? (size_t) K * sizeof(float) : 0);
    const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
    switch (epi) {
        case 0: hipLaunchKernelGGL((k_mmv_f16_x<NC, 0, U>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        case 1: hipLaunchKernelGGL((k_mmv_f16_x<NC, 1, U>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        case 2: hipLaunchKernelGGL((k_mmv_f16_x<NC, 2, U>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
        default: hipLaunchKernelGGL((k_mmv_f16_x<NC, 3, U>), grid, dim3(threads), lds, s, (const uint8_t *) W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro); break;
    }
}

template <int NC>
void launch_f16_x(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                  float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s) {
    // 64-lane workgroups (16 rows) while that still leaves >= 2 workgroups per CU, else 256;
    // deep prefetch when there are few rows (a few thousand quads cannot hide HBM latency)
    const int threads = N >= 16 * 1024 ? 256 : 64;
    const int variant = g_mi_tuning.f16_variant;
    // 16 lanes per row while the matrix is small enough that a quad per row leaves too few waves
    // to keep it in flight (measured on MI355X, GPT-2 shapes: K=3072 N=768 12.2 -> 8.2 us,
    // K=768 N=2304 with the norm prologue 6.8 -> 6.3 us); the quad kernel above that (lm_head
    // N=50257: 17 us vs 32 us -- four times fewer workgroups, each amortising its prologue).
    if (variant == 0 && (K >> 5) > 0 && N * ((ncols + NC - 1) / NC) < 16384) {
        const int t16 = g_mi_tuning.f16_threads ? g_mi_tuning.f16_threads : 256;
        if (K <= 48 * 32 * 2) launch_f16_w16<NC, 48>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, t16);
        else launch_f16_w16<NC, 16>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, t16);
        return;
    }
    if (N * ((ncols + NC - 1) / NC) <= 8192) launch_f16_x_u<NC, 32>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, threads);
    else launch_f16_x_u<NC, 8>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, threads);
}

// ---- attention block of the GPT-2 graph in one kernel (main-backend.cpp:552-608) -----------------
// For one (head h, query token t): KQ[k] = dot(K[:, k, h], Q[:, t, h]) over the head dim,
// w = KQ * pre_scale, masked to -inf for k > n_past + t, soft_max (fp16 exp table, exact double
// sum), then KQV[d] = dot(V_trans[:, d, h], p) over k, written straight into the merged [D*H, N]
// layout. Every dot is ggml_vec_dot_f32's CPU order (quad per dot, as k_mm_f32_ord), every
// rounding as the separate nodes do it, so the result is bit-identical to the unfused graph.

// ggml_vec_dot_f32 order for one dot on a quad; valid in lane q == 0
template <typename LX, typename LY>
__device__ __forceinline__ float dot_f32_cpu_order(LX ldx, LY ldy, int64_t K, int q) {
    float acc[8];
#pragma unroll
    for (int l = 0; l < 8; l++) acc[l] = 0.0f;
    const int64_t np = K & ~(int64_t) 31;
#pragma unroll 2
    for (int64_t i = 8 * q; i < np; i += 32) {
        float xv[8], yv[8];
#pragma unroll
        for (int l = 0; l < 8; l++) {
            xv[l] = ldx(i + l);
            yv[l] = ldy(i + l);
        }
#pragma unroll
        for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(xv[l], yv[l], acc[l]);
    }
    float s = quad_reduce_avx(acc);
    if (q == 0) {
        const int64_t L = K - np;
        const int64_t fused_from = (L >= 8 ? (L / 8) * 8 : 0) + (((L >= 8 ? L % 8 : L) >= 4) ? 4 : 0);
        for (int64_t j = 0; j < L; j++) {
            const float a = ldx(np + j), b = ldy(np + j);
            s = j < fused_from ? add_rn(s, mul_rn(a, b)) : __fmaf_rn(a, b, s);
        }
    }
    return s;
}

// 512 lanes = 128 quads. Latency is the cost at decode sizes, so the K rows of the first KQ round
// and the first 4 steps (128 positions) of every V column are requested before anything else.
constexpr int kAttnThreads = 512;
constexpr int kAttnVPre = 4;

__global__ __launch_bounds__(kAttnThreads) void k_attn_ordered(mi_attn_desc a, const uint16_t * __restrict__ exp_table) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // q[D] | p[n_kv]
    __shared__ float shf[kAttnThreads / 64];
    __shared__ double shd[kAttnThreads / 64];
    const int h = blockIdx.x, t = blockIdx.y;
    const int hk = h / a.r2;  // K/V head (broadcast when Q has more heads)
    const int q = threadIdx.x & 3, quad = threadIdx.x >> 2, nquads = blockDim.x >> 2;
    const int nw = (int) (blockDim.x >> 6);
    float * qv = sm;
    float * p = sm + a.D;

    // early V requests: quad d < D owns KQV column d; steps s < kAttnVPre of its ordered dot
    const int64_t npv = (int64_t) a.n_kv & ~(int64_t) 31;
    const int dq = quad < a.D ? quad : a.D - 1;
    const char * vcol = a.v + (size_t) dq * a.v_nb[1] + (size_t) hk * a.v_nb[2];
    const size_t vnb0 = a.v_nb[0];
    float vpre[kAttnVPre][8];
#pragma unroll
    for (int st = 0; st < kAttnVPre; st++)
#pragma unroll
        for (int l = 0; l < 8; l++) {
            const int64_t k = (int64_t) st * 32 + 8 * q + l;
            vpre[st][l] = k < npv ? *(const float *) (vcol + k * vnb0) : 0.0f;
        }

    for (int d = threadIdx.x; d < a.D; d += blockDim.x) qv[d] = *(const float *) (a.q + d * a.q_nb[0] + t * a.q_nb[1] + h * a.q_nb[2]);
    __syncthreads();
    // KQ row, then pre-scale / causal mask / soft_max scale
    for (int k0 = 0; k0 < a.n_kv; k0 += nquads) {
        const int k = k0 + quad;
        const int kk = k < a.n_kv ? k : a.n_kv - 1;
        const char * krow = a.k + (size_t) kk * a.k_nb[1] + (size_t) hk * a.k_nb[2];
        const size_t knb0 = a.k_nb[0];
        const float v = dot_f32_cpu_order([&](int64_t i) { return *(const float *) (krow + i * knb0); },
                                          [&](int64_t i) { return qv[i]; }, a.D, q);
        if (q == 0 && k < a.n_kv) {
            float w = mul_rn(v, a.pre_scale);
            if (a.mask) w = add_rn(w, *(const float *) (a.mask + (size_t) t * a.mask_nb1 + (size_t) k * 4));
            if (k >= a.n_past && k > a.n_past + t) w = -INFINITY;
            p[k] = mul_rn(w, a.sm_scale);
        }
    }
    __syncthreads();
    float mx = -INFINITY;
    for (int k = threadIdx.x; k < a.n_kv; k += blockDim.x) mx = fmaxf(mx, p[k]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0) shf[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = -INFINITY;
    for (int w = 0; w < nw; w++) mx = fmaxf(mx, shf[w]);
    double s = 0.0;
    for (int k = threadIdx.x; k < a.n_kv; k += blockDim.x) {
        const float w = p[k];
        const float v = w == -INFINITY ? 0.0f : mi_h2f(exp_table[mi_f2h(sub_rn(w, mx))]);
        p[k] = v;
        s += (double) v;  // fp16 values: every partial double sum is exact
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) shd[threadIdx.x >> 6] = s;
    __syncthreads();
    double sum = 0.0;
    for (int w = 0; w < nw; w++) sum += shd[w];
    const float inv = (float) (1.0 / sum);
    for (int k = threadIdx.x; k < a.n_kv; k += blockDim.x) p[k] = mul_rn(p[k], inv);
    __syncthreads();

    // KQV[d] = ggml_vec_dot_f32(n_kv, V_trans[:, d, h], p): quad d, first steps from vpre
    for (int d0 = 0; d0 < a.D; d0 += nquads) {
        const int d = d0 + quad;
        const bool first = d0 == 0;
        const int dd = d < a.D ? d : a.D - 1;
        const char * vc = a.v + (size_t) dd * a.v_nb[1] + (size_t) hk * a.v_nb[2];
        float acc[8];
#pragma unroll
        for (int l = 0; l < 8; l++) acc[l] = 0.0f;
        const int64_t nsteps = npv >> 5;
        int64_t st = 0;
        if (first) {
#pragma unroll
            for (int u = 0; u < kAttnVPre; u++) {
                if (u < nsteps) {
#pragma unroll
                    for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(vpre[u][l], p[u * 32 + 8 * q + l], acc[l]);
                }
            }
            st = nsteps < kAttnVPre ? nsteps : kAttnVPre;
        }
#pragma unroll 4
        for (; st < nsteps; st++) {
            const int64_t i = st * 32 + 8 * q;
#pragma unroll
            for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(*(const float *) (vc + (i + l) * vnb0), p[i + l], acc[l]);
        }
        float r = quad_reduce_avx(acc);
        if (q == 0 && d < a.D) {
            const int64_t L = a.n_kv - npv;
            const int64_t fused_from = (L >= 8 ? (L / 8) * 8 : 0) + (((L >= 8 ? L % 8 : L) >= 4) ? 4 : 0);
            for (int64_t j = 0; j < L; j++) {
                const float x = *(const float *) (vc + (npv + j) * vnb0), y = p[npv + j];
                r = j < fused_from ? add_rn(r, mul_rn(x, y)) : __fmaf_rn(x, y, r);
            }
            *(float *) (a.out + d * a.o_nb[0] + t * a.o_nb[1] + h * a.o_nb[2]) = r;
        }
    }
}

// One-round-trip variant of k_attn_ordered for decode-sized contexts (n_kv <= 32768 / D): every
// global load of the block -- q, the K rows of all key rounds, the whole V slab of the head -- is
// issued before any arithmetic, so the kernel pays one memory round trip instead of three (q ->
// K -> V in k_attn_ordered). K rows stay in registers for the KQ dots; the V slab lands in LDS
// (rows padded to D + 1 floats: conflict-free column walks) and the KQV chains read it from
// there. Every dot, mask, soft_max and rounding step is k_attn_ordered's, so the result is the
// same bit for bit.
// KVCAP: the key-count bucket the launch was sized for (n_kv <= KVCAP), so only the key rounds and
// V-slab loads the context needs are issued. q / K loads are 16-byte vector loads (host-checked
// contiguity and alignment): at decode the load phase is issue-bound on only H workgroups.
template <int D, int KVCAP, int ABL = 0>
__global__ __launch_bounds__(512) void k_attn_fast(mi_attn_desc a, const uint16_t * __restrict__ exp_table) {
    constexpr int KVMAX = KVCAP;               // keys this instantiation serves
    constexpr int KR = KVMAX / 128;            // key rounds of the 128 quads
    constexpr int QS = D / 32;                 // 32-element steps of one head-dim dot
    constexpr int VS = D + 1;                  // padded LDS row stride of the V slab
    constexpr int VREG = KVMAX * D / 512 / 4;  // float4 of the V slab per thread
    extern __shared__ __attribute__((aligned(16))) float sm[];  // vs[n_kv][VS] | p[n_kv]
    __shared__ float shf[8];
    __shared__ double shd[8];
    const int h = blockIdx.x, t = blockIdx.y;
    const int hk = h / a.r2;
    const int tid = threadIdx.x, q = tid & 3, quad = tid >> 2;
    const int n_kv = a.n_kv;
    float * vs = sm;
    float * p = sm + n_kv * VS;

    // ---- 1. all loads up front (addresses clamped into the tensors instead of predicated)
    float qv[QS][8];
    const char * qrow = a.q + (size_t) t * a.q_nb[1] + (size_t) h * a.q_nb[2];
#pragma unroll
    for (int st = 0; st < QS; st++) {
        const float4 u0 = *(const float4 *) (qrow + (size_t) (st * 32 + 8 * q) * 4);  // q_nb[0] == 4
        const float4 u1 = *(const float4 *) (qrow + (size_t) (st * 32 + 8 * q + 4) * 4);
        qv[st][0] = u0.x; qv[st][1] = u0.y; qv[st][2] = u0.z; qv[st][3] = u0.w;
        qv[st][4] = u1.x; qv[st][5] = u1.y; qv[st][6] = u1.z; qv[st][7] = u1.w;
    }
    float kv[KR][QS][8];
#pragma unroll
    for (int r = 0; r < KR; r++) {
        const int k = min(quad + 128 * r, n_kv - 1);
        const char * krow = a.k + (size_t) k * a.k_nb[1] + (size_t) hk * a.k_nb[2];
#pragma unroll
        for (int st = 0; st < QS; st++) {
            const float4 u0 = *(const float4 *) (krow + (size_t) (st * 32 + 8 * q) * 4);  // k_nb[0] == 4
            const float4 u1 = *(const float4 *) (krow + (size_t) (st * 32 + 8 * q + 4) * 4);
            kv[r][st][0] = u0.x; kv[r][st][1] = u0.y; kv[r][st][2] = u0.z; kv[r][st][3] = u0.w;
            kv[r][st][4] = u1.x; kv[r][st][5] = u1.y; kv[r][st][6] = u1.z; kv[r][st][7] = u1.w;
        }
    }
    float4 vr[VREG];
    const char * vh = a.v + (size_t) hk * a.v_nb[2];
#pragma unroll
    for (int i = 0; i < VREG; i++) {
        const int e = 4 * (tid + 512 * i);
        const int k = min(e / D, n_kv - 1), d = e % D;  // 4 consecutive d of one key (D % 4 == 0)
        vr[i] = *(const float4 *) (vh + (size_t) k * a.v_nb[0] + (size_t) d * 4);  // v_nb[1] == 4, 16-B aligned (host-checked)
    }

    // ---- 2. KQ from registers (ggml_vec_dot_f32 order per dot), pre-scale, causal mask, sm scale
#pragma unroll
    for (int r = 0; r < KR; r++) {
        const int k = quad + 128 * r;
        if (128 * r >= n_kv) break;  // block-uniform
        float acc[8];
#pragma unroll
        for (int l = 0; l < 8; l++) acc[l] = 0.0f;
#pragma unroll
        for (int st = 0; st < QS; st++)
#pragma unroll
            for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(kv[r][st][l], qv[st][l], acc[l]);
        const float v = quad_reduce_avx(acc);
        if (q == 0 && k < n_kv) {
            float w = mul_rn(v, a.pre_scale);
            if (a.mask) w = add_rn(w, *(const float *) (a.mask + (size_t) t * a.mask_nb1 + (size_t) k * 4));
            if (k >= a.n_past && k > a.n_past + t) w = -INFINITY;
            p[k] = mul_rn(w, a.sm_scale);
        }
    }
    if constexpr (ABL == 3) {  // timing ablation: loads + KQ only
        if (q == 0 && quad < n_kv) *(float *) (a.out + (size_t) quad * 4) = p[quad] + vr[0].x + vr[VREG - 1].w;
        return;
    }
    // ---- 3. V slab into LDS
#pragma unroll
    for (int i = 0; i < VREG; i++) {
        const int e = 4 * (tid + 512 * i);
        const int k = e / D, d = e % D;
        if (k < n_kv) {
            float * dstv = vs + k * VS + d;
            dstv[0] = vr[i].x;
            dstv[1] = vr[i].y;
            dstv[2] = vr[i].z;
            dstv[3] = vr[i].w;
        }
    }
    __syncthreads();

    // ---- 4. soft_max over p (as k_attn_ordered)
    const int nw = 8;
    float mx = -INFINITY;
    for (int k = tid; k < n_kv; k += 512) mx = fmaxf(mx, p[k]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if ((tid & 63) == 0) shf[tid >> 6] = mx;
    __syncthreads();
    mx = -INFINITY;
    for (int w = 0; w < nw; w++) mx = fmaxf(mx, shf[w]);
    double ssum = 0.0;
    for (int k = tid; k < n_kv; k += 512) {
        const float w = p[k];
        const float v = w == -INFINITY ? 0.0f : (ABL == 1 ? sub_rn(w, mx) : mi_h2f(exp_table[mi_f2h(sub_rn(w, mx))]));
        p[k] = v;
        ssum += (double) v;  // fp16 values: every partial double sum is exact
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ssum += __shfl_xor(ssum, off, 64);
    if ((tid & 63) == 0) shd[tid >> 6] = ssum;
    __syncthreads();
    double sum = 0.0;
    for (int w = 0; w < nw; w++) sum += shd[w];
    const float inv = (float) (1.0 / sum);
    for (int k = tid; k < n_kv; k += 512) p[k] = mul_rn(p[k], inv);
    __syncthreads();

    if constexpr (ABL == 2) {  // timing ablation: no KQV
        if (tid < D) *(float *) (a.out + (size_t) tid * a.o_nb[0] + (size_t) t * a.o_nb[1] + (size_t) h * a.o_nb[2]) = p[tid];
        return;
    }
    // ---- 5. KQV[d] = ggml_vec_dot_f32(n_kv, V_trans[:, d, h], p) from LDS, quad d
    const int npv = n_kv & ~31;
    for (int d0 = 0; d0 < D; d0 += 128) {
        const int d = d0 + quad;
        if (d >= D) break;
        float acc[8];
#pragma unroll
        for (int l = 0; l < 8; l++) acc[l] = 0.0f;
        for (int i = 8 * q; i < npv; i += 32) {
#pragma unroll
            for (int l = 0; l < 8; l++) acc[l] = __fmaf_rn(vs[(i + l) * VS + d], p[i + l], acc[l]);
        }
        float r = quad_reduce_avx(acc);
        if (q == 0) {
            const int L = n_kv - npv;
            const int fused_from = (L >= 8 ? (L / 8) * 8 : 0) + (((L >= 8 ? L % 8 : L) >= 4) ? 4 : 0);
            for (int j = 0; j < L; j++) {
                const float x = vs[(npv + j) * VS + d], y = p[npv + j];
                r = j < fused_from ? add_rn(r, mul_rn(x, y)) : __fmaf_rn(x, y, r);
            }
            *(float *) (a.out + (size_t) d * a.o_nb[0] + (size_t) t * a.o_nb[1] + (size_t) h * a.o_nb[2]) = r;
        }
    }
}

ord_geom make_ord_geom(const mi_mm_desc & m, int NC) {
    ord_geom g;
    g.K = m.K;
    g.N = m.N;
    g.ne11 = m.ne11;
    g.ne12 = m.ne12;
    g.ne13 = m.ne13;
    g.r2 = m.ne12 / m.ne02;
    g.r3 = m.ne13 / m.ne03;
    g.nb01 = m.nb01;
    g.nb02 = m.nb02;
    g.nb03 = m.nb03;
    g.nb1 = m.nb1;
    g.nb2 = m.nb2;
    g.nb3 = m.nb3;
    g.col_chunks = (m.ne11 + NC - 1) / NC;
    return g;
}

template <int NC> void launch_f16(const mi_mm_desc & m, const uint16_t * xh, hipStream_t s) {
    const ord_geom g = make_ord_geom(m, NC);
    const dim3 grid((unsigned) ((m.N + kQuadsPerBlock - 1) / kQuadsPerBlock), (unsigned) (g.col_chunks * m.ne12 * m.ne13));
    const bool aligned = m.K % 8 == 0 && ((uintptr_t) m.W | m.nb01 | m.nb02 | m.nb03 | (uintptr_t) xh) % 16 == 0;
    if (aligned) hipLaunchKernelGGL((k_mmv_f16_ord<NC, true>), grid, dim3(256), 0, s, (const uint8_t *) m.W, xh, m.dst, g);
    else hipLaunchKernelGGL((k_mmv_f16_ord<NC, false>), grid, dim3(256), 0, s, (const uint8_t *) m.W, xh, m.dst, g);
}

} // namespace

void mi_mul_mat_f16(const mi_mm_desc & m, const uint16_t * xh, hipStream_t s) {
    switch (m.ne11 >= 4 ? 4 : (int) m.ne11) {
        case 1: launch_f16<1>(m, xh, s); break;
        case 2: launch_f16<2>(m, xh, s); break;
        case 3: launch_f16<3>(m, xh, s); break;
        default: launch_f16<4>(m, xh, s); break;
    }
}

void mi_mul_mat_f32(const mi_mm_desc & m, const mi_src_cols & x, hipStream_t s) {
    const ord_geom g = make_ord_geom(m, 1);
    const dim3 grid((unsigned) ((m.N + kQuadsPerBlock - 1) / kQuadsPerBlock), (unsigned) (m.ne11 * m.ne12 * m.ne13));
    hipLaunchKernelGGL(k_mm_f32_ord, grid, dim3(256), 0, s, (const uint8_t *) m.W, x, m.dst, g);
}

bool mi_mul_mat_f16_fused_supported(int64_t K, int64_t ncols) { return ncols >= 1 && K >= 8 && K % 8 == 0 && K <= 10240; }

void mi_mul_mat_f16_fused(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh,
                          int64_t ncols, float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro,
                          hipStream_t s) {
    if (mi_mmv_order() == 0 && mi_mul_mat_f16_fast_supported(K, ncols, x, xh, pro)) {
        mi_mul_mat_f16_fast(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s);
        return;
    }
    // reference CPU order: columns per workgroup: up to 4, with the f16 activations (+ one f32 column) within 64 KB of LDS
    const int64_t cap = (32768 - (pro.mode ? 2 * K : 0)) / K;
    const int nc = (int) std::min<int64_t>(std::min<int64_t>(ncols, 4), std::max<int64_t>(cap, 1));
    switch (nc) {
        case 1: launch_f16_x<1>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s); break;
        case 2: launch_f16_x<2>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s); break;
        case 3: launch_f16_x<3>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s); break;
        default: launch_f16_x<4>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s); break;
    }
}

bool mi_attn_supported(int D, int n_kv) { return D >= 1 && D <= 256 && n_kv >= 1 && (size_t) (D + n_kv) * 4 <= 60 * 1024; }

void mi_attn_ordered(const mi_attn_desc & a, const uint16_t * exp_table, hipStream_t s) {
    if (mi_mmv_order() == 0 && g_mi_tuning.attn_variant == 0 && mi_attn_tree_supported(a)) {
        mi_attn_tree(a, s);  // attn_fast.hip: tree order (the default decode mode)
        return;
    }
    static const bool lds_ok = [] {  // the V slab needs more than the default 64 KB of dynamic LDS
        bool ok = true;
        for (const void * f : {(const void *) k_attn_fast<64, 128>, (const void *) k_attn_fast<64, 256>, (const void *) k_attn_fast<64, 512>,
                               (const void *) k_attn_fast<128, 128>, (const void *) k_attn_fast<128, 256>,
                               (const void *) k_attn_fast<64, 512, 1>, (const void *) k_attn_fast<64, 512, 2>, (const void *) k_attn_fast<64, 512, 3>})
            ok &= hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess;
        (void) hipGetLastError();
        return ok;
    }();
    const bool fast_ok = lds_ok && g_mi_tuning.attn_variant == 0 && a.v_nb[1] == 4 && a.q_nb[0] == 4 && a.k_nb[0] == 4 &&
                         ((uintptr_t) a.v | a.v_nb[0] | a.v_nb[2] | (uintptr_t) a.q | a.q_nb[1] | a.q_nb[2] | (uintptr_t) a.k | a.k_nb[1] |
                          a.k_nb[2]) % 16 == 0;
    const dim3 grid((unsigned) a.H, (unsigned) a.N);
    if (fast_ok && a.D == 64 && a.n_kv <= 512) {
        const size_t lds = (size_t) a.n_kv * (64 + 2) * sizeof(float);
#if MI_DIAG
        switch (g_mi_tuning.attn_abl) {  // timing ablations only (results invalid): make DIAG=1
            case 1: hipLaunchKernelGGL((k_attn_fast<64, 512, 1>), grid, dim3(512), lds, s, a, exp_table); return;
            case 2: hipLaunchKernelGGL((k_attn_fast<64, 512, 2>), grid, dim3(512), lds, s, a, exp_table); return;
            case 3: hipLaunchKernelGGL((k_attn_fast<64, 512, 3>), grid, dim3(512), lds, s, a, exp_table); return;
            default: break;
        }
#endif
        if (a.n_kv <= 128) hipLaunchKernelGGL((k_attn_fast<64, 128>), grid, dim3(512), lds, s, a, exp_table);
        else if (a.n_kv <= 256) hipLaunchKernelGGL((k_attn_fast<64, 256>), grid, dim3(512), lds, s, a, exp_table);
        else hipLaunchKernelGGL((k_attn_fast<64, 512>), grid, dim3(512), lds, s, a, exp_table);
        return;
    }
    if (fast_ok && a.D == 128 && a.n_kv <= 256) {
        const size_t lds = (size_t) a.n_kv * (128 + 2) * sizeof(float);
        if (a.n_kv <= 128) hipLaunchKernelGGL((k_attn_fast<128, 128>), grid, dim3(512), lds, s, a, exp_table);
        else hipLaunchKernelGGL((k_attn_fast<128, 256>), grid, dim3(512), lds, s, a, exp_table);
        return;
    }
    const size_t lds = (size_t) (a.D + a.n_kv) * sizeof(float);
    hipLaunchKernelGGL(k_attn_ordered, dim3((unsigned) a.H, (unsigned) a.N), dim3(kAttnThreads), lds, s, a, exp_table);
}
