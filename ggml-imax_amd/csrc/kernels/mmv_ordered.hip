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

#include "mi355x_common.h"
#include "mi355x_kernels.h"

// Bit-exactness with the CPU needs every multiply and add rounded separately unless written as
// __fmaf_rn: HIP's __fmul_rn/__fadd_rn are plain operators defined in a header (so this file's
// pragma does not reach them) that -ffp-contract=fast would fuse; mul_rn/add_rn below are
// written under the pragma instead.
#pragma clang fp contract(off)

namespace {
__device__ __forceinline__ float mul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float add_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float sub_rn(float a, float b) { return a - b; }
} // namespace

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

// F16 weights x f16 activation columns (xh: [ncols][K], the CPU's from_float rows).
// One quad per (row, chunk of NC columns).
template <int NC>
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
        h8_to_f(*(const uint4 *) (wrow + i), w);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (c < nc) {
                float x[8];
                h8_to_f(*(const uint4 *) (xh + (col0 + c) * g.K + i), x);
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
    hipLaunchKernelGGL(k_mmv_f16_ord<NC>, grid, dim3(256), 0, s, (const uint8_t *) m.W, xh, m.dst, g);
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
