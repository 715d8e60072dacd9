// ops.hip -- the non-matmul ops of the GPT-2 / LLaMA-style graphs on gfx950.
//
// All are memory- or launch-bound. Each follows the reference CPU forward's rounding sequence so
// that results are bit-identical where the CPU order is reproducible:
//   get_rows   src/ggml.c:12920 (f16) / :13006 (f32) / :12874 (Q4_0, Q8_0, Q4_K, Q5_K) -- exact
//   add / mul  src/ggml.c:8568 / :9687 (broadcast src1)      -- exact
//   scale      src/ggml.c:12637                              -- exact
//   norm       src/ggml.c:11353-11406 (double sums)          -- sums in double, then the same f32 ops
//   rms_norm   src/ggml.c:11428-11478 (double sums)
//   soft_max   src/ggml.c:13393-13508 (fp16 exp table, double sum, y *= (float)(1/sum))
//   diag_mask  src/ggml.c:13301-13390
//   gelu/silu  src/ggml.c:1966-1991 (fp16 lookup tables, built on the host with libm like the
//              reference's ggml_init, src/ggml.c:2884-2898)
//   rope       src/ggml.c:13719-13948 (modes 0 and 2)
//   cpy/cont/dup src/ggml.c:8062, :12818 -- element i of src (row-major logical order) to
//              element i of dst, with f32/f16 conversion (RNE)

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#include "cpu_order.h"

namespace {

// element index -> coordinates; 32-bit division (the launchers keep element counts below 2^32)
__device__ __forceinline__ void unflatten(int64_t i64, const int64_t * ne, int64_t & i0, int64_t & i1, int64_t & i2, int64_t & i3) {
    uint32_t i = (uint32_t) i64;
    const uint32_t n0 = (uint32_t) ne[0], n1 = (uint32_t) ne[1], n2 = (uint32_t) ne[2];
    i0 = i % n0;
    i /= n0;
    i1 = i % n1;
    i /= n1;
    i2 = i % n2;
    i3 = i / n2;
}

__device__ __forceinline__ size_t off4(const size_t * nb, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    return (size_t) i0 * nb[0] + (size_t) i1 * nb[1] + (size_t) i2 * nb[2] + (size_t) i3 * nb[3];
}

__device__ __forceinline__ float ld_f(const char * p, int type) {
    return type == 1 ? mi_h2f(*(const uint16_t *) p) : *(const float *) p;
}

__device__ __forceinline__ void st_f(char * p, int type, float v) {
    if (type == 1) *(uint16_t *) p = mi_f2h(v);
    else *(float *) p = v;
}

// ---- element-wise ----------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_binary(mi_tensor_desc d, mi_tensor_desc a, mi_tensor_desc b, int op, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unflatten(i, d.ne, i0, i1, i2, i3);
        const float x = ld_f(a.data + off4(a.nb, i0, i1, i2, i3), a.type);
        const float y = ld_f(b.data + off4(b.nb, (uint32_t) i0 % (uint32_t) b.ne[0], (uint32_t) i1 % (uint32_t) b.ne[1],
                                          (uint32_t) i2 % (uint32_t) b.ne[2], (uint32_t) i3 % (uint32_t) b.ne[3]), b.type);
        float r;
        switch (op) {
            case MI_OP_ADD: r = x + y; break;
            case MI_OP_MUL: r = x * y; break;
            case MI_OP_SUB: r = x - y; break;
            default: r = x / y; break;
        }
        st_f(d.data + off4(d.nb, i0, i1, i2, i3), d.type, r);
    }
}

__global__ __launch_bounds__(256) void k_unary(mi_tensor_desc d, mi_tensor_desc a, int op, float p0, const uint16_t * table, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unflatten(i, d.ne, i0, i1, i2, i3);
        const float x = ld_f(a.data + off4(a.nb, i0, i1, i2, i3), a.type);
        float r;
        switch (op) {
            case MI_OP_SCALE: r = x * p0; break;
            case MI_OP_GELU:  // ggml_vec_gelu_f32 with GGML_GELU_FP16 (src/ggml.c:1978-1991)
                r = x <= -10.0f ? 0.0f : (x >= 10.0f ? x : mi_h2f(table[mi_f2h(x)]));
                break;
            case MI_OP_SILU:  // ggml_vec_silu_f32 with GGML_SILU_FP16: table[fp16(x)]
                r = mi_h2f(table[mi_f2h(x)]);
                break;
            case MI_OP_CPY:
            default: r = x; break;
        }
        st_f(d.data + off4(d.nb, i0, i1, i2, i3), d.type, r);
    }
}

// element i of src (in src's logical order) -> element i of dst (dst's logical order)
__global__ __launch_bounds__(256) void k_cpy(mi_tensor_desc d, mi_tensor_desc a, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3, j0, j1, j2, j3;
        unflatten(i, a.ne, i0, i1, i2, i3);
        unflatten(i, d.ne, j0, j1, j2, j3);
        const char * sp = a.data + off4(a.nb, i0, i1, i2, i3);
        char * dp = d.data + off4(d.nb, j0, j1, j2, j3);
        if (a.type == d.type && a.type == 1) *(uint16_t *) dp = *(const uint16_t *) sp;
        else st_f(dp, d.type, ld_f(sp, a.type));
    }
}

// up to kMaxCopies independent copies in one launch (blockIdx.y selects the copy)
struct mi_cpy_batch {
    mi_tensor_desc d[kMiMaxCopies], a[kMiMaxCopies];
    int64_t n[kMiMaxCopies];
};

__global__ __launch_bounds__(256) void k_cpy_multi(mi_cpy_batch b) {
    const int c = blockIdx.y;
    const mi_tensor_desc & d = b.d[c];
    const mi_tensor_desc & a = b.a[c];
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < b.n[c]; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3, j0, j1, j2, j3;
        unflatten(i, a.ne, i0, i1, i2, i3);
        unflatten(i, d.ne, j0, j1, j2, j3);
        const char * sp = a.data + off4(a.nb, i0, i1, i2, i3);
        char * dp = d.data + off4(d.nb, j0, j1, j2, j3);
        if (a.type == d.type && a.type == 1) *(uint16_t *) dp = *(const uint16_t *) sp;
        else st_f(dp, d.type, ld_f(sp, a.type));
    }
}

__global__ __launch_bounds__(256) void k_get_rows(mi_tensor_desc d, mi_tensor_desc a, mi_tensor_desc idx, int64_t n) {
    // dst row (i10, i11, i12) = src0 row (src1[i10, i11, i12], i11, i12)
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const int64_t c = i % d.ne[0];
        int64_t r = i / d.ne[0];
        const int64_t i10 = r % idx.ne[0];
        r /= idx.ne[0];
        const int64_t i11 = r % idx.ne[1];
        const int64_t i12 = r / idx.ne[1];
        const int32_t i01 = *(const int32_t *) (idx.data + i10 * idx.nb[0] + i11 * idx.nb[1] + i12 * idx.nb[2]);
        const float v = ld_f(a.data + c * a.nb[0] + (size_t) i01 * a.nb[1] + i11 * a.nb[2] + i12 * a.nb[3], a.type);
        st_f(d.data + c * d.nb[0] + i10 * d.nb[1] + i11 * d.nb[2] + i12 * d.nb[3], d.type, v);
    }
}

// GET_ROWS of a quantized src0 (ggml_compute_forward_get_rows_q, src/ggml.c:12874-12918): each
// output element is the reference dequantize_row_* value, as its x86 build computes it --
// Q4_0 ((q & 15) - 8) * d (src/ggml-quants.c:980-998), Q8_0 q * d (:1074-1088), Q4_K / Q5_K
// fma(d * sc, q, -(dmin * m)) (:2181-2218, :2464-2507; the -mfma build emits vfmsub132ps there).
template <int TYPE>
__device__ __forceinline__ float dequant_elem(const uint8_t * row, int64_t c) {
    if constexpr (TYPE == 2 || TYPE == 8) {  // Q4_0 (18 B) / Q8_0 (34 B) blocks of 32
        constexpr int BS = TYPE == 2 ? 18 : 34;
        const uint8_t * blk = row + (c >> 5) * BS;
        const int j = (int) (c & 31);
        uint16_t dh;
        __builtin_memcpy(&dh, blk, 2);
        const float d = mi_h2f(dh);
        if constexpr (TYPE == 2) {
            const uint8_t b = blk[2 + (j & 15)];
            return (float) ((j < 16 ? (b & 0x0F) : (b >> 4)) - 8) * d;
        } else {
            return (float) (int8_t) blk[2 + j] * d;
        }
    } else {  // Q4_K (144 B) / Q5_K (176 B) superblocks of 256
        constexpr bool Q5 = TYPE == 13;
        const uint8_t * blk = row + (c >> 8) * (Q5 ? 176 : 144);
        const int e = (int) (c & 255), g = e >> 6, l = e & 31, hi = (e >> 5) & 1;
        uint16_t dh, mh;
        __builtin_memcpy(&dh, blk, 2);
        __builtin_memcpy(&mh, blk + 2, 2);
        uint32_t sc3[3];
        __builtin_memcpy(sc3, blk + 4, 12);
        int sc, m;
        mi_scale_min_k4(2 * g + hi, sc3[0], sc3[1], sc3[2], sc, m);
        const float d1 = mul_rn(mi_h2f(dh), (float) sc), m1 = mul_rn(mi_h2f(mh), (float) m);
        const uint8_t * qs = blk + (Q5 ? 48 : 16) + 32 * g;
        int q = hi ? (qs[l] >> 4) : (qs[l] & 0x0F);
        if constexpr (Q5) q += (blk[16 + l] >> (2 * g + hi)) & 1 ? 16 : 0;
        return __fmaf_rn(d1, (float) q, -m1);
    }
}

template <int TYPE>
__global__ __launch_bounds__(256) void k_get_rows_q(mi_tensor_desc d, mi_tensor_desc a, mi_tensor_desc idx, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const int64_t c = i % d.ne[0];
        int64_t r = i / d.ne[0];
        const int64_t i10 = r % idx.ne[0];
        r /= idx.ne[0];
        const int64_t i11 = r % idx.ne[1];
        const int64_t i12 = r / idx.ne[1];
        const int32_t i01 = *(const int32_t *) (idx.data + i10 * idx.nb[0] + i11 * idx.nb[1] + i12 * idx.nb[2]);
        const uint8_t * row = (const uint8_t *) a.data + (size_t) i01 * a.nb[1] + i11 * a.nb[2] + i12 * a.nb[3];
        st_f(d.data + c * d.nb[0] + i10 * d.nb[1] + i11 * d.nb[2] + i12 * d.nb[3], d.type, dequant_elem<TYPE>(row, c));
    }
}

// get_rows(a, ia) + get_rows(b, ib) in one pass (the GPT-2 token + position embedding,
// main-backend.cpp:475-478): each element is read exactly as k_get_rows / k_get_rows_q read it
// and the two f32 values are added once, as the ADD node does. 1-D index vectors, f32 dst rows.
template <int T>  // 0: f32 / f16 (ld_f), else the quantized type
__device__ __forceinline__ float emb_elem(const mi_tensor_desc & a, int32_t r, int64_t c) {
    // (f32 / f16 resolved at compile time: a runtime type select put the loads under a branch)
    if constexpr (T == 0) return *(const float *) (a.data + c * a.nb[0] + (size_t) r * a.nb[1]);
    else if constexpr (T == 1) return mi_h2f(*(const uint16_t *) (a.data + c * a.nb[0] + (size_t) r * a.nb[1]));
    else return dequant_elem<T>((const uint8_t *) a.data + (size_t) r * a.nb[1], c);
}

// grid (column chunks, rows). Both indices are read once per thread before any gather, the
// position index first: in a decode step the token id may sit in pinned host memory (a PCIe round
// trip) while the position table is device-resident, so the position row's loads issue while the
// id is still in flight (vmcnt retires in issue order).
template <int TA, int TB>
__global__ __launch_bounds__(256) void k_get_rows_add(mi_tensor_desc d, mi_tensor_desc a, mi_tensor_desc ia, mi_tensor_desc b,
                                                      mi_tensor_desc ib, int ne0, uint64_t * st) {
    MI_STAMP(st, 0);
    const int r = (int) blockIdx.y;
    const int32_t rb = *(const int32_t *) (ib.data + (size_t) r * ib.nb[0]);
    const int32_t ra = *(const int32_t *) (ia.data + (size_t) r * ia.nb[0]);
    // every element's loads before any store (the stores may alias the tables as far as the
    // compiler knows, so a load-add-store loop paid one memory round trip per iteration); clamped
    // unconditional loads
    constexpr int V = 4;
    const int stride = (int) (gridDim.x * blockDim.x);
    for (int c0 = (int) (blockIdx.x * blockDim.x + threadIdx.x); c0 < ne0; c0 += V * stride) {
        float v[V];
#pragma unroll
        for (int u = 0; u < V; u++) {
            const int c = min(c0 + u * stride, ne0 - 1);
            v[u] = emb_elem<TA>(a, ra, c) + emb_elem<TB>(b, rb, c);
        }
#pragma unroll
        for (int u = 0; u < V; u++) {
            const int c = c0 + u * stride;
            if (c < ne0) *(float *) (d.data + (size_t) c * d.nb[0] + (size_t) r * d.nb[1]) = v[u];
        }
    }
    MI_STAMP(st, 7);
}

__global__ __launch_bounds__(256) void k_diag_mask(mi_tensor_desc d, mi_tensor_desc a, int n_past, float value, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unflatten(i, d.ne, i0, i1, i2, i3);
        float v = *(const float *) (a.data + off4(a.nb, i0, i1, i2, i3));
        if (i0 >= n_past && i0 > n_past + i1) v = value;
        *(float *) (d.data + off4(d.nb, i0, i1, i2, i3)) = v;
    }
}

// ---- row reductions: one 256-thread workgroup per row ----------------------------------------

__device__ __forceinline__ float block_max_f(float v, float * sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    float t = -INFINITY;
    for (int w = 0; w < (int) (blockDim.x >> 6); w++) t = fmaxf(t, sh[w]);
    return t;
}

// rows of src0 / dst are addressed by (i1, i2, i3); elements along ne0 with stride nb[0]
__device__ __forceinline__ void row_coords(int64_t r, const int64_t * ne, int64_t & i1, int64_t & i2, int64_t & i3) {
    i1 = r % ne[1];
    r /= ne[1];
    i2 = r % ne[2];
    i3 = r / ne[2];
}

constexpr int kRowLds = 12288;  // floats staged in LDS (48 KB); longer rows stage in dst

// norm / rms_norm, optionally followed by the graph's  mul(., g)  and  add(., b)  with 1-D g, b
// broadcast over rows (each rounded separately, as the CPU's separate MUL and ADD nodes).
__global__ __launch_bounds__(256) void k_norm(mi_tensor_desc d, mi_tensor_desc a, float eps, int rms, const float * g,
                                              const float * bias) {
    __shared__ __attribute__((aligned(16))) float lds[kRowLds];
    __shared__ double shd[9];
    int64_t i1, i2, i3;
    row_coords(blockIdx.x, a.ne, i1, i2, i3);
    const char * x = a.data + off4(a.nb, 0, i1, i2, i3);
    char * y = d.data + off4(d.nb, 0, i1, i2, i3);
    const int64_t n = a.ne[0];
    float * buf = n <= kRowLds ? lds : (float *) y;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) buf[i] = *(const float *) (x + i * a.nb[0]);
    __syncthreads();
    float scale;
    if (rms) {
        // src/ggml.c:11428-11478: sum += (double)(x*x); mean = sum/n; y = x * (1/sqrtf(mean+eps))
        const float mean = row_mean_cpu_order<true>(buf, n, shd);
        scale = 1.0f / sqrtf(add_rn(mean, eps));
    } else {
        // src/ggml.c:11353-11406: mean = (float)(sum x / n); v = x - mean; sum2 += (double)(v*v)
        const float mean = row_mean_cpu_order<false>(buf, n, shd);
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) buf[i] = sub_rn(buf[i], mean);
        __syncthreads();
        const float variance = row_mean_cpu_order<true>(buf, n, shd);
        scale = 1.0f / sqrtf(add_rn(variance, eps));
    }
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float v = mul_rn(buf[i], scale);
        if (g) v = mul_rn(v, g[i]);
        if (bias) v = add_rn(v, bias[i]);
        *(float *) (y + i * d.nb[0]) = v;
    }
}

// src/ggml.c:13393-13508: w = x*scale (+ mask); max; val = table_exp[fp16(w - max)] (0 for -inf);
// sum += (double)val; y = val * (float)(1/sum). The vals are fp16 numbers in [0, 1] (multiples of
// 2^-24), so every double partial sum is exact and a tree reduction equals the CPU's chain.
// Optionally fused with the graph's preceding  scale(pre_scale)  and  diag_mask_inf(n_past)
// (n_past < 0: none), applied in the CPU's order before soft_max's own scale.
__global__ __launch_bounds__(256) void k_soft_max(mi_tensor_desc d, mi_tensor_desc a, mi_tensor_desc mask, float scale,
                                                  const uint16_t * exp_table, float pre_scale, int n_past) {
    __shared__ __attribute__((aligned(16))) float lds[kRowLds];
    __shared__ float shf[4];
    __shared__ double shd[4];
    int64_t i1, i2, i3;
    row_coords(blockIdx.x, a.ne, i1, i2, i3);
    const char * x = a.data + off4(a.nb, 0, i1, i2, i3);
    char * y = d.data + off4(d.nb, 0, i1, i2, i3);
    const int64_t n = a.ne[0];
    float * buf = n <= kRowLds ? lds : (float *) y;
    // the mask row is broadcast over rows: (i1 % mask.ne1), as (i1 % ne01) in the reference
    const char * mrow = mask.data ? mask.data + (size_t) (blockIdx.x % a.ne[1]) * mask.nb[1] : nullptr;
    float mx = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float w = *(const float *) (x + i * a.nb[0]);
        if (n_past >= 0) {
            w = mul_rn(w, pre_scale);
            if (i >= n_past && i > n_past + i1) w = -INFINITY;
        }
        w = mul_rn(w, scale);
        if (mrow) w = add_rn(w, ld_f(mrow + i * mask.nb[0], mask.type));  // slope = 1 (max_bias = 0)
        buf[i] = w;
        mx = fmaxf(mx, w);
    }
    mx = block_max_f(mx, shf);  // includes the barrier that publishes buf
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float w = buf[i];
        const float v = w == -INFINITY ? 0.0f : mi_h2f(exp_table[mi_f2h(sub_rn(w, mx))]);
        buf[i] = v;
        s += (double) v;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) shd[threadIdx.x >> 6] = s;
    __syncthreads();
    double sum = 0.0;
    for (int w = 0; w < (int) (blockDim.x >> 6); w++) sum += shd[w];
    const float inv = (float) (1.0 / sum);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) *(float *) (y + i * d.nb[0]) = mul_rn(buf[i], inv);
}

// rope f32 (src/ggml.c:13719-13948), modes 0 (adjacent pairs) and 2 (neox halves), forward.
// One thread per rotated pair. cos/sin come from the backend's host-built table (tab: the
// reference's own running product theta *= theta_scale and the host libm's sincosf, so bit for bit
// the reference CPU's values) for positions 0 <= p < tab_p; otherwise theta follows the same
// running product on the device (each thread replays k multiplications) and cos/sin are rounded
// from double (a correctly rounded libm: within an ulp of the host's). The pair is combined with
// the fmas the reference's -mfma build emits (checked against its outputs): mode 0 fma(x0, cos,
// -(x1 sin)) / fma(x1, cos, x0 sin), NeoX fma(x0, cos, -(x1 sin)) / fma(x0, sin, x1 cos).
struct mi_rope_params {
    int n_dims, mode;
    float freq_scale, ext_factor, attn_factor, theta_scale, inv_ndims, corr0, corr1;
    const float2 * tab;  // [tab_p][pairs] {cos, sin}, or null
    int tab_p;
};

__device__ __forceinline__ void rope_yarn_dev(float theta_extrap, const mi_rope_params & r, int64_t i0, float & c, float & s) {
    const float theta_interp = mul_rn(r.freq_scale, theta_extrap);
    float theta = theta_interp;
    float mscale = r.attn_factor;
    if (r.ext_factor != 0.0f) {
        const float y = ((float) (i0 / 2) - r.corr0) / fmaxf(0.001f, r.corr1 - r.corr0);
        const float ramp_mix = (1.0f - fminf(1.0f, fmaxf(0.0f, y))) * r.ext_factor;
        theta = add_rn(mul_rn(theta_interp, 1.0f - ramp_mix), mul_rn(theta_extrap, ramp_mix));
        mscale *= 1.0f + 0.1f * (float) log(1.0 / (double) r.freq_scale);
    }
    c = mul_rn((float) cos((double) theta), mscale);
    s = mul_rn((float) sin((double) theta), mscale);
}

__global__ __launch_bounds__(256) void k_rope(mi_tensor_desc d, mi_tensor_desc a, const int32_t * pos, mi_rope_params r) {
    const int64_t pairs = a.ne[0] / 2;
    const int64_t nrows = a.ne[1] * a.ne[2] * a.ne[3];
    const int64_t total = pairs * nrows;
    for (int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t) gridDim.x * blockDim.x) {
        const int64_t k = t % pairs;
        int64_t row = t / pairs;
        const int64_t i1 = row % a.ne[1];
        row /= a.ne[1];
        const int64_t i2 = row % a.ne[2];
        const int64_t i3 = row / a.ne[2];
        const float p = (float) pos[i2];
        const char * src = a.data + off4(a.nb, 0, i1, i2, i3);
        char * dst = d.data + off4(d.nb, 0, i1, i2, i3);
        const int32_t pi = pos[i2];
        const bool tabbed = r.tab && pi >= 0 && pi < r.tab_p;
        if (r.mode == 0) {
            float c, s;
            if (tabbed) {
                const float2 cs = r.tab[(int64_t) pi * pairs + k];
                c = cs.x;
                s = cs.y;
            } else {
                float theta = p;
                for (int64_t j = 0; j < k; j++) theta = mul_rn(theta, r.theta_scale);
                rope_yarn_dev(theta, r, 2 * k, c, s);
            }
            const float x0 = *(const float *) (src + 2 * k * a.nb[0]);
            const float x1 = *(const float *) (src + (2 * k + 1) * a.nb[0]);
            *(float *) (dst + 2 * k * d.nb[0]) = __builtin_fmaf(x0, c, -mul_rn(x1, s));
            *(float *) (dst + (2 * k + 1) * d.nb[0]) = __builtin_fmaf(x1, c, mul_rn(x0, s));
        } else {
            const int64_t ic = 2 * k;
            if (ic < r.n_dims) {
                float c, s;
                if (tabbed) {
                    const float2 cs = r.tab[(int64_t) pi * (r.n_dims / 2) + k];
                    c = cs.x;
                    s = cs.y;
                } else {
                    float theta = mul_rn(p, r.freq_scale);
                    for (int64_t j = 0; j < k; j++) theta = mul_rn(theta, r.theta_scale);
                    const float cur_rot = mul_rn(r.inv_ndims, (float) ic);
                    rope_yarn_dev(theta, r, (int64_t) cur_rot, c, s);
                }
                const int64_t i0 = ic / 2;
                const int64_t h = r.n_dims / 2;
                const float x0 = *(const float *) (src + i0 * a.nb[0]);
                const float x1 = *(const float *) (src + (i0 + h) * a.nb[0]);
                *(float *) (dst + i0 * d.nb[0]) = __builtin_fmaf(x0, c, -mul_rn(x1, s));
                *(float *) (dst + (i0 + h) * d.nb[0]) = __builtin_fmaf(x0, s, mul_rn(x1, c));
            } else {
                *(float *) (dst + ic * d.nb[0]) = *(const float *) (src + ic * a.nb[0]);
                *(float *) (dst + (ic + 1) * d.nb[0]) = *(const float *) (src + (ic + 1) * a.nb[0]);
            }
        }
    }
}

unsigned grid_for(int64_t n) {
    if (n >= (int64_t) 1 << 32) abort();  // element-wise kernels index with 32 bits
    int64_t g = (n + 255) / 256;
    return (unsigned) (g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

} // namespace

void mi_op_binary(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & b, int op, hipStream_t s) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_binary, dim3(grid_for(n)), dim3(256), 0, s, d, a, b, op, n);
}

void mi_op_unary(const mi_tensor_desc & d, const mi_tensor_desc & a, int op, float p0, const uint16_t * table, hipStream_t s) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_unary, dim3(grid_for(n)), dim3(256), 0, s, d, a, op, p0, table, n);
}

void mi_op_cpy(const mi_tensor_desc & d, const mi_tensor_desc & a, hipStream_t s) {
    const int64_t n = a.ne[0] * a.ne[1] * a.ne[2] * a.ne[3];
    hipLaunchKernelGGL(k_cpy, dim3(grid_for(n)), dim3(256), 0, s, d, a, n);
}

void mi_op_get_rows(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & idx, hipStream_t s) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    switch (a.type) {
        case 2: hipLaunchKernelGGL(k_get_rows_q<2>, dim3(grid_for(n)), dim3(256), 0, s, d, a, idx, n); break;
        case 8: hipLaunchKernelGGL(k_get_rows_q<8>, dim3(grid_for(n)), dim3(256), 0, s, d, a, idx, n); break;
        case 12: hipLaunchKernelGGL(k_get_rows_q<12>, dim3(grid_for(n)), dim3(256), 0, s, d, a, idx, n); break;
        case 13: hipLaunchKernelGGL(k_get_rows_q<13>, dim3(grid_for(n)), dim3(256), 0, s, d, a, idx, n); break;
        default: hipLaunchKernelGGL(k_get_rows, dim3(grid_for(n)), dim3(256), 0, s, d, a, idx, n); break;
    }
}

template <int TA>
static void launch_get_rows_add(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & ia, const mi_tensor_desc & b,
                                const mi_tensor_desc & ib, int64_t n, hipStream_t s) {
    (void) n;
    if (d.ne[0] >= ((int64_t) 1 << 31)) abort();  // row length indexed with 32 bits (never an embedding)
    const int ne0 = (int) d.ne[0];
    // grid.y is at most 65535 rows: longer index vectors in chunks (descriptors advanced by rows)
    for (int64_t r0 = 0; r0 < d.ne[1]; r0 += 65535) {
        const int64_t nr = std::min<int64_t>(65535, d.ne[1] - r0);
        mi_tensor_desc dc = d, iac = ia, ibc = ib;
        dc.data += r0 * d.nb[1];
        iac.data += r0 * ia.nb[0];
        ibc.data += r0 * ib.nb[0];
        dc.ne[1] = nr;
        const dim3 g((unsigned) std::min<int64_t>((ne0 + 1023) / 1024, 64), (unsigned) nr);
        uint64_t * st = mi_stamp_take("k_get_rows_add", g.x * g.y);
        switch (b.type) {
            case 2: hipLaunchKernelGGL((k_get_rows_add<TA, 2>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
            case 8: hipLaunchKernelGGL((k_get_rows_add<TA, 8>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
            case 12: hipLaunchKernelGGL((k_get_rows_add<TA, 12>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
            case 13: hipLaunchKernelGGL((k_get_rows_add<TA, 13>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
            case 1: hipLaunchKernelGGL((k_get_rows_add<TA, 1>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
            default: hipLaunchKernelGGL((k_get_rows_add<TA, 0>), g, dim3(256), 0, s, dc, a, iac, b, ibc, ne0, st); break;
        }
    }
}

void mi_op_get_rows_add(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & ia, const mi_tensor_desc & b,
                        const mi_tensor_desc & ib, hipStream_t s) {
    const int64_t n = d.ne[0] * d.ne[1];
    switch (a.type) {
        case 2: launch_get_rows_add<2>(d, a, ia, b, ib, n, s); break;
        case 8: launch_get_rows_add<8>(d, a, ia, b, ib, n, s); break;
        case 12: launch_get_rows_add<12>(d, a, ia, b, ib, n, s); break;
        case 13: launch_get_rows_add<13>(d, a, ia, b, ib, n, s); break;
        case 1: launch_get_rows_add<1>(d, a, ia, b, ib, n, s); break;
        default: launch_get_rows_add<0>(d, a, ia, b, ib, n, s); break;
    }
}

void mi_op_diag_mask(const mi_tensor_desc & d, const mi_tensor_desc & a, int n_past, float value, hipStream_t s) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_diag_mask, dim3(grid_for(n)), dim3(256), 0, s, d, a, n_past, value, n);
}

void mi_op_norm(const mi_tensor_desc & d, const mi_tensor_desc & a, float eps, bool rms, const float * g, const float * b,
                hipStream_t s) {
    const int64_t rows = a.ne[1] * a.ne[2] * a.ne[3];
    hipLaunchKernelGGL(k_norm, dim3((unsigned) rows), dim3(256), 0, s, d, a, eps, rms ? 1 : 0, g, b);
}

void mi_op_soft_max(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & mask, float scale,
                    const uint16_t * exp_table, float pre_scale, int n_past, hipStream_t s) {
    const int64_t rows = a.ne[1] * a.ne[2] * a.ne[3];
    hipLaunchKernelGGL(k_soft_max, dim3((unsigned) rows), dim3(256), 0, s, d, a, mask, scale, exp_table, pre_scale, n_past);
}

void mi_op_rope(const mi_tensor_desc & d, const mi_tensor_desc & a, const int32_t * pos, int n_dims, int mode, float freq_base,
                float freq_scale, float ext_factor, float attn_factor, float corr0, float corr1, const float * tab, int tab_p,
                hipStream_t s) {
    mi_rope_params r;
    r.tab = (const float2 *) tab;
    r.tab_p = tab ? tab_p : 0;
    r.n_dims = n_dims;
    r.mode = mode;
    r.freq_scale = freq_scale;
    r.ext_factor = ext_factor;
    r.attn_factor = attn_factor;
    r.theta_scale = powf(freq_base, -2.0f / n_dims);
    r.inv_ndims = -1.f / n_dims;
    r.corr0 = corr0;
    r.corr1 = corr1;
    const int64_t n = a.ne[0] / 2 * a.ne[1] * a.ne[2] * a.ne[3];
    hipLaunchKernelGGL(k_rope, dim3(grid_for(n)), dim3(256), 0, s, d, a, pos, r);
}

void mi_op_cpy_multi(const mi_tensor_desc * d, const mi_tensor_desc * a, int count, hipStream_t s) {
    mi_cpy_batch b;
    int64_t nmax = 1;
    for (int c = 0; c < count; c++) {
        b.d[c] = d[c];
        b.a[c] = a[c];
        b.n[c] = a[c].ne[0] * a[c].ne[1] * a[c].ne[2] * a[c].ne[3];
        nmax = b.n[c] > nmax ? b.n[c] : nmax;
    }
    hipLaunchKernelGGL(k_cpy_multi, dim3(grid_for(nmax), (unsigned) count), dim3(256), 0, s, b);
}
