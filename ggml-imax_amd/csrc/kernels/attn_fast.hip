// attn_fast.hip -- the attention block of the GPT-2 graph (KQ, scale, causal mask, soft_max, KQV,
// head merge; examples/gpt-2/main-backend.cpp:552-608) in tree order: the fast decode mode
// (mmv_order 0). mmv_ordered.hip's k_attn_fast / k_attn_ordered replay the reference CPU's exact
// summation order (mmv_order 1).
//
// What is kept from the reference: the scores are (q . k) * pre_scale (ggml_scale) masked to -inf
// past n_past + t (diag_mask_inf) times the soft_max scale; the soft_max weights are the
// reference's fp16 values exp(f16(s - max)) rounded to fp16 (ggml_compute_forward_soft_max_f32
// reads them from ggml_table_exp_f16, src/ggml.c:12196-12260: here computed with expf and rounded
// the same way, equal to the table entry except where expf and the host's expf straddle an fp16
// rounding boundary). What differs: every sum is an f32 tree (dots, the soft_max denominator and
// the KQV sums) and the KQV weights are applied unnormalized, the 1 / sum scaling once at the end.
//
// One workgroup (8 waves) per (head, query token). A key is handled by D / 8 lanes (8 head-dim
// elements each, 2 x 16-byte loads per row), 64 keys per pass of the workgroup; the K and V rows
// of the first 64 * KPG keys are all requested before any arithmetic. Pass 1: scores (kept in
// LDS) and the workgroup max (one barrier); pass 2: p = exp weights, unnormalized sum p * v per
// lane, then the waves' partial (sum p, sum p v) are added through LDS (one barrier).

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#pragma clang fp contract(off)

namespace {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int LPK>
__device__ __forceinline__ float group_sum(float v) {  // sum over each aligned group of LPK lanes
#pragma unroll
    for (int off = 1; off < LPK; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// One (head h, query token t) of the block by the workgroup's 8 waves. D: head dim (64 or 128);
// KPG: keys per lane group held in registers per pass. sm: LDS of n_kv + 8 (D + 8) floats.
// Returns, in threads d < D, element d of the head's output (num / den); other threads return 0.
template <int D, int KPG>
// st (diagnostic builds): phase stamps of the calling workgroup -- slot 2 the first chunk scored
// (q and the first K rows landed), 3 the max known (first barrier), 4 the p.v sums done
__device__ __forceinline__ float attn_head(const mi_attn_desc & a, int h, int t, float * sm, float * shm, uint64_t * st = nullptr) {
    constexpr int LPK = D / 8;          // lanes per key
    constexpr int GPW = 64 / LPK;       // key groups per wave
    constexpr int G = 8 * GPW;          // key groups per workgroup
    constexpr int CH = G * KPG;         // keys per pass
    const int hk = h / a.r2;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = lane % LPK;                       // 8-element slice of the head dim
    const int grp = wave * GPW + lane / LPK;        // key group of the workgroup
    const int n_kv = a.n_kv;
    float * s = sm;

    // q slice (8 floats), and the first pass's K and V rows, all requested up front
    const char * qrow = a.q + (size_t) t * a.q_nb[1] + (size_t) h * a.q_nb[2] + (size_t) j * 32;
    const float4 q0 = *(const float4 *) qrow, q1 = *(const float4 *) (qrow + 16);
    const char * kb = a.k + (size_t) hk * a.k_nb[2] + (size_t) j * 32;
    const char * vb = a.v + (size_t) hk * a.v_nb[2] + (size_t) j * 32;
    float4 kr[KPG][2], vr[KPG][2];
    auto load_rows = [&](const char * base, size_t nb, int c0, float4 (&r)[KPG][2]) {
#pragma unroll
        for (int kk = 0; kk < KPG; kk++) {
            const int key = min(c0 + kk * G + grp, n_kv - 1);  // clamped: unconditional loads
            const char * p = base + (size_t) key * nb;
            r[kk][0] = *(const float4 *) p;
            r[kk][1] = *(const float4 *) (p + 16);
        }
    };
    // KQ mask row (batched decode): its values for a chunk's keys requested with the chunk's K
    // rows, unconditionally from a valid address (K itself when there is no mask: n_kv floats of
    // it are readable) -- a load under a branch, or one issued next to its use, is waited for at
    // once; the values are used only with a mask
    const bool use_mask = a.mask != nullptr;
    const float * mrow = use_mask ? (const float *) (a.mask + (size_t) t * a.mask_nb1) : (const float *) a.k;
    float mk[KPG];
    auto load_mask = [&](int c0) {
#pragma unroll
        for (int kk = 0; kk < KPG; kk++) mk[kk] = mrow[min(c0 + kk * G + grp, n_kv - 1)];
    };
    load_rows(kb, a.k_nb[1], 0, kr);
    load_mask(0);
    load_rows(vb, a.v_nb[0], 0, vr);

    // ---- pass 1: scores and their max
    const int lim = a.n_past + t;  // keys k > lim are masked (diag_mask_inf)
    float mx = -INFINITY;
    for (int c0 = 0; c0 < n_kv; c0 += CH) {
        if (c0) {
            load_rows(kb, a.k_nb[1], c0, kr);
            load_mask(c0);
        }
#pragma unroll
        for (int kk = 0; kk < KPG; kk++) {
            float d = kr[kk][0].x * q0.x + kr[kk][0].y * q0.y + kr[kk][0].z * q0.z + kr[kk][0].w * q0.w +
                      (kr[kk][1].x * q1.x + kr[kk][1].y * q1.y + kr[kk][1].z * q1.z + kr[kk][1].w * q1.w);
            d = group_sum<LPK>(d);
            const int key = c0 + kk * G + grp;
            float w = d * a.pre_scale;
            if (use_mask) w = w + mk[kk];
            if (key >= a.n_past && key > lim) w = -INFINITY;
            w = w * a.sm_scale;
            if (key < n_kv) {
                mx = fmaxf(mx, w);
                if (j == 0) s[key] = w;
            }
        }
        if (c0 == 0) MI_STAMP(st, 2);
    }
    mx = mi_wave_max(mx);
    if (lane == 0) shm[wave] = mx;
    __syncthreads();  // s[] and shm[] complete
    MI_STAMP(st, 3);
    mx = shm[0];
#pragma unroll
    for (int w = 1; w < 8; w++) mx = fmaxf(mx, shm[w]);

    // ---- pass 2: p = fp16 exp(fp16(s - max)), unnormalized sums of p and p * v
    float l = 0.0f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < n_kv; c0 += CH) {
        if (c0) load_rows(vb, a.v_nb[0], c0, vr);
#pragma unroll
        for (int kk = 0; kk < KPG; kk++) {
            const int key = c0 + kk * G + grp;
            if (key < n_kv) {
                const float w = s[key];
                const float p = w == -INFINITY ? 0.0f : mi_h2f(mi_f2h(expf(mi_h2f(mi_f2h(w - mx)))));
                if (j == 0) l += p;
                o[0] += p * vr[kk][0].x; o[1] += p * vr[kk][0].y; o[2] += p * vr[kk][0].z; o[3] += p * vr[kk][0].w;
                o[4] += p * vr[kk][1].x; o[5] += p * vr[kk][1].y; o[6] += p * vr[kk][1].z; o[7] += p * vr[kk][1].w;
            }
        }
    }
    // the wave's groups: lanes of equal j hold the same head-dim slice
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
        l += __shfl_xor(l, off, 64);
#pragma unroll
        for (int e = 0; e < 8; e++) o[e] += __shfl_xor(o[e], off, 64);
    }
    MI_STAMP(st, 4);
    l = group_sum<LPK>(l);  // only lane j == 0 of each group accumulated l
    float * red = sm + n_kv;  // [8 waves][D + 8]: o slices, then l at [D]
    if (lane < LPK) {
        float * r = red + wave * (D + 8) + lane * 8;
#pragma unroll
        for (int e = 0; e < 8; e++) r[e] = o[e];
        if (lane == 0) red[wave * (D + 8) + D] = l;
    }
    __syncthreads();
    float res = 0.0f;
    if (threadIdx.x < D) {
        const int d = threadIdx.x;
        float num = red[d], den = red[D];
#pragma unroll
        for (int w = 1; w < 8; w++) {
            num += red[w * (D + 8) + d];
            den += red[w * (D + 8) + D];
        }
        res = num / den;
    }
    return res;
}

template <int D, int KPG>
__global__ __launch_bounds__(512) void k_attn_tree(mi_attn_desc a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // s[n_kv] | red[8][D + 8]
    __shared__ float shm[8];
    const int h = blockIdx.x, t = blockIdx.y;
    const float r = attn_head<D, KPG>(a, h, t, sm, shm);
    if (threadIdx.x < D)
        *(float *) (a.out + (size_t) threadIdx.x * a.o_nb[0] + (size_t) t * a.o_nb[1] + (size_t) h * a.o_nb[2]) = r;
}

// Attention of one decode token fused with the output projection that consumes it (GPT-2's
// c_proj, main-backend.cpp:610-620): workgroup (row block rb, head h) computes head h's output
// (attn_head; rounded to f16, as the F16 GEMV rounds its activations), then the partial product
// of rows rb * RPW .. + RPW of W over that head's D input columns: part[h][row]. Head 0 adds the
// bias and the residual (the graph's two ADDs), so that sum_h part[h] (in head order) is the
// projection's final output; the consumer (mi_sum_parts, or the next GEMV's norm prologue) adds
// the H partials. Each workgroup of a head repeats that head's attention (K/V rows from L2).
// Weights: D / 8 lanes per row, one 16-byte chunk each, requested before the attention.
template <int D, int KPG, bool XF>
__global__ __launch_bounds__(512) void k_attn_proj(mi_attn_desc a, mi_attn_proj_desc p) {
    constexpr int LPR = D / 8;           // lanes per weight row
    constexpr int RPW = 512 / LPR;       // rows per workgroup
    extern __shared__ __attribute__((aligned(16))) float sm[];  // s[n_kv] | red[8][D + 8] | (16 B aligned) oh[D] f16
    __shared__ float shm[8];
    MI_STAMP(p.stamps, 0);
    MI_STAMP_CLK(p.stamps, 6);
    const int rb = blockIdx.x, h = blockIdx.y;
    const int c = threadIdx.x % LPR;
    const int64_t row = (int64_t) rb * RPW + threadIdx.x / LPR;
    const int64_t rc = row < p.N ? row : p.N - 1;
    // the projection's weights: requested before the attention (their latency hidden under it), or
    // with xfirst after it, so that the attention's q / K / V loads do not queue behind them
    const uint8_t * wp = p.W + rc * p.nb01 + ((size_t) h * D + c * 8) * 2;
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (!XF) w = *(const uint4 *) wp;
    const float e_bias = p.bias[rc], e_res = p.resid[rc];  // requested before the attention too
    const float r = attn_head<D, KPG>(a, h, 0, sm, shm, p.stamps);
    if constexpr (XF) w = *(const uint4 *) wp;
    MI_STAMP(p.stamps, 1);  // the head's attention done
    uint16_t * oh = (uint16_t *) (sm + ((a.n_kv + 3) & ~3) + 8 * (D + 8));  // 16-byte aligned
    if (threadIdx.x < D) oh[threadIdx.x] = mi_f2h(r);
    __syncthreads();
    const uint4 x = *(const uint4 *) (oh + c * 8);
    float acc = 0.0f;
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.x), __builtin_bit_cast(f16x2, x.x), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.y), __builtin_bit_cast(f16x2, x.y), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.z), __builtin_bit_cast(f16x2, x.z), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.w), __builtin_bit_cast(f16x2, x.w), acc, false);
    acc = group_sum<LPR>(acc);
    // head 0: (x + bias) + resid, the order of the unfused epilogue
    if (c == 0 && row < p.N) p.parts[(size_t) h * p.N + row] = h == 0 ? (acc + e_bias) + e_res : acc;
    MI_STAMP_CLK(p.stamps, 5);
    MI_STAMP(p.stamps, 7);
}

// out[i] = sum_h parts[h][i], in head order
__global__ void k_sum_parts(float * __restrict__ out, const float * __restrict__ parts, int nparts, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = parts[i];
    for (int h = 1; h < nparts; h++) v += parts[(size_t) h * n + i];
    out[i] = v;
}

} // namespace

bool mi_attn_tree_supported(const mi_attn_desc & a) {
    return (a.D == 64 || a.D == 128) && a.n_kv >= 1 && a.q_nb[0] == 4 && a.k_nb[0] == 4 && a.v_nb[1] == 4 &&
           ((uintptr_t) a.q | (uintptr_t) a.k | (uintptr_t) a.v | a.q_nb[1] | a.q_nb[2] | a.k_nb[1] | a.k_nb[2] | a.v_nb[0] |
            a.v_nb[2]) % 16 == 0 &&
           (size_t) (a.n_kv + 8 * (a.D + 8)) * 4 <= 64 * 1024;
}

void mi_attn_tree(const mi_attn_desc & a, hipStream_t s) {
    const dim3 grid((unsigned) a.H, (unsigned) a.N);
    const size_t lds = (size_t) (a.n_kv + 8 * (a.D + 8)) * sizeof(float);
    if (a.D == 64) {
        if (a.n_kv <= 256) hipLaunchKernelGGL((k_attn_tree<64, 4>), grid, dim3(512), lds, s, a);
        else hipLaunchKernelGGL((k_attn_tree<64, 8>), grid, dim3(512), lds, s, a);
    } else {
        hipLaunchKernelGGL((k_attn_tree<128, 4>), grid, dim3(512), lds, s, a);
    }
}

bool mi_attn_proj_supported(const mi_attn_desc & a, int64_t K, int64_t N, size_t nb01, const void * W) {
    return a.D == 64 && a.N == 1 && mi_attn_tree_supported(a) && K == (int64_t) a.D * a.H && N >= 1 && N <= (1 << 20) &&
           nb01 % 16 == 0 && (uintptr_t) W % 16 == 0 && (size_t) (a.n_kv + 3 + 8 * (a.D + 8) + a.D) * 4 <= 64 * 1024;
}

void mi_attn_proj(const mi_attn_desc & a, const mi_attn_proj_desc & p, hipStream_t s) {
    constexpr int RPW = 512 / (64 / 8);
    const dim3 grid((unsigned) ((p.N + RPW - 1) / RPW), (unsigned) a.H);
    const size_t lds = (size_t) (a.n_kv + 3 + 8 * (a.D + 8) + a.D) * sizeof(float);
    mi_attn_proj_desc ps = p;
    ps.stamps = mi_stamp_take("k_attn_proj", grid.x * grid.y);
    if (g_mi_tuning.xfirst == 1) {  // (off by default, as the F16 GEMVs)
        if (a.n_kv <= 256) hipLaunchKernelGGL((k_attn_proj<64, 4, true>), grid, dim3(512), lds, s, a, ps);
        else hipLaunchKernelGGL((k_attn_proj<64, 8, true>), grid, dim3(512), lds, s, a, ps);
    } else {
        if (a.n_kv <= 256) hipLaunchKernelGGL((k_attn_proj<64, 4, false>), grid, dim3(512), lds, s, a, ps);
        else hipLaunchKernelGGL((k_attn_proj<64, 8, false>), grid, dim3(512), lds, s, a, ps);
    }
}

void mi_sum_parts(float * out, const float * parts, int nparts, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_parts, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, out, parts, nparts, n);
}
