// mmv_f16.hip -- decode-regime F16 mul_mat (GEMV, up to 8 columns) in tree order: the fast mode of
// the F16 decode path (mmv_order 0; mmv_ordered.hip's kernels replay the reference CPU's exact
// summation order, mmv_order 1).
//
// Same contract as mi_mul_mat_f16_fused (mi355x_kernels.h): the activations are rounded to f16 as
// the reference's vec_dot_type conversion does (ggml_fp32_to_fp16_row, src/ggml.c:610-612,
// RNE), optionally produced by the graph's norm -> mul(g) -> add(b) chain computed in the kernel
// (ggml_compute_forward_norm_f32 / rms_norm, src/ggml.c:10950-11050), and the graph's following
// bias / residual / GELU nodes and K/V row copies are applied in the store. What differs from the
// reference is only the order of the f32 sums (products of two halves are exact in f32; lane
// partial sums + a 16-lane tree instead of ggml_vec_dot_f16's 32 AVX partial sums + the
// GGML_F32x8_REDUCE tree, src/ggml.c:1680-1720), and the norm's sums (f32 tree instead of a
// sequential double), ~1e-7 relative per dot.
//
// Geometry (wave64): 16 lanes per weight row, four rows per wave, one to four waves per
// workgroup. Lane m of a row reads the row's 16-byte chunks m, m + 16, ... (a wave-instruction
// covers 4 rows x 256 contiguous bytes), every chunk of the row requested before the first
// v_dot2_f32_f16 when the row fits the register batch (K <= 3072), else a two-deep ring of
// 8-chunk batches. Activations: f16 columns staged once per workgroup in LDS (read back as
// 16-byte broadcast reads shared by the wave's four rows). Roofline: HBM (2*K bytes per row);
// GPT-2's matrices are 1.2-4.7 MB, so a launch is latency- not bandwidth-bound, and the lever is
// having every row of the matrix in flight at once (>= N/4 waves).

#include <algorithm>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#pragma clang fp contract(off)

namespace {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr int kLpr = 16;          // lanes per weight row
constexpr int kChunk = 8;         // f16 per lane per chunk (16 bytes)
constexpr int kKStep = kLpr * kChunk;  // K covered by one chunk step of a row (128)

__device__ __forceinline__ float dot8(const uint4 & w, const uint4 & x, float acc) {
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.x), __builtin_bit_cast(f16x2, x.x), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.y), __builtin_bit_cast(f16x2, x.y), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.z), __builtin_bit_cast(f16x2, x.z), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w.w), __builtin_bit_cast(f16x2, x.w), acc, false);
    return acc;
}

// zero a weight chunk past the row's end at its use, not at its load: a select right after the
// load was compiled into a branch whose register writes wait for the load (vmcnt(0)), which
// serialised the prologue's loads (k_gemv_f16_ps: one full memory round trip per chunk past nit)
__device__ __forceinline__ uint4 keep_if(bool keep, const uint4 & v) {
    return keep ? v : make_uint4(0u, 0u, 0u, 0u);
}

// sum over each aligned 16-lane row; every lane of the row gets it
__device__ __forceinline__ float row16_sum(float v) {
    auto f = [](int x) { return __int_as_float(x); };
    auto i = [](float x) { return __float_as_int(x); };
    v += f(mi_dpp<MI_DPP_QP_1032>(0, i(v)));
    v += f(mi_dpp<MI_DPP_QP_2301>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, i(v)));
    v += f(mi_dpp<MI_DPP_ROW_MIRROR>(0, i(v)));
    return v;
}

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
    return (uint32_t) mi_f2h(a) | ((uint32_t) mi_f2h(b) << 16);
}

// The graph's norm|rms_norm -> mul(g) -> add(b) of one column, by one wave, into f16 LDS (xs,
// padded with zeros to kp): lane l holds elements 256 j + 4 l .. + 3 (j < JM) in registers, and
// (GB) the g / b values of the same elements.
template <int JM, bool GB>
__device__ __forceinline__ void norm_load(const float * __restrict__ xc, int64_t K, int lane, const mi_norm_prologue & pro,
                                          float4 (&v)[JM], float4 (&g)[GB ? JM : 1], float4 (&bb)[GB ? JM : 1]) {
#pragma unroll
    for (int j = 0; j < JM; j++) {
        // unconditional loads at clamped addresses + selects: a load under a lane branch makes
        // the compiler wait for it at the branch's join (vmcnt(0)), serialising every load
        const int64_t k = (int64_t) j * 256 + lane * 4;
        const int64_t kc = k < K ? k : K - 4;
        v[j] = *(const float4 *) (xc + kc);  // (zeroed past K in norm_store, at use)
        if constexpr (GB) {
            // absent g / b: the load reads x instead (valid address, no branch), the value is
            // not used (norm_store checks pro.g / pro.b)
            g[j] = *(const float4 *) ((pro.g ? pro.g : xc) + kc);
            bb[j] = *(const float4 *) ((pro.b ? pro.b : xc) + kc);
        }
    }
}

template <int JM, bool GB>
__device__ __forceinline__ void norm_store(float4 (&v)[JM], const float4 (&g)[GB ? JM : 1], const float4 (&bb)[GB ? JM : 1], int64_t K,
                                           int64_t kp, const mi_norm_prologue & pro, uint16_t * xs, int lane) {
    const float fk = (float) K;
#pragma unroll
    for (int j = 0; j < JM; j++)  // elements past K (clamped loads) are zero
        if ((int64_t) j * 256 + lane * 4 >= K) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    float scale;
    if (pro.mode == 2) {
        float s2 = 0.0f;
#pragma unroll
        for (int j = 0; j < JM; j++) s2 += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
        scale = 1.0f / sqrtf(mi_wave_sum_u(s2) / fk + pro.eps);
    } else {
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < JM; j++) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
        const float mean = mi_wave_sum_u(s) / fk;
        float s2 = 0.0f;
#pragma unroll
        for (int j = 0; j < JM; j++) {
            const int64_t k = (int64_t) j * 256 + lane * 4;
            if (k < K) {
                v[j].x -= mean; v[j].y -= mean; v[j].z -= mean; v[j].w -= mean;
                s2 += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
            }
        }
        scale = 1.0f / sqrtf(mi_wave_sum_u(s2) / fk + pro.eps);
    }
#pragma unroll
    for (int j = 0; j < JM; j++) {
        const int64_t k = (int64_t) j * 256 + lane * 4;
        if (k < kp) {
            uint2 h = make_uint2(0u, 0u);
            if (k < K) {
                float y[4] = {v[j].x * scale, v[j].y * scale, v[j].z * scale, v[j].w * scale};
                float4 gg, bv;
                if constexpr (GB) {
                    gg = g[j];
                    bv = bb[j];
                } else {
                    gg = pro.g ? *(const float4 *) (pro.g + k) : make_float4(1.f, 1.f, 1.f, 1.f);
                    bv = pro.b ? *(const float4 *) (pro.b + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                if (pro.g) { y[0] *= gg.x; y[1] *= gg.y; y[2] *= gg.z; y[3] *= gg.w; }
                if (pro.b) { y[0] += bv.x; y[1] += bv.y; y[2] += bv.z; y[3] += bv.w; }
                h = make_uint2(pack_h2(y[0], y[1]), pack_h2(y[2], y[3]));
            }
            *(uint2 *) (xs + k) = h;
        }
    }
}

// f32 activation column -> f16 LDS (zero-padded to kp), JX float4 per thread per round, all of a
// round's loads in flight together
template <int JX>
struct ColStager {
    float4 v[JX];
    int64_t kk = 0;  // K of the last load
    __device__ __forceinline__ void load(const float * __restrict__ xc, int64_t K, int64_t base) {
#pragma unroll
        for (int j = 0; j < JX; j++) {
            const int64_t i = base + (int64_t) j * blockDim.x + threadIdx.x;  // float4 index
            // branch-free (see norm_load); past K zeroed at the store: a select right after the
            // load became a branch that waited for it (vmcnt(0) per load)
            v[j] = *(const float4 *) (xc + (i * 4 < K ? i * 4 : K - 4));
        }
        kk = K;
    }
    __device__ __forceinline__ void store(uint16_t * xd, int64_t kp, int64_t base) {
#pragma unroll
        for (int j = 0; j < JX; j++) {
            const int64_t i = base + (int64_t) j * blockDim.x + threadIdx.x;
            const float4 w = i * 4 < kk ? v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (i * 4 < kp) *(uint2 *) (xd + i * 4) = make_uint2(pack_h2(w.x, w.y), pack_h2(w.z, w.w));
        }
    }
    __device__ __forceinline__ void column(const float * __restrict__ xc, int64_t K, int64_t kp, uint16_t * xd, int64_t from) {
        // rounds pipelined (as stage_cols): the next round requested before this one is stored
        const int64_t step = (int64_t) JX * blockDim.x;
        if (from >= kp / 4) return;
        load(xc, K, from);
        for (int64_t base = from; base < kp / 4; base += step) {
            float4 cur[JX];
#pragma unroll
            for (int j = 0; j < JX; j++) cur[j] = v[j];
            if (base + step < kp / 4) load(xc, K, base + step);
#pragma unroll
            for (int j = 0; j < JX; j++) {
                const int64_t i = base + (int64_t) j * blockDim.x + threadIdx.x;
                const float4 w = i * 4 < kk ? cur[j] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (i * 4 < kp) *(uint2 *) (xd + i * 4) = make_uint2(pack_h2(w.x, w.y), pack_h2(w.z, w.w));
            }
        }
    }
};

// Several f32 activation columns -> f16 LDS (each zero-padded to kp), rounds of JX float4 per thread
// over the flattened [nc][K / 4] index space, every load of a round in flight together (a column
// per round costs a dependent memory round trip per column)
template <int JX>
__device__ __forceinline__ void stage_cols(const mi_src_cols & x, int64_t c0, int nc, int64_t K, int64_t kp, uint16_t * xs) {
    const int64_t k4 = K / 4, total = (int64_t) nc * k4;
    if (nc <= 8 && k4 <= 2 * (int64_t) blockDim.x) {
        // every (column, float4) of the thread requested at once -- up to 8 columns x 2 float4 --
        // with no index division (the flattened form below divides a 64-bit index by K / 4 twice
        // per element: GPT-2's 8-column MLP projection spent 4.2 us staging its 96 KB)
        const int tid = (int) threadIdx.x, nt = (int) blockDim.x, k4i = (int) k4;
        float4 v[8][2];
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int q = tid + j * nt;
                const char * col = x.base + (c0 + (c < nc ? c : nc - 1)) * x.nb1;
                v[c][j] = *(const float4 *) (col + (size_t) (q < k4i ? q : k4i - 1) * 16);
            }
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int q = tid + j * nt;
                if (c < nc && q < k4i)
                    *(uint2 *) (xs + (size_t) c * kp + (size_t) q * 4) = make_uint2(pack_h2(v[c][j].x, v[c][j].y), pack_h2(v[c][j].z, v[c][j].w));
            }
        if (kp > K) {
            const int pad = (int) (kp - K);
            for (int i = tid; i < nc * pad; i += nt) xs[(size_t) (i / pad) * kp + K + (i % pad)] = 0;
        }
        return;
    }
    const int64_t step = (int64_t) JX * blockDim.x;
    auto load = [&](float4 (&v)[JX], int64_t base) {
#pragma unroll
        for (int j = 0; j < JX; j++) {
            const int64_t i = base + (int64_t) j * blockDim.x + threadIdx.x;
            const int64_t ic = i < total ? i : total - 1;  // branch-free loads (see norm_load)
            const int64_t c = ic / k4, q = ic - c * k4;
            v[j] = *(const float4 *) (x.base + (c0 + c) * x.nb1 + q * 16);
        }
    };
    // rounds pipelined: the next round's loads are requested before this round is converted and
    // stored, so the rounds cost about one memory round trip instead of one each
    float4 v[JX], nv[JX];
    load(v, 0);
    for (int64_t base = 0; base < total; base += step) {
        if (base + step < total) load(nv, base + step);
#pragma unroll
        for (int j = 0; j < JX; j++) {
            const int64_t i = base + (int64_t) j * blockDim.x + threadIdx.x;
            if (i < total) {
                const int64_t c = i / k4, q = i - c * k4;
                *(uint2 *) (xs + c * kp + q * 4) = make_uint2(pack_h2(v[j].x, v[j].y), pack_h2(v[j].z, v[j].w));
            }
        }
#pragma unroll
        for (int j = 0; j < JX; j++) v[j] = nv[j];
    }
    for (int64_t i = threadIdx.x; i < (int64_t) nc * (kp - K); i += blockDim.x) {
        const int64_t c = i / (kp - K);
        xs[c * kp + K + (i - c * (kp - K))] = 0;
    }
}

// One workgroup = RGS row groups of 4 weight rows (16 lanes per row) x KS waves per group
// (runtime: KS = blockDim.x / 64 / RGS); a group's waves split the rows' 128-wide K steps: wave
// s of the group takes steps s, s + KS, ... -- at most U of them in registers when ONE, else a
// two-deep ring of U-step batches -- and the KS partial sums of a (row, column) are added in wave
// order through LDS. JM: register depth of the norm prologue (K <= 256 JM), 0 = no prologue.
// Many small waves rather than few long ones: a decode matrix is 1-5 MB, so what bounds a launch
// is how many rows' bytes are in flight at once; several row groups per workgroup only for very
// tall matrices (lm_head), where the per-workgroup staging of the activations would otherwise
// cost more L2 traffic than the weights.
template <int NC, int EPI, int U, bool ONE, int JM, bool XH = false>
__global__ __launch_bounds__(512) void k_gemv_f16(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                  mi_src_cols x, const uint16_t * __restrict__ xh, int64_t ncols,
                                                  float * __restrict__ dst, size_t ycol, mi_f16_epilogue e, mi_norm_prologue pro,
                                                  int64_t kp, int rgs) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [NC][kp] f16 (zero beyond K), then [waves][4][NC] f32
    MI_STAMP(e.stamps, 0);
    MI_STAMP_CLK(e.stamps, 6);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x >> 6) / rgs;
    const int grp = wid / nw, wave = wid % nw;  // row group, K slice
    const int m = lane & (kLpr - 1), rg = lane >> 4;
    const int64_t row = ((int64_t) blockIdx.x * rgs + grp) * 4 + rg;
    const bool live = row < N;
    const int64_t c0 = (int64_t) blockIdx.y * NC;
    const int nc = (int) std::min<int64_t>(NC, ncols - c0);
    const int nit = (int) ((K + kKStep - 1) / kKStep);   // K steps of a row (host: nw <= nit)
    const int nj = (nit - wave + nw - 1) / nw;            // this wave's steps
    const int64_t k8 = K / kChunk;  // whole 16-byte chunks of the row (K % 8 == 0)

    const uint8_t * wrow = W + (live ? row : 0) * nb01;
    // this wave's j-th step; branch-free (see norm_load): clamped address, then zero past the row
    auto ld = [&](int j) -> uint4 {
        const int it = wave + (j < nj ? j : nj - 1) * nw;
        const int64_t c = (int64_t) it * kLpr + m;
        return *(const uint4 *) (wrow + (c < k8 ? c : k8 - 1) * 16);  // (zeroed past K at use: keep_if)
    };

    // Everything that does not depend on the weights is requested before them (vmcnt retires in
    // order, so its consumers then do not wait for the weight stream): the first activation
    // column (or the norm prologue's column, g and b) and the epilogue's bias / residual. Loads
    // are unconditional (clamped indices): a load under a branch is waited for at its join.
    constexpr bool GB = JM > 0 && JM <= 4;
    constexpr int JX = ONE ? 4 : 8;
    float4 pv[JM > 0 ? JM : 1], pg[GB ? JM : 1], pb[GB ? JM : 1];
    ColStager<JX> st;
    if constexpr (JM > 0) {
        norm_load<JM, GB>((const float *) (x.base + (c0 + (wid < nc ? wid : 0)) * x.nb1), K, lane, pro, pv, pg, pb);
    } else {
        // (XH: f16 activations given; a template switch, not a runtime branch: a load under a
        // branch is waited for at its join, before the weights below are even requested)
        if constexpr (!XH) st.load((const float *) (x.base + c0 * x.nb1), K, 0);
    }
    // xfirst: the activation-side loads land before any weight load is queued behind them
    if (e.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 cur[U];
#pragma unroll
    for (int u = 0; u < U; u++) cur[u] = ld(u);
    // the epilogue's bias / residual right behind the weights (they land with them; requested
    // before, the compiler paired a loaded register into a weight-address computation and made the
    // weight requests wait for it)
    asm volatile("" ::: "memory");
    float e_bias = 0.0f, e_res = 0.0f;
    {
        const int64_t rc = live ? row : 0, cc = c0 + (m < nc ? m : nc - 1);
        if (EPI >= 1) e_bias = e.bias[rc];
        if (EPI == 2) e_res = *(const float *) (e.resid + cc * e.resid_nb1 + rc * sizeof(float));
    }

    // stage the f16 activation columns (zero-padded to kp). One column with the norm prologue:
    // every wave normalizes it into its own LDS copy (PRIV), so no wave waits for another's.
    const bool priv = JM > 0 && NC == 1 && rgs == 1;
    uint16_t * xw = priv ? xs + (size_t) wave * kp : xs;
    if constexpr (JM > 0) {
        if (priv) {
            norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xw, lane);
        } else {
            // several columns per wave: the next column's x is requested before this one is
            // normalized (g and b are the same for every column), so the columns' loads overlap
            const int nwt = blockDim.x >> 6;
            for (int c = wid; c < nc; c += nwt) {
                const int cn = c + nwt < nc ? c + nwt : nc - 1;
                float4 nv[JM > 0 ? JM : 1];
                {
                    const float * xc = (const float *) (x.base + (c0 + cn) * x.nb1);
#pragma unroll
                    for (int j = 0; j < JM; j++) {
                        const int64_t k = (int64_t) j * 256 + lane * 4;
                        nv[j] = *(const float4 *) (xc + (k < K ? k : K - 4));  // (zeroed in norm_store)
                    }
                }
                norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xs + (size_t) c * kp, lane);
#pragma unroll
                for (int j = 0; j < JM; j++) pv[j] = nv[j];
            }
        }
    } else if constexpr (XH) {
        for (int c = 0; c < nc; c++) {
            const uint4 * src = (const uint4 *) (xh + (c0 + c) * K);
            uint4 * xd = (uint4 *) (xs + (size_t) c * kp);
            for (int64_t k = threadIdx.x; k < kp / 8; k += blockDim.x) xd[k] = k < k8 ? src[k] : make_uint4(0u, 0u, 0u, 0u);
        }
    } else {
        if (nc == 1) {
            st.store(xs, kp, 0);
            st.column((const float *) (x.base + c0 * x.nb1), K, kp, xs, (int64_t) JX * blockDim.x);
        } else {
            (void) st;
            stage_cols<JX>(x, c0, nc, K, kp, xs);
        }
    }
    MI_STAMP(e.stamps, 1);  // activations staged (normalized) by wave 0
    if (!priv) mi_lds_barrier();

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = 0.0f;
    auto step = [&](const uint4 & wl, int j) {
        const int64_t k = ((int64_t) (wave + j * nw) * kLpr + m) * kChunk;
        const uint4 w = keep_if(k < K, wl);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if (c < nc) acc[c] = dot8(w, *(const uint4 *) (xw + (size_t) c * kp + k), acc[c]);
    };
    if constexpr (ONE) {
#pragma unroll
        for (int u = 0; u < U; u++)
            if (u < nj) step(cur[u], u);
    } else {
        uint4 nxt[U];
        for (int s0 = 0; s0 < nj; s0 += U) {
            const int s1 = s0 + U;
            if (s1 < nj) {
#pragma unroll
                for (int u = 0; u < U; u++) nxt[u] = ld(s1 + u);
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (s0 + u < nj) step(cur[u], s0 + u);
#pragma unroll
            for (int u = 0; u < U; u++) cur[u] = nxt[u];
        }
    }

    MI_STAMP(e.stamps, 3);  // wave 0's dots done (its weights landed)
    // this wave's row totals in every lane of the row; lane m < nc holds column m
    float mine = 0.0f;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float t = row16_sum(acc[c]);
        if (m == c) mine = t;
    }
    if (nw > 1) {
        // the waves' partial sums of each (row, column), added in wave order by wave 0
        float * red = (float *) (xs + (size_t) (priv ? nw : NC) * kp) + (size_t) grp * nw * 4 * NC;
        if (m < nc) red[(wave * 4 + rg) * NC + m] = mine;
        mi_lds_barrier();
        if (wave != 0) return;
        if (m < nc) {
            mine = red[rg * NC + m];
            for (int w = 1; w < nw; w++) mine += red[(w * 4 + rg) * NC + m];
        }
    }
    if (live && m < nc) {
        const int64_t col = c0 + m;
        float v = mine;
        if (EPI >= 1) v = v + e_bias;
        if (EPI == 2) v = v + e_res;
        if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
        *(float *) ((char *) dst + col * ycol + row * sizeof(float)) = v;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1)
                *(float *) (e.copy[k].ptr + col * e.copy[k].col_stride + (row - e.copy[k].row0) * sizeof(float)) = v;
        }
    }
    MI_STAMP_CLK(e.stamps, 5);
    MI_STAMP(e.stamps, 7);
}

// Tall matrices (lm_head, N = 50257): 1..8 columns (NC, padded), rows in one register pass (K <= 128 U).
// A fixed grid of 4-wave workgroups (~8 waves per CU) stages / normalizes the columns once per
// workgroup (wave w the columns w, w + 4: the columns' norms run in parallel), then every wave walks
// its row groups (4 rows) grid-stride, the next group's weights requested before the current group
// is reduced: the weight stream keeps two row groups per wave in flight instead of paying one
// launch-wide latency round per row group. (A per-row-group grid would stage the columns once per
// 4 rows: 12565 workgroups each normalizing every column for lm_head -- 66 us at 8 columns.)
template <int EPI, int U, int JM, int NC>
__global__ __launch_bounds__(256) void k_gemv_f16_tall(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                       mi_src_cols x, int ncols, float * __restrict__ dst, size_t ycol,
                                                       mi_f16_epilogue e, mi_norm_prologue pro, int64_t kp) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [NC][kp] f16
    MI_STAMP(e.stamps, 0);
    MI_STAMP_CLK(e.stamps, 6);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m = lane & (kLpr - 1), rg = lane >> 4;
    const int64_t ngroups = (N + 3) / 4, stride = (int64_t) gridDim.x * 4;
    const int nit = (int) ((K + kKStep - 1) / kKStep);
    const int64_t k8 = K / kChunk;
    int64_t grp = (int64_t) blockIdx.x * 4 + wid;
    auto row_of = [&](int64_t gi) { const int64_t r = gi * 4 + rg; return r < N ? r : N - 1; };
    auto load_group = [&](uint4 (&w)[U], float & eb, int64_t gi) {
        const int64_t r = row_of(gi < ngroups ? gi : ngroups - 1);
        const uint8_t * wrow = W + r * nb01;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int it = u < nit ? u : nit - 1;
            const int64_t c = (int64_t) it * kLpr + m;
#ifdef MI_TALL_NT  // (A/B builds: nontemporal weight loads for the lm_head)
            w[u] = __builtin_nontemporal_load((const uint4 *) (wrow + (c < k8 ? c : k8 - 1) * 16));
#else
            w[u] = *(const uint4 *) (wrow + (c < k8 ? c : k8 - 1) * 16);  // (zeroed past K at use)
#endif
        }
        if (EPI >= 1) eb = e.bias[r];
    };

    constexpr bool GB = JM > 0 && JM <= 4;
    const int nc = ncols < NC ? ncols : NC;
    float4 pv[JM > 0 ? JM : 1], pg[GB ? JM : 1], pb[GB ? JM : 1];
    ColStager<4> st;
    if constexpr (JM > 0) norm_load<JM, GB>((const float *) (x.base + (size_t) (wid < nc ? wid : 0) * x.nb1), K, lane, pro, pv, pg, pb);
    else if (NC == 1) st.load((const float *) x.base, K, 0);
    if (e.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 cur[U];
    float eb = 0.0f;
    load_group(cur, eb, grp);
    if constexpr (JM > 0) {
        // wave w normalizes columns w, w + 4 (the second one's x requested before the first's store)
        if (wid < nc) {
            if (NC > 4 && wid + 4 < nc) {
                float4 nv[JM];
                const float * xc2 = (const float *) (x.base + (size_t) (wid + 4) * x.nb1);
#pragma unroll
                for (int j = 0; j < JM; j++) {
                    const int64_t k = (int64_t) j * 256 + lane * 4;
                    nv[j] = *(const float4 *) (xc2 + (k < K ? k : K - 4));  // (zeroed in norm_store)
                }
                norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xs + (size_t) wid * kp, lane);
                norm_store<JM, GB>(nv, pg, pb, K, kp, pro, xs + (size_t) (wid + 4) * kp, lane);
            } else {
                norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xs + (size_t) wid * kp, lane);
            }
        }
    } else if (NC == 1) {
        st.store(xs, kp, 0);
        st.column((const float *) x.base, K, kp, xs, (int64_t) 4 * blockDim.x);
    } else {
        stage_cols<4>(x, 0, nc, K, kp, xs);
    }
    mi_lds_barrier();
    MI_STAMP(e.stamps, 2);

    for (; grp < ngroups; grp += stride) {
        uint4 nxt[U];
        float ebn = 0.0f;
        load_group(nxt, ebn, grp + stride);
        float acc[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) acc[c] = 0.0f;
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (u < nit) {
                const uint4 w = keep_if((int64_t) u * kLpr + m < k8, cur[u]);
#pragma unroll
                for (int c = 0; c < NC; c++)
                    if (c < nc) acc[c] = dot8(w, *(const uint4 *) (xs + (size_t) c * kp + ((int64_t) u * kLpr + m) * kChunk), acc[c]);
            }
        }
        float mine = 0.0f;  // lane m of the row holds column m
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const float t = row16_sum(acc[c]);
            if (m == c) mine = t;
        }
        const int64_t row = grp * 4 + rg;
        if (m < nc && row < N) {
            float v = mine;
            if (EPI >= 1) v = v + eb;
            if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
            *(float *) ((char *) dst + (size_t) m * ycol + row * sizeof(float)) = v;
            // a CPY of the output rows (e.g. the logits into the caller's pinned host buffer: the
            // stores go out over PCIe while the GEMV runs, instead of a copy queued behind it)
            if (e.copy[0].ptr && row >= e.copy[0].row0 && row < e.copy[0].row1)
                *(float *) (e.copy[0].ptr + (size_t) m * e.copy[0].col_stride + (row - e.copy[0].row0) * sizeof(float)) = v;
        }
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = nxt[u];
        eb = ebn;
    }
    MI_STAMP_CLK(e.stamps, 5);
    MI_STAMP(e.stamps, 7);
}

// Tall matrices (lm_head) with 2..8 columns on the matrix cores (round 6): k_gemv_f16_tall's dot8
// reads every column's 16 activation bytes from LDS for each 16 weight bytes, so at 8 columns the
// LDS traffic is 8x the weight stream (batched decode's lm_head: 28.7 us for 77 MB). Here each wave
// holds the normalized f16 columns once, as the B operands of v_mfma_f32_16x16x32_f16 for the whole
// K (lane l: column l % 16, K slice 8 (l / 16) of each 32-deep step; columns >= nc are zero), and
// streams 16-row weight tiles as the A operand (lane l: row l % 16, the same K slice): one MFMA per
// 32-deep step, the accumulator's lane l then holds column l % 16 of rows 4 (l / 16) .. + 3.
// f16 x f16 products are exact in f32; the accumulation order is the matrix core's (tree order:
// within 1e-5 of the reference's vec_dot_f16). Staging and the norm prologue as k_gemv_f16_tall.
// NK: 32-deep K steps (K <= 32 NK, K % 32 == 0).
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
template <int EPI, int JM, int NK>
__global__ __launch_bounds__(256) void k_gemv_f16_mt(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                     mi_src_cols x, int ncols, float * __restrict__ dst, size_t ycol,
                                                     mi_f16_epilogue e, mi_norm_prologue pro, int64_t kp) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [8][kp] f16
    MI_STAMP(e.stamps, 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nc = ncols < 8 ? ncols : 8;
    const int nk = (int) (K / 32);
    const int64_t ntiles = (N + 15) / 16, stride = (int64_t) gridDim.x * 4;
    int64_t tile = (int64_t) blockIdx.x * 4 + wid;
    auto load_tile = [&](half8 (&a)[NK], int64_t ti) {
        const int64_t r = ti * 16 + li;
        const uint8_t * wrow = W + (r < N ? r : N - 1) * nb01 + (size_t) lk * 16;
#pragma unroll
        for (int t = 0; t < NK; t++) a[t] = *(const half8 *) (wrow + (size_t) (t < nk ? t : nk - 1) * 64);
    };
    constexpr bool GB = JM > 0 && JM <= 4;
    float4 pv[JM > 0 ? JM : 1], pg[GB ? JM : 1], pb[GB ? JM : 1];
    if constexpr (JM > 0) norm_load<JM, GB>((const float *) (x.base + (size_t) (wid < nc ? wid : 0) * x.nb1), K, lane, pro, pv, pg, pb);
    half8 a[NK];
    load_tile(a, tile < ntiles ? tile : ntiles - 1);  // the first tile's weights in flight under the staging
    if constexpr (JM > 0) {
        if (wid < nc) {
            if (wid + 4 < nc) {
                float4 nv[JM];
                const float * xc2 = (const float *) (x.base + (size_t) (wid + 4) * x.nb1);
#pragma unroll
                for (int j = 0; j < JM; j++) {
                    const int64_t k = (int64_t) j * 256 + lane * 4;
                    nv[j] = *(const float4 *) (xc2 + (k < K ? k : K - 4));  // (zeroed in norm_store)
                }
                norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xs + (size_t) wid * kp, lane);
                norm_store<JM, GB>(nv, pg, pb, K, kp, pro, xs + (size_t) (wid + 4) * kp, lane);
            } else {
                norm_store<JM, GB>(pv, pg, pb, K, kp, pro, xs + (size_t) wid * kp, lane);
            }
        }
    } else {
        stage_cols<4>(x, 0, nc, K, kp, xs);
    }
    mi_lds_barrier();
    MI_STAMP(e.stamps, 2);
    // the columns as B operands for the whole K (zero past nc)
    half8 b[NK];
#pragma unroll
    for (int t = 0; t < NK; t++) {
        const half8 v = *(const half8 *) (xs + (size_t) (li < nc ? li : 0) * kp + (size_t) (t < nk ? t : 0) * 32 + lk * 8);
        b[t] = li < nc && t < nk ? v : half8{};
    }
    typedef float f32x4v_t __attribute__((ext_vector_type(4)));
    for (; tile < ntiles; tile += stride) {
        f32x4v_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < NK; t++)
            if (t < nk) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[t], acc, 0, 0, 0);
        if (tile + stride < ntiles) load_tile(a, tile + stride);  // (the registers are free once the MFMAs read them)
        const float v4[4] = {acc.x, acc.y, acc.z, acc.w};
        if (li < nc) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t row = tile * 16 + lk * 4 + q;
                if (row < N) {
                    float v = v4[q];
                    if (EPI >= 1) v = v + e.bias[row];
                    if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
                    *(float *) ((char *) dst + (size_t) li * ycol + row * sizeof(float)) = v;
                    if (e.copy[0].ptr && row >= e.copy[0].row0 && row < e.copy[0].row1)
                        *(float *) (e.copy[0].ptr + (size_t) li * e.copy[0].col_stride + (row - e.copy[0].row0) * sizeof(float)) = v;
                }
            }
        }
    }
    MI_STAMP(e.stamps, 7);
}

#if MI_DIAG
// (diagnostic builds only: measured slower than k_gemv_f16 on batched decode, 0.515 -> 0.568 ms/step,
// profiles/r06s2k_batched_f16_m8_ab.txt -- a 16-row tile per workgroup leaves 48 workgroups for the
// 768-row projections, fewer than the streams the weight rows need)
// Plain (no norm prologue) F16 GEMVs of 2..8 columns on the matrix cores (round 6, batched decode's
// attention / MLP output projections): one workgroup of NW waves per 16-row tile, the K steps
// (32 deep) dealt to the waves in contiguous runs of at most NKW; each lane loads its A operand (row
// l % 16, K slice 8 (l / 16) of a step) straight from the weights and its B operand (column l % 16,
// the same K slice) straight from the f32 columns, rounded to f16 in registers -- no LDS staging of
// the columns, each workgroup reads only its K runs of them once. The waves' 16 x 16 partial tiles
// are added in wave order by wave 0, which applies the epilogue (bias, residual, GELU, row copies).
// Tree order (f32 sums in the matrix core's order): within 1e-5 of the reference's vec_dot_f16.
template <int EPI, int NKW, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemv_f16_m8(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                         mi_src_cols x, int ncols, float * __restrict__ dst, size_t ycol,
                                                         mi_f16_epilogue e) {
    __shared__ float red[NW][64][4];
    MI_STAMP(e.stamps, 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nc = ncols < 8 ? ncols : 8;
    const int nk = (int) (K / 32);
    const int spw = (nk + NW - 1) / NW;                 // steps per wave (<= NKW, launcher)
    const int t0 = wid * spw, t1 = t0 + spw < nk ? t0 + spw : nk;
    const int64_t r0 = (int64_t) blockIdx.x * 16;
    const int64_t r = r0 + li;
    const uint8_t * wrow = W + (r < N ? r : N - 1) * nb01 + (size_t) lk * 16;
    const char * xc = x.base + (size_t) (li < nc ? li : 0) * x.nb1 + (size_t) lk * 32;
    half8 a[NKW];
    float4 xv[NKW][2];
#pragma unroll
    for (int i = 0; i < NKW; i++) {
        const int t = t0 + i < t1 ? t0 + i : (t1 > t0 ? t1 - 1 : 0);  // (clamped: unconditional loads)
        a[i] = *(const half8 *) (wrow + (size_t) t * 64);
    }
    // (the epilogue operands ride behind the weights)
    float e_bias[4], e_res[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int64_t rq = r0 + lk * 4 + q;
        const int64_t rc = rq < N ? rq : N - 1;
        e_bias[q] = EPI >= 1 ? e.bias[rc] : 0.0f;
        e_res[q] = EPI == 2 ? *(const float *) (e.resid + (size_t) (li < nc ? li : 0) * e.resid_nb1 + rc * sizeof(float)) : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < NKW; i++) {
        const int t = t0 + i < t1 ? t0 + i : (t1 > t0 ? t1 - 1 : 0);
        xv[i][0] = *(const float4 *) (xc + (size_t) t * 128);
        xv[i][1] = *(const float4 *) (xc + (size_t) t * 128 + 16);
    }
    typedef float f32x4v_t __attribute__((ext_vector_type(4)));
    f32x4v_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < NKW; i++) {
        if (t0 + i < t1) {
            half8 b;
            b[0] = (_Float16) xv[i][0].x; b[1] = (_Float16) xv[i][0].y; b[2] = (_Float16) xv[i][0].z; b[3] = (_Float16) xv[i][0].w;
            b[4] = (_Float16) xv[i][1].x; b[5] = (_Float16) xv[i][1].y; b[6] = (_Float16) xv[i][1].z; b[7] = (_Float16) xv[i][1].w;
            if (li >= nc) b = half8{};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b, acc, 0, 0, 0);
        }
    }
    MI_STAMP(e.stamps, 3);
    red[wid][lane][0] = acc.x;
    red[wid][lane][1] = acc.y;
    red[wid][lane][2] = acc.z;
    red[wid][lane][3] = acc.w;
    mi_lds_barrier();
    if (wid != 0) return;
    float v4[4] = {red[0][lane][0], red[0][lane][1], red[0][lane][2], red[0][lane][3]};
#pragma unroll
    for (int w = 1; w < NW; w++)
#pragma unroll
        for (int q = 0; q < 4; q++) v4[q] += red[w][lane][q];
    if (li < nc) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int64_t row = r0 + lk * 4 + q;
            if (row < N) {
                float v = v4[q];
                if (EPI >= 1) v = v + e_bias[q];
                if (EPI == 2) v = v + e_res[q];
                if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
                *(float *) ((char *) dst + (size_t) li * ycol + row * sizeof(float)) = v;
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1)
                        *(float *) (e.copy[k].ptr + (size_t) li * e.copy[k].col_stride + (row - e.copy[k].row0) * sizeof(float)) = v;
                }
            }
        }
    }
    MI_STAMP(e.stamps, 7);
}
#endif  // MI_DIAG

// The F16 GEMV of one column whose input is a norm chain over a value still held as partial sums
// (mi_attn_proj's per-head parts, mi_norm_prologue::parts): workgroup = RW waves x 4 rows (RW =
// blockDim / 64), each wave the whole K of its rows in one register pass. The workgroup adds the
// parts once (QPT groups of 4 elements per thread, parts in order, all loads before the
// weights') into LDS, the first workgroup also storing the sum (the graph value it stands for);
// then every wave normalizes the column into its own f16 copy (no second barrier) and runs its
// rows. NPM: parts capacity (registers), >= pro.nparts.
constexpr int kPsMaxParts = 16;
template <int EPI, int U, int JM, int NPM, int QPT>
__global__ __launch_bounds__(512) void k_gemv_f16_ps(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                     float * __restrict__ dst, mi_f16_epilogue e, mi_norm_prologue pro, int64_t kp) {
    const int rw = blockDim.x >> 6;
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [rw][kp] f16 per wave, then [kp] f32 (the sum)
    MI_STAMP(e.stamps, 0);
    MI_STAMP_CLK(e.stamps, 6);
    float * xf = (float *) (xs + (size_t) rw * kp);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m = lane & (kLpr - 1), rg = lane >> 4;
    const int64_t row = ((int64_t) blockIdx.x * rw + wid) * 4 + rg;
    const bool live = row < N;
    const int nit = (int) ((K + kKStep - 1) / kKStep);
    const int64_t k8 = K / kChunk;
    const uint8_t * wrow = W + (live ? row : 0) * nb01;

    // the parts of this thread's QPT x 4 elements (threads past K share one clamped line)
    float4 pp[QPT][NPM];
#pragma unroll
    for (int r = 0; r < QPT; r++) {
        const int64_t q4 = ((int64_t) r * blockDim.x + threadIdx.x) * 4;
        const int64_t kq = q4 < K ? q4 : K - 4;
#pragma unroll
        for (int q = 0; q < NPM; q++) pp[r][q] = *(const float4 *) (pro.parts + (int64_t) (q < pro.nparts ? q : 0) * K + kq);
    }
    // g, b of the lane's norm elements, the epilogue's bias / residual
    float4 pg[JM], pb[JM];
#pragma unroll
    for (int j = 0; j < JM; j++) {
        const int64_t k = (int64_t) j * 256 + lane * 4;
        const int64_t kc = k < K ? k : K - 4;
        pg[j] = *(const float4 *) ((pro.g ? pro.g : pro.parts) + kc);
        pb[j] = *(const float4 *) ((pro.b ? pro.b : pro.parts) + kc);
    }
    float e_bias = 0.0f, e_res = 0.0f;
    {
        const int64_t rc = live ? row : 0;
        if (EPI >= 1) e_bias = e.bias[rc];
        if (EPI == 2) e_res = *(const float *) (e.resid + rc * sizeof(float));
    }
    if (e.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 cur[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int it = u < nit ? u : nit - 1;
        const int64_t c = (int64_t) it * kLpr + m;
        cur[u] = *(const uint4 *) (wrow + (c < k8 ? c : k8 - 1) * 16);  // (zeroed past K at use)
    }

#pragma unroll
    for (int r = 0; r < QPT; r++) {
        float4 sum = pp[r][0];
#pragma unroll
        for (int q = 1; q < NPM; q++) {
            if (q < pro.nparts) {
                sum.x += pp[r][q].x; sum.y += pp[r][q].y; sum.z += pp[r][q].z; sum.w += pp[r][q].w;
            }
        }
        const int64_t q4 = ((int64_t) r * blockDim.x + threadIdx.x) * 4;
        if (q4 < K) {
            *(float4 *) (xf + q4) = sum;
            if (blockIdx.x == 0) *(float4 *) (pro.store + q4) = sum;
        }
    }
    MI_STAMP(e.stamps, 1);  // parts landed and summed (wave 0)
    __syncthreads();
    MI_STAMP(e.stamps, 2);
    float4 v[JM];
#pragma unroll
    for (int j = 0; j < JM; j++) {
        const int64_t k = (int64_t) j * 256 + lane * 4;
        v[j] = k < K ? *(const float4 *) (xf + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint16_t * xw = xs + (size_t) wid * kp;
    norm_store<JM, true>(v, pg, pb, K, kp, pro, xw, lane);
    MI_STAMP(e.stamps, 4);  // normalized

    float acc = 0.0f;
#pragma unroll
    for (int u = 0; u < U; u++)
        if (u < nit) acc = dot8(keep_if((int64_t) u * kLpr + m < k8, cur[u]), *(const uint4 *) (xw + ((int64_t) u * kLpr + m) * kChunk), acc);
    acc = row16_sum(acc);
    if (live && m == 0) {
        float r = acc;
        if (EPI >= 1) r = r + e_bias;
        if (EPI == 2) r = r + e_res;
        if (EPI == 3) r = r <= -10.0f ? 0.0f : (r >= 10.0f ? r : mi_h2f(e.gelu_table[mi_f2h(r)]));
        dst[row] = r;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1)
                *(float *) (e.copy[k].ptr + (row - e.copy[k].row0) * sizeof(float)) = r;
        }
    }
    MI_STAMP_CLK(e.stamps, 5);
    MI_STAMP(e.stamps, 7);
}

// Several columns (2..8) with the norm prologue (round 6; batched decode's c_attn / c_fc, K <= 1024):
// one workgroup of NW waves normalizes every column ONCE -- wave w the columns w, w + NW, ..., all of
// a wave's columns requested together with g and b (shared by the columns) -- into f16 LDS, and its
// waves then stream 4 rows each over the whole K with every row's chunks requested at kernel entry
// (before the norm), reading the columns back as 16-byte broadcast reads. The one-column-per-
// workgroup form (f16_nc 10, the default before) normalized each column in N / 4 workgroups and
// re-read every weight row once per column; staging all columns in the row-group kernel serialized
// the norms (k_gemv_f16 with 8 columns, ~0.9 us per column). Same per-element arithmetic (norm_store,
// dot8, row16_sum): tree order, within the F16 tolerance of the reference.
// KS > 1: the KS waves of a 4-row group split the row's chunks (wave part p takes chunks i = p mod KS)
// and their partial sums meet in LDS, added in part order.
// JM == 0 (plain, no norm: batched decode's c_proj / mlp projection): every thread stages the f32
// columns to f16 LDS (stage_cols) instead; NCHT = 16-byte chunks per lane and row (K <= 128 NCHT).
template <int EPI, int JM, int NW, int KS = 1, int NCHT = JM * 2>
__global__ __launch_bounds__(64 * NW) void k_gemv_f16_bn(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                        mi_src_cols x, int64_t ncols, float * __restrict__ dst, size_t ycol,
                                                        mi_f16_epilogue e, mi_norm_prologue pro, int64_t kp) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [8][kp] f16, then [NW][4][8] f32 partials
    constexpr int CPW = (8 + NW - 1) / NW;  // columns per wave
    constexpr int NCH = NCHT / KS;           // 16-byte chunks per lane and row of this wave
    constexpr int JMV = JM > 0 ? JM : 1;
    MI_STAMP(e.stamps, 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m = lane & (kLpr - 1), rg = lane >> 4;
    const int grp = wid / KS, part = wid % KS;
    const int64_t row = ((int64_t) blockIdx.x * (NW / KS) + grp) * 4 + rg;
    const bool live = row < N;
    const int nc = (int) std::min<int64_t>(8, ncols);
    const int64_t k8 = K / kChunk;

    // the wave's columns, g and b first (vmcnt retires in order), then the rows' weight chunks
    float4 pv[CPW][JMV], pg[JMV], pb[JMV];
    if constexpr (JM > 0) {
#pragma unroll
        for (int j = 0; j < CPW; j++) {
            const int c = wid + NW * j;
            const float * xc = (const float *) (x.base + (c < nc ? c : nc - 1) * x.nb1);
            if (j == 0) {
                norm_load<JM, true>(xc, K, lane, pro, pv[0], pg, pb);
            } else {
                float4 dg[1], db[1];
                norm_load<JM, false>(xc, K, lane, pro, pv[j], dg, db);
            }
        }
    }
    asm volatile("" ::: "memory");
    const uint8_t * wrow = W + (live ? row : 0) * nb01;
    uint4 cur[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        const int64_t c = (int64_t) (i * KS + part) * kLpr + m;
        cur[i] = *(const uint4 *) (wrow + (c < k8 ? c : k8 - 1) * 16);  // (zeroed past K at use)
    }
    asm volatile("" ::: "memory");
    float e_bias = 0.0f, e_res = 0.0f;
    {
        const int64_t rc = live ? row : 0, cc = m < nc ? m : nc - 1;
        if (EPI >= 1) e_bias = e.bias[rc];
        if (EPI == 2) e_res = *(const float *) (e.resid + cc * e.resid_nb1 + rc * sizeof(float));
    }
    if constexpr (JM > 0) {
#pragma unroll
        for (int j = 0; j < CPW; j++) {
            const int c = wid + NW * j;
            if (c < nc) norm_store<JM, true>(pv[j], pg, pb, K, kp, pro, xs + (size_t) c * kp, lane);
        }
    } else {
        (void) pv; (void) pg; (void) pb;
        stage_cols<8>(x, 0, nc, K, kp, xs);
    }
    MI_STAMP(e.stamps, 1);
    mi_lds_barrier();

    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; c++) acc[c] = 0.0f;
#pragma unroll
    for (int i = 0; i < NCH; i++) {
        const int64_t k = ((int64_t) (i * KS + part) * kLpr + m) * kChunk;
        const uint4 w = keep_if(k < K, cur[i]);
        if (k < kp) {
#pragma unroll
            for (int c = 0; c < 8; c++)
                if (c < nc) acc[c] = dot8(w, *(const uint4 *) (xs + (size_t) c * kp + k), acc[c]);
        }
    }
    MI_STAMP(e.stamps, 3);
    float mine = 0.0f;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const float t = row16_sum(acc[c]);
        if (m == c) mine = t;
    }
    if constexpr (KS > 1) {
        float * red = (float *) (xs + (size_t) 8 * kp);
        if (m < 8) red[(wid * 4 + rg) * 8 + m] = mine;
        mi_lds_barrier();
        if (part != 0) return;
        if (m < 8) {
            for (int p = 1; p < KS; p++) mine += red[((wid + p) * 4 + rg) * 8 + m];
        }
    }
    if (live && m < nc) {
        const int64_t col = m;
        float v = mine;
        if (EPI >= 1) v = v + e_bias;
        if (EPI == 2) v = v + e_res;
        if (EPI == 3) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
        *(float *) ((char *) dst + col * ycol + row * sizeof(float)) = v;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1)
                *(float *) (e.copy[k].ptr + col * e.copy[k].col_stride + (row - e.copy[k].row0) * sizeof(float)) = v;
        }
    }
    MI_STAMP(e.stamps, 7);
}

template <int NC, int U, bool ONE, int JM>
void launch_nc(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols, float * dst,
               size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s, int ks, int rgs) {
    const int64_t kp = (K + kKStep - 1) / kKStep * kKStep;
    const dim3 grid((unsigned) ((N + 4 * rgs - 1) / (4 * rgs)), (unsigned) ((ncols + NC - 1) / NC));
    const bool priv = JM > 0 && NC == 1 && rgs == 1;
    const size_t lds = (size_t) (priv ? ks : NC) * kp * sizeof(uint16_t) + (size_t) ks * rgs * 4 * NC * sizeof(float);
    const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
    const uint8_t * w = (const uint8_t *) W;
    mi_f16_epilogue es = e;
    es.stamps = mi_stamp_take(JM ? "k_gemv_f16_norm" : "k_gemv_f16", grid.x * grid.y);
    es.xfirst = g_mi_tuning.xfirst == 1;  // (off by default: GPT-2 decode 304 -> 316 us per token with it)
#define MI_GEMV_F16X(EP, XHV) hipLaunchKernelGGL((k_gemv_f16<NC, EP, U, ONE, JM, XHV>), grid, dim3(64 * ks * rgs), lds, s, w, nb01, K, N, x, xh, ncols, dst, ycol, es, pro, kp, rgs)
#define MI_GEMV_F16(EP) do { if constexpr (JM == 0) { if (xh) MI_GEMV_F16X(EP, true); else MI_GEMV_F16X(EP, false); } else MI_GEMV_F16X(EP, false); } while (0)
    switch (epi) {
        case 0: MI_GEMV_F16(0); break;
        case 1: MI_GEMV_F16(1); break;
        case 2: MI_GEMV_F16(2); break;
        default: MI_GEMV_F16(3); break;
    }
#undef MI_GEMV_F16
#undef MI_GEMV_F16X
}

template <int U, bool ONE, int JM>
void launch_u(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols, float * dst,
              size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s, int nc, int ks, int rgs) {
    switch (nc) {
        case 1: launch_nc<1, U, ONE, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, ks, rgs); break;
        case 2: launch_nc<2, U, ONE, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, ks, rgs); break;
        case 4: launch_nc<4, U, ONE, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, ks, rgs); break;
        default: launch_nc<8, U, ONE, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, ks, rgs); break;
    }
}

// one register pass of `per` steps per wave: U = per rounded up to 1/2/4/8 (no wasted loads)
template <int JM>
void launch_one(int per, const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s, int nc, int ks, int rgs) {
    if (per <= 1) launch_u<1, true, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    else if (per <= 2) launch_u<2, true, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    else if (per <= 4) launch_u<4, true, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    else launch_u<8, true, JM>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
}

} // namespace

bool mi_mul_mat_f16_fast_supported(int64_t K, int64_t ncols, const mi_src_cols & x, const uint16_t * xh, const mi_norm_prologue & pro) {
    if (ncols < 1 || ncols > 8 || K < 8 || K % 8 != 0 || K > 16384) return false;
    if (!xh && (x.nb1 % 16 != 0 || (uintptr_t) x.base % 16 != 0)) return false;
    // norm prologue: column in registers (K <= 3072), one register pass per wave (K <= 1024 or >= 3 waves)
    if (pro.mode && (K > 3072 || xh || ((uintptr_t) pro.g | (uintptr_t) pro.b) % 16 != 0)) return false;
    // summed-partials prologue (k_gemv_f16_ps): one column, K <= 1024
    if (pro.parts && (!pro.mode || ncols != 1 || K > 1024 || pro.nparts < 1 || pro.nparts > kPsMaxParts || !pro.store ||
                      ((uintptr_t) pro.parts | (uintptr_t) pro.store) % 16 != 0 || K % 8 != 0)) return false;
    return true;
}

void mi_mul_mat_f16_fast(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                         float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s) {
    // columns per workgroup: ncols rounded up to 1/2/4/8, within 64 KB of f16 columns in LDS
    const int64_t kp = (K + kKStep - 1) / kKStep * kKStep;
    int nc = ncols >= 8 ? 8 : ncols >= 3 ? 4 : (int) ncols;
    while (nc > 1 && (int64_t) nc * kp * 2 > 60000) nc /= 2;
    // columns per workgroup capped by the knob f16_nc (not for lm_head; ones digit: the plain GEMVs,
    // tens digit: those with the norm prologue; 0 = up to 8). Default 10: the norm GEMVs stage one
    // column per workgroup, so every wave normalizes its own copy with no barrier (batched decode,
    // 8 columns: 0.666-0.669 -> 0.650-0.657 ms/step; 2 or 4 columns per workgroup are slower, and so
    // is one column for the plain GEMVs: profiles/r05nc_batched_cols_per_wg.txt)
    const int nc_cap = pro.mode ? g_mi_tuning.f16_nc / 10 : g_mi_tuning.f16_nc % 10;
    if (nc_cap > 0 && (N + 3) / 4 < 4096)
        while (nc > 1 && nc > nc_cap) nc /= 2;
    // waves per workgroup (K split): about kWaves waves on the chip (~8 per CU), at most 8 per
    // workgroup and no more than the row's K steps, then as few as give the same steps per wave
    const int nit = (int) (kp / kKStep);
    const int64_t groups = (N + 3) / 4 * ((ncols + nc - 1) / nc);
    // target waves: ~8 per CU; with the norm prologue every wave reads the whole column, g and b
    // (12 K bytes, the same lines for every wave of the chip), so fewer (~3 per CU)
    const int64_t want = g_mi_tuning.f16_waves > 0 ? g_mi_tuning.f16_waves : (pro.mode ? 768 : 2048);
    int ks = (int) std::max<int64_t>(1, std::min<int64_t>(8, want / std::max<int64_t>(groups, 1)));
    // very tall matrices (lm_head): row groups share one staging of the activations per workgroup
    ks = std::min(ks, nit);
    if (pro.mode) ks = std::max(ks, (nit + 7) / 8);  // the prologue path runs one register pass
    // several columns with the norm prologue: the columns' norms spread over 3 waves (a lone wave
    // normalizes its columns one after the other, ~0.9 us each: 8 columns 8.2 us of prologue; one
    // column per wave makes 6-wave workgroups of which only two fit a CU at 106 VGPRs, so GPT-2's
    // 768 c_fc workgroups ran in two rounds: batched decode 0.700 -> 0.672 ms/step with 3,
    // profiles/r05r_batched_norm_waves.txt)
    if (pro.mode && nc > 1) ks = std::max(ks, std::min(g_mi_tuning.f16_norm_waves > 0 ? g_mi_tuning.f16_norm_waves : 3, nit));
    const int per = (nit + ks - 1) / ks;  // steps per wave
    ks = (nit + per - 1) / per;
    const bool one = per <= 8;
    const int rgs = g_mi_tuning.f16_rgs > 0 ? std::max(1, std::min(g_mi_tuning.f16_rgs, 8 / ks)) : 1;
    if (groups / ((ncols + nc - 1) / nc) >= 4096 && K <= 1024 && !xh && !e.resid && !e.copy[1].ptr && g_mi_tuning.f16_rgs == 0 &&
        !pro.parts && (ncols == 1 || ncols == nc)) {
        // tall matrix: grid-stride row groups (k_gemv_f16_tall), 1..8 columns in one launch
        const int64_t rgroups = (N + 3) / 4;
        const dim3 grid((unsigned) std::min<int64_t>((rgroups + 3) / 4, 512));
        const size_t lds = (size_t) nc * kp * sizeof(uint16_t);
        const int epi = e.gelu_table ? 3 : (e.bias ? 1 : 0);
        const uint8_t * w = (const uint8_t *) W;
        mi_f16_epilogue es = e;
        if (nc >= 2 && ncols >= 2 && K % 32 == 0 && K <= 768 && g_mi_tuning.f16_mt) {
            // several columns on the matrix cores (k_gemv_f16_mt): 16-row tiles, grid-stride
            const dim3 gridm((unsigned) std::min<int64_t>(((N + 15) / 16 + 3) / 4, 512));
            const size_t ldsm = (size_t) 8 * kp * sizeof(uint16_t);
            es.stamps = mi_stamp_take("k_gemv_f16_mt", gridm.x);
#define MI_GEMV_MT(EP, JMV) hipLaunchKernelGGL((k_gemv_f16_mt<EP, JMV, 24>), gridm, dim3(256), ldsm, s, w, nb01, K, N, x, (int) ncols, dst, ycol, es, pro, kp)
            if (pro.mode) {
                if (epi == 0) MI_GEMV_MT(0, 4); else if (epi == 1) MI_GEMV_MT(1, 4); else MI_GEMV_MT(3, 4);
            } else {
                if (epi == 0) MI_GEMV_MT(0, 0); else if (epi == 1) MI_GEMV_MT(1, 0); else MI_GEMV_MT(3, 0);
            }
#undef MI_GEMV_MT
            return;
        }
        es.stamps = mi_stamp_take("k_gemv_f16_tall", grid.x);
        es.xfirst = g_mi_tuning.xfirst == 1;  // (off by default: GPT-2 decode 304 -> 316 us per token with it)
#define MI_GEMV_TALL_N(EP, JMV, NCV) hipLaunchKernelGGL((k_gemv_f16_tall<EP, 8, JMV, NCV>), grid, dim3(256), lds, s, w, nb01, K, N, x, (int) ncols, dst, ycol, es, pro, kp)
#define MI_GEMV_TALL(EP, JMV) do { switch (nc) { case 1: MI_GEMV_TALL_N(EP, JMV, 1); break; case 2: MI_GEMV_TALL_N(EP, JMV, 2); break; \
                                                  case 4: MI_GEMV_TALL_N(EP, JMV, 4); break; default: MI_GEMV_TALL_N(EP, JMV, 8); break; } } while (0)
        if (pro.mode) {
            if (epi == 0) MI_GEMV_TALL(0, 4); else if (epi == 1) MI_GEMV_TALL(1, 4); else MI_GEMV_TALL(3, 4);
        } else {
            if (epi == 0) MI_GEMV_TALL(0, 0); else if (epi == 1) MI_GEMV_TALL(1, 0); else MI_GEMV_TALL(3, 0);
        }
#undef MI_GEMV_TALL
#undef MI_GEMV_TALL_N
        return;
    }
    if (pro.parts) {  // supported(): one column, K <= 1024, <= 16 parts
        // waves per workgroup: enough workgroups to cover the CUs, few enough that the parts
        // (nparts x 4 K bytes read per workgroup) stay a small fraction of the weight bytes
        // (rw >= 2 and K <= 1024: at most 2 groups of 4 elements per thread)
        const int rw = g_mi_tuning.f16_ps_waves > 0 ? g_mi_tuning.f16_ps_waves : 4;
        const int qpt = (int) ((K / 4 + 64 * rw - 1) / (64 * rw));
        const dim3 grid((unsigned) ((N + 4 * rw - 1) / (4 * rw)));
        const size_t lds = (size_t) rw * kp * sizeof(uint16_t) + (size_t) kp * sizeof(float);
        const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
        const uint8_t * w = (const uint8_t *) W;
        mi_f16_epilogue es = e;
        es.stamps = mi_stamp_take("k_gemv_f16_ps", grid.x);
        es.xfirst = g_mi_tuning.xfirst == 1;  // (off by default: GPT-2 decode 304 -> 316 us per token with it)
#define MI_GEMV_PS(EP, NPM, QPT) hipLaunchKernelGGL((k_gemv_f16_ps<EP, 8, 4, NPM, QPT>), grid, dim3(64 * rw), lds, s, w, nb01, K, N, dst, es, pro, kp)
#define MI_GEMV_PS_E(NPM, QPT)                     \
        switch (epi) {                             \
            case 0: MI_GEMV_PS(0, NPM, QPT); break; \
            case 1: MI_GEMV_PS(1, NPM, QPT); break; \
            case 2: MI_GEMV_PS(2, NPM, QPT); break; \
            default: MI_GEMV_PS(3, NPM, QPT); break; \
        }
        if (qpt <= 1) {
            if (pro.nparts <= 12) { MI_GEMV_PS_E(12, 1) } else { MI_GEMV_PS_E(16, 1) }
        } else {
            if (pro.nparts <= 12) { MI_GEMV_PS_E(12, 2) } else { MI_GEMV_PS_E(16, 2) }
        }
#undef MI_GEMV_PS_E
#undef MI_GEMV_PS
    } else if (pro.mode && (ncols > 1 || g_mi_tuning.f16_bn >= 10) && K <= 1024 && g_mi_tuning.f16_bn > 0) {
        // several columns with the norm prologue: normalized once per workgroup (k_gemv_f16_bn)
        // f16_bn: 1 = 4 waves, 2 = 8 waves, 3 = 8 waves with K split over wave pairs, 4 = 8 waves K split
        // over 4, 5 = 16 waves K split over 4
        const int bn = g_mi_tuning.f16_bn % 10;  // (+10: one column too)
        const int NWv = bn == 5 ? 16 : bn >= 2 ? 8 : 4, KSv = bn == 3 ? 2 : bn >= 4 ? 4 : 1;
        const dim3 grid((unsigned) ((N + 4 * (NWv / KSv) - 1) / (4 * (NWv / KSv))));
        const size_t lds = (size_t) 8 * kp * sizeof(uint16_t) + (size_t) NWv * 4 * 8 * sizeof(float);
        const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
        const uint8_t * w = (const uint8_t *) W;
        mi_f16_epilogue es = e;
        es.stamps = mi_stamp_take("k_gemv_f16_bn", grid.x);
#define MI_GEMV_BN(EP, NWV, KSV) hipLaunchKernelGGL((k_gemv_f16_bn<EP, 4, NWV, KSV>), grid, dim3(64 * NWV), lds, s, w, nb01, K, N, x, ncols, dst, ycol, es, pro, kp)
#define MI_GEMV_BN_E(NWV, KSV) switch (epi) { case 0: MI_GEMV_BN(0, NWV, KSV); break; case 1: MI_GEMV_BN(1, NWV, KSV); break; \
                                                  case 2: MI_GEMV_BN(2, NWV, KSV); break; default: MI_GEMV_BN(3, NWV, KSV); break; }
        if (bn == 5) { MI_GEMV_BN_E(16, 4) } else if (bn == 4) { MI_GEMV_BN_E(8, 4) } else if (KSv == 2) { MI_GEMV_BN_E(8, 2) }
        else if (NWv == 8) { MI_GEMV_BN_E(8, 1) } else { MI_GEMV_BN_E(4, 1) }
#undef MI_GEMV_BN_E
#undef MI_GEMV_BN
#if MI_DIAG
    } else if (!pro.mode && ncols > 1 && K % 32 == 0 && K <= 4096 && !xh && g_mi_tuning.f16_m8 > 0 && (N + 3) / 4 < 4096) {
        // several plain columns on the matrix cores (k_gemv_f16_m8): per 16-row tile 4 waves (K <= 1024,
        // at most 8 steps of 32 each) or 8 (at most 16 steps each)
        const int nk = (int) (K / 32);
        const dim3 grid((unsigned) ((N + 15) / 16));
        const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
        const uint8_t * w = (const uint8_t *) W;
        mi_f16_epilogue es = e;
        es.stamps = mi_stamp_take("k_gemv_f16_m8", grid.x);
#define MI_GEMV_M8(EP, NKWV, NWV) hipLaunchKernelGGL((k_gemv_f16_m8<EP, NKWV, NWV>), grid, dim3(64 * NWV), 0, s, w, nb01, K, N, x, (int) ncols, dst, ycol, es)
#define MI_GEMV_M8_E(NKWV, NWV) switch (epi) { case 0: MI_GEMV_M8(0, NKWV, NWV); break; case 1: MI_GEMV_M8(1, NKWV, NWV); break; \
                                                   case 2: MI_GEMV_M8(2, NKWV, NWV); break; default: MI_GEMV_M8(3, NKWV, NWV); break; }
        if (nk <= 32) { MI_GEMV_M8_E(8, 4) } else { MI_GEMV_M8_E(16, 8) }
#undef MI_GEMV_M8_E
#undef MI_GEMV_M8
#endif
    } else if (!pro.mode && ncols > 1 && K <= 3072 && !xh && g_mi_tuning.f16_bp > 0 && (N + 3) / 4 < 4096) {
        // several plain columns: 16 waves, 4 row groups x K split over 4 (k_gemv_f16_bn, JM = 0). Measured
        // slower than k_gemv_f16 on batched decode (profiles/r06r_batched_plain_gemv_ab.txt): opt-in,
        // f16_bp 1 is accepted by diagnostic builds only
        const dim3 grid((unsigned) ((N + 15) / 16));
        const size_t lds = (size_t) 8 * kp * sizeof(uint16_t) + (size_t) 16 * 4 * 8 * sizeof(float);
        const int epi = e.gelu_table ? 3 : (e.resid ? 2 : (e.bias ? 1 : 0));
        const uint8_t * w = (const uint8_t *) W;
        mi_f16_epilogue es = e;
        es.stamps = mi_stamp_take("k_gemv_f16_bp", grid.x);
#define MI_GEMV_BP(EP, NCHT) hipLaunchKernelGGL((k_gemv_f16_bn<EP, 0, 16, 4, NCHT>), grid, dim3(1024), lds, s, w, nb01, K, N, x, ncols, dst, ycol, es, pro, kp)
#define MI_GEMV_BP_E(NCHT) switch (epi) { case 0: MI_GEMV_BP(0, NCHT); break; case 1: MI_GEMV_BP(1, NCHT); break; \
                                              case 2: MI_GEMV_BP(2, NCHT); break; default: MI_GEMV_BP(3, NCHT); break; }
        if (K <= 1024) { MI_GEMV_BP_E(8) } else { MI_GEMV_BP_E(24) }
#undef MI_GEMV_BP_E
#undef MI_GEMV_BP
    } else if (pro.mode) {  // supported() guarantees one pass (K <= 3072)
        if (K <= 1024) launch_one<4>(per, W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
        else launch_one<12>(per, W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    } else if (one) {
        launch_one<0>(per, W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    } else {
        launch_u<8, false, 0>(W, nb01, K, N, x, xh, ncols, dst, ycol, e, pro, s, nc, ks, rgs);
    }
}
