// mmv_fused_impl.h -- the streaming decode GEMV k_mmv_stream (see mmv_fused.hip for the design),
// its weight-format policies and launchers. Included by one translation unit per weight format
// (mmv_fused_q4k.hip, _q5k, _q40, _q80) so that the kernel instances compile in parallel; each
// exports one mi_mmv_launch_* entry point that mmv_fused.hip's dispatcher calls.
#pragma once

#include <type_traits>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

// the norm prologue replays the CPU's rounding (cpu_order.h turns FMA contraction off); the rest
// of this file keeps the default contraction
#include "cpu_order.h"
#pragma clang fp contract(fast)

namespace {

// ------------------------------------------------------------------ activations in LDS
// layout per member: qs [NC][K] int8 | d [NC][K/QKA] f32 | s32 [NC][K/32] int16

struct lds_act {
    int8_t * qs;
    float * d;
    int16_t * s32;
};

template <int QKA>
__device__ __forceinline__ lds_act lds_carve(uint8_t * lds, int NC, int64_t K) {
    lds_act a;
    a.qs = (int8_t *) lds;
    a.d = (float *) (lds + NC * K);
    a.s32 = (int16_t *) (lds + NC * K + NC * (K / QKA) * 4);
    return a;
}

template <int QKA>
__host__ __device__ constexpr size_t lds_bytes(int NC, int64_t K) {
    return (size_t) NC * (K + (K / QKA) * 4 + (K / 32) * 2);
}

// reference-order scratch (per wave: rows x columns x F::ord_words), after the activations
__host__ __device__ constexpr size_t ord_offset(size_t act) { return (act + 15) & ~(size_t) 15; }

// one 256-element slice (four floats per lane) of column c into LDS
template <int QKA>
__device__ __forceinline__ void quantize_slice(float4 v4, int lane, const lds_act & a, int64_t K, int c, int sl) {
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    int8_t * qs = a.qs + c * K + sl * 256;
    if constexpr (QKA == 256) {
        // Q8_K (quantize_row_q8_K_reference as the reference's gcc -mfma build rounds it)
        uint32_t packed;
        int sum32;
        float dd;
        mi_q8K_superblock(v, lane, packed, sum32, dd);
        *(uint32_t *) (qs + lane * 4) = packed;
        if ((lane & 7) == 0) a.s32[c * (K / 32) + sl * 8 + (lane >> 3)] = (int16_t) sum32;
        if (lane == 0) a.d[c * (K / 256) + sl] = dd;
    } else {
        // Q8_0, AVX2 branch of quantize_row_q8_0 (src/ggml-quants.c:535-618): per 32-block
        // amax, d = amax/127 -> fp16 (RNE), id = 127/amax, q = round-half-even(x*id).
        // 8 lanes hold one block; max over the 8-lane group with DPP.
        float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        uint32_t ab = __float_as_uint(am);
        ab = max(ab, (uint32_t) mi_dpp<MI_DPP_QP_1032>(0, (int) ab));
        ab = max(ab, (uint32_t) mi_dpp<MI_DPP_QP_2301>(0, (int) ab));
        ab = max(ab, (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, (int) ab));
        const float amax = __uint_as_float(ab);
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        uint32_t packed = 0;
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int q = (int) __builtin_rintf(__fmul_rn(v[i], id));
            s += q;
            packed |= ((uint32_t) (q & 0xFF)) << (8 * i);
        }
        s = mi_sum8(s);
        *(uint32_t *) (qs + lane * 4) = packed;
        if ((lane & 7) == 0) {
            const int blk = sl * 8 + (lane >> 3);
            a.d[c * (K / 32) + blk] = mi_h2f(mi_f2h(amax / 127.f));
            a.s32[c * (K / 32) + blk] = (int16_t) s;
        }
    }
}

// Q8_K of one superblock held by a 16-lane row, 16 consecutive elements per lane (a wave quantizes
// four superblocks at once): quantize_row_q8_K_reference (src/ggml-quants.c:3370-3407) as the
// reference's gcc -mfma build rounds it -- the first element of largest |x| keeps its sign
// (a row's max and min decide it; only when +a and -a both occur is the first index looked up),
// iscale = -127/max, q = min(127, RNE(iscale x)) by the fma bit trick, d = 1/iscale, zero
// superblocks d = 0. 16-lane DPP reductions (4 steps) instead of whole-wave ones with readlanes.
// `live`: this row's superblock exists (every lane takes part in the reductions).
__device__ __forceinline__ float mi_dppf_max16(float v) {
    auto f = [](int x) { return __int_as_float(x); };
    auto i = [](float x) { return __float_as_int(x); };
    v = fmaxf(v, f(mi_dpp<MI_DPP_QP_1032>(0, i(v))));
    v = fmaxf(v, f(mi_dpp<MI_DPP_QP_2301>(0, i(v))));
    v = fmaxf(v, f(mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, i(v))));
    v = fmaxf(v, f(mi_dpp<MI_DPP_ROW_MIRROR>(0, i(v))));
    return v;
}
__device__ __forceinline__ uint32_t mi_dpp_umin16(uint32_t v) {
    v = min(v, (uint32_t) mi_dpp<MI_DPP_QP_1032>(0, (int) v));
    v = min(v, (uint32_t) mi_dpp<MI_DPP_QP_2301>(0, (int) v));
    v = min(v, (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, (int) v));
    v = min(v, (uint32_t) mi_dpp<MI_DPP_ROW_MIRROR>(0, (int) v));
    return v;
}
__device__ __forceinline__ void quantize_row16(const float4 (&v4)[4], int lane, const lds_act & a, int64_t K, int c, int sl, bool live) {
    float x[16];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        x[4 * u] = v4[u].x; x[4 * u + 1] = v4[u].y; x[4 * u + 2] = v4[u].z; x[4 * u + 3] = v4[u].w;
    }
    float mx = x[0], mn = x[0];
#pragma unroll
    for (int i = 1; i < 16; i++) {
        mx = fmaxf(mx, x[i]);
        mn = fminf(mn, x[i]);
    }
    mx = mi_dppf_max16(mx);
    mn = -mi_dppf_max16(-mn);
    float vmax = mx >= -mn ? mx : mn;
    const bool tie = mx == -mn && mx != 0.0f;
    if (__any(tie)) {  // +a and -a both largest in some row: the first one (key = 2 index + sign) wins
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 15; i >= 0; i--)
            if (fabsf(x[i]) == mx) key = (uint32_t) ((((lane & 15) * 16 + i) << 1) | (x[i] < 0.0f ? 1 : 0));
        key = mi_dpp_umin16(key);
        if (tie) vmax = (key & 1) ? mn : mx;
    }
    const float iscale = vmax != 0.0f ? -127.f / vmax : 0.0f;
    uint32_t w[4];
    int s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t pk = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float t = __builtin_fmaf(iscale, x[4 * j + e], 12582912.f);
            int q = (__float_as_int(t) & 0x007fffff) - 0x00400000;
            q = q < 127 ? q : 127;
            pk |= ((uint32_t) (q & 0xFF)) << (8 * e);
        }
        w[j] = pk;
        s = mi_dot4((int) pk, 0x01010101, s);
    }
    const int s32 = s + mi_dpp<MI_DPP_QP_1032>(0, s);  // lanes 2m, 2m + 1 of the row: elements 32 m ..
    if (live) {
        *(uint4 *) (a.qs + c * K + sl * 256 + (lane & 15) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
        if ((lane & 1) == 0) a.s32[c * (K / 32) + sl * 8 + ((lane & 15) >> 1)] = (int16_t) s32;
        if ((lane & 15) == 0) a.d[c * (K / 256) + sl] = vmax != 0.0f ? 1.0f / iscale : 0.0f;
    }
}

// ------------------------------------------------------------------ weight formats

template <bool Q5>
struct FmtKQ {
    static constexpr bool KL = false;  // load() does not need K
    static constexpr int QKA = 256;  // activation block
    static constexpr int ITEM = 64;  // elements per item
    static constexpr int BS = Q5 ? 176 : 144;
    struct Regs {
        uint4 hdr, qa, qb;
        uint4 ha, hb;  // Q5 only
    };
    __device__ static __forceinline__ void load(Regs & r, const uint8_t * row, int item) {
        // row is wave-uniform and the lane offsets are 32-bit: scalar base + vector offset
        // addressing, no per-lane 64-bit address arithmetic per row
        const uint32_t s = (uint32_t) item >> 2, j = (uint32_t) item & 3;
        const uint32_t blk = s * BS;
        const uint32_t qp = blk + (Q5 ? 48 : 16) + 32 * j;
        r.hdr = *(const uint4 *) (row + blk);
        r.qa = *(const uint4 *) (row + qp);
        r.qb = *(const uint4 *) (row + qp + 16);
        if constexpr (Q5) {
            r.ha = *(const uint4 *) (row + blk + 16);
            r.hb = *(const uint4 *) (row + blk + 32);
        }
    }
    template <int NC>
    __device__ static __forceinline__ void dot(const Regs & r, int item, const lds_act & a, int64_t K, int ncols, float (&acc)[NC]) {
        const int s = item >> 2, j = item & 3;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) s * 256 + 64 * j);
            const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
            const int alo[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const int ahi[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            const int ss = *(const int *) (a.s32 + c * (K / 32) + s * 8 + 2 * j);
            acc[c] = item_dot(r, j, alo, ahi, ss, a.d[c * (K / 256) + s], acc[c]);
        }
    }
    // one column's operands of an item, held in registers across rows (the item of a lane is the
    // same in every row)
    struct Act {
        int alo[8], ahi[8];
        int ss;
        float ad;
    };
    __device__ static __forceinline__ void act_load(Act & v, int item, const lds_act & a, int64_t K) {
        const int s = item >> 2, j = item & 3;
        const int4 * p = (const int4 *) (a.qs + (int64_t) s * 256 + 64 * j);
        const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
        const int l8[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const int h8[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v.alo[i] = l8[i];
            v.ahi[i] = h8[i];
        }
        v.ss = *(const int *) (a.s32 + s * 8 + 2 * j);
        v.ad = a.d[s];
    }
    __device__ static __forceinline__ float dot_act(const Regs & r, int item, const Act & v, float acc) {
        return item_dot(r, item & 3, v.alo, v.ahi, v.ss, v.ad, acc);
    }
    // one item (superblock s, 64-group j) of one column, the column's quants / 32-sums / scale given
    __device__ static __forceinline__ float item_dot(const Regs & r, int j, const int (&alo)[8], const int (&ahi)[8], int ss, float ad, float acc) {
        const uint32_t q[8] = {r.qa.x, r.qa.y, r.qa.z, r.qa.w, r.qb.x, r.qb.y, r.qb.z, r.qb.w};
        uint32_t qlo[8], qhi[8];
        if constexpr (Q5) {
            const uint32_t h[8] = {r.ha.x, r.ha.y, r.ha.z, r.ha.w, r.hb.x, r.hb.y, r.hb.z, r.hb.w};
#pragma unroll
            for (int i = 0; i < 8; i++) {
                qlo[i] = (q[i] & 0x0F0F0F0Fu) | (((h[i] >> (2 * j)) & 0x01010101u) << 4);
                qhi[i] = ((q[i] >> 4) & 0x0F0F0F0Fu) | (((h[i] >> (2 * j + 1)) & 0x01010101u) << 4);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                qlo[i] = q[i] & 0x0F0F0F0Fu;
                qhi[i] = (q[i] >> 4) & 0x0F0F0F0Fu;
            }
        }
        const float dw = mi_h2f((uint16_t) (r.hdr.x & 0xFFFF));
        const float dmw = mi_h2f((uint16_t) (r.hdr.x >> 16));
        // 6-bit scales / mins of sub-blocks 2j and 2j+1 (get_scale_min_k4,
        // src/ggml-quants.c:1357-1365) without divergent branches: j is lane-dependent
        const uint32_t sh = 16u * (uint32_t) (j & 1);
        const uint32_t x0 = r.hdr.y >> sh, x1 = r.hdr.z >> sh, x2 = r.hdr.w >> sh;
        int sc0, m0, sc1, m1;
        if (j < 2) {  // sub-blocks 0..3: plain 6-bit fields (a select, both sides are cheap)
            sc0 = (int) (x0 & 63);
            sc1 = (int) ((x0 >> 8) & 63);
            m0 = (int) (x1 & 63);
            m1 = (int) ((x1 >> 8) & 63);
        } else {      // sub-blocks 4..7: low 4 bits from bytes 8..11, high 2 bits from bytes 0..7
            sc0 = (int) ((x2 & 0xF) | (((x0 >> 6) & 3) << 4));
            sc1 = (int) (((x2 >> 8) & 0xF) | (((x0 >> 14) & 3) << 4));
            m0 = (int) (((x2 >> 4) & 0xF) | (((x1 >> 6) & 3) << 4));
            m1 = (int) (((x2 >> 12) & 0xF) | (((x1 >> 14) & 3) << 4));
        }
        int lo = 0, hi = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            lo = mi_dot4((int) qlo[i], alo[i], lo);
            hi = mi_dot4((int) qhi[i], ahi[i], hi);
        }
        // sc*lo + sc*hi and m*bsum + m*bsum in f32 are exact (|.| < 2^24: 63*32*31*127 and
        // 63*32*128 per term), i.e. (float) of the reference's int32 sums, without the
        // quarter-rate 32-bit integer multiplies
        const float sumi = fmaf((float) sc1, (float) hi, (float) sc0 * (float) lo);
        const float summ = fmaf((float) m1, (float) (ss >> 16), (float) m0 * (float) (int) (int16_t) (ss & 0xFFFF));
        // explicit fmas (the file contracts freely): the same bits in every kernel that inlines this
        return fmaf(ad, fmaf(-dmw, summ, dw * sumi), acc);
    }

    // CPU order (see ord_* below): per item (superblock s, 64-group j) the reference's eight int32
    // lanes l -- sc[2j] * (bytes 4l..4l+3 of the low nibbles . q8) + sc[2j+1] * (high nibbles) --
    // summed over the superblock's four items (a DPP quad: items 4s..4s+3 sit on adjacent lanes),
    // plus the mins lane m[2j] * bsum32[2j] + m[2j+1] * bsum32[2j+1]. Entry of superblock sb in the
    // scratch: [0..7] the eight int32 sums, [8..11] the four mins lanes (Q5_K: [8] their sum),
    // [12] d = y.d * x.d, [13] dmin = -(y.d * x.dmin).
    template <int NC>
    __device__ static __forceinline__ void dot_ord(const Regs & r, int item, int slot, const lds_act & a, int64_t K, int ncols,
                                                   uint32_t * scr, int cs, int) {
        const int s = item >> 2, j = item & 3;
        const uint32_t q[8] = {r.qa.x, r.qa.y, r.qa.z, r.qa.w, r.qb.x, r.qb.y, r.qb.z, r.qb.w};
        uint32_t qlo[8], qhi[8];
        if constexpr (Q5) {
            const uint32_t h[8] = {r.ha.x, r.ha.y, r.ha.z, r.ha.w, r.hb.x, r.hb.y, r.hb.z, r.hb.w};
#pragma unroll
            for (int i = 0; i < 8; i++) {
                qlo[i] = (q[i] & 0x0F0F0F0Fu) | (((h[i] >> (2 * j)) & 0x01010101u) << 4);
                qhi[i] = ((q[i] >> 4) & 0x0F0F0F0Fu) | (((h[i] >> (2 * j + 1)) & 0x01010101u) << 4);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                qlo[i] = q[i] & 0x0F0F0F0Fu;
                qhi[i] = (q[i] >> 4) & 0x0F0F0F0Fu;
            }
        }
        const float dw = mi_h2f((uint16_t) (r.hdr.x & 0xFFFF));
        const float dmw = mi_h2f((uint16_t) (r.hdr.x >> 16));
        const uint32_t sh = 16u * (uint32_t) (j & 1);
        const uint32_t x0 = r.hdr.y >> sh, x1 = r.hdr.z >> sh, x2 = r.hdr.w >> sh;
        int sc0, m0, sc1, m1;
        if (j < 2) {
            sc0 = (int) (x0 & 63);
            sc1 = (int) ((x0 >> 8) & 63);
            m0 = (int) (x1 & 63);
            m1 = (int) ((x1 >> 8) & 63);
        } else {
            sc0 = (int) ((x2 & 0xF) | (((x0 >> 6) & 3) << 4));
            sc1 = (int) (((x2 >> 8) & 0xF) | (((x0 >> 14) & 3) << 4));
            m0 = (int) (((x2 >> 4) & 0xF) | (((x1 >> 6) & 3) << 4));
            m1 = (int) (((x2 >> 12) & 0xF) | (((x1 >> 14) & 3) << 4));
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) s * 256 + 64 * j);
            const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
            const int alo[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const int ahi[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            int v[8];
#pragma unroll
            for (int l = 0; l < 8; l++) {
                // |products| < 2^23: the 24-bit multiplier is exact
                v[l] = __mul24(sc0, mi_dot4((int) qlo[l], alo[l], 0)) + __mul24(sc1, mi_dot4((int) qhi[l], ahi[l], 0));
                v[l] += mi_dpp<MI_DPP_QP_1032>(0, v[l]);
                v[l] += mi_dpp<MI_DPP_QP_2301>(0, v[l]);
            }
            const int ss = *(const int *) (a.s32 + c * (K / 32) + s * 8 + 2 * j);
            int pm = __mul24(m0, (int) (int16_t) (ss & 0xFFFF)) + __mul24(m1, ss >> 16);
            if constexpr (Q5) {
                pm += mi_dpp<MI_DPP_QP_1032>(0, pm);
                pm += mi_dpp<MI_DPP_QP_2301>(0, pm);
            }
            uint32_t * e = scr + c * cs + (slot >> 2) * 16;
            // lane j stores sums 2j and 2j+1 (all four lanes hold all eight after the quad sums),
            // as floats (exact: |sum| < 2^24), i.e. the reference's _mm256_cvtepi32_ps
            const int w0 = j == 0 ? v[0] : j == 1 ? v[2] : j == 2 ? v[4] : v[6];
            const int w1 = j == 0 ? v[1] : j == 1 ? v[3] : j == 2 ? v[5] : v[7];
            *(uint2 *) (e + 2 * j) = make_uint2(__float_as_uint((float) w0), __float_as_uint((float) w1));
            if (!Q5 || j == 0) e[8 + j] = __float_as_uint((float) pm);
            const float yd = a.d[c * (K / 256) + s];
            if (j == 2) e[12] = __float_as_uint(yd * dw);
            if (j == 3) e[13] = __float_as_uint(-(yd * dmw));
        }
    }
    // one chain step per superblock: acc[l] = fma(d, (float) sumi[l], acc[l]) (the reference's
    // _mm256_fmadd_ps) and the mins accumulator: Q4_K four lanes acc_m[k] = fma(dmin, prod[k],
    // acc_m[k]) (_mm_fmadd_ps), Q5_K one scalar summs += dmin * hsum(prod) (contracted by the
    // reference's -mfma build)
    __device__ static __forceinline__ void chain(const uint32_t * scr, int l, int n_items, int, float & A, float & M) {
        const float * e = (const float *) scr;
        const int nsb = n_items >> 2;
        const int lm = 8 + (Q5 ? 0 : (l & 3));
        for (int sb = 0; sb < nsb; sb++, e += 16) {
            A = fmaf(e[12], e[l], A);
            M = fmaf(e[13], e[lm], M);
        }
    }
    // scratch words per (row, column): one 16-word entry per superblock (+8: bank spread)
    static int ord_words(int nitems, int & stride) {
        stride = 0;
        return 16 * (nitems / 4) + 8;
    }
    __device__ static __forceinline__ float finish(float A, float M) {
        float z = A + __shfl_xor(A, 4, 8);
        z = z + __shfl_xor(z, 2, 8);
        z = z + __shfl_xor(z, 1, 8);
        if constexpr (Q5) return z + M;
        float m = M + __shfl_xor(M, 2, 8);
        m = m + __shfl_xor(m, 1, 8);
        return z + m;
    }
};

// Q4_0 (18 B) / Q8_0 (34 B) blocks: 2-byte aligned. Load the dwords covering the quants
// (aligned down) and re-align with v_alignbyte; d is a separate 2-byte load.
template <bool Q8>
struct FmtQ0 {
    static constexpr bool KL = false;
    static constexpr int QKA = 32;
    static constexpr int ITEM = 32;
    static constexpr int BS = Q8 ? 34 : 18;
    static constexpr int NQ = Q8 ? 8 : 4;  // quant dwords per block
    struct Regs {
        uint32_t w[NQ + 1];  // the dwords covering d and the quants
        uint32_t off;        // byte offset of the block in w[0]: 0 or 2
    };
    __device__ static __forceinline__ void load(Regs & r, const uint8_t * row, int item) {
        // rows start 16-byte aligned (fused_mv_eligible), so the block's misalignment is a
        // function of the item alone; dword loads only (a 16-bit load of d gets a zero-extend
        // the compiler places right behind the load, which waits for it), on 32-bit lane offsets
        // from the wave-uniform row pointer
        const uint32_t blk = (uint32_t) item * BS;
        r.off = blk & 2;
        const uint32_t base = blk - r.off;
#pragma unroll
        for (int i = 0; i <= NQ; i++) r.w[i] = *(const uint32_t *) (row + base + 4 * i);  // 256 B tail slack
    }
    template <int NC>
    __device__ static __forceinline__ void dot(const Regs & r, int item, const lds_act & a, int64_t K, int ncols, float (&acc)[NC]) {
        // d = bytes off..off+1 of w[0]; the quants start at byte off + 2
        uint32_t t[NQ];
#pragma unroll
        for (int i = 0; i < NQ; i++) t[i] = r.off ? r.w[i + 1] : __builtin_amdgcn_alignbyte(r.w[i + 1], r.w[i], 2);
        const uint32_t dbits = (r.off ? r.w[0] >> 16 : r.w[0]) & 0xFFFF;
        const float dw = mi_h2f((uint16_t) dbits);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) item * 32);
            const int4 a0 = p[0], a1 = p[1];
            const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            acc[c] = block_dot(t, dw, av, Q8 ? 0 : (int) a.s32[c * (K / 32) + item], a.d[c * (K / 32) + item], acc[c]);
        }
    }
    __device__ static __forceinline__ float block_dot(const uint32_t (&t)[NQ], float dw, const int (&av)[8], int s32, float da, float acc) {
        int sumi = 0;
        if constexpr (Q8) {
#pragma unroll
            for (int i = 0; i < 8; i++) sumi = mi_dot4((int) t[i], av[i], sumi);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                sumi = mi_dot4((int) (t[i] & 0x0F0F0F0Fu), av[i], sumi);
                sumi = mi_dot4((int) ((t[i] >> 4) & 0x0F0F0F0Fu), av[i + 4], sumi);
            }
            sumi -= 8 * s32;  // (q - 8) * y
        }
        return fmaf((float) sumi, dw * da, acc);
    }
    struct Act {
        int av[8];
        int s32;
        float da;
    };
    __device__ static __forceinline__ void act_load(Act & v, int item, const lds_act & a, int64_t K) {
        const int4 * p = (const int4 *) (a.qs + (int64_t) item * 32);
        const int4 a0 = p[0], a1 = p[1];
        const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int i = 0; i < 8; i++) v.av[i] = av[i];
        v.s32 = Q8 ? 0 : (int) a.s32[item];
        v.da = a.d[item];
    }
    __device__ static __forceinline__ float dot_act(const Regs & r, int, const Act & v, float acc) {
        uint32_t t[NQ];
#pragma unroll
        for (int i = 0; i < NQ; i++) t[i] = r.off ? r.w[i + 1] : __builtin_amdgcn_alignbyte(r.w[i + 1], r.w[i], 2);
        const uint32_t dbits = (r.off ? r.w[0] >> 16 : r.w[0]) & 0xFFFF;
        return block_dot(t, mi_h2f((uint16_t) dbits), v.av, v.s32, v.da, acc);
    }

    // CPU order: the reference's eight int32 lanes l of mul_sum_i8_pairs_float -- elements 4l..4l+3
    // (Q4_0: low nibbles for l < 4, high nibbles of bytes 4(l-4).. for l >= 4, minus 8) -- and
    // d = x.d * y.d, stored transposed: scratch [l][slot] (row stride 68 words), d at [8][slot].
    template <int NC>
    __device__ static __forceinline__ void dot_ord(const Regs & r, int item, int slot, const lds_act & a, int64_t K, int ncols,
                                                   uint32_t * scr, int cs, int S) {
        uint32_t t[NQ];
#pragma unroll
        for (int i = 0; i < NQ; i++) t[i] = r.off ? r.w[i + 1] : __builtin_amdgcn_alignbyte(r.w[i + 1], r.w[i], 2);
        const uint32_t dbits = (r.off ? r.w[0] >> 16 : r.w[0]) & 0xFFFF;
        const float dw = mi_h2f((uint16_t) dbits);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) item * 32);
            const int4 a0 = p[0], a1 = p[1];
            const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            uint32_t * e = scr + c * cs + slot;
#pragma unroll
            for (int l = 0; l < 8; l++) {
                int q;
                if constexpr (Q8) {
                    q = mi_dot4((int) t[l], av[l], 0);
                } else {
                    const uint32_t nib = l < 4 ? (t[l] & 0x0F0F0F0Fu) : ((t[l - 4] >> 4) & 0x0F0F0F0Fu);
                    q = mi_dot4((int) nib, av[l], mi_dot4((int) 0xF8F8F8F8u, av[l], 0));  // (q - 8) . y
                }
                e[l * S] = __float_as_uint((float) q);  // exact; _mm256_cvtepi32_ps
            }
            e[8 * S] = __float_as_uint(dw * a.d[c * (K / 32) + item]);
        }
    }
    // acc[l] = fma(d_i, (float) q[i][l], acc[l]) over the blocks in order (_mm256_fmadd_ps)
    __device__ static __forceinline__ void chain(const uint32_t * scr, int l, int n_items, int S, float & A, float & M) {
        (void) M;
        const float * q = (const float *) scr + l * S;
        const float * d = (const float *) scr + 8 * S;
        int i = 0;
        for (; i + 4 <= n_items; i += 4) {
            const float4 qq = *(const float4 *) (q + i);
            const float4 dd = *(const float4 *) (d + i);
            A = fmaf(dd.x, qq.x, A);
            A = fmaf(dd.y, qq.y, A);
            A = fmaf(dd.z, qq.z, A);
            A = fmaf(dd.w, qq.w, A);
        }
        for (; i < n_items; i++) A = fmaf(d[i], q[i], A);
    }
    // scratch words per (row, column): 9 rows (8 lanes + d) of S >= nitems words; S = 4 (mod 32)
    // keeps the eight lanes' 16-byte chain reads on distinct banks
    static int ord_words(int nitems, int & stride) {
        int S = (nitems + 3) & ~3;
        while (S % 32 != 4) S += 4;
        stride = S;
        return 9 * S;
    }
    __device__ static __forceinline__ float finish(float A, float) {
        // hsum_float_8: ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
        float z = A + __shfl_xor(A, 4, 8);
        z = z + __shfl_xor(z, 2, 8);
        return z + __shfl_xor(z, 1, 8);
    }
};

// Q4_0 in pairs of blocks (tree order only): an item is 2 blocks = 36 B, 4-byte aligned, so 9
// dword loads cover it with no slack, the second block's quants are whole dwords (only the
// first's need v_alignbyte), and a K = 4096 row is one item per lane.
// one pair of Q4_0 blocks against its q8_0 activations: block quants t0 / t1 (16 bytes each), scales
// dw0 / dw1; shared by FmtQ0Pair and FmtQ0R, so the canonical and the repacked layouts give the
// same bits
__device__ __forceinline__ float q0pair_dot(const uint32_t (&t0)[4], const uint32_t (&t1)[4], float dw0, float dw1, const int (&av0)[8],
                                            const int (&av1)[8], uint32_t ss, float2 da, float acc) {
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s0 = mi_dot4((int) (t0[i] & 0x0F0F0F0Fu), av0[i], s0);
        s0 = mi_dot4((int) ((t0[i] >> 4) & 0x0F0F0F0Fu), av0[i + 4], s0);
        s1 = mi_dot4((int) (t1[i] & 0x0F0F0F0Fu), av1[i], s1);
        s1 = mi_dot4((int) ((t1[i] >> 4) & 0x0F0F0F0Fu), av1[i + 4], s1);
    }
    s0 -= 8 * (int) (int16_t) (ss & 0xFFFF);
    s1 -= 8 * (int) (int16_t) (ss >> 16);
    acc = fmaf((float) s0, dw0 * da.x, acc);
    return fmaf((float) s1, dw1 * da.y, acc);
}

struct FmtQ0Pair {
    static constexpr bool KL = false;
    static constexpr int QKA = 32;
    static constexpr int ITEM = 64;
    struct Regs {
        uint32_t w[9];
    };
    __device__ static __forceinline__ void load(Regs & r, const uint8_t * row, int item) {
        const uint8_t * p = row + (uint32_t) item * 36;
#pragma unroll
        for (int i = 0; i < 9; i++) r.w[i] = *(const uint32_t *) (p + 4 * i);
    }
    template <int NC>
    __device__ static __forceinline__ void dot(const Regs & r, int item, const lds_act & a, int64_t K, int ncols, float (&acc)[NC]) {
        // block 0: d = bytes 0..1, quants bytes 2..17; block 1: d = bytes 18..19, quants 20..35
        uint32_t t0[4];
#pragma unroll
        for (int i = 0; i < 4; i++) t0[i] = __builtin_amdgcn_alignbyte(r.w[i + 1], r.w[i], 2);
        const float dw0 = mi_h2f((uint16_t) (r.w[0] & 0xFFFF));
        const float dw1 = mi_h2f((uint16_t) (r.w[4] >> 16));
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) item * 64);
            const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
            const int av0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const int av1[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            const uint32_t ss = *(const uint32_t *) (a.s32 + c * (K / 32) + 2 * item);  // both blocks' sums
            const float2 da = *(const float2 *) (a.d + c * (K / 32) + 2 * item);
            acc[c] = pair_dot(r, t0, dw0, dw1, av0, av1, ss, da, acc[c]);
        }
    }
    __device__ static __forceinline__ float pair_dot(const Regs & r, const uint32_t (&t0)[4], float dw0, float dw1, const int (&av0)[8],
                                                     const int (&av1)[8], uint32_t ss, float2 da, float acc) {
        const uint32_t t1[4] = {r.w[5], r.w[6], r.w[7], r.w[8]};
        return q0pair_dot(t0, t1, dw0, dw1, av0, av1, ss, da, acc);
    }
    struct Act {
        int av0[8], av1[8];
        uint32_t ss;
        float2 da;
    };
    __device__ static __forceinline__ void act_load(Act & v, int item, const lds_act & a, int64_t K) {
        const int4 * p = (const int4 *) (a.qs + (int64_t) item * 64);
        const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
        const int av0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const int av1[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v.av0[i] = av0[i];
            v.av1[i] = av1[i];
        }
        v.ss = *(const uint32_t *) (a.s32 + 2 * item);
        v.da = *(const float2 *) (a.d + 2 * item);
    }
    __device__ static __forceinline__ float dot_act(const Regs & r, int, const Act & v, float acc) {
        uint32_t t0[4];
#pragma unroll
        for (int i = 0; i < 4; i++) t0[i] = __builtin_amdgcn_alignbyte(r.w[i + 1], r.w[i], 2);
        return pair_dot(r, t0, mi_h2f((uint16_t) (r.w[0] & 0xFFFF)), mi_h2f((uint16_t) (r.w[4] >> 16)), v.av0, v.av1, v.ss, v.da, acc);
    }
};

// Q4_0 block pairs on the 16-byte-aligned repacked copy (tree order only; mmq_planes.hip
// k_q40_repack): per row [K/32 blocks x 16 quant bytes][K/32 x f16 d], so item (pair) p is two
// aligned dwordx4 at 32 p and one dword at K/2 + 4 p -- consecutive lanes read consecutive bytes.
// The same pair arithmetic as FmtQ0Pair (q0pair_dot): bit-identical outputs.
struct FmtQ0R {
    static constexpr bool KL = true;  // load() needs K (the scales follow the row's quants)
    static constexpr int QKA = 32;
    static constexpr int ITEM = 64;
    struct Regs {
        uint4 q0, q1;
        uint32_t d;
    };
    __device__ static __forceinline__ void load(Regs & r, const uint8_t * row, int item, int64_t K) {
        const uint32_t o = (uint32_t) item * 32;
        r.q0 = *(const uint4 *) (row + o);
        r.q1 = *(const uint4 *) (row + o + 16);
        r.d = *(const uint32_t *) (row + (uint32_t) (K / 2) + 4 * (uint32_t) item);
    }
    __device__ static __forceinline__ float pdot(const Regs & r, const int (&av0)[8], const int (&av1)[8], uint32_t ss, float2 da, float acc) {
        const uint32_t t0[4] = {r.q0.x, r.q0.y, r.q0.z, r.q0.w};
        const uint32_t t1[4] = {r.q1.x, r.q1.y, r.q1.z, r.q1.w};
        return q0pair_dot(t0, t1, mi_h2f((uint16_t) (r.d & 0xFFFF)), mi_h2f((uint16_t) (r.d >> 16)), av0, av1, ss, da, acc);
    }
    template <int NC>
    __device__ static __forceinline__ void dot(const Regs & r, int item, const lds_act & a, int64_t K, int ncols, float (&acc)[NC]) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) item * 64);
            const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
            const int av0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const int av1[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            const uint32_t ss = *(const uint32_t *) (a.s32 + c * (K / 32) + 2 * item);
            const float2 da = *(const float2 *) (a.d + c * (K / 32) + 2 * item);
            acc[c] = pdot(r, av0, av1, ss, da, acc[c]);
        }
    }
    using Act = FmtQ0Pair::Act;
    __device__ static __forceinline__ void act_load(Act & v, int item, const lds_act & a, int64_t K) { FmtQ0Pair::act_load(v, item, a, K); }
    __device__ static __forceinline__ float dot_act(const Regs & r, int, const Act & v, float acc) { return pdot(r, v.av0, v.av1, v.ss, v.da, acc); }
};

// Q8_0 blocks on the 16-byte-aligned repacked copy (tree order only; k_q80_repack): per row [K/32
// blocks x 32 quant bytes][K/32 x f16 d], item = one block as for FmtQ0<true> (lane l: blocks l,
// l + 64, ...) with FmtQ0<true>'s arithmetic (block_dot): bit-identical outputs. A lane's block is
// two aligned dwordx4; its scale comes with its neighbour's in one dword (selected by parity).
struct FmtQ8R {
    static constexpr bool KL = true;
    static constexpr int QKA = 32;
    static constexpr int ITEM = 32;
    using Q = FmtQ0<true>;
    struct Regs {
        uint4 q0, q1;
        uint32_t dd;
        uint32_t odd;  // 16 if the item is odd (its d in the high half of dd)
    };
    __device__ static __forceinline__ void load(Regs & r, const uint8_t * row, int item, int64_t K) {
        const uint32_t o = (uint32_t) item * 32;
        r.q0 = *(const uint4 *) (row + o);
        r.q1 = *(const uint4 *) (row + o + 16);
        r.dd = *(const uint32_t *) (row + (uint32_t) K + 4 * ((uint32_t) item >> 1));
        r.odd = ((uint32_t) item & 1) * 16;
    }
    __device__ static __forceinline__ float bdot(const Regs & r, const int (&av)[8], float da, float acc) {
        const uint32_t t[8] = {r.q0.x, r.q0.y, r.q0.z, r.q0.w, r.q1.x, r.q1.y, r.q1.z, r.q1.w};
        return Q::block_dot(t, mi_h2f((uint16_t) ((r.dd >> r.odd) & 0xFFFF)), av, 0, da, acc);
    }
    template <int NC>
    __device__ static __forceinline__ void dot(const Regs & r, int item, const lds_act & a, int64_t K, int ncols, float (&acc)[NC]) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            const int4 * p = (const int4 *) (a.qs + c * K + (int64_t) item * 32);
            const int4 a0 = p[0], a1 = p[1];
            const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            acc[c] = bdot(r, av, a.d[c * (K / 32) + item], acc[c]);
        }
    }
    using Act = Q::Act;
    __device__ static __forceinline__ void act_load(Act & v, int item, const lds_act & a, int64_t K) { Q::act_load(v, item, a, K); }
    __device__ static __forceinline__ float dot_act(const Regs & r, int, const Act & v, float acc) { return bdot(r, v.av, v.da, acc); }
};

// a format's weight load (FmtQ0R's needs the row length)
template <class F>
__device__ __forceinline__ void fmt_load(typename F::Regs & r, const uint8_t * row, int item, int64_t K) {
    if constexpr (F::KL) F::load(r, row, item, K);
    else F::load(r, row, item);
}

// ------------------------------------------------------------------ the streaming kernel

// IPL = items per lane held in the prefetch ring (further items of long rows are loaded
// in-line); PD = rows in flight ahead of the row being computed.
// norm|rms_norm -> mul(g) -> add(b) of the group's activation columns into LDS (f32), by wave 0
// with each column in registers -- the arithmetic of k_norm (ops.hip) and of the F16 GEMV's
// prologue: certified double means, then every step rounded separately. norm_cols: a column's x,
// g, b in registers (every load unconditional at a clamped index, then a select: a load under a
// lane branch makes the compiler wait for it at the branch's join; absent g / b read x instead).
struct norm_cols {
    static constexpr int kJ = (int) (kMiMmvProMaxK / 64);
    float v[kJ], gv[kJ], bv[kJ];
};

__device__ __forceinline__ void norm_cols_load(const mi_mmv_group & g, const char * X, int c, norm_cols & r) {
    const int lane = threadIdx.x & 63;
    const int64_t K = g.K;
    const float * xc = (const float *) (X + c * g.xcol);
    const float * gp = g.pro.g ? g.pro.g : xc;
    const float * bp = g.pro.b ? g.pro.b : xc;
#pragma unroll
    for (int j = 0; j < norm_cols::kJ; j++) {
        const int64_t k = (int64_t) j * 64 + lane;
        const bool in = k < K;
        const int64_t kc = in ? k : K - 1;
        const float xv = xc[kc], gl = gp[kc], bl = bp[kc];
        r.v[j] = in ? xv : 0.0f;
        r.gv[j] = in && g.pro.g ? gl : 1.0f;
        r.bv[j] = in && g.pro.b ? bl : 0.0f;
    }
}

// r: column 0, already loaded (before the weight stream, so that vmcnt does not make it wait for
// the weights); the other columns are loaded here
__device__ void norm_prologue(const mi_mmv_group & g, const char * X, int ncols, float * xn, norm_cols & r) {
    constexpr int kJ = norm_cols::kJ;
    const int lane = threadIdx.x & 63;
    const int64_t K = g.K;
    for (int c = 0; c < ncols; c++) {
        if (c > 0) norm_cols_load(g, X, c, r);
        float scale;
        if (g.pro.mode == 2) {
            const float mean = wave_mean_cpu_order<true, kJ>(r.v, K);
            if (c == 0) MI_STAMP(g.stamps, 6);  // (diagnostic: first column's x landed, mean certified)
            scale = 1.0f / sqrtf(add_rn(mean, g.pro.eps));
        } else {
            const float mean = wave_mean_cpu_order<false, kJ>(r.v, K);
            if (c == 0) MI_STAMP(g.stamps, 6);
#pragma unroll
            for (int j = 0; j < kJ; j++) r.v[j] = sub_rn(r.v[j], mean);
            const float variance = wave_mean_cpu_order<true, kJ>(r.v, K);
            scale = 1.0f / sqrtf(add_rn(variance, g.pro.eps));
        }
        if (c == 0) MI_STAMP(g.stamps, 5);  // (diagnostic: first column's scale)
#pragma unroll
        for (int j = 0; j < kJ; j++) {
            const int64_t k = (int64_t) j * 64 + lane;
            if (k < K) {
                float y = mul_rn(r.v[j], scale);
                if (g.pro.g) y = mul_rn(y, r.gv[j]);
                if (g.pro.b) y = add_rn(y, r.bv[j]);
                xn[c * K + k] = y;
            }
        }
    }
}

// One column with a Q8_K activation (Q4_K / Q5_K weights), K a multiple of 256 up to
// kMiMmvProMaxK: wave 0 holds the column four consecutive elements per lane (k = 256 j + 4 l + i,
// float4 loads), normalizes it in registers and quantizes each 256-slice straight into the LDS
// activations (quantize_slice: the layout mi_q8K_superblock takes) -- no normalized copy through
// LDS, no second barrier and no re-read (round 6). The arithmetic of norm_prologue element for
// element: certified double mean / variance (wave_mean_cpu_order4), then every step rounded.
struct norm_cols4 {
    static constexpr int kJ = (int) (kMiMmvProMaxK / 256);
    float4 v[kJ], gv[kJ], bv[kJ];
};

__device__ __forceinline__ void norm_cols4_load(const mi_mmv_group & g, const char * X, norm_cols4 & r) {
    const int lane = threadIdx.x & 63;
    const int64_t K = g.K;
    const float * xc = (const float *) X;
    const float * gp = g.pro.g ? g.pro.g : xc;
    const float * bp = g.pro.b ? g.pro.b : xc;
#pragma unroll
    for (int j = 0; j < norm_cols4::kJ; j++) {
        const int64_t k = (int64_t) j * 256 + lane * 4;
        const int64_t kc = k < K ? k : K - 4;  // (unconditional loads at clamped addresses; unused past K)
        r.v[j] = *(const float4 *) (xc + kc);
        r.gv[j] = *(const float4 *) (gp + kc);
        r.bv[j] = *(const float4 *) (bp + kc);
    }
}

// Q8_K of J 256-slices held four consecutive floats per lane (slice j: v[j]), all slices' steps
// interleaved (mi_q8K_superblock's arithmetic per slice: the first element of largest |x| keeps its
// sign, iscale = -127 / max, q = min(127, RNE via the fma bit trick), d = 1 / iscale; zero slices
// d = 0), so the slices' wave reductions and divisions overlap instead of running one after the other
template <int J>
__device__ __forceinline__ void quantize_slices_q8K(const float (&v)[J][4], int nsl, int lane, const lds_act & a, int64_t K) {
    uint32_t ab[J];
    int bi[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        float best = 0.0f;
        int bidx = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float ax = fabsf(v[j][i]);
            if (ax > best) { best = ax; bidx = i; }  // first occurrence within the lane
        }
        ab[j] = __float_as_uint(best);
        bi[j] = bidx;
    }
    uint32_t am[J], key[J];
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = ab[j];
    auto mx = [](uint32_t x, uint32_t y) { return x > y ? x : y; };
    auto mn = [](uint32_t x, uint32_t y) { return x < y ? x : y; };
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_QP_1032>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_QP_2301>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_ROW_MIRROR>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_ROW_BCAST15, 0xA>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) am[j] = mx(am[j], (uint32_t) mi_dpp<MI_DPP_ROW_BCAST31, 0xC>(0, (int) am[j]));
#pragma unroll
    for (int j = 0; j < J; j++) {
        am[j] = (uint32_t) __builtin_amdgcn_readlane((int) am[j], 63);
        key[j] = ab[j] == am[j] ? (uint32_t) (lane * 4 + bi[j]) : 0xFFFFFFFFu;
    }
    constexpr int kId = -1;
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_QP_1032>(kId, (int) key[j]));
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_QP_2301>(kId, (int) key[j]));
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_ROW_HALF_MIRROR>(kId, (int) key[j]));
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_ROW_MIRROR>(kId, (int) key[j]));
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_ROW_BCAST15, 0xA>(kId, (int) key[j]));
#pragma unroll
    for (int j = 0; j < J; j++) key[j] = mn(key[j], (uint32_t) mi_dpp<MI_DPP_ROW_BCAST31, 0xC>(kId, (int) key[j]));
    float iscale[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        const uint32_t idx = (uint32_t) __builtin_amdgcn_readlane((int) key[j], 63);
        const int owner = (int) (idx >> 2), sel = (int) (idx & 3);
        const float mine = sel == 0 ? v[j][0] : sel == 1 ? v[j][1] : sel == 2 ? v[j][2] : v[j][3];
        const float vmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), owner & 63));
        iscale[j] = am[j] != 0 ? -127.f / vmax : 0.0f;
    }
    int s[J];
    uint32_t packed[J];
#pragma unroll
    for (int j = 0; j < J; j++) {
        packed[j] = 0;
        s[j] = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float t = __builtin_fmaf(iscale[j], v[j][i], 12582912.f);
            int q = (__float_as_int(t) & 0x007fffff) - 0x00400000;
            q = q < 127 ? q : 127;
            if (am[j] == 0) q = 0;
            s[j] += q;
            packed[j] |= ((uint32_t) (q & 0xFF)) << (8 * i);
        }
    }
#pragma unroll
    for (int j = 0; j < J; j++) s[j] = mi_sum8(s[j]);
#pragma unroll
    for (int j = 0; j < J; j++) {
        if (j >= nsl) break;  // wave-uniform
        *(uint32_t *) (a.qs + j * 256 + lane * 4) = packed[j];
        if ((lane & 7) == 0) a.s32[j * 8 + (lane >> 3)] = (int16_t) s[j];
        if (lane == 0) a.d[j] = am[j] != 0 ? 1.0f / iscale[j] : 0.0f;
    }
}

__device__ void norm_quant_prologue1(const mi_mmv_group & g, norm_cols4 & r, const lds_act & act) {
    constexpr int kJ = norm_cols4::kJ;
    const int lane = threadIdx.x & 63;
    const int64_t K = g.K;
    const int nsl = (int) (K / 256);
    float scale;
    if (g.pro.mode == 2) {
        const float mean = wave_mean_cpu_order4<true, kJ>(r.v, K);
        MI_STAMP(g.stamps, 6);
        scale = 1.0f / sqrtf(add_rn(mean, g.pro.eps));
    } else {
        const float mean = wave_mean_cpu_order4<false, kJ>(r.v, K);
        MI_STAMP(g.stamps, 6);
#pragma unroll
        for (int j = 0; j < kJ; j++) {
            r.v[j].x = sub_rn(r.v[j].x, mean);
            r.v[j].y = sub_rn(r.v[j].y, mean);
            r.v[j].z = sub_rn(r.v[j].z, mean);
            r.v[j].w = sub_rn(r.v[j].w, mean);
        }
        const float variance = wave_mean_cpu_order4<true, kJ>(r.v, K);
        scale = 1.0f / sqrtf(add_rn(variance, g.pro.eps));
    }
    MI_STAMP(g.stamps, 5);
    float y[kJ][4];
#pragma unroll
    for (int j = 0; j < kJ; j++) {
        const float e[4] = {r.v[j].x, r.v[j].y, r.v[j].z, r.v[j].w};
        const float ge[4] = {r.gv[j].x, r.gv[j].y, r.gv[j].z, r.gv[j].w};
        const float be[4] = {r.bv[j].x, r.bv[j].y, r.bv[j].z, r.bv[j].w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            float t = mul_rn(e[i], scale);
            if (g.pro.g) t = mul_rn(t, ge[i]);
            if (g.pro.b) t = add_rn(t, be[i]);
            y[j][i] = j < nsl ? t : 0.0f;  // (slices past K: zero, not stored)
        }
    }
    quantize_slices_q8K<kJ>(y, nsl, lane, act, K);
}

// one output element, through the graph's epilogue: + bias[row], then + resid or GELU (the fp16
// table lookup of ggml_vec_gelu_f32 with its +-10 clamps), then the K/V-cache row copies -- each
// step rounded as its own node would round it
// The epilogue operands of a wave's first row, requested in the prologue (a load at store time adds
// a dependent memory round trip at the end of the kernel -- at GPT-2's sizes one row per wave)
template <int NC>
struct epi_pre {
    int row = -1;
    float bias = 0.0f;
    float res[NC];
};
template <int NC>
__device__ __forceinline__ void epi_prefetch(const mi_mmv_group & g, int row, const char * any, epi_pre<NC> & p) {
    const mi_mmv_group::epilogue & e = g.epi;
    p.row = row;
    // unconditional loads at valid addresses (an absent operand reads `any`; its value is unused)
    p.bias = *(e.bias ? e.bias + row : (const float *) any);
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const int cc = c < g.ncols ? c : g.ncols - 1;
        p.res[c] = *(const float *) (e.resid ? e.resid + cc * e.resid_nb1 + (size_t) row * sizeof(float) : any);
    }
}

template <bool X, int NC = 1>
__device__ __forceinline__ void store_out(const mi_mmv_group & g, float * dst, int c, int row, float v, const epi_pre<NC> * pre = nullptr) {
    if constexpr (!X) {
        *(float *) ((char *) dst + c * g.ycol + (size_t) row * sizeof(float)) = v;
        return;
    }
    const mi_mmv_group::epilogue & e = g.epi;
    const bool hit = pre && row == pre->row;
    float pr = pre ? pre->res[0] : 0.0f;
    if (pre) {
#pragma unroll
        for (int cc = 1; cc < NC; cc++)
            if (c == cc) pr = pre->res[cc];
    }
    if (e.bias) v = v + (hit ? pre->bias : e.bias[row]);
    if (e.resid) v = v + (hit ? pr : *(const float *) (e.resid + c * e.resid_nb1 + (size_t) row * sizeof(float)));
    else if (e.gelu_table) v = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : mi_h2f(e.gelu_table[mi_f2h(v)]));
    *(float *) ((char *) dst + c * g.ycol + (size_t) row * sizeof(float)) = v;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (e.copy[k].ptr && row >= e.copy[k].row0 && row < e.copy[k].row1) {
            *(float *) (e.copy[k].ptr + c * e.copy[k].col_stride + (size_t) (row - e.copy[k].row0) * sizeof(float)) = v;
        }
    }
}

// ORD: combine in the reference CPU's order (bit-identical results, see dot_ord / chain): each
// 64-item chunk of a row leaves its per-item lane sums in the wave's LDS scratch, then lane
// (column c, CPU lane l) runs the reference's sequential fma chain over the chunk.
// PRO: the graph's norm prologue (g.pro) and store epilogue (g.epi) are compiled in
// XF (lone members): the activation side first -- its loads issued and waited for before any weight
// load, so they do not queue behind every workgroup's weight stream (phase stamps: with the weights
// requested first, a lone Q4_K 4096^2 member's activations took 3.6 us to land and quantize,
// profiles/r05b_lone_gemv_stamps.txt); the weights are then requested while the activations are
// quantized (PRO: after the prologue's quantization)
// MR > 1 (one column, rows of at most 16 items: tall short-K matrices such as GPT-2's lm_head,
// K = 768 = 12 Q4_K items): each wave step covers MR rows, 16 lanes per row (lane 16 r + i: item i
// of the step's row r) instead of one row on 64 lanes of which K / ITEM do work
template <class F, int NC, int PD, int IPL, bool TAIL, bool ORD, bool PRO, bool XF, int MR = 1>
__global__ __launch_bounds__(256) void k_mmv_stream(mi_mmv_group g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    MI_STAMP(g.stamps, 0);
    if (!(PRO && g.pro.mode)) MI_STAMP_CLK(g.stamps, 6);  // (norm prologue: slots 6, 5 time its phases)
    constexpr int NB = PD + 1;  // ring slots
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int member = blockIdx.x / g.blocks_per_member;
    const int rb = blockIdx.x - member * g.blocks_per_member;
    const uint8_t * W = (const uint8_t *) g.m[member].W;
    const char * X = g.m[member].X;
    float * dst = g.m[member].dst;
    const int64_t K = g.K;
    const int nitems = (int) (K / F::ITEM);
    const int ncols = g.ncols;
    const lds_act act = lds_carve<F::QKA>(lds, NC, K);
    uint32_t * scr = (uint32_t *) (lds + ord_offset(lds_bytes<F::QKA>(NC, K))) + wave * (g.ord_rows ? g.ord_rows : 1) * NC * g.ord_cs;

    // 32-bit row bookkeeping (N < 2^31): scalar compares, no 64-bit VGPR temporaries in the loop
    const int Nr = (int) g.N;
    const int row_begin = rb * (int) g.rows_per_block;
    const int row_end = row_begin + (int) g.rows_per_block < Nr ? row_begin + (int) g.rows_per_block : Nr;
    const int nrows = row_end - row_begin > wave ? (row_end - row_begin - wave + 3) / 4 : 0;
    auto wrow_of = [&](int k) {
        const int r = row_begin + 4 * k + wave;
        return W + (size_t) (r < Nr ? r : Nr - 1) * g.nb01;
    };

    // Every load of the ring is unconditional, with clamped row / item indices: a load under a
    // branch makes the compiler merge the ring registers after it, and the merge copy waits for
    // the load just issued (vmcnt(0)), which serialises the prefetch.
    typename F::Regs ring[NB][IPL];
    auto prefetch = [&](typename F::Regs (&slot)[IPL], int k) {
        const uint8_t * wr = wrow_of(k);
#pragma unroll
        for (int i = 0; i < IPL; i++) {
            const int item = lane + 64 * i;
            fmt_load<F>(slot[i], wr, item < nitems ? item : nitems - 1, K);
        }
    };
    // MR > 1: ring slot = one step of MR rows; lane 16 r + i loads item i of row MR k + r
    auto prefetch_mr = [&](typename F::Regs (&slot)[IPL], int k) {
        const uint8_t * wr = wrow_of(MR * k + (lane >> 4));
        const int item = lane & 15;
        fmt_load<F>(slot[0], wr, item < nitems ? item : nitems - 1, K);
    };
    const int nsteps = MR > 1 ? (nrows + MR - 1) / MR : nrows;
    const int klast = nsteps > 0 ? nsteps - 1 : 0;

    // 0) what the prologue reads first, requested before the weights (vmcnt retires in order: a
    //    use of it would otherwise wait for the weight loads too): the norm prologue's first
    //    column, g and b (wave 0), or the activation slices of the first quantization round
    norm_cols nc0;
    // one Q8_K column: normalized and quantized in wave 0's registers (norm_quant_prologue1)
    constexpr bool P4 = PRO && NC == 1 && F::QKA == 256;
    norm_cols4 nc4;
    const bool p4 = P4 && g.pro.mode && g.pro_q;
    const int nsl = (int) (K / 256);
    const int total = nsl * ncols;
    float4 xfirst[4];
    // Q8_K (R16): a round of a wave = slices p0 .. p0 + 3, one per 16-lane row (lane: 16 consecutive
    // elements, quantize_row16); Q8_0: slices p0, p0 + 4, p0 + 8, p0 + 12, four elements per lane
    constexpr bool R16 = F::QKA == 256;
    const int p_first = R16 ? 4 * wave : wave;
    auto load_round = [&](float4 (&v)[4], const char * Xs, size_t xcs, int p0) {
        // unconditional (clamped) loads: a predicated load makes hipcc wait vmcnt(0) per load
        if constexpr (R16) {
            const int p = min(p0 + (lane >> 4), total - 1);
            const int c = p / nsl, sl = p - c * nsl;
            const float4 * src = (const float4 *) (Xs + c * xcs + ((size_t) sl * 256 + (lane & 15) * 16) * sizeof(float));
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = src[u];
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = min(p0 + 4 * u, total - 1);
                const int c = p / nsl, sl = p - c * nsl;
                v[u] = *(const float4 *) (Xs + c * xcs + ((size_t) sl * 256 + lane * 4) * sizeof(float));
            }
        }
    };
    epi_pre<NC> epre;
    if constexpr (PRO) {
        // wave 0 alone requests the norm's column. (The load under this branch is waited for at
        // its join, before wave 0 requests its weights; every wave loading the column instead --
        // unconditional, ahead of the weights -- queued waves 1-3's weights behind it: Q4_K GPT-2
        // decode 0.417 -> 0.443 ms/token, profiles/r05t_bench_quick.json)
        if (g.pro.mode && wave == 0) {
            if (p4) norm_cols4_load(g, X, nc4);
            else norm_cols_load(g, X, 0, nc0);
        }
        epi_prefetch<NC>(g, row_begin + wave < Nr ? row_begin + wave : Nr - 1, X, epre);
    } else {
        load_round(xfirst, X, g.xcol, p_first);
    }
    // (keep these loads ahead of the weight prefetch: the scheduler hoisted the prefetch above
    // them, and vmcnt retires in order -- the activations then waited for the weights)
#ifndef MI_AB_NO_ACT_ORDER  // (A/B builds only)
    asm volatile("" ::: "memory");
#endif
    if constexpr (XF && !PRO) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // 1) the first PD rows' weights in flight
    if constexpr (!(XF && PRO)) {
#pragma unroll
        for (int u = 0; u < PD; u++) {
            if constexpr (MR > 1) prefetch_mr(ring[u], u < klast ? u : klast);
            else prefetch(ring[u], u < klast ? u : klast);
        }
    }

    // 2) quantize the member's activation columns into LDS (wave w: 256-slices w, w+4, ...),
    //    from the normalized columns when the graph's norm chain is fused in
    const char * Xq = X;
    size_t xcolq = g.xcol;
    if (PRO && g.pro.mode && p4) {
        // (the activations complete in LDS once wave 0 is through: the barrier below publishes them)
        if (wave == 0) norm_quant_prologue1(g, nc4, act);
        MI_STAMP(g.stamps, 2);
    } else if (PRO && g.pro.mode) {
        float * xn = (float *) (lds + g.pro_off);
        if (wave == 0) norm_prologue(g, X, ncols, xn, nc0);
        MI_STAMP(g.stamps, 2);  // (norm prologue: slot 2 = wave 0's norm done, instead of the barrier below)
        __syncthreads();
        Xq = (const char *) xn;
        xcolq = (size_t) K * sizeof(float);
    }
    if (!p4) {
        for (int p0 = p_first; p0 < total; p0 += 16) {
            float4 v[4];
            if (!PRO && p0 == p_first) {
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = xfirst[u];
            } else {
                load_round(v, Xq, xcolq, p0);
            }
            if constexpr (R16) {
                const int p = min(p0 + (lane >> 4), total - 1);
                const int c = p / nsl, sl = p - c * nsl;
                quantize_row16(v, lane, act, K, c, sl, p0 + (lane >> 4) < total);
            } else {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int p = p0 + 4 * u;
                    if (p < total) {
                        const int c = p / nsl, sl = p - c * nsl;
                        quantize_slice<F::QKA>(v[u], lane, act, K, c, sl);
                    }
                }
            }
        }
    }
    MI_STAMP(g.stamps, 1);  // wave 0's activation slices loaded and quantized
    if constexpr (XF && PRO) {
#pragma unroll
        for (int u = 0; u < PD; u++) {
            if constexpr (MR > 1) prefetch_mr(ring[u], u < klast ? u : klast);
            else prefetch(ring[u], u < klast ? u : klast);
        }
    }
    __syncthreads();
    if (!(PRO && g.pro.mode)) MI_STAMP(g.stamps, 2);  // every wave's

    if constexpr (MR > 1) {
        static_assert(NC == 1 && IPL == 1 && !TAIL, "multi-row steps: one column, one item per lane");
        const int rr = lane >> 4, it = lane & 15;
        auto sync = [] {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        };
        for (int k0 = 0; k0 < nsteps; k0 += NB) {
#pragma unroll
            for (int u = 0; u < NB; u++) {
                const int k = k0 + u;
                if (k >= nsteps) break;  // wave-uniform
                prefetch_mr(ring[(u + PD) % NB], k + PD < klast ? k + PD : klast);
                const int j = MR * k + rr;  // this lane's row of the wave
                if constexpr (ORD) {
                    // R = g.ord_rows rows (a multiple of MR) collect their lane sums, then one
                    // chain pass: lane 8 r + l runs CPU lane l of row slot r (as the one-row form)
                    const int RS = g.ord_rows / MR, cs = g.ord_cs, S = g.ord_s;
                    const int slot = k % RS;
                    if (it < nitems) F::template dot_ord<1>(ring[u][0], it, it, act, K, ncols, scr + (slot * MR + rr) * cs, cs, S);
                    if (slot == RS - 1 || k == nsteps - 1) {  // wave-uniform
                        sync();
                        if (k == nsteps - 1) MI_STAMP(g.stamps, 3);
                        const int r = lane >> 3, ll = lane & 7;
                        const int jr = (k - slot) * MR + r;
                        const bool mine = r < (slot + 1) * MR && jr < nrows;
                        float A = 0.0f, M = 0.0f;
                        if (mine && !g.abl) F::chain(scr + r * cs, ll, nitems, S, A, M);
                        const float v = F::finish(A, M);
                        if (k == nsteps - 1) MI_STAMP(g.stamps, 4);
                        if (ll == 0 && mine) store_out<PRO, 1>(g, dst, 0, row_begin + 4 * jr + wave, v, &epre);
                        sync();
                    }
                } else {
                    float acc[1] = {0.0f};
                    if (it < nitems) F::template dot<1>(ring[u][0], it, act, K, ncols, acc);
                    // sum over the row's 16 lanes (DPP within a 16-lane row)
                    auto f = [](int x) { return __int_as_float(x); };
                    auto i = [](float x) { return __float_as_int(x); };
                    float v = acc[0];
                    v += f(mi_dpp<MI_DPP_QP_1032>(0, i(v)));
                    v += f(mi_dpp<MI_DPP_QP_2301>(0, i(v)));
                    v += f(mi_dpp<MI_DPP_ROW_HALF_MIRROR>(0, i(v)));
                    v += f(mi_dpp<MI_DPP_ROW_MIRROR>(0, i(v)));
                    if (it == 0 && j < nrows) store_out<PRO, 1>(g, dst, 0, row_begin + 4 * j + wave, v, &epre);
                    if (k == 0) MI_STAMP(g.stamps, 3);
                }
            }
        }
    } else {
    // (one column, tree order: the lane's items are the same in every row, so their activation
    // operands are read from LDS once, here, instead of per row)
    constexpr bool AREG = NC == 1 && !ORD && !TAIL;
    typename F::Act areg[AREG ? IPL : 1];
    if constexpr (AREG) {
#pragma unroll
        for (int i = 0; i < IPL; i++) {
            const int item = lane + 64 * i;
            F::act_load(areg[i], item < nitems ? item : nitems - 1, act, K);
        }
    }
    // 3) stream: ring slot u holds row k0+u; refill it with row k0+u+PD right before using it
    //    (the last row again past the end: an L2 hit)
    for (int k0 = 0; k0 < nrows; k0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int k = k0 + u;
            if (k >= nrows) break;  // wave-uniform
            prefetch(ring[(u + PD) % NB], k + PD < klast ? k + PD : klast);
            const int row = row_begin + 4 * k + wave;
            if constexpr (ORD) {
                const int R = g.ord_rows, cs = g.ord_cs, S = g.ord_s;
                auto sync = [] {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_wave_barrier();
                };
                if (R == 0) {
                    // rows too long for the scratch: one chain pass per 64-item chunk of the row
                    const int cl = lane >> 3, ll = lane & 7;
                    float A = 0.0f, M = 0.0f;
                    auto chunk_done = [&](int base) {
                        sync();
                        if (cl < ncols && !g.abl) F::chain(scr + cl * cs, ll, min(64, nitems - base), S, A, M);
                        sync();
                    };
#pragma unroll
                    for (int i = 0; i < IPL; i++) {
                        if (64 * i >= nitems) break;  // wave-uniform
                        const int item = lane + 64 * i;
                        if (item < nitems) F::template dot_ord<NC>(ring[u][i], item, lane, act, K, ncols, scr, cs, S);
                        chunk_done(64 * i);
                    }
                    if constexpr (TAIL) {
                        const uint8_t * wr = wrow_of(k);
                        for (int base = 64 * IPL; base < nitems; base += 64) {
                            const int item = base + lane;
                            if (item < nitems) {
                                typename F::Regs rr;
                                fmt_load<F>(rr, wr, item, K);
                                F::template dot_ord<NC>(rr, item, lane, act, K, ncols, scr, cs, S);
                            }
                            chunk_done(base);
                        }
                    }
                    const float v = F::finish(A, M);
                    if (ll == 0 && cl < ncols) store_out<PRO, NC>(g, dst, cl, row, v, &epre);
                    continue;
                }
                // whole rows in the scratch: R rows' lane sums are collected, then one chain pass
                // runs them all, lane = (row r, column c, CPU lane l), 8 * NC * R <= 64
                const int slot = k % R;
                uint32_t * srow = scr + slot * NC * cs;
#pragma unroll
                for (int i = 0; i < IPL; i++) {
                    const int item = lane + 64 * i;
                    if (item < nitems) F::template dot_ord<NC>(ring[u][i], item, item, act, K, ncols, srow, cs, S);
                }
                if constexpr (TAIL) {
                    const uint8_t * wr = wrow_of(k);
                    for (int item = lane + 64 * IPL; item < nitems; item += 64) {
                        typename F::Regs rr;
                        fmt_load<F>(rr, wr, item, K);
                        F::template dot_ord<NC>(rr, item, item, act, K, ncols, srow, cs, S);
                    }
                }
                if (slot == R - 1 || k == nrows - 1) {  // wave-uniform
                    sync();
                    if (k == nrows - 1) MI_STAMP(g.stamps, 3);  // (reference order) the last rows' lane sums in the scratch
                    const int r = lane / (8 * NC), cl = (lane >> 3) % NC, ll = lane & 7;
                    const bool mine = r <= slot && cl < ncols;
                    float A = 0.0f, M = 0.0f;
                    if (mine && !g.abl) F::chain(scr + (r * NC + cl) * cs, ll, nitems, S, A, M);
                    const float v = F::finish(A, M);
                    if (k == nrows - 1) MI_STAMP(g.stamps, 4);  // (reference order) chains done
                    if (ll == 0 && mine) {
                        store_out<PRO, NC>(g, dst, cl, row_begin + 4 * (k - slot + r) + wave, v, &epre);
                    }
                    sync();
                }
                continue;
            }
            float acc[NC];
#pragma unroll
            for (int c = 0; c < NC; c++) acc[c] = 0.0f;
#pragma unroll
            for (int i = 0; i < IPL; i++) {
                const int item = lane + 64 * i;
                if constexpr (AREG) {
                    if (item < nitems) acc[0] = F::dot_act(ring[u][i], item, areg[i], acc[0]);
                } else {
                    if (item < nitems) F::template dot<NC>(ring[u][i], item, act, K, ncols, acc);
                }
            }
            if constexpr (TAIL) {
                // items beyond the ring's IPL per lane, loaded in-line (long rows only: a loop
                // with loads here makes the compiler drain vmcnt at the top of every row group)
                const uint8_t * wr = wrow_of(k);
                for (int item = lane + 64 * IPL; item < nitems; item += 64) {
                    typename F::Regs rr;
                    fmt_load<F>(rr, wr, item, K);
                    F::template dot<NC>(rr, item, act, K, ncols, acc);
                }
            }
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const float v = mi_wave_sum_u(acc[c]);
                if (lane == 0 && c < ncols) store_out<PRO, NC>(g, dst, c, row, v, &epre);
            }
            if (k == 0) MI_STAMP(g.stamps, 3);  // first row reduced and stored
        }
    }
    }
    if (!(PRO && g.pro.mode)) MI_STAMP_CLK(g.stamps, 5);
    MI_STAMP(g.stamps, 7);
}

// ------------------------------------------------------------------ LDS-DMA weight stream (round 6)
#if MI_DIAG
// k_mmv_dma: the tree-order Q4_K GEMV of one column with the weights moved by LDS-DMA. Measured
// (profiles/r06h_gemv_lds_dma_ab.txt, headline workload): 5.6-6.0 TB/s against k_mmv_stream's
// 6.2-6.3 on the same box (nt 3-7 % faster than the default policy); diagnostic builds only.
// Design:
// (global_load_lds_dwordx4, 1 KB per wave-instruction, every weight byte fetched exactly once --
// k_mmv_stream's lanes load each 16-byte superblock header four times) into wave-private rings,
// optionally with the nontemporal policy (NT; the guide's nt-weights row: LDS-DMA streams reach
// 6.5-6.8 TB/s chip-wide nt, 6.4 default, MI355X_MICROARCH.md "ldsdma-fill"). Wave w of a workgroup
// owns a contiguous run of rows, i.e. a contiguous byte stream (rows of 144 K / 256 bytes, packed);
// a ring slot is a group of 4 rows = 9 x 1 KB pieces for K = 4096 (GR = 4 rows x BS x K / 256 / 1024
// pieces; K = 4096 only, as the waits' immediates assume), G slots, G - 1 groups in flight. The dot products read the
// slot with ds_read_b128 and use FmtKQ's arithmetic (the same per-item sums and wave reduction as
// k_mmv_stream: the same bits); the 4 rows' results leave as one 16-byte store by lane 0. The DMAs
// are inline asm outside the compiler's vmcnt bookkeeping: per group a wave issues exactly GR DMAs
// and one store, so "group g landed" is s_waitcnt vmcnt((G - 1) (GR + 1)).
__device__ __forceinline__ uint32_t mi_lds_addr_u8(const uint8_t * p) {  // LDS byte address, wave-uniform
    return (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (uintptr_t) p);
}
__device__ __forceinline__ void mi_glds16_nt(const void * gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds));
}
__device__ __forceinline__ void mi_glds16_dflt(const void * gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds));
}
template <int G> struct dma_wait;
template <> struct dma_wait<2> { __device__ static void run() { asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); } };
template <> struct dma_wait<3> { __device__ static void run() { asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); } };
template <> struct dma_wait<4> { __device__ static void run() { asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); } };

constexpr int kDmaRowsPerGroup = 4;

template <int NW, int G, bool NT>
__global__ __launch_bounds__(64 * NW) void k_mmv_dma(mi_mmv_group g) {
    using F = FmtKQ<false>;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int64_t K = 4096;
    constexpr int nsl = K / 256;
    constexpr int RB = nsl * F::BS;                   // row bytes (rows packed: nb01 == RB)
    constexpr int GB = kDmaRowsPerGroup * RB;         // group bytes
    constexpr int GR = GB / 1024;                     // DMA pieces per group
    static_assert(GB % 1024 == 0 && GR == 9, "dma_wait assumes 9 pieces + 1 store per group");
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int member = blockIdx.x / g.blocks_per_member;
    const int rb = blockIdx.x - member * g.blocks_per_member;
    const uint8_t * W = (const uint8_t *) g.m[member].W;
    const char * X = g.m[member].X;
    float * dst = g.m[member].dst;
    const lds_act act = lds_carve<256>(lds, 1, K);
    uint8_t * ring = lds + ord_offset(lds_bytes<256>(1, K)) + (size_t) wave * G * GB;

    // rows of this workgroup, then of this wave (contiguous, whole groups except the member's last)
    const int Nr = (int) g.N;
    const int row_begin = rb * (int) g.rows_per_block;
    const int row_end = min(row_begin + (int) g.rows_per_block, Nr);
    const int rpw = (int) g.rows_per_block / NW;  // a multiple of kDmaRowsPerGroup (launcher)
    const int r0 = min(row_begin + wave * rpw, row_end), r1 = min(r0 + rpw, row_end);
    const int ngroups = (r1 - r0 + kDmaRowsPerGroup - 1) / kDmaRowsPerGroup;
    const uint8_t * wbase = W + (size_t) r0 * RB;
    const uint8_t * wlast = W + (size_t) Nr * RB - 16;  // (clamp: pieces past the member's end re-read its last bytes)
    auto issue = [&](int grp) {
        const int gc = grp < ngroups ? grp : (ngroups > 0 ? ngroups - 1 : 0);  // (past the end: the last group again)
        const uint8_t * src = wbase + (size_t) gc * GB + 16 * lane;
        const uint32_t dsts = mi_lds_addr_u8(ring + (grp % G) * GB);
#pragma unroll
        for (int p = 0; p < GR; p++) {
            const uint8_t * a = src + 1024 * p;
            a = a < wlast ? a : wlast;
            if constexpr (NT) mi_glds16_nt(a, dsts + 1024 * p);
            else mi_glds16_dflt(a, dsts + 1024 * p);
        }
    };

    // activations: the column's slices quantized into LDS by every wave (as k_mmv_stream), requested
    // before the first groups' DMAs
    auto load_round = [&](float4 (&v)[4], int p0) {
        const int p = min(p0 + (lane >> 4), nsl - 1);
        const float4 * src = (const float4 *) (X + ((size_t) p * 256 + (lane & 15) * 16) * sizeof(float));
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = src[u];
    };
    float4 xfirst[4];
    load_round(xfirst, 4 * wave);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the compiler does not count the DMAs below)
    for (int grp = 0; grp < G - 1; grp++) issue(grp);
    for (int p0 = 4 * wave; p0 < nsl; p0 += 4 * NW) {
        float4 v[4];
        if (p0 == 4 * wave) {
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = xfirst[u];
        } else {
            load_round(v, p0);
        }
        const int p = min(p0 + (lane >> 4), nsl - 1);
        quantize_row16(v, lane, act, K, 0, p, p0 + (lane >> 4) < nsl);
    }
    __syncthreads();
    // this lane's item (superblock s, 64-group j) is the same in every row: its activation operands
    // stay in registers
    const int s = lane >> 2, j = lane & 3;
    int alo[8], ahi[8];
    {
        const int4 * p = (const int4 *) (act.qs + (int64_t) s * 256 + 64 * j);
        const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
        const int l8[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const int h8[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            alo[i] = l8[i];
            ahi[i] = h8[i];
        }
    }
    const int ss = *(const int *) (act.s32 + s * 8 + 2 * j);
    const float ad = act.d[s];
    const uint32_t ioff = (uint32_t) (s * F::BS);

    // stream: group grp in slot grp % G; its refill (group grp + G - 1) issued first
    for (int grp = 0; grp < ngroups; grp++) {
        issue(grp + G - 1);
        dma_wait<G>::run();
        const uint8_t * slot = ring + (grp % G) * GB + ioff;
        typename F::Regs rg[kDmaRowsPerGroup];
#pragma unroll
        for (int r = 0; r < kDmaRowsPerGroup; r++) {
            rg[r].hdr = *(const uint4 *) (slot + r * RB);
            rg[r].qa = *(const uint4 *) (slot + r * RB + 16 + 32 * j);
            rg[r].qb = *(const uint4 *) (slot + r * RB + 32 + 32 * j);
        }
        float res[kDmaRowsPerGroup];
#pragma unroll
        for (int r = 0; r < kDmaRowsPerGroup; r++) res[r] = mi_wave_sum_u(F::item_dot(rg[r], j, alo, ahi, ss, ad, 0.0f));
        const int row = r0 + kDmaRowsPerGroup * grp;
        if (lane == 0) {
            if (row + kDmaRowsPerGroup <= r1) {
                *(float4 *) (dst + row) = make_float4(res[0], res[1], res[2], res[3]);
            } else {
                for (int r = 0; r < kDmaRowsPerGroup; r++)
                    if (row + r < r1) dst[row + r] = res[r];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the re-read DMAs past the end have landed)
}
#endif  // MI_DIAG

// Workgroups that fit on the chip at once for this kernel instance (all of them are launched
// in one wave, so no workgroup waits for another to retire). Speed only: nothing relies on
// co-residency. Cached per kernel.
int resident_blocks(const void * fn, size_t lds) {
    struct entry { const void * fn; size_t lds; int n; };
    static entry cache[64];
    static int ncache = 0;
    for (int i = 0; i < ncache; i++) if (cache[i].fn == fn && cache[i].lds == lds) return cache[i].n;
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    (void) hipGetDevice(&dev);
    (void) hipGetDeviceProperties(&prop, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    const int n = per_cu * prop.multiProcessorCount;
    if (ncache < 64) cache[ncache++] = entry{fn, lds, n};
    return n;
}

static int mi_cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        (void) hipGetDevice(&dev);
        n = hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    }
    return n;
}

template <class F, int NC, int PD, int IPL, bool TAIL, bool ORD, bool PRO = false, bool XF = false, int MR = 1>
void launch_one(mi_mmv_group g, hipStream_t s) {
    const size_t act = lds_bytes<F::QKA>(NC, g.K);
    size_t lds = act;
    if constexpr (ORD) {
        // whole rows in the scratch when R >= 1 rows per wave fit a 36 KB budget (the kernel is
        // VGPR-limited to ~4 workgroups per CU anyway), else one chunk of 64 items per wave
        const int nitems = (int) (g.K / F::ITEM);
        int S = 0;
        const int cs = F::ord_words(nitems, S);
        int R = (int) ((36 * 1024) / ((size_t) 4 * NC * cs * 4));
        if (R > 8 / NC) R = 8 / NC;
        if (MR > 1) R = R >= MR ? R / MR * MR : 0;  // whole multi-row steps per chain pass (0: refused below)
        if (R >= 1) {
            g.ord_rows = R;
            g.ord_cs = cs;
            g.ord_s = S;
        } else {
            g.ord_rows = 0;
            g.ord_cs = F::ord_words(64, S);
            g.ord_s = S;
        }
        lds = ord_offset(act) + (size_t) 4 * (g.ord_rows ? g.ord_rows : 1) * NC * g.ord_cs * 4;
    }
    if constexpr (MR > 1 && ORD) {
        if (g.ord_rows < MR) {  // a chain pass must hold whole multi-row steps: the one-row form
            launch_one<F, NC, PD, IPL, TAIL, ORD, PRO, XF, 1>(g, s);
            return;
        }
    }
    g.pro_q = PRO && NC == 1 && F::QKA == 256 && g_mi_tuning.mmv_pro4 ? 1 : 0;
    if (PRO && g.pro.mode) {
        g.pro_off = (int) ord_offset(lds);
        lds = (size_t) g.pro_off + (size_t) NC * g.K * sizeof(float);
    }
    const void * fn = (const void *) k_mmv_stream<F, NC, PD, IPL, TAIL, ORD, PRO, XF, MR>;
    if (lds > 64 * 1024) {
        static bool attr_set = false;  // per instance
        if (!attr_set) {
            (void) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_set = true;
        }
    }
    // automatic grid: the resident workgroup count, split over the members. A lone member at
    // K >= 4096 gets one workgroup per CU instead: every workgroup quantizes the whole activation
    // in its prologue, so at 4 rows per workgroup that redundant work dominates (Q4_K 4096^2 alone
    // in its graph 7.96 -> 6.57 us, profiles/r04e_pf_single_blocks.txt)
    int target = g_mi_tuning.mmv_blocks > 0 ? g_mi_tuning.mmv_blocks : resident_blocks(fn, lds);
    if (g_mi_tuning.mmv_blocks <= 0 && g.n == 1 && g.K >= 4096) target = std::min(target, mi_cu_count());
    // Q5_K grouped launches: twice the resident count (smaller workgroups, a later tail; 4096 x 11008
    // 5.56 -> 5.75 TB/s, r04r_gemv_sweep.txt)
    // Q4_K tall members (4096 x 11008): the same (5.47-5.49 -> 5.56-5.62 TB/s on one box,
    // profiles/r05sw_gemv_blocks_sweep.txt; 4096^2 members unchanged within noise, left alone)
    else if (g_mi_tuning.mmv_blocks <= 0 && !ORD && !PRO &&
             (std::is_same<F, FmtKQ<true>>::value || (std::is_same<F, FmtKQ<false>>::value && g.N >= 8192))) target *= 2;
    int bpm = target / g.n;
    if (bpm < 1) bpm = 1;
    int64_t rows = (g.N + bpm - 1) / bpm;
    rows = (rows + 3) / 4 * 4;
    g.rows_per_block = rows;
    g.blocks_per_member = (int) ((g.N + rows - 1) / rows);
    g.stamps = mi_stamp_take(ORD ? "k_mmv_stream_ord" : "k_mmv_stream", (unsigned) (g.blocks_per_member * g.n));
    hipLaunchKernelGGL((k_mmv_stream<F, NC, PD, IPL, TAIL, ORD, PRO, XF, MR>), dim3((unsigned) (g.blocks_per_member * g.n)), dim3(256), lds,
                       s, g);
}

#if MI_DIAG
// k_mmv_dma for a group (tree order, one column, packed Q4_K rows, K = 4096); false: not taken.
// mmv_dma: 1 = 4 waves x 3 slots, 2 = 8 waves x 2 slots, 3 = 4 waves x 4 slots (+10: default load
// policy instead of nontemporal); one workgroup per CU
bool launch_dma(mi_mmv_group g, hipStream_t s) {
    const int v = g_mi_tuning.mmv_dma;
    const int64_t RB = g.K / 256 * 144;
    if (g.K != 4096 || (int64_t) g.nb01 != RB || g.N >= (1 << 30)) return false;  // (9 pieces per group: the waits' immediates)
    for (int i = 0; i < g.n; i++)
        if (((uintptr_t) g.m[i].dst | (uintptr_t) g.m[i].W) % 16 != 0) return false;
    const int shape = v % 10;
    const bool nt = v < 10;
    const int NW = shape == 2 ? 8 : 4, G = shape == 2 ? 2 : shape == 3 ? 4 : 3;
    const size_t lds = ord_offset(lds_bytes<256>(1, g.K)) + (size_t) NW * G * 4 * RB;
    if (lds > 160 * 1024) return false;
    const int target = mi_cu_count();
    int bpm = target / g.n;
    if (bpm < 1) bpm = 1;
    int64_t rows = (g.N + bpm - 1) / bpm;
    const int64_t unit = (int64_t) NW * kDmaRowsPerGroup;
    rows = (rows + unit - 1) / unit * unit;
    g.rows_per_block = rows;
    g.blocks_per_member = (int) ((g.N + rows - 1) / rows);
    const void * fn;
#define MI_DMA_K(NW_, G_, NT_) (const void *) k_mmv_dma<NW_, G_, NT_>
    if (NW == 8) fn = nt ? MI_DMA_K(8, 2, true) : MI_DMA_K(8, 2, false);
    else if (G == 4) fn = nt ? MI_DMA_K(4, 4, true) : MI_DMA_K(4, 4, false);
    else fn = nt ? MI_DMA_K(4, 3, true) : MI_DMA_K(4, 3, false);
#undef MI_DMA_K
    (void) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const dim3 grid((unsigned) (g.blocks_per_member * g.n)), block((unsigned) (64 * NW));
    void * args[] = {&g};
    return hipLaunchKernel(fn, grid, block, args, lds, s) == hipSuccess;
}
#endif  // MI_DIAG

template <class F, int NC, int PD, int IPL, bool ORD, bool XF = false>
void launch_tail(const mi_mmv_group & g, hipStream_t s) {
    if (g.K / F::ITEM > 64 * IPL) launch_one<F, NC, PD, IPL, true, ORD, false, XF>(g, s);
    else launch_one<F, NC, PD, IPL, false, ORD, false, XF>(g, s);
}

template <class F, int NC, bool ORD>
void launch_stream(const mi_mmv_group & g, int variant, hipStream_t s) {
    const int items = (int) (g.K / F::ITEM);
    const mi_mmv_group::epilogue & e = g.epi;
    // XF (activations landed before any weight request) is opt-in only (xfirst 1). It was the
    // automatic choice for lone members at K >= 2048 while the scheduler hoisted the weight prefetch
    // above the activation loads (lone Q4_K 4096^2 6.93 -> 6.11 us per graph then); with the
    // activation loads pinned ahead of the prefetch, both stream together and XF only serializes
    // them: 5.45 -> 4.95 us per graph without it (profiles/r05xf_xfirst_ab.txt)
    const bool xf = g.n == 1 && g_mi_tuning.xfirst == 1;
    const bool pro_epi = g.pro.mode || e.bias || e.resid || e.gelu_table || e.copy[0].ptr || e.copy[1].ptr;
#if MI_DIAG  // measured slower (profiles/r06h_gemv_lds_dma_ab.txt): diagnostic builds only
    if constexpr (NC == 1 && !ORD && std::is_same<F, FmtKQ<false>>::value) {
        if (!pro_epi && g_mi_tuning.mmv_dma > 0 && launch_dma(g, s)) return;
    }
#endif
    if constexpr (NC == 1) {
        // tall lone members with rows of <= 16 items (GPT-2 lm_head: 50257 x 768, 12 Q4_K items per
        // row): four rows per wave step on 16 lanes each (MR = 4); variant 9x: the one-row form
        if (g.n == 1 && g.N >= 16384 && items <= 16 && variant / 10 != 9) {
            if (pro_epi) launch_one<F, 1, 4, 1, false, ORD, true, false, 4>(g, s);
            else launch_one<F, 1, 4, 1, false, ORD, false, false, 4>(g, s);
            return;
        }
    }
    if (pro_epi) {
        // the graph's norm prologue and/or epilogue: instances of their own (prefetch depth 1) so
        // that their registers and per-row branches do not weigh on the plain kernels
        if (xf) {
            if (items > 128) launch_one<F, NC, 2, 2, true, ORD, true, true>(g, s);
            else if (items > 64) launch_one<F, NC, 2, 2, false, ORD, true, true>(g, s);
            else launch_one<F, NC, 4, 1, false, ORD, true, true>(g, s);
            return;
        }
        if (items > 128) launch_one<F, NC, 1, 2, true, ORD, true>(g, s);
        else if (items > 64) launch_one<F, NC, 1, 2, false, ORD, true>(g, s);
        else launch_one<F, NC, 1, 1, false, ORD, true>(g, s);
        return;
    }
    if (items > 64) {
        // two items per lane in the ring (Q4_0 / Q8_0 at K=4096)
        if (xf) launch_tail<F, NC, 2, 2, ORD, true>(g, s);
        else if (variant / 10 == 1) launch_tail<F, NC, 1, 2, ORD>(g, s);
        else launch_tail<F, NC, 2, 2, ORD>(g, s);
        return;
    }
    if (xf) {
        launch_one<F, NC, 4, 1, false, ORD, false, true>(g, s);
        return;
    }
    switch (variant / 10) {
        case 1: launch_one<F, NC, 1, 1, false, ORD>(g, s); break;
        case 3: launch_one<F, NC, 3, 1, false, ORD>(g, s); break;
        default: launch_one<F, NC, 2, 1, false, ORD>(g, s); break;
    }
}

template <class F, bool ORD>
void launch_stream_nc(const mi_mmv_group & g, int variant, hipStream_t s) {
    switch (g.ncols) {
        case 1: launch_stream<F, 1, ORD>(g, variant, s); break;
        case 2: launch_stream<F, 2, ORD>(g, variant, s); break;
        case 3: case 4: launch_stream<F, 4, ORD>(g, variant, s); break;
        default: launch_stream<F, 8, ORD>(g, variant, s); break;
    }
}

template <class F>
void launch_stream_ord(const mi_mmv_group & g, int variant, hipStream_t s) {
    if (mi_mmv_order()) {
        mi_mmv_group h = g;
        h.abl = mi_mmv_order() == 2;
        launch_stream_nc<F, true>(h, variant, s);
    } else
        launch_stream_nc<F, false>(g, variant, s);
}


} // namespace
