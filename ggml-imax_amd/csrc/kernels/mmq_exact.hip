// mmq_exact.hip -- batched (prompt / prefill) GGML_OP_MUL_MAT for Q4_K / Q5_K weights on the
// gfx950 int8 matrix cores, with the reference's exact integer block sums.
//
// The reference dot product (vec_dot_q4_K_q8_K, src/ggml-quants.c:7089-7152 AVX2; q5_K :7920-8003)
// is, per superblock s of 256 weights of a row n and activation column b,
//     y += d_a(b,s) * d_w(n,s) * T  -  d_a(b,s) * dmin_w(n,s) * U
//     T = sum_j sc_j * sum_{k in j} q_k * q8_k        (exact int32; 8 sub-blocks j of 32)
//     U = sum_j m_j  * (bsums_2j + bsums_2j+1)        (exact int32)
// with q = 4-bit (Q4_K) or 5-bit (Q5_K) weight quants, sc_j / m_j the 6-bit sub-block scales /
// mins, q8 the Q8_K activation quants (quantize_row_q8_K_reference, :3370-3407). Here both T and
// U come out of the matrix cores exactly:
//   * T: sc_j * q does not fit int8 (<= 945), so the weights are staged as NP int8 "planes"
//     q * (sc_j's bit field p) -- Q4_K: sc = 8*hi3 + lo3, 2 planes (<= 15*7); Q5_K: sc = 16*f2 +
//     4*f1 + f0, 3 planes (<= 31*3) -- each a v_mfma_i32_32x32x32_i8 operand against the int8 q8
//     activations; T = (P1 << 3) + P0 (Q4_K) or ((P2 << 2) + P1 << 2) + P0 (Q5_K), exact.
//   * U: one v_mfma_f32_32x32x16_f16 per superblock with exact small integers: A = [m_j, 64 m_j]
//     (<= 4032), B = [S_j & 63, S_j >> 6] where S_j = sum of 32 q8 (the activation quantizer
//     writes these), so every product and partial sum is an integer < 2^24: exact.
// The float combine per superblock and the order of the superblock chain are fixed (mmqx_term
// and the two-halves chain below) and shared by every kernel of this file, so column shards of a
// prompt (prompt-sharded multi-GPU) give the same bits as the whole prompt. Against the
// reference CPU the only difference is the f32 combine order (reference: 8-lane partial chains
// + hsum): ~1e-7 relative.
//
// Workgroup = 2 groups x 4 wave64s, tile 64 weight rows x 128 columns; group g owns half of the
// superblocks of K (the canonical chain split) and dequantizes its 64 x 128 weight slab of a stage
// (half a superblock) into double-buffered LDS planes once for its four waves; each wave owns all
// 64 rows x its own 32 columns (two 32x32 MFMA tiles sharing one activation fragment), which it
// loads straight from HBM/L2 into a register ring (16 B per lane per 32-deep K step).
// Roofline: 2*N*K*B flops; at B=512 MFMA-bound. The NP planes make the int8 rate per weight
// 2 (Q4_K) or 3 (Q5_K) i8 MFMAs per 32 K, i.e. Q4_K runs at the dense f16 rate (2.5 PF/s).

#include <algorithm>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#pragma clang fp contract(off)

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));     // 16 int8 (MFMA i8 operand)
typedef int i32x16 __attribute__((ext_vector_type(16)));   // 32x32 i32 accumulator
typedef float f32x16 __attribute__((ext_vector_type(16)));  // 32x32 f32 accumulator
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr int XBM = 64;            // weight rows per workgroup
constexpr int XBN = 128;           // activation columns per workgroup (4 waves x 32)
constexpr int XSK = 128;           // K per LDS stage (half a superblock)
constexpr int XROW = XSK + 16;     // LDS row stride of a plane (bytes)

// packed bytes times a small factor (every byte product < 256: no carry between bytes)
__device__ __forceinline__ uint32_t mulb(uint32_t x, uint32_t m) {
    u16x2 a = __builtin_bit_cast(u16x2, x);
    const u16x2 b = {(unsigned short) m, (unsigned short) m};
    return __builtin_bit_cast(uint32_t, a * b);
}

// the canonical per-superblock combine (every kernel of the family uses exactly this)
__device__ __forceinline__ float mmqx_term(float y, int T, float U, float dw, float dm, float da) {
    const float t = __builtin_fmaf(-dm, U, dw * (float) T);
    return __builtin_fmaf(da, t, y);
}

template <int TYPE>
struct XFmt {
    static constexpr bool Q5 = TYPE == 13;
    static constexpr int NP = Q5 ? 3 : 2;
    static constexpr int BS = Q5 ? 176 : 144;
    static constexpr int SHIFT = Q5 ? 2 : 3;  // T = sum_p P_p << (SHIFT * p)
    __device__ static __forceinline__ uint32_t factor(int sc, int p) {
        if constexpr (Q5) return (uint32_t) ((sc >> (2 * p)) & 3);
        else return (uint32_t) (p ? sc >> 3 : sc & 7);
    }
};

// raw bytes of one thread's share of a stage: header + 16 quant bytes (+ 16 high-bit bytes)
template <int TYPE>
struct XRaw {
    uint4 hdr, qs, qh;
};

} // namespace

// ---- activations: q8_K quants in the MFMA layouts ------------------------------------------------
// xq [K/64][ncols][64] int8, xd [K/256][ncols] f32 (d), xu [K/256][ncols][16] f16 (S_j & 63,
// S_j >> 6 for j = 0..7, S_j = sum of the 32 quants of sub-block j). One superblock per wave.
__global__ __launch_bounds__(256) void k_quantize_q8_K_mmx(mi_src_cols x, int64_t K, mi_act_mmx act, int64_t nblocks_total) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t blk = (int64_t) blockIdx.x * 4 + wave;
    if (blk >= nblocks_total) return;  // wave-uniform
    const int64_t nb_per_col = K / 256;
    const int64_t c = blk / nb_per_col;
    const int64_t b = blk % nb_per_col;
    const int64_t i1 = c % x.ne1, i2 = (c / x.ne1) % x.ne2, i3 = c / (x.ne1 * x.ne2);
    const float * col = (const float *) (x.base + i1 * x.nb1 + i2 * x.nb2 + i3 * x.nb3);
    const float4 v4 = *(const float4 *) (col + b * 256 + lane * 4);
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    // quantize_row_q8_K_reference: first max-|x| element (sign kept), iscale = -127/max,
    // q = min(127, nearest_int(iscale*x)) -- as quantize.hip's k_quantize_q8_K, bit for bit
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
    uint32_t packed = 0;
    int sum = 0;
    float d = 0.0f;
    if (amax != 0.0f) {
        const float iscale = -127.f / vmax;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int bits = __float_as_int(__builtin_fmaf(iscale, v[i], 12582912.f));
            int q = (bits & 0x007fffff) - 0x00400000;
            q = q < 127 ? q : 127;
            sum += q;
            packed |= ((uint32_t) (q & 0xFF)) << (8 * i);
        }
        d = 1.0f / iscale;
    }
    const int64_t ncols = act.ncols;
    // element k = lane*4 .. +3 of the superblock: 64-block lane/16, offset (lane%16)*4
    *(uint32_t *) (act.xq + ((b * 4 + (lane >> 4)) * ncols + c) * 64 + (lane & 15) * 4) = packed;
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);  // lanes 8j..8j+7: S_j (sub-block j of 32)
    if ((lane & 7) == 0) {
        const int j = lane >> 3;
        const uint32_t lo = mi_f2h((float) (sum & 63)), hi = mi_f2h((float) (sum >> 6));
        *(uint32_t *) (act.xu + (b * ncols + c) * 16 + 2 * j) = lo | (hi << 16);
    }
    if (lane == 0) act.xd[b * ncols + c] = d;
}

size_t mi_act_mmx_bytes(int64_t K, int64_t ncols) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t) 255; };
    return al((size_t) K * ncols) + al((size_t) (K / 256) * ncols * 4) + al((size_t) (K / 256) * ncols * 32);
}

mi_act_mmx mi_act_mmx_carve(void * base, int64_t K, int64_t ncols) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t) 255; };
    char * p = (char *) base;
    mi_act_mmx a;
    a.K = K;
    a.ncols = ncols;
    a.xq = (int8_t *) p;
    p += al((size_t) K * ncols);
    a.xd = (float *) p;
    p += al((size_t) (K / 256) * ncols * 4);
    a.xu = (uint16_t *) p;
    return a;
}

void mi_quantize_q8_K_mmx(const mi_src_cols & x, int64_t K, const mi_act_mmx & act, hipStream_t s) {
    const int64_t nblk = (K / 256) * act.ncols;
    hipLaunchKernelGGL(k_quantize_q8_K_mmx, dim3((unsigned) ((nblk + 3) / 4)), dim3(256), 0, s, x, K, act, nblk);
}

namespace {

// ---- the GEMM -----------------------------------------------------------------------------------
// SK = 2: two groups of 4 waves (512 threads, 2 waves per SIMD), group g sums chain half g;
// SK = 1: one group of 4 waves (256 threads, 1 wave per SIMD with the whole register file), each
// wave runs both chain halves in turn. PF = stages of weight and activation loads in flight.
template <int TYPE, int SK, int PF, bool XCD>
__global__ __launch_bounds__(256 * SK) void k_mmqx(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                   mi_act_mmx act, float * __restrict__ dst, size_t ycol) {
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    constexpr int kPlane = XBM * XROW;                       // one plane of a stage
    constexpr int kAu = XBM * 32;                            // U operand rows (16 halves each)
    constexpr int kBuf = NP * kPlane + kAu + XBM * 8;        // + d_w, dmin_w per row
    constexpr int kRed = 256 * 32 * 4;                       // group 1's partial tile
    constexpr int kLds = 2 * SK * kBuf > kRed ? 2 * SK * kBuf : kRed;
    __shared__ __attribute__((aligned(16))) char lds[kLds];

    const int grp = SK == 2 ? (int) threadIdx.x >> 8 : 0;
    const int tid = (int) threadIdx.x & 255;
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t ncols = act.ncols;
    int64_t n0, b0;
    {
        const int64_t nrt = (N + XBM - 1) / XBM, nct = (ncols + XBN - 1) / XBN;
        int64_t t = blockIdx.x;
        if constexpr (XCD) {
            // workgroup i runs on XCD i % 8: give each XCD a contiguous run of tiles, row tiles
            // fastest, so an XCD's L2 holds few activation column tiles
            const int64_t T = nrt * nct, per = (T + 7) / 8;
            t = (int64_t) (blockIdx.x % 8) * per + blockIdx.x / 8;
            if (t >= T) return;
        }
        n0 = (t % nrt) * XBM;
        b0 = (t / nrt) * XBN;
    }
    char * const lds_g = lds + grp * 2 * kBuf;

    // canonical chain split: half 0 sums superblocks [0, S/2), half 1 [S/2, S)
    const int S = (int) (K / 256);
    const int half = S / 2;
    const int sb_first = grp ? half : 0;
    const int n_sb = SK == 1 ? S : (grp ? S - half : half);
    const int n_sb_max = SK == 1 ? S : S - half;
    const int nst = 2 * n_sb;  // stages of this group (2 per superblock)

    // staging role: row ar, quarter q of the stage's 128 K (16 bytes of one 64-group's quants)
    const int ar = tid >> 2, q4 = tid & 3;
    const int64_t arow = std::min<int64_t>(n0 + ar, N - 1);
    const uint8_t * wrow = W + arow * nb01;

    // activation fragments: column b0 + 32 wave + (lane & 31), 16 bytes at 16 (lane >> 5)
    const int r = lane & 31, h = lane >> 5;
    const int64_t bcol = std::min<int64_t>(b0 + 32 * wave + r, ncols - 1);
    const int8_t * xcol = act.xq + bcol * 64 + 16 * h;
    const int64_t xstep = ncols * 64;  // bytes per 64-deep K block

    auto clamp_st = [&](int st) { return st < nst ? st : (nst > 0 ? nst - 1 : 0); };
    auto load_raw = [&](XRaw<TYPE> & raw, int st) {
        st = clamp_st(st);
        const int sb = sb_first + (st >> 1), hs = st & 1;
        const uint8_t * blk = wrow + (int64_t) sb * F::BS;
        const int j = 2 * hs + (q4 >> 1);
        raw.hdr = *(const uint4 *) blk;
        raw.qs = *(const uint4 *) (blk + (F::Q5 ? 48 : 16) + 32 * j + 16 * (q4 & 1));
        if constexpr (F::Q5) raw.qh = *(const uint4 *) (blk + 16 + 16 * (q4 & 1));
    };
    // activations of stage st; the second stage of a superblock also brings the superblock's U
    // operand and scale (one ring, so every load is consumed in issue order: vmcnt is in-order)
    auto load_x = [&](i32x4 (&xv)[4], half8 & bu, float & da, int st) {
        st = clamp_st(st);
        const int sb = sb_first + (st >> 1);
        const int64_t kb = (int64_t) sb * 4 + 2 * (st & 1);  // first 64-block
#pragma unroll
        for (int kk = 0; kk < 4; kk++) xv[kk] = *(const i32x4 *) (xcol + (kb + (kk >> 1)) * xstep + 32 * (kk & 1));
        if (st & 1) {
            bu = *(const half8 *) (act.xu + ((int64_t) sb * ncols + bcol) * 16 + 8 * h);
            da = act.xd[(int64_t) sb * ncols + bcol];
        }
    };
    // dequantize this thread's share of stage `st` into LDS buffer `buf`
    auto store_stage = [&](int buf, const XRaw<TYPE> & raw, int st) {
        char * base = lds_g + buf * kBuf;
        const int hs = st & 1;
        const int j = 2 * hs + (q4 >> 1);
        int sc0, m0, sc1, m1;
        mi_scale_min_k4(2 * j, raw.hdr.y, raw.hdr.z, raw.hdr.w, sc0, m0);
        mi_scale_min_k4(2 * j + 1, raw.hdr.y, raw.hdr.z, raw.hdr.w, sc1, m1);
        const uint32_t qs[4] = {raw.qs.x, raw.qs.y, raw.qs.z, raw.qs.w};
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            lo[i] = qs[i] & 0x0F0F0F0Fu;
            hi[i] = (qs[i] >> 4) & 0x0F0F0F0Fu;
            if constexpr (F::Q5) {
                const uint32_t qh[4] = {raw.qh.x, raw.qh.y, raw.qh.z, raw.qh.w};
                lo[i] |= ((qh[i] >> (2 * j)) & 0x01010101u) << 4;
                hi[i] |= ((qh[i] >> (2 * j + 1)) & 0x01010101u) << 4;
            }
        }
        const int off = ar * XROW + 64 * (q4 >> 1) + 16 * (q4 & 1);
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const uint32_t f0 = F::factor(sc0, p), f1 = F::factor(sc1, p);
            char * pl = base + p * kPlane + off;
            *(uint4 *) pl = make_uint4(mulb(lo[0], f0), mulb(lo[1], f0), mulb(lo[2], f0), mulb(lo[3], f0));
            *(uint4 *) (pl + 32) = make_uint4(mulb(hi[0], f1), mulb(hi[1], f1), mulb(hi[2], f1), mulb(hi[3], f1));
        }
        if (hs) return;
        // (first stage of a superblock) U operand of the row: halves [m_j, 64 m_j] for
        // j = 2 q4, 2 q4 + 1; and d_w / dmin_w
        int mA, mB, scA, scB;
        mi_scale_min_k4(2 * q4, raw.hdr.y, raw.hdr.z, raw.hdr.w, scA, mA);
        mi_scale_min_k4(2 * q4 + 1, raw.hdr.y, raw.hdr.z, raw.hdr.w, scB, mB);
        (void) scA;
        (void) scB;
        uint2 au;
        au.x = (uint32_t) mi_f2h((float) mA) | ((uint32_t) mi_f2h((float) (64 * mA)) << 16);
        au.y = (uint32_t) mi_f2h((float) mB) | ((uint32_t) mi_f2h((float) (64 * mB)) << 16);
        *(uint2 *) (base + NP * kPlane + ar * 32 + 8 * q4) = au;
        if (q4 < 2) {
            float * dwm = (float *) (base + NP * kPlane + kAu);
            dwm[q4 * XBM + ar] = mi_h2f((uint16_t) (q4 == 0 ? (raw.hdr.x & 0xFFFF) : (raw.hdr.x >> 16)));
        }
    };

    i32x16 acc[2][NP];
    f32x16 y[2], y1[2];  // y: this group's chain half (SK = 1: half 0), y1: half 1 (SK = 1 only)
#pragma unroll
    for (int t = 0; t < 2; t++) y[t] = y1[t] = f32x16{};
    XRaw<TYPE> raw[PF];
    i32x4 xb[PF][4];
    half8 bu[PF];
    float da[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) {
        load_raw(raw[u], u + 1);
        load_x(xb[u], bu[u], da[u], u);
    }
    {
        XRaw<TYPE> r0;
        load_raw(r0, 0);
        store_stage(0, r0, 0);
    }
    mi_lds_barrier();

    const int nst_max = 2 * n_sb_max;
    for (int s0 = 0; s0 < nst_max; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int st = s0 + u;
            if (st >= nst_max) break;  // uniform across the workgroup
            const int cur = st & 1;
            const bool active = st < nst;  // group-uniform
            const char * base = lds_g + cur * kBuf;
            const int sb = sb_first + (st >> 1);
            if (active) {
                const int hs = st & 1;
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                    i32x4 a[2][NP];
#pragma unroll
                    for (int t = 0; t < 2; t++)
#pragma unroll
                        for (int p = 0; p < NP; p++)
                            a[t][p] = *(const i32x4 *) (base + p * kPlane + (32 * t + r) * XROW + 32 * kk + 16 * h);
#pragma unroll
                    for (int t = 0; t < 2; t++)
#pragma unroll
                        for (int p = 0; p < NP; p++)
                            acc[t][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[t][p], xb[u][kk], (hs == 0 && kk == 0) ? i32x16{} : acc[t][p], 0, 0, 0);
                }
                if (hs == 1) {
                    // end of superblock: U on the f16 MFMA, then the canonical combine; the
                    // row operands were staged with the superblock's first stage (other buffer)
                    const char * base0 = lds_g + (cur ^ 1) * kBuf;
                    const float * dwv = (const float *) (base0 + NP * kPlane + kAu);
                    const bool second = SK == 1 && sb >= half;
#pragma unroll
                    for (int t = 0; t < 2; t++) {
                        const half8 au = *(const half8 *) (base0 + NP * kPlane + (32 * t + r) * 32 + 16 * h);
                        const f32x16 U = __builtin_amdgcn_mfma_f32_32x32x16_f16(au, bu[u], f32x16{}, 0, 0, 0);
#pragma unroll
                        for (int g = 0; g < 4; g++) {
                            const float4 dw4 = *(const float4 *) (dwv + 32 * t + 8 * g + 4 * h);
                            const float4 dm4 = *(const float4 *) (dwv + XBM + 32 * t + 8 * g + 4 * h);
                            const float dw[4] = {dw4.x, dw4.y, dw4.z, dw4.w};
                            const float dm[4] = {dm4.x, dm4.y, dm4.z, dm4.w};
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const int i = 4 * g + e;
                                int T = acc[t][NP - 1][i];
#pragma unroll
                                for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[t][p][i];
                                if (second) y1[t][i] = mmqx_term(y1[t][i], T, U[i], dw[e], dm[e], da[u]);
                                else y[t][i] = mmqx_term(y[t][i], T, U[i], dw[e], dm[e], da[u]);
                            }
                        }
                    }
                }
            }
            if (st + 1 < nst) store_stage(cur ^ 1, raw[u], st + 1);
            // slot u is consumed: refill it (weights for stage st + 1 + PF, activations st + PF)
            load_raw(raw[u], st + 1 + PF);
            load_x(xb[u], bu[u], da[u], st + PF);
            mi_lds_barrier();
        }
    }

    if constexpr (SK == 2) {
        // group 1 hands its partial tile (chain half 1) to group 0 through LDS
        float * red = (float *) lds;
        __syncthreads();
        if (grp == 1) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                red[(i * 2 + 0) * 256 + tid] = y[0][i];
                red[(i * 2 + 1) * 256 + tid] = y[1][i];
            }
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            y1[0][i] = red[(i * 2 + 0) * 256 + tid];
            y1[1][i] = red[(i * 2 + 1) * 256 + tid];
        }
    }
    // y = half 0 + half 1
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int i = 0; i < 16; i++) y[t][i] += y1[t][i];
    // D[n][b]: column b = lane & 31 of this wave's 32, rows n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    const int64_t b = b0 + 32 * wave + r;
    if (b >= ncols) return;
    float * out = (float *) ((char *) dst + b * ycol);
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int64_t n = n0 + 32 * t + 8 * g + 4 * h;
            if (n + 3 < N) {
                *(float4 *) (out + n) = make_float4(y[t][4 * g], y[t][4 * g + 1], y[t][4 * g + 2], y[t][4 * g + 3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = y[t][4 * g + e];
            }
        }
    }
}

} // namespace

bool mi_mmqx_supported(int type, int64_t K, size_t ycol) {
    return (type == 12 || type == 13) && K % 256 == 0 && K >= 256 && ycol % 16 == 0;
}

void mi_mul_mat_mmqx(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_mmx & act, float * dst,
                     size_t ycol, hipStream_t s) {
    const int64_t nrt = (N + XBM - 1) / XBM, nct = (act.ncols + XBN - 1) / XBN;
    const int64_t T = nrt * nct;
    // variant bits (GGML_MI355X_MMQ_VARIANT): 64 = XCD-contiguous tile order, 128 = two 4-wave
    // groups splitting the chain halves (2 waves per SIMD) instead of one group with both halves
    const int var = g_mi_tuning.mmq_variant;
    const bool xcd = (var & 64) != 0;
    const bool sk2 = (var & 128) != 0;
    const dim3 grid((unsigned) (xcd ? (T + 7) / 8 * 8 : T));
    const uint8_t * w = (const uint8_t *) W;
#define MI_MMQX(TY, SKV, PF)                                                                                              \
    if (xcd) hipLaunchKernelGGL((k_mmqx<TY, SKV, PF, true>), grid, dim3(256 * SKV), 0, s, w, nb01, K, N, act, dst, ycol);  \
    else hipLaunchKernelGGL((k_mmqx<TY, SKV, PF, false>), grid, dim3(256 * SKV), 0, s, w, nb01, K, N, act, dst, ycol);
    if (type == 12) {
        if (sk2) { MI_MMQX(12, 2, 2) } else { MI_MMQX(12, 1, 4) }
    } else {
        if (sk2) { MI_MMQX(13, 2, 2) } else { MI_MMQX(13, 1, 3) }
    }
#undef MI_MMQX
}
