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
// The float combine per superblock and the combine order are fixed (mmqx_pre, then cfold: the
// values scaled by d_a and summed in a fixed tree of superblock groups) and shared by every kernel
// of this file, so column shards of a
// prompt (prompt-sharded multi-GPU) give the same bits as the whole prompt, whichever kernel runs
// them. Against the
// reference CPU the only difference is the f32 combine order (reference: 8-lane partial chains
// + hsum): ~1e-7 relative.
//
// Workgroup and pipeline: k_mmqx below. Activation fragments come straight from HBM/L2 into a
// register ring (16 B per lane per 32-deep K step); the dequantized weight planes are shared by
// the workgroup's waves through LDS.
// Roofline: 2*N*K*B flops; at B=512 MFMA-bound. The NP planes make the int8 rate per weight
// 2 (Q4_K) or 3 (Q5_K) i8 MFMAs per 32 K, i.e. Q4_K runs at the dense f16 rate (2.5 PF/s).

#include <algorithm>
#include <type_traits>
#include <utility>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#pragma clang fp contract(off)

#include "mmq_exact_common.h"

// ---- activations: q8_K quants in the MFMA layouts ------------------------------------------------
// xq [K/32][ncols][32] int8 (a 32-deep MFMA step of 32 columns is one contiguous 1 KB), xd
// [K/256][ncols] f32 (d), xu [K/256][ncols][16] f16 (S_j & 63,
// S_j >> 6 for j = 0..7, S_j = sum of the 32 quants of sub-block j). One superblock per wave;
// grid (column, group of 4 superblocks): the column's address is wave-uniform scalar arithmetic
// (32-bit, and no divisions at all for a plain 2-D src1), so the load issues at once.
__global__ __launch_bounds__(256) void k_quantize_q8_K_mmx(mi_mmx_qgroup q) {
    const int wave = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t K = q.K;
    const uint32_t nb_per_col = (uint32_t) (K / 256);
    const uint32_t b = blockIdx.y * 4 + (uint32_t) wave;
    if (b >= nb_per_col) return;  // wave-uniform
    // the member this column belongs to (scalar scan over the kernel arguments)
    int mi = 0;
    while (mi + 1 < q.n && (int64_t) blockIdx.x >= q.m[mi + 1].col_begin) mi++;
    const mi_src_cols x = q.m[mi].x;
    const mi_act_mmx act = q.m[mi].act;
    const uint32_t c = (uint32_t) ((int64_t) blockIdx.x - q.m[mi].col_begin);
    const char * cbase;
    if (x.ne2 == 1 && x.ne3 == 1) {
        cbase = x.base + (size_t) c * x.nb1;
    } else {
        const uint32_t ne1 = (uint32_t) x.ne1, ne2 = (uint32_t) x.ne2;
        const uint32_t i1 = c % ne1, i2 = (c / ne1) % ne2, i3 = c / (ne1 * ne2);
        cbase = x.base + (size_t) i1 * x.nb1 + (size_t) i2 * x.nb2 + (size_t) i3 * x.nb3;
    }
    const float * col = (const float *) cbase;
    const float4 v4 = *(const float4 *) (col + b * 256 + lane * 4);
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    // quantize_row_q8_K_reference as the reference's -mfma build computes it (mi355x_common.h:
    // first max-|x| element keeps its sign, iscale = -127/max, fma rounding trick); DPP
    // reductions, sums of 32 per 8-lane group
    uint32_t packed;
    int sum;
    float d;
    mi_q8K_superblock(v, lane, packed, sum, d);
    const int64_t ncols = act.ncols;
    // element k = lane*4 .. +3 of the superblock: 32-block lane/8, offset (lane%8)*4
    *(uint32_t *) (act.xq + ((b * 8 + (lane >> 3)) * ncols + c) * 32 + (lane & 7) * 4) = packed;
    if ((lane & 7) == 0) {
        const int j = lane >> 3;
        const uint32_t lo = mi_f2h((float) (sum & 63)), hi = mi_f2h((float) (sum >> 6));
        *(uint32_t *) (act.xu + (b * ncols + c) * 16 + 2 * j) = lo | (hi << 16);
    }
    if (lane == 0) act.xd[b * ncols + c] = d;
}

// q8_0 activations (Q4_0 / Q8_0 weights) in the same MFMA layout: xq [K/32][ncols][32] int8, xd
// [K/32][ncols] f32 (the fp16-rounded d). quantize_row_q8_0 as the reference's AVX2 build computes
// it (src/ggml-quants.c:535-618: amax, d = amax / 127 -> fp16, id = 127 / amax, round-half-even
// of x * id); one 32-block per half-wave, grid (column, group of 8 blocks).
__global__ __launch_bounds__(256) void k_quantize_q8_0_mmx(mi_mmx_qgroup q) {
    const int64_t K = q.K;
    const int64_t nb_per_col = K / 32;
    const int64_t b = (int64_t) blockIdx.y * 8 + (threadIdx.x >> 5);
    const int l = threadIdx.x & 31;
    if (b >= nb_per_col) return;  // whole half-waves exit together
    int mi = 0;
    while (mi + 1 < q.n && (int64_t) blockIdx.x >= q.m[mi + 1].col_begin) mi++;
    const mi_src_cols x = q.m[mi].x;
    const mi_act_mmx act = q.m[mi].act;
    const uint32_t c = (uint32_t) ((int64_t) blockIdx.x - q.m[mi].col_begin);
    const char * cbase;
    if (x.ne2 == 1 && x.ne3 == 1) {
        cbase = x.base + (size_t) c * x.nb1;
    } else {
        const uint32_t ne1 = (uint32_t) x.ne1, ne2 = (uint32_t) x.ne2;
        const uint32_t i1 = c % ne1, i2 = (c / ne1) % ne2, i3 = c / (ne1 * ne2);
        cbase = x.base + (size_t) i1 * x.nb1 + (size_t) i2 * x.nb2 + (size_t) i3 * x.nb3;
    }
    const float v = ((const float *) cbase)[b * 32 + l];
    float amax = fabsf(v);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 32));
    const float d = amax / 127.f;
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    const float qv = __builtin_rintf(__fmul_rn(v, id));
    act.xq[(b * act.ncols + c) * 32 + l] = (int8_t) (int) qv;
    if (l == 0) act.xd[b * act.ncols + c] = mi_h2f(mi_f2h(d));
}

size_t mi_act_mmx0_bytes(int64_t K, int64_t ncols) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t) 255; };
    return al((size_t) K * ncols) + al((size_t) (K / 32) * ncols * 4);
}

mi_act_mmx mi_act_mmx0_carve(void * base, int64_t K, int64_t ncols) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t) 255; };
    char * p = (char *) base;
    mi_act_mmx a;
    a.K = K;
    a.ncols = ncols;
    a.xq = (int8_t *) p;
    a.xd = (float *) (p + al((size_t) K * ncols));
    a.xu = nullptr;
    return a;
}

void mi_quantize_q8_0_mmx_group(mi_mmx_qgroup & q, hipStream_t s) {
    int64_t cols = 0;
    for (int i = 0; i < q.n; i++) {
        q.m[i].col_begin = cols;
        cols += q.m[i].act.ncols;
    }
    if (cols == 0 || q.K < 32) return;
    hipLaunchKernelGGL(k_quantize_q8_0_mmx, dim3((unsigned) cols, (unsigned) ((q.K / 32 + 7) / 8)), dim3(256), 0, s, q);
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

void mi_quantize_q8_K_mmx_group(mi_mmx_qgroup & q, hipStream_t s) {
    int64_t cols = 0;
    for (int i = 0; i < q.n; i++) {
        q.m[i].col_begin = cols;
        cols += q.m[i].act.ncols;
    }
    if (cols == 0 || q.K < 256) return;
    hipLaunchKernelGGL(k_quantize_q8_K_mmx, dim3((unsigned) cols, (unsigned) ((q.K / 256 + 3) / 4)), dim3(256), 0, s, q);
}

void mi_quantize_q8_K_mmx(const mi_src_cols & x, int64_t K, const mi_act_mmx & act, hipStream_t s) {
    mi_mmx_qgroup q;
    q.n = 1;
    q.K = K;
    q.m[0].x = x;
    q.m[0].act = act;
    mi_quantize_q8_K_mmx_group(q, s);
}

namespace {

// ---- the GEMM -----------------------------------------------------------------------------------
// One workgroup = 8 wave64s (two per SIMD), tile 64 weight rows x 128 columns; wave (rw, cw) owns
// rows 32 rw.. x columns 32 cw.. (one 32x32 tile: one int8 MFMA per plane per 32-deep K step).
// A stage is one superblock (256 K): the 512 threads dequantize the next superblock's 64 rows
// (eight lanes per row, each a contiguous 16-byte chunk of its quants: coalesced loads) into
// the other LDS plane buffer, plus the row operands of the combine. Activations and weights arrive a stage ahead (vmcnt is in-order: every load is
// consumed in the order it was issued, each with one stage of lead). Two waves per SIMD: while
// one issues its MFMAs the other runs its dequantization / combine VALU.
// Canonical combine (shared by every kernel of this file): mmqx_pre per superblock, cfold's order.
// NWV = 4: half-width workgroups (64 rows x 64 columns, 4 waves, each thread stages two rows), two
// per CU, so one workgroup's barrier wait overlaps the other's MFMA steps.
template <int TYPE, bool XCD, int ABL = 0, int LEAD = 4, int SCT = 0, int NWV = 8>
__global__ __launch_bounds__(64 * NWV) void k_mmqx(mi_mmx_group g) {
    MI_MMX_MEMBER(g);
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    constexpr int XR = 256 + 16;             // LDS row stride of a plane (bytes): conflict-free b128 reads / writes
    constexpr int kPlane = XBM * XR;         // one plane of a superblock
    constexpr int kRow = XBM * 32 + XBM * 8; // row operands of the combine: U halves, d_w, dmin_w
    constexpr int kBuf = NP * kPlane + kRow;
    constexpr int XBN_ = 16 * NWV;              // columns per workgroup
    constexpr int ROWP = 8 / NWV;               // staging passes (rows per thread)
    constexpr int RSTEP = 8 * NWV;              // rows per staging pass
    __shared__ __attribute__((aligned(16))) char lds[2 * kBuf];

    const int tid = (int) threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int rw = wave & 1, cw = wave >> 1;
    const int64_t ncols = act.ncols;
    int64_t n0, b0;
    {
        const int64_t nrt = (N + XBM - 1) / XBM, nct = (ncols + XBN_ - 1) / XBN_;
        int64_t t = mmx_tile;
        if constexpr (XCD) {
            // workgroup i runs on XCD i % 8: give each XCD a contiguous run of tiles, row tiles
            // fastest, so an XCD's L2 holds few activation column tiles (one-member launches)
            const int64_t T = nrt * nct, per = (T + 7) / 8;
            t = (int64_t) (blockIdx.x % 8) * per + blockIdx.x / 8;
            if (t >= T) return;
        }
        n0 = (t % nrt) * XBM;
        b0 = (t / nrt) * XBN_;
    }
    const int S = (int) (K / 256);
    // timing diagnostics (ABL & 8; results invalid): s_memtime of wave 0 of workgroups 0 and 97 into
    // dst as uint64 [2][80]: 0 start, 1 after the prologue, 2 + 4 sb + {0 stage start, 1 after the
    // MFMA steps, 2 after the combine, 3 after the barrier}
    auto stamp = [&](int slot) {
        if constexpr ((ABL & 8) != 0) {
            const int wsel = blockIdx.x == 0 ? 0 : blockIdx.x == 97 ? 1 : -1;
            if (wsel >= 0 && (threadIdx.x >> 6) == 0 && (threadIdx.x & 63) == 0 && slot < 80)
                ((uint64_t *) dst)[wsel * 80 + slot] = __builtin_amdgcn_s_memtime();
        }
    };
    // and every workgroup's start / end on the constant 100 MHz clock: uint64 [gridDim][2] at 160
    auto rstamp = [&](int e) {
        if constexpr ((ABL & 8) != 0) {
            if (threadIdx.x == 0) ((uint64_t *) dst)[160 + 2 * blockIdx.x + e] = __builtin_amdgcn_s_memrealtime();
        }
    };
    rstamp(0);
    stamp(0);

    // All global loads go through buffer descriptors with 32-bit per-lane offsets (the host
    // checks the sizes): one address register per load instead of a 64-bit pointer.
    // staging role: row ar = tid / 8, 16-byte quant chunk c = tid % 8 of the superblock (eight
    // lanes read a row's 128 quant bytes contiguously): elements 16 (c & 1).. of sub-blocks
    // 2 (c / 2) (low nibbles) and 2 (c / 2) + 1 (high nibbles)
    const int ar = tid >> 3, c8 = tid & 7;
    const int nrows = (int) std::min<int64_t>(XBM, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    uint32_t wrow[ROWP];
#pragma unroll
    for (int pr = 0; pr < ROWP; pr++) wrow[pr] = (uint32_t) (std::min(ar + pr * RSTEP, nrows - 1) * nb01);
    const uint32_t qoff = (F::Q5 ? 48 : 16) + 16 * c8;
    const int j0 = 2 * (c8 >> 1), hf = c8 & 1;

    // activation fragments: column b0 + 32 cw + (lane & 31), 16 bytes at 16 (lane >> 5)
    const int r = lane & 31, h = lane >> 5;
    const uint32_t bcol = (uint32_t) std::min<int64_t>(b0 + 32 * cw + r, ncols - 1);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t ures = __builtin_amdgcn_make_buffer_rsrc((void *) act.xu, (short) 0, (int) (S * ncols * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) (S * ncols * 4), 0x00020000);
    const uint32_t xcol = bcol * 32 + 16 * h;
    const uint32_t xstep = (uint32_t) ncols * 32;  // bytes per 32-deep K step

    struct Raw {
        uint4 hdr, qs, qh;
    };
    auto load_raw = [&](Raw & raw, int sb, int pr) {
        sb = sb < S ? sb : S - 1;
        const uint32_t blk = wrow[pr] + (uint32_t) sb * F::BS;
        raw.hdr = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, blk, 0, 0));
        raw.qs = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, blk + qoff, 0, 0));
        if constexpr (F::Q5) raw.qh = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, blk + 16 + 16 * hf, 0, 0));
    };
    struct Xs {
        i32x4 q[8];
        half8 bu;
        float da;
    };
    auto load_x = [&](Xs & xs, int sb) {
        sb = sb < S ? sb : S - 1;
        const uint32_t kb = (uint32_t) sb * 8;  // first 32-deep step
#pragma unroll
        for (int kk = 0; kk < 8; kk++)
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol + (kb + kk) * xstep, 0, 0));
        const uint32_t sc = (uint32_t) sb * (uint32_t) ncols + bcol;
        xs.bu = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, sc * 32 + 16 * h, 0, 0));
        xs.da = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, sc * 4, 0, 0));
    };
    // 6-bit scale / min of sub-block j from the 12 scale bytes (words w0 w1 w2), as
    // get_scale_min_k4 (ggml-quants.c): field positions fixed per thread, so each is two
    // bit-field extracts and an or
    struct KSel {
        bool hi;
        uint32_t sh, w, shh, wh;
    };
    auto ksel = [](int j) { const int jj = j & 3; const bool hi = j >= 4; return KSel{hi, (uint32_t) (8 * jj), hi ? 4u : 6u, (uint32_t) (8 * jj + 6), hi ? 2u : 0u}; };
    const KSel k0 = ksel(j0), k1 = ksel(j0 + 1), kc = ksel(c8);
    auto kscale = [](const KSel & k, uint32_t w0, uint32_t w2) {
        return __builtin_amdgcn_ubfe(k.hi ? w2 : w0, k.sh, k.w) | (__builtin_amdgcn_ubfe(w0, k.shh, k.wh) << 4);
    };
    auto kmin = [](const KSel & k, uint32_t w1, uint32_t w2) {
        return __builtin_amdgcn_ubfe(k.hi ? w2 : w1, k.hi ? k.sh + 4 : k.sh, k.w) | (__builtin_amdgcn_ubfe(w1, k.shh, k.wh) << 4);
    };
    // dequantization of one thread's share of a superblock into LDS buffer `buf`, in pieces that
    // the stage loop interleaves with its MFMAs: unpack (dq_prep), plane p half hh (dq_piece, k =
    // 2 p + hh), the combine's row operands (dq_rows)
    struct Dq {
        uint32_t lo[4], hi[4], sc0, sc1;
    };
    auto dq_prep = [&](Dq & dq, const Raw & raw) {
        dq.sc0 = kscale(k0, raw.hdr.y, raw.hdr.w);
        dq.sc1 = kscale(k1, raw.hdr.y, raw.hdr.w);
        const uint32_t q[4] = {raw.qs.x, raw.qs.y, raw.qs.z, raw.qs.w};
        const uint32_t qh[4] = {raw.qh.x, raw.qh.y, raw.qh.z, raw.qh.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            dq.lo[i] = q[i] & 0x0F0F0F0Fu;
            dq.hi[i] = (q[i] >> 4) & 0x0F0F0F0Fu;
            if constexpr (F::Q5) {
                dq.lo[i] |= ((qh[i] >> j0) & 0x01010101u) << 4;
                dq.hi[i] |= ((qh[i] >> (j0 + 1)) & 0x01010101u) << 4;
            }
        }
    };
    auto dq_piece = [&](int buf, const Dq & dq, int k, int pr) {
        if constexpr ((ABL & 1) != 0) return;  // timing ablation: no dequantization
        char * pl0 = lds + buf * kBuf + (ar + pr * RSTEP) * XR + 32 * j0 + 16 * hf;
        const int p = k >> 1;
        if ((k & 1) == 0) {
            const uint32_t f0 = F::factor((int) dq.sc0, p);
            *(uint4 *) (pl0 + p * kPlane) = make_uint4(mulb(dq.lo[0], f0), mulb(dq.lo[1], f0), mulb(dq.lo[2], f0), mulb(dq.lo[3], f0));
        } else {
            const uint32_t f1 = F::factor((int) dq.sc1, p);
            *(uint4 *) (pl0 + p * kPlane + 32) = make_uint4(mulb(dq.hi[0], f1), mulb(dq.hi[1], f1), mulb(dq.hi[2], f1), mulb(dq.hi[3], f1));
        }
    };
    auto dq_rows = [&](int buf, const Raw & raw, int pr) {
        if constexpr ((ABL & 1) != 0) return;
        const int ar = (tid >> 3) + pr * RSTEP;
        // row operands: U halves [m_c, 64 m_c] at slot c; d_w (c = 0), dmin_w (c = 1)
        char * ro = lds + buf * kBuf + NP * kPlane;
        const uint32_t mc = kmin(kc, raw.hdr.z, raw.hdr.w);
        *(uint32_t *) (ro + ar * 32 + 4 * c8) = (uint32_t) mi_f2h((float) mc) | ((uint32_t) mi_f2h((float) (64 * mc)) << 16);
        if (c8 < 2) ((float *) (ro + XBM * 32))[c8 * XBM + ar] = mi_h2f((uint16_t) (c8 == 0 ? (raw.hdr.x & 0xFFFF) : (raw.hdr.x >> 16)));
    };
    auto store_stage = [&](int buf, const Raw & raw, int pr) {
        Dq dq;
        dq_prep(dq, raw);
#pragma unroll
        for (int k = 0; k < 2 * NP; k++) dq_piece(buf, dq, k, pr);
        dq_rows(buf, raw, pr);
    };

    f32x16 y = f32x16(-0.0f), gsum = {};  // y = -0: cfold_vec's first group sum lands exactly
    // the thread's output elements D[n][b]: column b = lane & 31 of this wave's 32, rows n = (reg & 3)
    // + 8 (reg >> 2) + 4 (lane >> 5); also where the low half's sum is parked (no register to spare)
    const int64_t bo = b0 + 32 * cw + r;
    auto y_io = [&](f32x16 & v, bool st) {
        if (bo >= ncols) return;
        float * out = (float *) ((char *) dst + bo * ycol);
#pragma unroll
        for (int gq = 0; gq < 4; gq++) {
            const int64_t n = n0 + 32 * rw + 8 * gq + 4 * h;
            if (n + 3 < N) {
                if (st) {
                    *(float4 *) (out + n) = make_float4(v[4 * gq], v[4 * gq + 1], v[4 * gq + 2], v[4 * gq + 3]);
                } else {
                    const float4 t = *(const float4 *) (out + n);
                    v[4 * gq] = t.x; v[4 * gq + 1] = t.y; v[4 * gq + 2] = t.z; v[4 * gq + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    if (n + e < N) {
                        if (st) out[n + e] = v[4 * gq + e];
                        else v[4 * gq + e] = out[n + e];
                    }
                }
            }
        }
    };
    auto park = [&](const f32x16 & v) {
        if constexpr ((ABL & 8) == 0) {
            f32x16 t = v;
            y_io(t, true);
        }
    };
    const int gs = cfold_gs(S);
    // The raw weights of superblock sb + 1 are dequantized into LDS at the end of stage sb; they
    // were requested LEAD stages earlier (a ring of LEAD raw slots: HBM latency is several stage
    // times). The activation fragment of step kk of sb + 1 is loaded into the register that step kk
    // of sb has just consumed (L2-resident: one stage of lead is enough).
    Raw raw[LEAD][ROWP];
    Xs xs;
#pragma unroll
    for (int pr = 0; pr < ROWP; pr++) {
        Raw r0;
        load_raw(r0, 0, pr);
        store_stage(0, r0, pr);
    }
    load_x(xs, 0);
#pragma unroll
    for (int u = 0; u < LEAD; u++)
#pragma unroll
        for (int pr = 0; pr < ROWP; pr++) load_raw(raw[u][pr], 1 + u, pr);
    mi_lds_barrier();
    stamp(1);

    // one stage = superblock sb; LDS buffer sb & 1. Unrolled by LEAD so every ring slot index is
    // static (slot u = sb % LEAD holds superblock sb + 1); fully unrolled when S is a template
    // constant (SCT), so no loop back-edge makes the compiler drain the ring.
    const int S_ = SCT > 0 ? SCT : S;
    auto stage = [&](const int sb, Raw (&rslot)[ROWP]) {
        stamp(2 + 4 * sb);
        const int cur = sb & 1;
        const char * base = lds + cur * kBuf;
        const char * arow_p = base + (32 * rw + r) * XR + 16 * h;
        const int nx = sb + 1 < S ? sb + 1 : S - 1;
        const uint32_t kbn = (uint32_t) nx * 8;
        i32x16 acc[NP];
        // weight fragments two 32-deep steps ahead (explicit ring; the sched_barrier per step
        // keeps the compiler from hoisting every step's LDS reads: registers)
        i32x4 an[2][NP];
#pragma unroll
        for (int p = 0; p < NP; p++) {
            an[0][p] = *(const i32x4 *) (arow_p + p * kPlane);
            an[1][p] = *(const i32x4 *) (arow_p + p * kPlane + 32);
        }
        // the dequantization of superblock sb + 1 (raw loaded LEAD stages ago) into the other LDS
        // buffer, one piece per 32-deep step, between this stage's MFMAs (the other buffer's
        // readers finished at the previous stage's barrier); then the slot's next load
        Dq dq[ROWP];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            i32x4 a[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) a[p] = an[kk & 1][p];
            if (kk < 6) {
#pragma unroll
                for (int p = 0; p < NP; p++) an[kk & 1][p] = *(const i32x4 *) (arow_p + p * kPlane + 32 * (kk + 2));
            }
#pragma unroll
            for (int p = 0; p < NP; p++) {
                if constexpr ((ABL & 4) != 0) {  // timing ablation: no MFMAs
                    acc[p][kk] = (kk == 0 ? 0 : acc[p][kk]) + a[p][0] * xs.q[kk][0];
                } else {
                    acc[p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[p], xs.q[kk], kk == 0 ? i32x16{} : acc[p], 0, 0, 0);
                }
            }
            // step kk of the next superblock into the register just consumed
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol + (kbn + kk) * xstep, 0, 0));
#pragma unroll
            for (int pr = 0; pr < ROWP; pr++) {
                if (kk == 0) dq_prep(dq[pr], rslot[pr]);
                if (kk >= 1 && kk <= 2 * NP) dq_piece(cur ^ 1, dq[pr], kk - 1, pr);
                if (kk == 7) {
                    dq_rows(cur ^ 1, rslot[pr], pr);
                    load_raw(rslot[pr], sb + 1 + LEAD, pr);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        stamp(3 + 4 * sb);
        // U on the f16 MFMA, then the canonical combine
        if constexpr ((ABL & 2) != 0) {  // timing ablation: no combine
#pragma unroll
            for (int i = 0; i < 16; i++) {
                float gg = gsum[i], yy = y[i], ll = -0.0f;  // (timing ablation: results invalid)
                cfold(gg, yy, ll, (float) acc[0][i], 1.0f, sb, gs, S);
                gsum[i] = gg;
                y[i] = yy;
            }
        } else {
            const char * ro = base + NP * kPlane;
            const float * dwv = (const float *) (ro + XBM * 32);
            const half8 au = *(const half8 *) (ro + (32 * rw + r) * 32 + 16 * h);
            const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(au, xs.bu, f32x16{}, 0, 0, 0);
            const float da = xs.da;
            {
                const uint32_t sc = (uint32_t) nx * (uint32_t) ncols + bcol;
                xs.bu = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, sc * 32 + 16 * h, 0, 0));
                xs.da = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, sc * 4, 0, 0));
            }
            f32x16 tv;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const float4 dw4 = *(const float4 *) (dwv + 32 * rw + 8 * g + 4 * h);
                const float4 dm4 = *(const float4 *) (dwv + XBM + 32 * rw + 8 * g + 4 * h);
                const float dw[4] = {dw4.x, dw4.y, dw4.z, dw4.w};
                const float dm[4] = {dm4.x, dm4.y, dm4.z, dm4.w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int i = 4 * g + e;
                    int T = acc[NP - 1][i];
#pragma unroll
                    for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[p][i];
                    tv[i] = mmqx_pre(T, Uv[i], dw[e], dm[e]);
                }
            }
            cfold_vec_park(gsum, y, tv, f32x16(da), sb, gs, S, park);
        }
        stamp(4 + 4 * sb);
        mi_lds_barrier();
        stamp(5 + 4 * sb);
    };
    if constexpr (SCT > 0) {
#pragma unroll
        for (int sb = 0; sb < SCT; sb++) stage(sb, raw[sb % LEAD]);
    } else {
        for (int sb0 = 0; sb0 < S_; sb0 += LEAD) {
#pragma unroll
            for (int u = 0; u < LEAD; u++) {
                if (sb0 + u < S_) stage(sb0 + u, raw[u]);
            }
        }
    }

    rstamp(1);
    if constexpr ((ABL & 8) != 0) {
        // dst holds the stamps; keep the results alive (an unlikely-value store) so nothing is
        // eliminated
        float t = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; i++) t += y[i];
        if (t == 1.2345e-30f) dst[4096 + threadIdx.x] = t;
        return;
    }
    if (cfold_split(S) < S) {  // cfold_end: the parked low half + the high half
        f32x16 lo = {};
        y_io(lo, false);
        y = lo + y;
    }
    y_io(y, true);
}


// ---- long prompts, warp-specialized: loader waves stage, MFMA waves compute ----------------------
// k_mmqx's tile (64 weight rows x 128 columns) and stage structure, with the roles split: 8 MFMA
// waves (rw, cw) compute their 32 x 32 tiles from the LDS planes of superblock sb while 4 loader
// waves turn superblock sb + 1 (requested LEAD stages earlier) into the other LDS buffer's planes
// and row operands. Every wave passes the same one barrier per stage. In k_mmqx each wave does its
// MFMA steps, its share of the dequantization and the combine, and the barrier then waits for the
// slowest; here the MFMA waves' stage is only MFMAs + combine. Same operands, same canonical combine
// (mmqx_pre, cfold_vec): bit-identical to k_mmqx.
// ABL 8: timing stamps of MFMA wave 0 (workgroups 0 and 97) into dst, as k_mmqx (results invalid)
template <int TYPE, int LEAD, int ABL = 0>
__global__ __launch_bounds__(768, 1) void k_mmqw(mi_mmx_group g) {
    MI_MMX_MEMBER(g);
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    constexpr int XR = 256 + 16;
    constexpr int kPlane = XBM * XR;
    constexpr int kRow = XBM * 32 + XBM * 8;
    constexpr int kBuf = NP * kPlane + kRow;
    constexpr int NCW = 8;       // MFMA waves
    constexpr int ROWP = 2;      // loader threads (256) x 2 rows = 64 rows
    constexpr int RSTEP = 32;
    __shared__ __attribute__((aligned(16))) char lds[2 * kBuf];

    const int tid = (int) threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const bool loader = wave >= NCW;  // wave-uniform role
    const int rw = wave & 1, cw = (wave >> 1) & 3;
    const int64_t ncols = act.ncols;
    const int64_t nrt = (N + XBM - 1) / XBM;
    const int64_t n0 = (mmx_tile % nrt) * XBM, b0 = (mmx_tile / nrt) * XBN;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);

    // loader role: thread lt = tid - 512, row ar (+ 32), 16-byte quant chunk c8 of the superblock
    const int lt = tid - 64 * NCW;
    const int ar = (lt >> 3) & 31, c8 = lt & 7;
    const int nrows = (int) std::min<int64_t>(XBM, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    uint32_t wrow[ROWP];
#pragma unroll
    for (int pr = 0; pr < ROWP; pr++) wrow[pr] = (uint32_t) (std::min(ar + pr * RSTEP, nrows - 1) * nb01);
    const uint32_t qoff = (F::Q5 ? 48 : 16) + 16 * c8;
    const int j0 = 2 * (c8 >> 1), hf = c8 & 1;

    // MFMA role: column b0 + 32 cw + (lane & 31), 16 bytes at 16 (lane >> 5)
    const int r = lane & 31, h = lane >> 5;
    const uint32_t bcol = (uint32_t) std::min<int64_t>(b0 + 32 * cw + r, ncols - 1);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t ures = __builtin_amdgcn_make_buffer_rsrc((void *) act.xu, (short) 0, (int) (S * ncols * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) (S * ncols * 4), 0x00020000);
    const uint32_t xcol = bcol * 32 + 16 * h;
    const uint32_t xstep = (uint32_t) ncols * 32;

    struct Raw {
        uint4 hdr, qs, qh;
    };
    auto load_raw = [&](Raw & raw, int sb, int pr) {
        sb = sb < S ? sb : S - 1;
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(sb * F::BS);
        raw.hdr = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wrow[pr], so, 0));
        raw.qs = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wrow[pr] + qoff, so, 0));
        if constexpr (F::Q5) raw.qh = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wrow[pr] + 16 + 16 * hf, so, 0));
    };
    struct Xs {
        i32x4 q[8];
        half8 bu;
        float da;
    };
    auto load_x = [&](Xs & xs, int sb) {
        sb = sb < S ? sb : S - 1;
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((sb * 8 + kk) * (int) xstep);
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol, so, 0));
        }
        const uint32_t sc = (uint32_t) sb * (uint32_t) ncols + bcol;
        xs.bu = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, sc * 32 + 16 * h, 0, 0));
        xs.da = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, sc * 4, 0, 0));
    };
    struct KSel {
        bool hi;
        uint32_t sh, w, shh, wh;
    };
    auto ksel = [](int j) { const int jj = j & 3; const bool hi = j >= 4; return KSel{hi, (uint32_t) (8 * jj), hi ? 4u : 6u, (uint32_t) (8 * jj + 6), hi ? 2u : 0u}; };
    const KSel k0 = ksel(j0), k1 = ksel(j0 + 1), kc = ksel(c8);
    auto kscale = [](const KSel & k, uint32_t w0, uint32_t w2) {
        return __builtin_amdgcn_ubfe(k.hi ? w2 : w0, k.sh, k.w) | (__builtin_amdgcn_ubfe(w0, k.shh, k.wh) << 4);
    };
    auto kmin = [](const KSel & k, uint32_t w1, uint32_t w2) {
        return __builtin_amdgcn_ubfe(k.hi ? w2 : w1, k.hi ? k.sh + 4 : k.sh, k.w) | (__builtin_amdgcn_ubfe(w1, k.shh, k.wh) << 4);
    };
    // one loader thread's share of a superblock (rows ar, ar + 32) into LDS buffer `buf`
    auto store_stage = [&](int buf, const Raw & raw, int pr) {
        const int row = ar + pr * RSTEP;
        const uint32_t sc0 = kscale(k0, raw.hdr.y, raw.hdr.w), sc1 = kscale(k1, raw.hdr.y, raw.hdr.w);
        const uint32_t q[4] = {raw.qs.x, raw.qs.y, raw.qs.z, raw.qs.w};
        const uint32_t qh[4] = {raw.qh.x, raw.qh.y, raw.qh.z, raw.qh.w};
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            lo[i] = q[i] & 0x0F0F0F0Fu;
            hi[i] = (q[i] >> 4) & 0x0F0F0F0Fu;
            if constexpr (F::Q5) {
                lo[i] |= ((qh[i] >> j0) & 0x01010101u) << 4;
                hi[i] |= ((qh[i] >> (j0 + 1)) & 0x01010101u) << 4;
            }
        }
        char * pl0 = lds + buf * kBuf + row * XR + 32 * j0 + 16 * hf;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const uint32_t f0 = F::factor((int) sc0, p), f1 = F::factor((int) sc1, p);
            *(uint4 *) (pl0 + p * kPlane) = make_uint4(mulb(lo[0], f0), mulb(lo[1], f0), mulb(lo[2], f0), mulb(lo[3], f0));
            *(uint4 *) (pl0 + p * kPlane + 32) = make_uint4(mulb(hi[0], f1), mulb(hi[1], f1), mulb(hi[2], f1), mulb(hi[3], f1));
        }
        char * ro = lds + buf * kBuf + NP * kPlane;
        const uint32_t mc = kmin(kc, raw.hdr.z, raw.hdr.w);
        *(uint32_t *) (ro + row * 32 + 4 * c8) = (uint32_t) mi_f2h((float) mc) | ((uint32_t) mi_f2h((float) (64 * mc)) << 16);
        if (c8 < 2) ((float *) (ro + XBM * 32))[c8 * XBM + row] = mi_h2f((uint16_t) (c8 == 0 ? (raw.hdr.x & 0xFFFF) : (raw.hdr.x >> 16)));
    };

    // The roles run separate loops (so their registers are not live at once), each passing the
    // same 1 + S barriers.
    if (loader) {
        Raw raw[LEAD][ROWP];
#pragma unroll
        for (int pr = 0; pr < ROWP; pr++) {
            Raw r0;
            load_raw(r0, 0, pr);
            store_stage(0, r0, pr);
        }
#pragma unroll
        for (int u = 0; u < LEAD; u++)
#pragma unroll
            for (int pr = 0; pr < ROWP; pr++) load_raw(raw[u][pr], 1 + u, pr);
        mi_lds_barrier();
        // S % LEAD == 0 (host-checked) and no branch in the body, so the waits are exact (vmcnt
        // retires in order: a slot's loads wait only for themselves). Past the end the loads are
        // clamped re-reads and the last store fills the buffer nobody reads any more.
        for (int sb0 = 0; sb0 < S; sb0 += LEAD) {
#pragma unroll
            for (int u = 0; u < LEAD; u++) {
                const int sb = sb0 + u;
                // superblock sb + 1 into the other buffer (its readers passed the last barrier),
                // then the slot's next request
#pragma unroll
                for (int pr = 0; pr < ROWP; pr++) store_stage((sb + 1) & 1, raw[u][pr], pr);
#pragma unroll
                for (int pr = 0; pr < ROWP; pr++) load_raw(raw[u][pr], sb + 1 + LEAD, pr);
                mi_lds_barrier();
            }
        }
        return;
    }

    auto stamp = [&](int slot) {
        if constexpr ((ABL & 8) != 0) {
            const int wsel = blockIdx.x == 0 ? 0 : blockIdx.x == 97 ? 1 : -1;
            if (wsel >= 0 && wave == 0 && lane == 0 && slot < 80) ((uint64_t *) dst)[wsel * 80 + slot] = __builtin_amdgcn_s_memtime();
        }
    };
    auto rstamp = [&](int e) {
        if constexpr ((ABL & 8) != 0) {
            if (threadIdx.x == 0) ((uint64_t *) dst)[160 + 2 * blockIdx.x + e] = __builtin_amdgcn_s_memrealtime();
        }
    };
    rstamp(0);
    stamp(0);
    f32x16 y = f32x16(-0.0f), gsum = {};
    // the thread's output elements D[n][b]: column b = lane & 31 of this wave's 32, rows n = (reg & 3)
    // + 8 (reg >> 2) + 4 (lane >> 5); also where the low half's sum is parked (no register to spare)
    const int64_t bo = b0 + 32 * cw + r;
    auto y_io = [&](f32x16 & v, bool st) {
        if (bo >= ncols) return;
        float * out = (float *) ((char *) dst + bo * ycol);
#pragma unroll
        for (int gq = 0; gq < 4; gq++) {
            const int64_t n = n0 + 32 * rw + 8 * gq + 4 * h;
            if (n + 3 < N) {
                if (st) {
                    *(float4 *) (out + n) = make_float4(v[4 * gq], v[4 * gq + 1], v[4 * gq + 2], v[4 * gq + 3]);
                } else {
                    const float4 t = *(const float4 *) (out + n);
                    v[4 * gq] = t.x; v[4 * gq + 1] = t.y; v[4 * gq + 2] = t.z; v[4 * gq + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    if (n + e < N) {
                        if (st) out[n + e] = v[4 * gq + e];
                        else v[4 * gq + e] = out[n + e];
                    }
                }
            }
        }
    };
    auto park = [&](const f32x16 & v) {
        if constexpr ((ABL & 8) == 0) {
            f32x16 t = v;
            y_io(t, true);
        }
    };
    Xs xs;
    load_x(xs, 0);
    mi_lds_barrier();
    stamp(1);
    for (int sb = 0; sb < S; sb++) {
        stamp(2 + 4 * sb);
        const char * base = lds + (sb & 1) * kBuf;
        const char * arow_p = base + (32 * rw + r) * XR + 16 * h;
        const int nx = sb + 1 < S ? sb + 1 : S - 1;
        const uint32_t kbn = (uint32_t) nx * 8;
        i32x16 acc[NP];
        i32x4 an[2][NP];
#pragma unroll
        for (int p = 0; p < NP; p++) {
            an[0][p] = *(const i32x4 *) (arow_p + p * kPlane);
            an[1][p] = *(const i32x4 *) (arow_p + p * kPlane + 32);
        }
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            i32x4 a[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) a[p] = an[kk & 1][p];
            if (kk < 6) {
#pragma unroll
                for (int p = 0; p < NP; p++) an[kk & 1][p] = *(const i32x4 *) (arow_p + p * kPlane + 32 * (kk + 2));
            }
#pragma unroll
            for (int p = 0; p < NP; p++)
                acc[p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[p], xs.q[kk], kk == 0 ? i32x16{} : acc[p], 0, 0, 0);
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((int) (kbn + kk) * (int) xstep);
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol, so, 0));
            __builtin_amdgcn_sched_barrier(0);
        }
        stamp(3 + 4 * sb);
        const char * ro = base + NP * kPlane;
        const float * dwv = (const float *) (ro + XBM * 32);
        const half8 au = *(const half8 *) (ro + (32 * rw + r) * 32 + 16 * h);
        const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(au, xs.bu, f32x16{}, 0, 0, 0);
        const float da = xs.da;
        {
            const uint32_t sc = (uint32_t) nx * (uint32_t) ncols + bcol;
            xs.bu = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, sc * 32 + 16 * h, 0, 0));
            xs.da = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, sc * 4, 0, 0));
        }
        f32x16 tv;
#pragma unroll
        for (int gq = 0; gq < 4; gq++) {
            const float4 dw4 = *(const float4 *) (dwv + 32 * rw + 8 * gq + 4 * h);
            const float4 dm4 = *(const float4 *) (dwv + XBM + 32 * rw + 8 * gq + 4 * h);
            const float dw[4] = {dw4.x, dw4.y, dw4.z, dw4.w};
            const float dm[4] = {dm4.x, dm4.y, dm4.z, dm4.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int i2 = 4 * gq + e;
                int T = acc[NP - 1][i2];
#pragma unroll
                for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[p][i2];
                tv[i2] = mmqx_pre(T, Uv[i2], dw[e], dm[e]);
            }
        }
        cfold_vec_park(gsum, y, tv, f32x16(da), sb, gs, S, park);
        stamp(4 + 4 * sb);
        mi_lds_barrier();
        stamp(5 + 4 * sb);
    }
    rstamp(1);
    if constexpr ((ABL & 8) != 0) {
        float t = 0.0f;
#pragma unroll
        for (int i2 = 0; i2 < 16; i2++) t += y[i2];
        if (t == 1.2345e-30f) dst[4096 + threadIdx.x] = t;
        return;
    }
    if (cfold_split(S) < S) {  // cfold_end: the parked low half + the high half
        f32x16 lo = {};
        y_io(lo, false);
        y = lo + y;
    }
    y_io(y, true);
}

// ---- short prompts, pipelined: 8 waves per tile, one superblock group each -----------------------
// A workgroup computes one tile of 32 weight rows x 32 NC prompt columns; wave w computes the terms
// of superblock group w of the canonical order (cfold: kCfoldGroups = 8 contiguous groups) one
// superblock after the other and left-folds them in registers. The weights of the next superblock
// are requested before the current one's MFMAs (register double buffer); each 32-deep activation
// fragment of the next superblock is requested into the register its step has just consumed. The
// 8 group sums meet in LDS and are folded by the whole workgroup. With NC = 2 a wave's dequantized
// weight planes feed two column tiles (half the dequantization VALU per MFMA).
// VALU economy: the plane factors of all 8 sub-blocks come from 2 SWAR extractions of the header's
// scale bytes (one bit-field extract per factor), loads advance by a wave-uniform SGPR offset (no
// per-load address VALU), and the activation scales travel as one float per lane through a
// wave-private LDS row.
// MFMA orientation as k_mmqd1: A = activation fragment (accumulator row = prompt column), B = the
// dequantized weight planes (accumulator column = the lane's own weight row r).
// NW = 4: two workgroups per CU (<= 256 VGPRs at two waves per SIMD), each wave computing groups
// w and w + 4 one after the other (each group's sum goes to LDS when it ends).
// RING: weight register buffers; superblock k + RING - 1's weights are requested when step k starts.
// r03v counters (RING 2, B = 32, 16 members): waves wait ~45 % of their cycles (SQ_WAIT_INST_ANY),
// MFMA 9 % busy, 18 VALU per MFMA. RING 4 measured slower (r03w): the activation fragments of step
// k + 1 are requested after those weights, and vmcnt retires in order.
template <int TYPE, int NC, int NW, int ABL = 0, int RING = 4>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void k_mmqp(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    constexpr int NE = 16 * NC;  // accumulator elements per lane
    constexpr int NG = kCfoldGroups / NW;  // groups per wave
    __shared__ __attribute__((aligned(16))) float red[kCfoldGroups * NE * 64];  // [group][el][lane] group sums
    __shared__ __attribute__((aligned(16))) float dal[NW][32 * NC];              // per-wave da row
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);
    // this wave's superblocks: groups w, w + NW, ... -> the list [g gs, min(S, (g + 1) gs)) of each
    auto gbeg = [&](int i) { return min(S, (w + NW * i) * gs); };
    auto gend = [&](int i) { return min(S, (w + NW * i + 1) * gs); };
    const int nsb = [&] { int n = 0; for (int i = 0; i < NG; i++) n += gend(i) - gbeg(i); return n; }();
    // the wave's k-th superblock (clamped to its last one)
    auto sb_at = [&](int k) {
        k = min(k, nsb - 1);
#pragma unroll
        for (int i = 0; i < NG; i++) {
            const int len = gend(i) - gbeg(i);
            if (k < len) return gbeg(i) + k;
            k -= len;
        }
        return S - 1;
    };
    const int64_t nrt = (N + 31) / 32;
    const int64_t n0 = (mmx_tile % nrt) * 32, c0 = (mmx_tile / nrt) * (32 * NC);

    const int nrows = (int) std::min<int64_t>(32, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t ures = __builtin_amdgcn_make_buffer_rsrc((void *) act.xu, (short) 0, (int) (S * ncols * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) (S * ncols * 4), 0x00020000);
    constexpr uint32_t kQs = F::Q5 ? 48 : 16;
    // lane-constant parts of every offset; the superblock / step advance is an SGPR
    const uint32_t wv = (uint32_t) (min(r, nrows - 1) * nb01);
    uint32_t acol[NC];
#pragma unroll
    for (int t = 0; t < NC; t++) acol[t] = (uint32_t) std::min<int64_t>(c0 + 32 * t + r, ncols - 1);
    const uint32_t xstep = (uint32_t) ncols * 32;

    auto ld = [](__amdgpu_buffer_rsrc_t res, uint32_t voff, uint32_t soff) -> uint4 {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(res, voff, soff, 0));
    };
    struct Wt {
        uint4 hdr, q4[4], qh;
    };
    auto load_w = [&](Wt & o, int sb) {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(sb * F::BS);
        o.hdr = ld(wres, wv, so);
#pragma unroll
        for (int p = 0; p < 4; p++) o.q4[p] = ld(wres, wv + kQs + 32 * p + 16 * h, so);
        if constexpr (F::Q5) o.qh = ld(wres, wv + 16 + 16 * h, so);
    };
    auto ld_x = [&](int sb, int kk, int t) -> i32x4 {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((sb * 8 + kk) * (int) xstep);
        return __builtin_bit_cast(i32x4, ld(xres, acol[t] * 32 + 16 * h, so));
    };
    auto ld_u = [&](int sb, int t) -> half8 {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(sb * (int) ncols * 32);
        return __builtin_bit_cast(half8, ld(ures, acol[t] * 32 + 16 * h, so));
    };
    auto ld_d = [&](int sb, int t) -> float {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(sb * (int) ncols * 4);
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, acol[t] * 4, so, 0));
    };

    f32x16 gsum[NC];
#pragma unroll
    for (int t = 0; t < NC; t++) gsum[t] = f32x16{};
    if (nsb > 0) {
        Wt wt[RING];
        i32x4 xa[NC][8];
        half8 xu[NC];
        float da[NC];
        const int sbf = sb_at(0);
#pragma unroll
        for (int u = 0; u < RING - 1; u++) load_w(wt[u], sb_at(u));
#pragma unroll
        for (int t = 0; t < NC; t++) {
#pragma unroll
            for (int kk = 0; kk < 8; kk++) xa[t][kk] = ld_x(sbf, kk, t);
            xu[t] = ld_u(sbf, t);
            da[t] = ld_d(sbf, t);
        }
        // the wave's k-th superblock: `cur` holds its weights; superblock k + RING - 1's weights go
        // into `nxt` (the buffer the previous step consumed), the next superblock's activations are
        // requested step by step as their registers free up
        auto step = [&](const Wt & cur, Wt & nxt, const int k) {
            const int sb = sb_at(k);
            const int sn = sb_at(k + 1);  // clamped: a past-the-end prefetch re-reads the last one
            const bool first = sb % gs == 0, last = sb % gs == gs - 1 || sb == S - 1;
            load_w(nxt, sb_at(k + RING - 1));
            const uint32_t w0 = cur.hdr.y, w1 = cur.hdr.z, w2 = cur.hdr.w;
            // the 6-bit scales of sub-blocks 0..3 / 4..7 as bytes (get_scale_min_k4)
            const uint32_t sca = w0 & 0x3F3F3F3Fu;
            const uint32_t scb = (w2 & 0x0F0F0F0Fu) | ((w0 >> 2) & 0x30303030u);
            const float dw = mi_h2f((uint16_t) (cur.hdr.x & 0xFFFF)), dm = mi_h2f((uint16_t) (cur.hdr.x >> 16));
            i32x16 acc[NC][NP];
            uint32_t lo[4], hi[4];
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                if ((kk & 1) == 0) {
                    const uint4 q = cur.q4[kk >> 1];
                    const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        lo[e] = qv[e] & 0x0F0F0F0Fu;
                        hi[e] = (qv[e] >> 4) & 0x0F0F0F0Fu;
                    }
                }
                uint32_t v[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    v[e] = (kk & 1) ? hi[e] : lo[e];
                    if constexpr (F::Q5) {
                        const uint32_t hb[4] = {cur.qh.x, cur.qh.y, cur.qh.z, cur.qh.w};
                        v[e] |= ((hb[e] >> kk) & 0x01010101u) << 4;
                    }
                }
                const uint32_t scw = kk < 4 ? sca : scb;
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    // plane factor: Q4_K sc = 8 hi3 + lo3; Q5_K sc = 16 f2 + 4 f1 + f0
                    const uint32_t f = __builtin_amdgcn_ubfe(scw, 8 * (kk & 3) + (F::Q5 ? 2 * p : 3 * p), F::Q5 ? 2 : 3);
                    const i32x4 b = {(int) mulb(v[0], f), (int) mulb(v[1], f), (int) mulb(v[2], f), (int) mulb(v[3], f)};
#pragma unroll
                    for (int t = 0; t < NC; t++) {
                        if constexpr ((ABL & 4) != 0) acc[t][p][kk] = (kk == 0 ? 0 : acc[t][p][kk]) + xa[t][kk][0] * b[0];
                        else acc[t][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[t][kk], b, kk == 0 ? i32x16{} : acc[t][p], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int t = 0; t < NC; t++) xa[t][kk] = ld_x(sn, kk, t);
            }
            // U on the f16 MFMA: A = [S & 63, S >> 6] of the lane's column, B = [m, 64 m] of its row
            const uint32_t ma = w1 & 0x3F3F3F3Fu;
            const uint32_t mb = ((w2 >> 4) & 0x0F0F0F0Fu) | ((w1 >> 2) & 0x30303030u);
            const uint32_t mw = h ? mb : ma;  // this lane's k-halves: sub-blocks 4h .. 4h + 3
            half8 mu;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t m = (mw >> (8 * q)) & 0xFF;
                mu[2 * q] = (_Float16) (float) m;
                mu[2 * q + 1] = (_Float16) (float) (64 * m);
            }
            // the activation scales of the tile's columns, redistributed through this wave's LDS row
            if (h == 0) {
#pragma unroll
                for (int t = 0; t < NC; t++) dal[w][32 * t + r] = da[t];
            }
            __builtin_amdgcn_wave_barrier();
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (first) {  // uniform: a group starts at -0 (-0 + t == t), kept a branch (no selects)
                asm volatile("" ::: "memory");
#pragma unroll
                for (int t = 0; t < NC; t++) gsum[t] = f32x16(-0.0f);
            }
#pragma unroll
            for (int t = 0; t < NC; t++) {
                const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(xu[t], mu, f32x16{}, 0, 0, 0);
                xu[t] = ld_u(sn, t);
                da[t] = ld_d(sn, t);
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const float4 d4 = *(const float4 *) &dal[w][32 * t + 8 * g + 4 * h];
                    const float dav[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const int el = 4 * g + e;
                        int T = acc[t][NP - 1][el];
#pragma unroll
                        for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[t][p][el];
                        gsum[t][el] = __builtin_fmaf(dav[e], mmqx_pre(T, Uv[el], dw, dm), gsum[t][el]);
                    }
                }
            }
            if (last) {  // the group's sum -> LDS slot of group sb / gs
                const int grp_i = sb / gs;
#pragma unroll
                for (int t = 0; t < NC; t++)
#pragma unroll
                    for (int el = 0; el < 16; el++) red[(grp_i * NE + 16 * t + el) * 64 + lane] = gsum[t][el];
            }
            __builtin_amdgcn_wave_barrier();  // the LDS row is rewritten by the next superblock
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
        };
        for (int k = 0; k < nsb; k += RING) {
#pragma unroll
            for (int u = 0; u < RING; u++) {
                if (k + u >= nsb) break;
                step(wt[u], wt[(u + RING - 1) % RING], k + u);
            }
        }
    }
    mi_lds_barrier();
    // the group sums folded (canonical order) by the whole workgroup: output o = el 64 + l
    // (el: accumulator element of tile el / 16, l: lane) -- lanes 0..31 store 32 consecutive rows
    const int ngroups = (S + gs - 1) / gs;
#pragma unroll
    for (int i = 0; i < NE / NW; i++) {
        const int o = (int) threadIdx.x + 64 * NW * i;
        const int el = o >> 6, l = o & 63;
        const float y = cfold_groups(ngroups, [&](int v) { return red[(v * NE + el) * 64 + l]; });
        const int e = el & 15, t = el >> 4;
        const int64_t n = n0 + (l & 31);
        const int64_t c = c0 + 32 * t + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
        if (n < N && c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = y;
    }
}

// ---- long prompts, K split over wave pairs: k_mmqt ------------------------------------------------
// A kernel that stages the shared operands once per workgroup in LDS and dequantizes each wave's 32
// weight rows in registers (round 4's k_mmqs: 38.6 us at B = 512, MFMA 26 % busy,
// profiles/r04c_pf_long.txt, r04d_mmqs_*_pmc.txt; removed) dequantizes them once per 32 columns,
// and the dequantization is the larger share of its VALU (~112 of ~300 instructions per 17 MFMAs). Here each wave runs 32 rows x 64
// columns -- two 32 x 32 tiles per dequantized plane, 34 MFMAs per superblock -- and the 8 waves of
// the 128-row x 64-column tile split K in two: waves 0-3 fold the low half of the canonical order
// (superblocks [0, SK), groups 0..3), waves 4-7 the high half ([SK, S), groups 4..7), and the
// halves meet once at the end in LDS (y = lo + hi: the canonical combine, bit-identical to every
// kernel of this file). A stage holds one superblock of each half: per half the activation quants
// [8 steps][64 columns][32] (16 KB, 16-byte halves swapped for columns 16-31 of a 32-column group,
// so the ds_read_b128 lane groups hit 64 distinct banks), the U halves (2 KB), the raw weight
// blocks of the 128 rows (18 KB) and d_a (256 B).
// Staging is LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write pass): a stage is
// 72 one-KB wave-instructions, 9 per wave (each a per-lane source address, the destination
// lane-linear), plus one 256-byte d_a DMA per half. The next stage's DMAs are issued as a step
// starts; the step ends with s_waitcnt vmcnt(0) + s_barrier (two LDS buffers; every global load of
// this kernel is a DMA, so vmcnt(0) waits for exactly the next stage). Q4_K only: a Q5_K stage pair
// (2 x 161 KB) exceeds the LDS.
// Per superblock and wave: 34 MFMAs (2 tiles x (2 planes x 8 steps + 1 U)) for one dequantization.
// (LDS-DMA helpers mi_glds16 / mi_glds4 / mi_lds_addr: mmq_exact_common.h)

// ABL (diagnostic builds only, results invalid): 8 s_memtime stamps of waves 0 and 4 of workgroups 0
// and 97 into dst as uint64 [2][2][80] (0 start, 1 after the prologue, 2 + 4 u + {0 step start, 1
// after the MFMA steps, 2 after the combine, 3 after the DMA wait}); 1 no weight DMAs after the
// prologue, 2 no combine, 4 no DMAs at all after the prologue (profiles/r04l_mmqt_stamps.txt).
// HS (round 6): the two K halves synchronize separately. Each half's 36 pieces are issued by its own
// four waves (9 each, as before) and the stage barrier is a per-half LDS counter (arrive after the
// wave's DMAs and LDS reads have completed, spin until the half's four waves have arrived) instead of
// the workgroup's s_barrier, so waves w and w + 4 -- the two waves of one SIMD, one of each half --
// are no longer held in lock step: one half's combine (VALU) can run under the other half's MFMAs.
// The halves have equal stage counts and meet at a full barrier before the final lo + hi.
// ST (round 6, diagnostic builds: measured 3-9 % slower than the lock-step form at B = 64..512,
// profiles/r06s2h_mmqt_stagger_ab.txt): a stagger of the two waves of a SIMD (MI355X_MICROARCH.md, "Two waves per SIMD",
// item 9): the high half (waves 4-7) defers each stage's combine into the next stage, ahead of that
// stage's MFMAs -- so while waves 0-3 issue their MFMAs their partner wave runs the previous
// combine, and the other way round. The deferred combine's LDS operands (the weight header, the U
// fragments, d_a) are copied to registers before the stage barrier (the next DMAs overwrite that
// buffer); the accumulators stay live until the combine. Same operations in the same order per
// element: bit-identical.
template <int TYPE, int ABL = 0, bool HS = false, bool ST = false>
__global__ __launch_bounds__(512, 1) void k_mmqt(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    using F = XFmt<TYPE>;
    static_assert(!F::Q5, "Q4_K only");
    constexpr int NP = F::NP;
    constexpr int BM = 128, BN = 64;
    constexpr int XB = 8 * BN * 32;           // activation quants of one superblock
    constexpr int UB = BN * 32;               // U halves
    constexpr int WB = BM * F::BS;            // raw weight blocks
    constexpr int DB = BN * 4;                // d_a
    constexpr int HB = XB + UB + WB + DB;     // one K half of a stage: [X | U | W | d_a]
    constexpr int SB = 2 * HB;                // a stage
    constexpr int NPIECE = (XB + UB + WB) / 1024;  // 1-KB DMA pieces per half (36)
    static_assert((XB + UB + WB) % 1024 == 0 && (2 * NPIECE) % 8 == 0, "whole pieces, evenly dealt");
    constexpr int NI = 2 * NPIECE / 8;        // pieces per wave and stage (9)
    constexpr int SINK = 2 * SB;              // d_a DMAs of waves 2-7 land here
    __shared__ __attribute__((aligned(16))) char lds[SINK + DB];
    __shared__ uint32_t hbar[2];              // HS: per-half arrival counters
    constexpr int kDefB = UB + DB + BM * 16;  // ST: the high half's deferred combine operands, per area
    static_assert(!ST || UB + DB == 2304, "deferred-area offsets");
    __shared__ __attribute__((aligned(16))) char ldef[ST ? 2 * kDefB : 16];

    const int tid = (int) threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int rw = w & 3, kh = w >> 2;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);
    const int SK = cfold_split(S);            // superblocks of the low half (>= those of the high)
    const int64_t nrt = (N + BM - 1) / BM;
    const int64_t n0 = (mmx_tile % nrt) * BM, c0 = (mmx_tile / nrt) * BN;
    const int nrows = (int) std::min<int64_t>(BM, N - n0);
    auto col_of = [&](int c) { return (uint32_t) std::min<int64_t>(c0 + c, ncols - 1); };

    // ---- staging: piece q = w + 8 i of a stage (half q / NPIECE, piece t = q % NPIECE of the half):
    // a wave-uniform global base and superblock stride, a per-lane 32-bit offset
    const char * pbase[NI];
    uint32_t pstride[NI], poff[NI], pdst[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int q = w + 8 * i;
        const int hf = HS ? kh : q / NPIECE, t = HS ? (w & 3) + 4 * i : q % NPIECE;
        pdst[i] = (uint32_t) (hf * HB + 1024 * t);
        if (t < 16) {  // activation quants: step kk, 32-column group cg
            const int kk = t >> 1, cg = t & 1, col = 32 * cg + (lane >> 1);
            pbase[i] = (const char *) act.xq + (size_t) kk * ncols * 32;
            pstride[i] = 8 * (uint32_t) ncols * 32;
            poff[i] = col_of(col) * 32 + 16 * ((lane & 1) ^ ((lane >> 5) & 1));
        } else if (t < 18) {  // U halves
            const int col = 32 * (t - 16) + (lane >> 1);
            pbase[i] = (const char *) act.xu;
            pstride[i] = (uint32_t) ncols * 32;
            poff[i] = col_of(col) * 32 + 16 * ((lane & 1) ^ ((lane >> 5) & 1));
        } else {  // raw weight blocks: 1 KB of the [128 rows][BS] image
            const int o = 1024 * (t - 18) + 16 * lane, row = o / F::BS;
            pbase[i] = (const char *) W + (size_t) n0 * nb01;
            pstride[i] = F::BS;
            poff[i] = (uint32_t) (std::min(row, nrows - 1) * nb01 + o % F::BS);
        }
    }
    const uint32_t doff = col_of(lane) * 4;
    // stage u: superblock u of the low half, SK + u of the high half (clamped: a high half shorter
    // than the low one re-reads its last superblock, whose terms are not folded) into buffer u & 1.
    // Piece i < NI; i == NI: d_a (wave 0 the low half's, wave 1 the high half's, the others into the
    // sink).
    auto stage_piece = [&](int u, int i) {
        if constexpr ((ABL & 4) != 0) if (u > 0) return;
        if constexpr ((ABL & 1) != 0) if (u > 0 && i < NI && (w + 8 * i) % NPIECE >= 18) return;
        char * sbuf = lds + (u & 1) * SB;
        if (i < NI) {
            const int hf = HS ? kh : (w + 8 * i) / NPIECE;
            const int sb = std::min(hf ? SK + u : u, S - 1);
            const char * src = pbase[i] + (size_t) sb * pstride[i] + poff[i];
            mi_glds16(src, mi_lds_addr(sbuf + pdst[i]));
        } else if constexpr (HS) {  // wave 0 of each half its d_a, the others into the sink
            const int sb = std::min(kh ? SK + u : u, S - 1);
            const char * src = (const char *) act.xd + (size_t) sb * ncols * 4 + doff;
            char * dd = (w & 3) ? lds + SINK : sbuf + kh * HB + XB + UB + WB;
            mi_glds4(src, mi_lds_addr(dd));
        } else {
            const int sb = std::min(w == 1 ? SK + u : u, S - 1);
            const char * src = (const char *) act.xd + (size_t) sb * ncols * 4 + doff;
            char * dd = w >= 2 ? lds + SINK : sbuf + w * HB + XB + UB + WB;
            mi_glds4(src, mi_lds_addr(dd));
        }
    };
    auto stage_dma = [&](int u) {
#pragma unroll
        for (int i = 0; i <= NI; i++) stage_piece(u, i);
    };
    auto stamp = [&](int slot) {
        if constexpr ((ABL & 8) != 0) {
            const int wsel = blockIdx.x == 0 ? 0 : blockIdx.x == 97 ? 1 : -1;
            if (wsel >= 0 && (w & 3) == 0 && lane == 0 && slot < 80)
                ((uint64_t *) dst)[(wsel * 2 + (w >> 2)) * 80 + slot] = __builtin_amdgcn_s_memtime();
        }
    };
    int stamp_slot = 0;
    auto stage_wait = [&] {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(stamp_slot);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    // HS: the half's barrier for the stage-u wait (u >= 1: the 4 u-th arrival of the half's waves)
    auto half_wait = [&](int u) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        stamp(stamp_slot);
        if (lane == 0) __hip_atomic_fetch_add(&hbar[kh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t target = 4u * (uint32_t) u;
        // (bounded: every wave arrives once per stage, so the bound is never reached; it only keeps
        // a fault from hanging the device)
        for (int spin = 0; spin < (1 << 24) && __hip_atomic_load(&hbar[kh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target; spin++)
            __builtin_amdgcn_s_sleep(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    if constexpr (HS) {
        if (tid < 2) hbar[tid] = 0;  // (ordered before any arrival by the prologue's full barrier)
    }

    // ---- compute: rows n0 + 32 rw + r of half kh; tiles ct = columns 32 ct ..
    const uint32_t xoff0 = (uint32_t) (r * 32 + 16 * (h ^ ((r >> 4) & 1)));  // tile 0; tile 1 at + 1024
    constexpr uint32_t kQs = 16;
    const uint32_t woff = (uint32_t) (kh * HB + XB + UB + (32 * rw + r) * F::BS);
    const int sb_end = kh ? S : SK;
    f32x16 y[2] = {f32x16(-0.0f), f32x16(-0.0f)}, gsum[2] = {};
    i32x16 acc[2][NP];

    // superblock MFMAs from stage buffer buf into acc; `hook(kk)` after step kk's MFMAs
    auto mfma = [&](int buf, auto && hook) {
        const char * base = lds + buf * SB;
        const char * hb = base + kh * HB;
        const char * wr = base + woff;
        const uint4 hdr = *(const uint4 *) wr;
        uint4 q4[4];
#pragma unroll
        for (int p = 0; p < 4; p++) q4[p] = *(const uint4 *) (wr + kQs + 32 * p + 16 * h);
        const uint32_t w0 = hdr.y, w2 = hdr.w;
        const uint32_t sca = w0 & 0x3F3F3F3Fu;
        const uint32_t scb = (w2 & 0x0F0F0F0Fu) | ((w0 >> 2) & 0x30303030u);
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const i32x4 xa0 = *(const i32x4 *) (hb + kk * (BN * 32) + xoff0);
            const i32x4 xa1 = *(const i32x4 *) (hb + kk * (BN * 32) + 1024 + xoff0);
            if ((kk & 1) == 0) {
                const uint4 q = q4[kk >> 1];
                const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    lo[e] = qv[e] & 0x0F0F0F0Fu;
                    hi[e] = (qv[e] >> 4) & 0x0F0F0F0Fu;
                }
            }
            const uint32_t scw = kk < 4 ? sca : scb;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const uint32_t f = __builtin_amdgcn_ubfe(scw, 8 * (kk & 3) + 3 * p, 3);
                const uint32_t * v = (kk & 1) ? hi : lo;
                const i32x4 b = {(int) mulb(v[0], f), (int) mulb(v[1], f), (int) mulb(v[2], f), (int) mulb(v[3], f)};
                acc[0][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa0, b, kk == 0 ? i32x16{} : acc[0][p], 0, 0, 0);
                acc[1][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa1, b, kk == 0 ? i32x16{} : acc[1][p], 0, 0, 0);
            }
            hook(kk);
        }
    };
    // the combine of superblock sb from acc: U on the f16 MFMA (A = [S & 63, S >> 6] of the lane's
    // column from xup, B = [m, 64 m] of its row from the header at hdrp), then mmqx_pre per element
    // (d_a from dal), folded into this half's sum
    auto combine = [&](const char * hdrp, const char * xup, const float * dal, int sb) {
        if constexpr ((ABL & 2) != 0) {  // timing ablation: no combine (keep the accumulators alive)
            if (acc[0][0][0] == 0x7fffffff && acc[1][1][5] == 0x7fffffff) y[0][0] += 1.0f;
            return;
        }
        const uint4 hdr = *(const uint4 *) hdrp;
        const float dw = mi_h2f((uint16_t) (hdr.x & 0xFFFF)), dm = mi_h2f((uint16_t) (hdr.x >> 16));
        const uint32_t ma = hdr.z & 0x3F3F3F3Fu;
        const uint32_t mb = ((hdr.w >> 4) & 0x0F0F0F0Fu) | ((hdr.z >> 2) & 0x30303030u);
        const uint32_t mw = h ? mb : ma;
        half8 mu;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t m = (mw >> (8 * q)) & 0xFF;
            mu[2 * q] = (_Float16) (float) m;
            mu[2 * q + 1] = (_Float16) (float) (64 * m);
        }
        const bool fold = sb < sb_end;  // wave-uniform
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const half8 xu = *(const half8 *) (xup + 1024 * ct);
            const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(xu, mu, f32x16{}, 0, 0, 0);
            f32x16 tv, dv;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float2 d2 = *(const float2 *) &dal[32 * ct + 8 * (j >> 1) + 4 * h + 2 * (j & 1)];
                dv[2 * j] = d2.x;
                dv[2 * j + 1] = d2.y;
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int el = 2 * j + e;
                    const int T = (acc[ct][1][el] << F::SHIFT) + acc[ct][0][el];
                    tv[el] = mmqx_pre(T, Uv[el], dw, dm);
                }
            }
            if (fold) {
                // one half's fold: groups end at multiples of gs, y = y + g (the high half's
                // first group lands exactly on y = -0)
                const int pos = sb % gs;
                if (pos == 0) {  // bitwise fma(dv, tv, -0)
                    asm volatile("" ::: "memory");
                    gsum[ct] = dv * tv;
                } else {
                    gsum[ct] = fma_vec(dv, tv, gsum[ct]);
                }
                if (pos == gs - 1 || sb == S - 1) {
                    asm volatile("" ::: "memory");
                    y[ct] = y[ct] + gsum[ct];
                }
            }
        }
    };
    auto combine_stage = [&](int buf, int sb) {  // operands from the stage buffer
        const char * hb = lds + buf * SB + kh * HB;
        combine(lds + buf * SB + woff, hb + XB + xoff0, (const float *) (hb + XB + UB + WB), sb);
    };
    const int sb0 = kh ? SK : 0;
    stamp(0);
    stage_dma(0);
    stamp_slot = 1;
    stage_wait();
    if constexpr (ST) {
        // the deferred combine's operands of stage u, copied by waves 4-7 into area u & 1 behind their
        // MFMAs: [U halves 2 KB | d_a 256 B | the 128 rows' headers 2 KB] (the stage buffer itself is
        // refilled by the next stage's DMAs)
        auto def_area = [&](int u) { return ldef + (u & 1) * kDefB; };
        for (int u = 0; u < SK; u++) {
            auto dma_hook = [&](int kk) {
                if (kk < 7) {
                    stage_piece(u + 1, kk);
                } else {
#pragma unroll
                    for (int i = 7; i <= NI; i++) stage_piece(u + 1, i);
                }
            };
            if (kh && u > 0) {  // the previous stage's combine, under waves 0-3's MFMAs
                const char * d = def_area(u - 1);
                combine(d + 2304 + (32 * rw + r) * 16, d + xoff0, (const float *) (d + 2048), sb0 + u - 1);
            }
            mfma(u & 1, dma_hook);
            if (kh) {
                const char * hb = lds + (u & 1) * SB + HB;  // (the high half's stage image)
                char * d = def_area(u);
                if (lane < 32) {
                    *(uint4 *) (d + 2304 + (32 * rw + lane) * 16) = *(const uint4 *) (hb + XB + UB + (32 * rw + lane) * F::BS);
                    if (lane < 4) *(uint4 *) (d + 2048 + 64 * rw + 16 * lane) = *(const uint4 *) (hb + XB + UB + WB + 64 * rw + 16 * lane);
                } else {
                    *(uint4 *) (d + 512 * rw + 16 * (lane - 32)) = *(const uint4 *) (hb + XB + 512 * rw + 16 * (lane - 32));
                }
            } else {
                combine_stage(u & 1, sb0 + u);
            }
            stage_wait();
        }
        if (kh && SK > 0) {
            const char * d = def_area(SK - 1);
            combine(d + 2304 + (32 * rw + r) * 16, d + xoff0, (const float *) (d + 2048), sb0 + SK - 1);
        }
    } else
    for (int u = 0; u < SK; u++) {
        stamp(2 + 4 * u);
        stamp_slot = 5 + 4 * u;
        // the next stage's DMAs (past the end: clamped re-reads into the idle buffer), one piece
        // behind each 32-deep step's MFMAs, the rest after the last
        auto dma_hook = [&](int kk) {
            if (kk < 7) {
                stage_piece(u + 1, kk);
            } else {
#pragma unroll
                for (int i = 7; i <= NI; i++) stage_piece(u + 1, i);
            }
        };
        mfma(u & 1, dma_hook);
        stamp(3 + 4 * u);
        combine_stage(u & 1, sb0 + u);
        stamp(4 + 4 * u);
        if constexpr (HS) half_wait(u + 1);
        else stage_wait();
    }
    if constexpr ((ABL & 8) != 0) {  // dst holds the stamps; keep the results alive
        float t = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; i++) t += y[0][i] + y[1][i];
        if (t == 1.2345e-30f) dst[8192 + threadIdx.x] = t;
        return;
    }

    // the halves meet: waves 4-7 leave their sums in LDS (the stage buffers are idle: every DMA
    // has landed and every wave has passed the last barrier), waves 0-3 add and store
    f32x16 * ex = (f32x16 *) lds;
    if constexpr (HS) mi_lds_barrier();  // the halves drift: both done with the stage buffers
    if (kh) {
        ex[(rw * 2 + 0) * 64 + lane] = y[0];
        ex[(rw * 2 + 1) * 64 + lane] = y[1];
    }
    mi_lds_barrier();
    if (kh) return;
    const int64_t n = n0 + 32 * rw + r;
    if (n >= N) return;
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const f32x16 yv = y[ct] + ex[(rw * 2 + ct) * 64 + lane];  // cfold_end: lo + hi
        // element el: prompt column c0 + 32 ct + (el & 3) + 8 (el >> 2) + 4 h
#pragma unroll
        for (int el = 0; el < 16; el++) {
            const int64_t c = c0 + 32 * ct + (el & 3) + 8 * (el >> 2) + 4 * h;
            if (c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = yv[el];
        }
    }
}

// ---- long prompts, one wave per SIMD, software-pipelined: k_mmqv (round 6) --------------------------
// k_mmqt's phases run in lock step per stage: every wave issues its MFMAs, then its combine (VALU),
// and the two waves of a SIMD do so together (stamps: MFMA steps ~2500-3200 cycles, combine ~1800,
// barrier ~1200 per stage, profiles/r04l_mmqt_stamps.txt; synchronizing the halves separately did not
// separate them, profiles/r06d_mmqt_stamps.txt). Here one wave per SIMD (4 waves, 128 rows x 64
// columns, each wave 32 rows x 64 columns over the WHOLE K) overlaps the two inside itself: the
// combine of superblock s - 1 (T = (P1 << 3) + P0, t = fma(-dmin_w, U, d_w T): 4 VALU per element, no
// branches) is issued between the MFMAs of superblock s, so the MFMA pipe hides the VALU latency
// chains; only the group fold (cfold_vec: g = fma(d_a, t, g), group ends) runs on its own. Stage =
// one superblock: activation quants [8][64][32] (swizzled halves), U halves, the 128 rows' raw
// blocks, d_a (k_mmqt's half-stage image, 36.4 KB) by LDS-DMA, 4 buffers, issued two stages ahead (9
// one-KB pieces + one d_a DMA per wave and stage: s_waitcnt vmcnt(10) leaves the next stage in
// flight). Same operands, same canonical combine: bit-identical to every kernel of the family.
template <int TYPE>
__global__ __launch_bounds__(256, 1) void k_mmqv(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    using F = XFmt<TYPE>;
    static_assert(!F::Q5, "Q4_K only");
    constexpr int NP = F::NP;
    constexpr int BM = 128, BN = 64;
    constexpr int XB = 8 * BN * 32;           // activation quants of one superblock
    constexpr int UB = BN * 32;               // U halves
    constexpr int WB = BM * F::BS;            // raw weight blocks
    constexpr int DB = BN * 4;                // d_a
    constexpr int HB = XB + UB + WB + DB;     // a stage: [X | U | W | d_a]
    constexpr int NBUF = 4;
    constexpr int NPIECE = (XB + UB + WB) / 1024;  // 36
    constexpr int NI = NPIECE / 4;            // 9 per wave
    static_assert(NPIECE % 4 == 0, "pieces evenly dealt");
    constexpr int SINK = NBUF * HB;
    __shared__ __attribute__((aligned(16))) char lds[SINK + DB];

    const int tid = (int) threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);
    const int64_t nrt = (N + BM - 1) / BM;
    const int64_t n0 = (mmx_tile % nrt) * BM, c0 = (mmx_tile / nrt) * BN;
    const int nrows = (int) std::min<int64_t>(BM, N - n0);
    auto col_of = [&](int c) { return (uint32_t) std::min<int64_t>(c0 + c, ncols - 1); };

    const char * pbase[NI];
    uint32_t pstride[NI], poff[NI], pdst[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int t = w + 4 * i;
        pdst[i] = (uint32_t) (1024 * t);
        if (t < 16) {  // activation quants: step kk, 32-column group cg
            const int kk = t >> 1, cg = t & 1, col = 32 * cg + (lane >> 1);
            pbase[i] = (const char *) act.xq + (size_t) kk * ncols * 32;
            pstride[i] = 8 * (uint32_t) ncols * 32;
            poff[i] = col_of(col) * 32 + 16 * ((lane & 1) ^ ((lane >> 5) & 1));
        } else if (t < 18) {  // U halves
            const int col = 32 * (t - 16) + (lane >> 1);
            pbase[i] = (const char *) act.xu;
            pstride[i] = (uint32_t) ncols * 32;
            poff[i] = col_of(col) * 32 + 16 * ((lane & 1) ^ ((lane >> 5) & 1));
        } else {  // raw weight blocks: 1 KB of the [128 rows][BS] image
            const int o = 1024 * (t - 18) + 16 * lane, row = o / F::BS;
            pbase[i] = (const char *) W + (size_t) n0 * nb01;
            pstride[i] = F::BS;
            poff[i] = (uint32_t) (std::min(row, nrows - 1) * nb01 + o % F::BS);
        }
    }
    const uint32_t doff = col_of(lane) * 4;
    // stage u (clamped: past the end re-reads the last superblock into an idle buffer) into buffer u % 4
    auto stage_piece = [&](int u, int i) {
        char * sbuf = lds + (u % NBUF) * HB;
        const int sb = std::min(u, S - 1);
        if (i < NI) {
            mi_glds16(pbase[i] + (size_t) sb * pstride[i] + poff[i], mi_lds_addr(sbuf + pdst[i]));
        } else {
            const char * src = (const char *) act.xd + (size_t) sb * ncols * 4 + doff;
            mi_glds4(src, mi_lds_addr(w ? lds + SINK : sbuf + XB + UB + WB));
        }
    };

    const uint32_t xoff0 = (uint32_t) (r * 32 + 16 * (h ^ ((r >> 4) & 1)));  // tile 0; tile 1 at + 1024
    const uint32_t woff = (uint32_t) (XB + UB + (32 * w + r) * F::BS);
    f32x16 g[2] = {}, y[2] = {f32x16(-0.0f), f32x16(-0.0f)}, lo[2] = {f32x16(-0.0f), f32x16(-0.0f)};
    i32x16 accA[2][NP], accB[2][NP];

    // U of superblock sb (its stage buffer) on the f16 MFMA (A = [S & 63, S >> 6] of the lane's
    // column, B = [m, 64 m] of its row); returns d_w, dmin_w of the row
    auto u_of = [&](int sb, f32x16 (&Uo)[2]) {
        const char * base = lds + (sb % NBUF) * HB;
        const uint4 hdr = *(const uint4 *) (base + woff);
        const uint32_t ma = hdr.z & 0x3F3F3F3Fu;
        const uint32_t mb = ((hdr.w >> 4) & 0x0F0F0F0Fu) | ((hdr.z >> 2) & 0x30303030u);
        const uint32_t mw = h ? mb : ma;
        half8 mu;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t m = (mw >> (8 * q)) & 0xFF;
            mu[2 * q] = (_Float16) (float) m;
            mu[2 * q + 1] = (_Float16) (float) (64 * m);
        }
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const half8 xu = *(const half8 *) (base + XB + xoff0 + 1024 * ct);
            Uo[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xu, mu, f32x16{}, 0, 0, 0);
        }
        return std::make_pair(mi_h2f((uint16_t) (hdr.x & 0xFFFF)), mi_h2f((uint16_t) (hdr.x >> 16)));
    };

    // superblock u: its MFMAs into acc; the previous superblock's t values (accp; when `pre`)
    // computed between the MFMA steps into tv; the stage two ahead's DMAs behind the steps
    auto body = [&](auto pre_c, int u, i32x16 (&acc)[2][NP], const i32x16 (&accp)[2][NP], f32x16 (&tv)[2]) {
        constexpr bool pre = decltype(pre_c)::value;
        const char * base = lds + (u % NBUF) * HB;
        const char * wr = base + woff;
        f32x16 Up[2];
        float dwp = 0.0f, dmp = 0.0f;
        if constexpr (pre) {
            const auto dd = u_of(u - 1, Up);
            dwp = dd.first;
            dmp = dd.second;
        }
        const uint4 hdr = *(const uint4 *) wr;
        uint4 q4[4];
#pragma unroll
        for (int p = 0; p < 4; p++) q4[p] = *(const uint4 *) (wr + 16 + 32 * p + 16 * h);
        const uint32_t w0 = hdr.y, w2 = hdr.w;
        const uint32_t sca = w0 & 0x3F3F3F3Fu;
        const uint32_t scb = (w2 & 0x0F0F0F0Fu) | ((w0 >> 2) & 0x30303030u);
        uint32_t lq[4], hq[4];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const i32x4 xa0 = *(const i32x4 *) (base + kk * (BN * 32) + xoff0);
            const i32x4 xa1 = *(const i32x4 *) (base + kk * (BN * 32) + 1024 + xoff0);
            if ((kk & 1) == 0) {
                const uint4 q = q4[kk >> 1];
                const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    lq[e] = qv[e] & 0x0F0F0F0Fu;
                    hq[e] = (qv[e] >> 4) & 0x0F0F0F0Fu;
                }
            }
            const uint32_t scw = kk < 4 ? sca : scb;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const uint32_t f = __builtin_amdgcn_ubfe(scw, 8 * (kk & 3) + 3 * p, 3);
                const uint32_t * v = (kk & 1) ? hq : lq;
                const i32x4 b = {(int) mulb(v[0], f), (int) mulb(v[1], f), (int) mulb(v[2], f), (int) mulb(v[3], f)};
                acc[0][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa0, b, kk == 0 ? i32x16{} : acc[0][p], 0, 0, 0);
                acc[1][p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa1, b, kk == 0 ? i32x16{} : acc[1][p], 0, 0, 0);
            }
            // the previous superblock's values of elements 2 kk, 2 kk + 1 (both tiles)
            if constexpr (pre) {
#pragma unroll
                for (int ct = 0; ct < 2; ct++) {
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const int el = 2 * kk + e;
                        const int T = (accp[ct][1][el] << F::SHIFT) + accp[ct][0][el];
                        tv[ct][el] = mmqx_pre(T, Up[ct][el], dwp, dmp);
                    }
                }
            }
            // the stage two ahead: one piece behind each step (steps 0..NI-1), the d_a DMA after the last
            if (kk < NI) stage_piece(u + 2, kk);
        }
#pragma unroll
        for (int i = 8; i <= NI; i++) stage_piece(u + 2, i);
    };
    // the last superblock's values (after its MFMAs, no next superblock to hide them under)
    auto last_pre = [&](int sb, const i32x16 (&accp)[2][NP], f32x16 (&tv)[2]) {
        f32x16 Up[2];
        const auto dd = u_of(sb, Up);
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int el = 0; el < 16; el++) {
                const int T = (accp[ct][1][el] << F::SHIFT) + accp[ct][0][el];
                tv[ct][el] = mmqx_pre(T, Up[ct][el], dd.first, dd.second);
            }
    };
    // the fold of superblock sb's values tv (d_a from its stage buffer)
    auto fold = [&](int sb, const f32x16 (&tv)[2]) {
        const float * dal = (const float *) (lds + (sb % NBUF) * HB + XB + UB + WB);
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            f32x16 dv;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float2 d2 = *(const float2 *) &dal[32 * ct + 8 * (j >> 1) + 4 * h + 2 * (j & 1)];
                dv[2 * j] = d2.x;
                dv[2 * j + 1] = d2.y;
            }
            cfold_vec(g[ct], y[ct], lo[ct], tv[ct], dv, sb, gs, S);
        }
    };
    auto stage_wait = [&] {
        asm volatile("s_waitcnt vmcnt(10)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };

    // prologue: stages 0 and 1 in flight
#pragma unroll
    for (int i = 0; i <= NI; i++) stage_piece(0, i);
#pragma unroll
    for (int i = 0; i <= NI; i++) stage_piece(1, i);
    f32x16 tv[2];
    using no_pre = std::integral_constant<bool, false>;
    using with_pre = std::integral_constant<bool, true>;
    stage_wait();
    body(no_pre{}, 0, accA, accB, tv);
    if (S == 1) {
        last_pre(0, accA, tv);
        fold(0, tv);
    }
    for (int u = 1; u < S; u += 2) {
        stage_wait();
        body(with_pre{}, u, accB, accA, tv);
        fold(u - 1, tv);
        if (u + 1 >= S) {  // the last superblock from accB
            last_pre(u, accB, tv);
            fold(u, tv);
            break;
        }
        stage_wait();
        body(with_pre{}, u + 1, accA, accB, tv);
        fold(u, tv);
        if (u + 2 >= S) {  // the last superblock from accA
            last_pre(u + 1, accA, tv);
            fold(u + 1, tv);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the clamped DMAs past the end have landed)

    const int64_t n = n0 + 32 * w + r;
    if (n >= N) return;
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const f32x16 yv = cfold_end_vec(lo[ct], y[ct]);
        // element el: prompt column c0 + 32 ct + (el & 3) + 8 (el >> 2) + 4 h
#pragma unroll
        for (int el = 0; el < 16; el++) {
            const int64_t c = c0 + 32 * ct + (el & 3) + 8 * (el >> 2) + 4 * h;
            if (c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = yv[el];
        }
    }
}

// ---- Q4_0 / Q8_0 prefill: the reference's exact int32 block sums on the int8 matrix cores --------
// The reference dots (vec_dot_q4_0_q8_0, src/ggml-quants.c:3469-3874, AVX2 :3600-3623;
// vec_dot_q8_0_q8_0, :4819, AVX2 :4925+) compute, per 32-block b, the exact int32
// T_b = sum (q_w - 8 | q_w) q_a and combine in f32: acc = fma(fp16(d_w) fp16(d_a), (float) T_b, acc).
// Here T_b is ONE v_mfma_i32_32x32x32_i8 (the instruction's K is exactly one block) on the weight
// quants -- Q4_0: the nibble minus 8, by the byte-wise bias trick (q + 0x78) ^ 0x80 (no carry
// between bytes for q <= 15); Q8_0: the bytes -- and the q8_0 activation quants; per block
// f = d_w d_a and g = fma(f, T, g). Canonical order of this family: blocks in kCfoldGroups groups of
// whole 8-block units (gs = ceil(K / 256 / kCfoldGroups) units each), fma-chained in block order
// from +0 inside a group, the group sums left-folded. Against the reference only that order differs.
// Workgroup: 4 waves on a tile of 32 weight rows x 32 prompt columns, two per CU; wave w computes
// groups w and w + 4, unit after unit, the next unit's weight bytes and scales requested into a
// second register set before the current unit's blocks are processed (Q4_0: the 144-byte unit of
// the lane's row, nine 16-byte loads, 16-byte aligned at K % 256 == 0; Q8_0: per block the five
// dwords covering the lane's 16 quant bytes and the scale -- blocks are 2-byte aligned). A block's
// operand is extracted with v_alignbyte right before its MFMA. Accumulator element el: prompt
// column c0 + (el & 3) + 8 (el >> 2) + 4 h, weight row n0 + r (as k_mmqp); the activation scales
// reach that layout through a wave-private LDS row per block.
template <bool Q8>
struct Q0Raw {
    // Q4_0: the unit's 144 bytes; Q8_0: per block 5 dwords from byte 34 j + 16 h (4-aligned down)
    uint32_t v[Q8 ? 40 : 36];
    float da[8];  // this lane's column's activation scales of the unit's 8 blocks
};

template <bool Q8, int RING = 2>
__global__ __launch_bounds__(256, 2) void k_mmq0p(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    constexpr int NW = 4;
    constexpr int BS = Q8 ? 34 : 18;
    constexpr int UB = 8 * BS;  // bytes of a row's 8-block unit: 144 / 272
    constexpr int NG = kCfoldGroups / NW;
    __shared__ __attribute__((aligned(16))) float red[kCfoldGroups * 16 * 64];  // [group][el][lane]
    __shared__ __attribute__((aligned(16))) float dal[NW][8][32];                // per-wave da rows
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);  // 8-block units
    const int gs = cfold_gs(S);
    auto gbeg = [&](int i) { return min(S, (w + NW * i) * gs); };
    auto gend = [&](int i) { return min(S, (w + NW * i + 1) * gs); };
    const int nsb = [&] { int n = 0; for (int i = 0; i < NG; i++) n += gend(i) - gbeg(i); return n; }();
    auto sb_at = [&](int k) {
        k = min(k, nsb - 1);
#pragma unroll
        for (int i = 0; i < NG; i++) {
            const int len = gend(i) - gbeg(i);
            if (k < len) return gbeg(i) + k;
            k -= len;
        }
        return S - 1;
    };
    const int64_t nrt = (N + 31) / 32;
    const int64_t n0 = (mmx_tile % nrt) * 32, c0 = (mmx_tile / nrt) * 32;
    const int nrows = (int) std::min<int64_t>(32, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) ((K / 32) * ncols * 4), 0x00020000);
    const uint32_t wv = (uint32_t) (min(r, nrows - 1) * nb01);
    const uint32_t acol = (uint32_t) std::min<int64_t>(c0 + r, ncols - 1);
    const uint32_t xstep = (uint32_t) ncols * 32;

    auto load_unit = [&](Q0Raw<Q8> & o, int u) {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(u * UB);
        if constexpr (Q8) {
            // block j: quants at 34 j + 2 + 16 h .. + 15, scale at 34 j; dwords from 4-aligned 34 j + 16 h - 2 (j odd)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t b0 = (uint32_t) ((BS * j) & ~3);  // 4-aligned start of block j
                const uint32_t q0 = b0 + 16 * h;                 // this half's first covering dword
#pragma unroll
                for (int i = 0; i < 5; i++) o.v[5 * j + i] = __builtin_amdgcn_raw_buffer_load_b32(wres, wv + q0 + 4 * i, so, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 9; i++) {
                const uint4 x = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wv + 16 * i, so, 0));
                o.v[4 * i] = x.x; o.v[4 * i + 1] = x.y; o.v[4 * i + 2] = x.z; o.v[4 * i + 3] = x.w;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t sd = (uint32_t) __builtin_amdgcn_readfirstlane((u * 8 + j) * (int) ncols * 4);
            o.da[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, acol * 4, sd, 0));
        }
    };
    // block j's 16 quant bytes (and its scale) from the unit registers
    auto operand = [&](const Q0Raw<Q8> & o, const int j, i32x4 & b, float & dw) {
        uint32_t t[4];
        if constexpr (Q8) {
            const int base = (BS * j) & 3;    // 0 (j even) or 2 (j odd): block start within its first dword
            const int qo = base + 2;          // quant byte offset within this half's covering dwords
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int ob = qo + 4 * e;
                t[e] = (ob & 3) == 0 ? o.v[5 * j + (ob >> 2)] : __builtin_amdgcn_alignbyte(o.v[5 * j + (ob >> 2) + 1], o.v[5 * j + (ob >> 2)], ob & 3);
            }
            // scale: half 0 holds it at byte `base` of its first dword; half 1 takes it from half 0
            const uint32_t d0w = o.v[5 * j] >> (8 * base);
            const uint32_t dsh = (uint32_t) __shfl_xor((int) d0w, 32, 64);
            dw = mi_h2f((uint16_t) ((h ? dsh : d0w) & 0xFFFF));
        } else {
            const int oq = BS * j + 2;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int ob = oq + 4 * e;
                const uint32_t x = (ob & 3) == 0 ? o.v[ob >> 2] : __builtin_amdgcn_alignbyte(o.v[(ob >> 2) + 1], o.v[ob >> 2], ob & 3);
                t[e] = (((x >> (4 * h)) & 0x0F0F0F0Fu) + 0x78787878u) ^ 0x80808080u;
            }
            const int od = BS * j;
            const uint32_t x = (od & 3) == 0 ? o.v[od >> 2] : __builtin_amdgcn_alignbyte(o.v[(od >> 2) + 1], o.v[od >> 2], od & 3);
            dw = mi_h2f((uint16_t) (x & 0xFFFF));
        }
        b = i32x4{(int) t[0], (int) t[1], (int) t[2], (int) t[3]};
    };
    auto ld_x = [&](int u, int j) -> i32x4 {
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((u * 8 + j) * (int) xstep);
        return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, acol * 32 + 16 * h, so, 0));
    };

    f32x16 gsum = {};
    if (nsb > 0) {
        Q0Raw<Q8> ru[RING];  // unit k + RING - 1's weights are requested when unit k starts (k_mmqp)
        i32x4 xa[8];
        const int uf = sb_at(0);
#pragma unroll
        for (int v = 0; v < RING - 1; v++) load_unit(ru[v], sb_at(v));
#pragma unroll
        for (int j = 0; j < 8; j++) xa[j] = ld_x(uf, j);
        auto unit = [&](const Q0Raw<Q8> & cur, Q0Raw<Q8> & nxt, const int k) {
            const int u = sb_at(k);
            const int un = sb_at(k + 1);  // clamped: a past-the-end prefetch re-reads the last one
            const bool last = u % gs == gs - 1 || u == S - 1;
            if (u % gs == 0) gsum = f32x16{};
            load_unit(nxt, sb_at(k + RING - 1));
            if (h == 0) {
#pragma unroll
                for (int j = 0; j < 8; j++) dal[w][j][r] = cur.da[j];
            }
            __builtin_amdgcn_wave_barrier();
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                i32x4 bq;
                float dw;
                operand(cur, j, bq, dw);
                const i32x16 T = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[j], bq, i32x16{}, 0, 0, 0);
                xa[j] = ld_x(un, j);
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const float4 d4 = *(const float4 *) &dal[w][j][8 * g + 4 * h];
                    const float dav[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const int el = 4 * g + e;
                        gsum[el] = __builtin_fmaf(dw * dav[e], (float) T[el], gsum[el]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // one block's accumulator at a time
            }
            __builtin_amdgcn_wave_barrier();  // the LDS rows are rewritten by the next unit
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (last) {
                const int gi = u / gs;
#pragma unroll
                for (int el = 0; el < 16; el++) red[(gi * 16 + el) * 64 + lane] = gsum[el];
            }
        };
        for (int k = 0; k < nsb; k += RING) {
#pragma unroll
            for (int v = 0; v < RING; v++) {
                if (k + v >= nsb) break;
                unit(ru[v], ru[(v + RING - 1) % RING], k + v);
            }
        }
    }
    mi_lds_barrier();
    const int ngroups = (S + gs - 1) / gs;
#pragma unroll
    for (int i = 0; i < 16 / NW; i++) {
        const int o = (int) threadIdx.x + 64 * NW * i;
        const int el = o >> 6, l = o & 63;
        float y = red[el * 64 + l];
        for (int v = 1; v < ngroups; v++) y = y + red[(v * 16 + el) * 64 + l];
        const int64_t n = n0 + (l & 31);
        const int64_t c = c0 + (el & 3) + 8 * (el >> 2) + 4 * (l >> 5);
        if (n < N && c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = y;
    }
}

// ---- Q4_0 / Q8_0, long prompts: weights staged once per workgroup ---------------------------------
// k_mmqx's structure for the one-MFMA-per-block family: a workgroup of NWV waves computes 64 weight
// rows x 16 NWV prompt columns, wave (rw, cw) one 32 x 32 tile. A stage is one 8-block unit (256
// K): its threads turn the next unit's 64 rows into MFMA operands in the other LDS buffer (thread =
// (row, block): the block's dwords, 8 lanes per row contiguous -- coalesced -- re-aligned with
// v_alignbyte; Q4_0 nibbles biased to q - 8), plus the rows' d_w; the raw weights were requested
// LEAD stages earlier. Per block: one v_mfma_i32_32x32x32_i8 whose accumulator input is the
// constant 0x4B400000, so the int32 result's bits are the float 1.5 * 2^23 + T (|T| < 2^22): one
// subtraction gives (float) T exactly; then f = d_w d_a (exact: two fp16 values) and
// g = fma(f, T, g). The MFMA of block j + 1 is issued before block j's combine (two accumulators).
// Combine order: the family's canonical one (k_mmq0p): bit-identical to it.
// NR = 2: each wave computes both 32-row halves of its 32 columns (64 x 32: every activation
// fragment feeds two MFMAs, half the activation traffic per MFMA); the workgroup's NWV waves then
// cover 32 NWV columns.
template <bool Q8, int NWV, int LEAD, int NR = 1>
__global__ __launch_bounds__(64 * NWV, NR == 2 ? 2 : 1) void k_mmq0x(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    constexpr int BS = Q8 ? 34 : 18;
    constexpr int UB = 8 * BS;                // bytes of a row's unit
    constexpr int ND = Q8 ? 9 : 5;            // dwords covering a block (2-byte aligned)
    constexpr int XR = 256 + 16;              // LDS row stride of the operand plane
    constexpr int kPlane = XBM * XR;
    constexpr int DWS = XBM + 4;              // d_w row stride: a row's 8 blocks on 8 distinct banks
    constexpr int kBuf = kPlane + 8 * DWS * 4;  // + d_w [block][row]
    constexpr int XBN_ = NR == 2 ? 32 * NWV : 16 * NWV;
    constexpr int ROWP = 8 / NWV;             // staging passes (rows per thread)
    constexpr int RSTEP = 8 * NWV;
    __shared__ __attribute__((aligned(16))) char lds[2 * kBuf];

    const int tid = (int) threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int rw = NR == 2 ? 0 : (wave & 1), cw = NR == 2 ? wave : (wave >> 1);
    const int64_t ncols = act.ncols;
    const int64_t nrt = (N + XBM - 1) / XBM;
    const int64_t n0 = (mmx_tile % nrt) * XBM, b0 = (mmx_tile / nrt) * XBN_;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);

    // staging role: row ar (+ RSTEP per pass), block j of the unit
    const int ar = tid >> 3, j = tid & 7;
    const int nrows = (int) std::min<int64_t>(XBM, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    const uint32_t boff = (uint32_t) (BS * j);
    const uint32_t bal = boff & 3;  // 0 or 2: the block's offset in its first dword
    uint32_t wrow[ROWP];
#pragma unroll
    for (int pr = 0; pr < ROWP; pr++) wrow[pr] = (uint32_t) (std::min(ar + pr * RSTEP, nrows - 1) * nb01) + (boff & ~3u);

    // activation fragments: column b0 + 32 cw + (lane & 31), 16 bytes at 16 (lane >> 5)
    const int r = lane & 31, h = lane >> 5;
    const uint32_t bcol = (uint32_t) std::min<int64_t>(b0 + 32 * cw + r, ncols - 1);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) ((K / 32) * ncols * 4), 0x00020000);
    const uint32_t xcol = bcol * 32 + 16 * h;
    const uint32_t xstep = (uint32_t) ncols * 32;

    struct Raw {
        uint32_t w[ND];
    };
    auto load_raw = [&](Raw & raw, int u, int pr) {
        u = u < S ? u : S - 1;
        const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane(u * UB);
#pragma unroll
        for (int i = 0; i < ND; i++) raw.w[i] = __builtin_amdgcn_raw_buffer_load_b32(wres, wrow[pr] + 4 * i, so, 0);
    };
    struct Xs {
        i32x4 q[8];
        float da[8];
    };
    auto load_x = [&](Xs & xs, int u) {
        u = u < S ? u : S - 1;
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((u * 8 + kk) * (int) xstep);
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol, so, 0));
        }
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((u * 8 + kk) * (int) ncols * 4);
            xs.da[kk] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, bcol * 4, so, 0));
        }
    };
    // one thread's block into LDS buffer `buf`: 32 operand bytes at [row][32 j] and d_w
    auto store_block = [&](int buf, const Raw & raw, int pr) {
        const int row = ar + pr * RSTEP;
        char * pl = lds + buf * kBuf + row * XR + 32 * j;
        float * dwv = (float *) (lds + buf * kBuf + kPlane);
        const uint32_t dbits = (bal ? raw.w[0] >> 16 : raw.w[0]) & 0xFFFF;
        dwv[j * DWS + row] = mi_h2f((uint16_t) dbits);
        // quants start at byte bal + 2 of w[0]: 2 -> alignbyte, 4 -> whole dwords from w[1]
        if constexpr (Q8) {
            uint32_t t[8];
#pragma unroll
            for (int i = 0; i < 8; i++) t[i] = bal ? raw.w[i + 1] : __builtin_amdgcn_alignbyte(raw.w[i + 1], raw.w[i], 2);
            *(uint4 *) pl = make_uint4(t[0], t[1], t[2], t[3]);
            *(uint4 *) (pl + 16) = make_uint4(t[4], t[5], t[6], t[7]);
        } else {
            uint32_t t[4];
#pragma unroll
            for (int i = 0; i < 4; i++) t[i] = bal ? raw.w[i + 1] : __builtin_amdgcn_alignbyte(raw.w[i + 1], raw.w[i], 2);
            uint32_t lo[4], hi[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                lo[i] = ((t[i] & 0x0F0F0F0Fu) + 0x78787878u) ^ 0x80808080u;          // elements 4i..: q - 8
                hi[i] = (((t[i] >> 4) & 0x0F0F0F0Fu) + 0x78787878u) ^ 0x80808080u;   // elements 16 + 4i..
            }
            *(uint4 *) pl = make_uint4(lo[0], lo[1], lo[2], lo[3]);
            *(uint4 *) (pl + 16) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
        }
    };

    f32x16 y[NR], gsum[NR];
#pragma unroll
    for (int ri = 0; ri < NR; ri++) {
        y[ri] = f32x16(-0.0f);
        gsum[ri] = f32x16{};
    }
    Raw raw[LEAD][ROWP];
    Xs xs;
#pragma unroll
    for (int pr = 0; pr < ROWP; pr++) {
        Raw r0;
        load_raw(r0, 0, pr);
        store_block(0, r0, pr);
    }
    load_x(xs, 0);
#pragma unroll
    for (int u = 0; u < LEAD; u++)
#pragma unroll
        for (int pr = 0; pr < ROWP; pr++) load_raw(raw[u][pr], 1 + u, pr);
    mi_lds_barrier();

    const i32x16 kBias = {0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000,
                          0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000};
    auto stage = [&](const int u, Raw (&rslot)[ROWP]) {
        const int cur = u & 1;
        const char * base = lds + cur * kBuf;
        const char * arow_p = base + (32 * rw + r) * XR + 16 * h;
        const float * dwv = (const float *) (base + kPlane);
        const int un = u + 1 < S ? u + 1 : S - 1;
        if (u % gs == 0) {  // uniform; kept a branch (no per-element selects)
            asm volatile("" ::: "memory");
#pragma unroll
            for (int ri = 0; ri < NR; ri++) gsum[ri] = f32x16{};
        }
        float da[8];
#pragma unroll
        for (int kk = 0; kk < 8; kk++) da[kk] = xs.da[kk];
        // NR = 1: two accumulators, block kk + 1's MFMA issued before block kk's combine; NR = 2:
        // one per row half, in the order M0(kk) C1(kk-1) M1(kk) C0(kk)
        i32x16 acc[NR == 1 ? 2 : NR];
        auto combine = [&](int kk, int ri, const i32x16 & T) {
            const f32x16 tv = __builtin_bit_cast(f32x16, T) - 12582912.0f;  // exact (float) T
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const float4 d4 = *(const float4 *) (dwv + kk * DWS + 32 * (rw + ri) + 8 * g + 4 * h);
                const float dw[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int i = 4 * g + e;
                    gsum[ri][i] = __builtin_fmaf(dw[e] * da[kk], tv[i], gsum[ri][i]);
                }
            }
        };
        auto mfma = [&](int kk, int ri) {
            const i32x4 a = *(const i32x4 *) (arow_p + ri * 32 * XR + 32 * kk);
            return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, xs.q[kk], kBias, 0, 0, 0);
        };
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            if constexpr (NR == 1) {
                acc[kk & 1] = mfma(kk, 0);
            } else {
                acc[0] = mfma(kk, 0);
                if (kk > 0) combine(kk - 1, 1, acc[1]);
                acc[1] = mfma(kk, 1);
            }
            // step kk of the next unit into the register just consumed
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((un * 8 + kk) * (int) xstep);
            xs.q[kk] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol, so, 0));
            if constexpr (NR == 1) {
                if (kk > 0) combine(kk - 1, 0, acc[(kk - 1) & 1]);
            } else {
                combine(kk, 0, acc[0]);
            }
#pragma unroll
            for (int pr = 0; pr < ROWP; pr++) {
                if (kk == 2 * pr + 1) store_block(cur ^ 1, rslot[pr], pr);
                if (kk == 2 * pr + 2) load_raw(rslot[pr], u + 1 + LEAD, pr);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const uint32_t so = (uint32_t) __builtin_amdgcn_readfirstlane((un * 8 + kk) * (int) ncols * 4);
            xs.da[kk] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, bcol * 4, so, 0));
        }
        combine(7, NR - 1, acc[1]);
        if (u % gs == gs - 1 || u == S - 1) {  // y starts at -0: -0 + g0 == g0 exactly
            asm volatile("" ::: "memory");
#pragma unroll
            for (int ri = 0; ri < NR; ri++) y[ri] = y[ri] + gsum[ri];
        }
        mi_lds_barrier();
    };
    for (int u0 = 0; u0 < S; u0 += LEAD) {
#pragma unroll
        for (int v = 0; v < LEAD; v++) {
            if (u0 + v < S) stage(u0 + v, raw[v]);
        }
    }

    // D[n][b]: column b = lane & 31 of this wave's 32, rows n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    const int64_t b = b0 + 32 * cw + r;
    if (b >= ncols) return;
    float * out = (float *) ((char *) dst + b * ycol);
#pragma unroll
    for (int ri = 0; ri < NR; ri++)
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int64_t n = n0 + 32 * (rw + ri) + 8 * g + 4 * h;
        if (n + 3 < N) {
            *(float4 *) (out + n) = make_float4(y[ri][4 * g], y[ri][4 * g + 1], y[ri][4 * g + 2], y[ri][4 * g + 3]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = y[ri][4 * g + e];
        }
    }
}

// ---- short prompts, K <= 4096: one round -------------------------------------------------------
// A workgroup of S waves (one superblock each) per 32 x 32 tile, so every load of the tile is
// requested at once and no wave runs a second round (k_mmqd's rounds each wait a full memory
// latency: the load -> MFMA -> fold phases of the two waves of a SIMD do not overlap). Four waves
// per SIMD at S = 16: <= 128 VGPRs, so the 16 da of a lane's accumulator elements go through a
// wave-private LDS row instead of registers. Same operands, same exact T / U and the same
// canonical fold (terms left-folded in superblock order) as k_mmqd / k_mmqx: bit-identical.
// ABL (timing ablations, results invalid): 1 no MFMAs, 2 one activation load reused, 4 no fold,
// 8 weight header only, 16 weight loads addressed as a wave-contiguous repacked layout ([chunk][row]
// 16-byte chunks per 32-row x superblock tile: every load instruction one contiguous 1 KB)
template <int TYPE, int ABL = 0>
__global__ __launch_bounds__(1024) void k_mmqd1(mi_mmx_group g) {
    MI_MMX_MEMBER(g);
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    extern __shared__ __attribute__((aligned(16))) float red[];  // [wave][lane][16] terms, then [wave][32] da
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);  // == waves of the workgroup
    const int64_t nrt = (N + 31) / 32;
    const int64_t n0 = (mmx_tile % nrt) * 32, c0 = (mmx_tile / nrt) * 32;
    const int sb = w;

    const int nrows = (int) std::min<int64_t>(32, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    const uint32_t wrow = (uint32_t) (min(r, nrows - 1) * nb01) + (uint32_t) sb * F::BS;
    const uint32_t acol = (uint32_t) std::min<int64_t>(c0 + r, ncols - 1);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t ures = __builtin_amdgcn_make_buffer_rsrc((void *) act.xu, (short) 0, (int) (S * ncols * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) (S * ncols * 4), 0x00020000);
    const uint32_t xstep = (uint32_t) ncols * 32;
    const uint32_t xcol = acol * 32 + 16 * h + (uint32_t) sb * 8 * xstep;
    constexpr uint32_t kQs = F::Q5 ? 48 : 16;

    // every load of the wave, weights first (HBM), then the activation fragments (L2)
    auto ld_w = [&](uint32_t off) -> uint4 { return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wrow + off, 0, 0)); };
    // ABL 16: the same loads at the offsets of a [chunk][row] repacked tile (chunk 0 = header,
    // 1 + 2 p + h = quant chunk p, half h)
    const uint32_t wtile = (uint32_t) sb * 32 * F::BS;
    auto ld_wc = [&](int chunk) -> uint4 {
        return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wtile + (uint32_t) (chunk * 32 + r) * 16, 0, 0));
    };
    const uint4 hdr = (ABL & 16) ? ld_wc(0) : ld_w(0);
    uint4 q4[4];
#pragma unroll
    for (int p = 0; p < 4; p++) q4[p] = (ABL & 8) ? hdr : (ABL & 16) ? ld_wc(1 + 2 * p + h) : ld_w(kQs + 32 * p + 16 * h);
    const uint4 qh = F::Q5 ? ld_w(16 + 16 * h) : uint4{};
    i32x4 xa[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++)
        xa[kk] = ((ABL & 2) && kk) ? xa[0] : __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol + kk * xstep, 0, 0));
    const half8 xu = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, ((uint32_t) sb * (uint32_t) ncols + acol) * 32 + 16 * h, 0, 0));
    // da of prompt column c0 + r (lanes >= 32 duplicate), parked in this wave's LDS row: columns
    // past ncols read a clamped column's value (never stored)
    const float dal = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, ((uint32_t) sb * (uint32_t) ncols + acol) * 4, 0, 0));
    float * dal_row = red + (size_t) S * 64 * 16 + w * 32;
    if (h == 0) dal_row[r] = dal;
    __builtin_amdgcn_wave_barrier();  // wave-private row: LDS ops of a wave complete in order
    __atomic_signal_fence(__ATOMIC_SEQ_CST);

    const uint32_t w0 = hdr.y, w1 = hdr.z, w2 = hdr.w;
    const float dw = mi_h2f((uint16_t) (hdr.x & 0xFFFF)), dm = mi_h2f((uint16_t) (hdr.x >> 16));
    i32x16 acc[NP];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
        const int jj = kk & 3;
        const uint32_t sc = kk < 4 ? ((w0 >> (8 * jj)) & 63) : (((w2 >> (8 * jj)) & 0xF) | (((w0 >> (8 * jj + 6)) & 3) << 4));
        const uint4 q = q4[kk >> 1];
        uint32_t v[4] = {q.x, q.y, q.z, q.w};
        const uint32_t hb[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[e] = (kk & 1) ? (v[e] >> 4) & 0x0F0F0F0Fu : v[e] & 0x0F0F0F0Fu;
            if constexpr (F::Q5) v[e] |= ((hb[e] >> kk) & 0x01010101u) << 4;
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            uint32_t f = F::factor((int) sc, p);
            f |= f << 16;
            const i32x4 b = {(int) mulb(v[0], f), (int) mulb(v[1], f), (int) mulb(v[2], f), (int) mulb(v[3], f)};
            if constexpr ((ABL & 1) != 0) acc[p][kk] = (kk == 0 ? 0 : acc[p][kk]) + xa[kk][0] * b[0];
            else acc[p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa[kk], b, kk == 0 ? i32x16{} : acc[p], 0, 0, 0);
        }
    }
    half8 mu;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int j = 4 * h + q;  // this lane's k-halves of the U MFMA: sub-blocks 4h .. 4h + 3
        const int jj = j & 3;
        const uint32_t m = j < 4 ? ((w1 >> (8 * jj)) & 63) : (((w2 >> (8 * jj + 4)) & 0xF) | (((w1 >> (8 * jj + 6)) & 3) << 4));
        mu[2 * q] = (_Float16) (float) m;
        mu[2 * q + 1] = (_Float16) (float) (64 * m);
    }
    const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(xu, mu, f32x16{}, 0, 0, 0);
    float * mine = red + ((size_t) w * 64 + lane) * 16;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const float4 d4 = *(const float4 *) (dal_row + 8 * g + 4 * h);
        const float dav[4] = {d4.x, d4.y, d4.z, d4.w};
        float term[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int el = 4 * g + e;
            int T = acc[NP - 1][el];
#pragma unroll
            for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[p][el];
            term[e] = mmqx_pre(T, Uv[el], dw, dm);
        }
        (void) dav;
        *(float4 *) (mine + 4 * g) = make_float4(term[0], term[1], term[2], term[3]);
    }
    mi_lds_barrier();
    // The 1024 outputs of the tile are folded by all S waves together: output o = 64 (w + S i) +
    // lane is accumulator element el = o % 16 of lane lo = o / 16; its terms (one per superblock =
    // per wave) are combined in the canonical order (cfold). Reads red[v][lo][el]: 64 consecutive
    // floats per wave-load.
    const int gs = cfold_gs(S);
    for (int o = 64 * w + lane; o < 1024; o += 64 * S) {
        const int lo = o >> 4, el = o & 15;
        const float * src = red + (size_t) lo * 16 + el;
        // d_a of superblock v for this output's column (the waves' da rows after the terms)
        const float * dsrc = red + (size_t) S * 64 * 16 + ((el & 3) + 8 * (el >> 2) + 4 * (lo >> 5));
        float y = -0.0f, ylo = -0.0f, gsum = 0.0f;
        for (int v = 0; v < ((ABL & 4) ? 1 : S); v++) cfold(gsum, y, ylo, src[(size_t) v * 64 * 16], dsrc[v * 32], v, gs, S);
        y = cfold_end(ylo, y);
        if (ABL & 4) y = gsum;
        // element el of lane lo = prompt column c0 + (el & 3) + 8 (el >> 2) + 4 (lo >> 5), row n0 + lo % 32
        const int64_t n = n0 + (lo & 31);
        const int64_t c = c0 + (el & 3) + 8 * (el >> 2) + 4 * (lo >> 5);
        if (n < N && c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = y;
    }
}

// ---- very short prompts (<= 16 columns), K <= 4096: 16 x 16 tiles --------------------------------
// k_mmqd1 on v_mfma_i32_16x16x64_i8: a 16-row x 16-column tile per workgroup (one wave per
// superblock), so a 16-column prompt spreads over N / 16 workgroups (every CU at N = 4096) instead
// of N / 32 with half of each 32-column tile idle. Lane (g = lane / 16, i = lane % 16): prompt
// column / weight row i, K bytes 16 g .. 16 g + 15 of each 64-deep step (step t = sub-blocks 2t,
// 2t + 1: Q4_K quant bytes 32 t + 16 (g & 1), low nibbles for g < 2, high for g >= 2). The
// accumulator element e of a lane is prompt column 4 g + e, weight row i. Same exact T / U and
// the same fold as every kernel of this file: bit-identical.
template <int TYPE>
__global__ __launch_bounds__(1024) void k_mmqd16(mi_mmx_group grp) {
    MI_MMX_MEMBER(grp);
    using F = XFmt<TYPE>;
    constexpr int NP = F::NP;
    extern __shared__ __attribute__((aligned(16))) float red[];  // [wave][lane][4] terms, then [wave][16] da
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);  // == waves of the workgroup
    const int64_t nrt = (N + 15) / 16;
    const int64_t n0 = (mmx_tile % nrt) * 16, c0 = (mmx_tile / nrt) * 16;
    const int sb = w;

    const int nrows = (int) std::min<int64_t>(16, N - n0);
    const __amdgpu_buffer_rsrc_t wres = __builtin_amdgcn_make_buffer_rsrc((void *) (W + n0 * nb01), (short) 0, (int) (nrows * nb01), 0x00020000);
    const uint32_t wrow = (uint32_t) (min(i, nrows - 1) * nb01) + (uint32_t) sb * F::BS;
    const uint32_t acol = (uint32_t) std::min<int64_t>(c0 + i, ncols - 1);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xq, (short) 0, (int) (K * ncols), 0x00020000);
    const __amdgpu_buffer_rsrc_t ures = __builtin_amdgcn_make_buffer_rsrc((void *) act.xu, (short) 0, (int) (S * ncols * 32), 0x00020000);
    const __amdgpu_buffer_rsrc_t dres = __builtin_amdgcn_make_buffer_rsrc((void *) act.xd, (short) 0, (int) (S * ncols * 4), 0x00020000);
    // 64-deep step t of this superblock = 32-deep steps 2 t (lanes g < 2) and 2 t + 1 (g >= 2)
    const uint32_t xstep = (uint32_t) ncols * 32;
    const uint32_t xcol = acol * 32 + 16 * (g & 1) + ((uint32_t) sb * 8 + (uint32_t) (g >> 1)) * xstep;
    constexpr uint32_t kQs = F::Q5 ? 48 : 16;

    auto ld_w = [&](uint32_t off) -> uint4 { return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wres, wrow + off, 0, 0)); };
    const uint4 hdr = ld_w(0);
    uint4 q4[4];
#pragma unroll
    for (int t = 0; t < 4; t++) q4[t] = ld_w(kQs + 32 * t + 16 * (g & 1));
    const uint4 qh = F::Q5 ? ld_w(16 + 16 * (g & 1)) : uint4{};
    i32x4 xa[4];
#pragma unroll
    for (int t = 0; t < 4; t++) xa[t] = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(xres, xcol + 2 * t * xstep, 0, 0));
    // U operand: sub-block halves of lanes g < 2 (g >= 2: zero K padding of the 16x16x32 MFMA)
    half8 xu = {};
    {
        const half8 u = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(ures, ((uint32_t) sb * (uint32_t) ncols + acol) * 32 + 16 * (g & 1), 0, 0));
        if (g < 2) xu = u;
    }
    const float dal = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dres, ((uint32_t) sb * (uint32_t) ncols + acol) * 4, 0, 0));
    float * dal_row = red + (size_t) S * 64 * 4 + w * 16;
    if (g == 0) dal_row[i] = dal;
    __builtin_amdgcn_wave_barrier();  // wave-private row: LDS ops of a wave complete in order
    __atomic_signal_fence(__ATOMIC_SEQ_CST);

    const uint32_t w0 = hdr.y, w1 = hdr.z, w2 = hdr.w;
    const float dw = mi_h2f((uint16_t) (hdr.x & 0xFFFF)), dm = mi_h2f((uint16_t) (hdr.x >> 16));
    const int hi = g >> 1;  // high nibbles: the odd sub-block of each step
    i32x4 acc[NP];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int j = 2 * t + hi;  // this lane's sub-block (lane-dependent: no unrolled constant)
        const int jj = j & 3;
        const uint32_t sc = j < 4 ? ((w0 >> (8 * jj)) & 63) : (((w2 >> (8 * jj)) & 0xF) | (((w0 >> (8 * jj + 6)) & 3) << 4));
        const uint4 q = q4[t];
        uint32_t v[4] = {q.x, q.y, q.z, q.w};
        const uint32_t hb[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[e] = (v[e] >> (4 * hi)) & 0x0F0F0F0Fu;
            if constexpr (F::Q5) v[e] |= ((hb[e] >> j) & 0x01010101u) << 4;
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            uint32_t f = F::factor((int) sc, p);
            f |= f << 16;
            const i32x4 b = {(int) mulb(v[0], f), (int) mulb(v[1], f), (int) mulb(v[2], f), (int) mulb(v[3], f)};
            acc[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[t], b, t == 0 ? i32x4{} : acc[p], 0, 0, 0);
        }
    }
    half8 mu = {};
    if (g < 2) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = 4 * g + q;  // K halves 8 g .. 8 g + 7: sub-blocks 4 g .. 4 g + 3
            const int jj = j & 3;
            const uint32_t m = j < 4 ? ((w1 >> (8 * jj)) & 63) : (((w2 >> (8 * jj + 4)) & 0xF) | (((w1 >> (8 * jj + 6)) & 3) << 4));
            mu[2 * q] = (_Float16) (float) m;
            mu[2 * q + 1] = (_Float16) (float) (64 * m);
        }
    }
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    const f32x4v Uv = __builtin_amdgcn_mfma_f32_16x16x32_f16(xu, mu, f32x4v{}, 0, 0, 0);
    float * mine = red + ((size_t) w * 64 + lane) * 4;
    {
        const float4 d4 = *(const float4 *) (dal_row + 4 * g);
        const float dav[4] = {d4.x, d4.y, d4.z, d4.w};
        float term[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            int T = acc[NP - 1][e];
#pragma unroll
            for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[p][e];
            term[e] = mmqx_pre(T, Uv[e], dw, dm);
        }
        (void) dav;
        *(float4 *) mine = make_float4(term[0], term[1], term[2], term[3]);
    }
    mi_lds_barrier();
    if (w != 0) return;
    float4 y = {-0.0f, -0.0f, -0.0f, -0.0f}, lo = y, gsum = {};
    const int gs = cfold_gs(S);
    for (int v = 0; v < S; v++) {
        const float4 t4 = *(const float4 *) (red + ((size_t) v * 64 + lane) * 4);
        const float4 d4 = *(const float4 *) (red + (size_t) S * 64 * 4 + v * 16 + 4 * g);  // d_a of columns 4 g ..
        cfold(gsum.x, y.x, lo.x, t4.x, d4.x, v, gs, S);
        cfold(gsum.y, y.y, lo.y, t4.y, d4.y, v, gs, S);
        cfold(gsum.z, y.z, lo.z, t4.z, d4.z, v, gs, S);
        cfold(gsum.w, y.w, lo.w, t4.w, d4.w, v, gs, S);
    }
    y = make_float4(cfold_end(lo.x, y.x), cfold_end(lo.y, y.y), cfold_end(lo.z, y.z), cfold_end(lo.w, y.w));
    const int64_t n = n0 + i;
    if (n >= N) return;
    const float yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int64_t c = c0 + 4 * g + e;
        if (c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = yv[e];
    }
}

} // namespace

bool mi_mmqx_supported(int type, int64_t K, size_t ycol, int64_t ncols, size_t nb01) {
    // buffer descriptors address < 2 GiB: activations K * ncols bytes, a 64-row weight block;
    // Q4_0 / Q8_0: 16-byte aligned 8-block units (K % 256 == 0, rows of 16-byte multiples)
    if (type == 2 || type == 8) {
        return K % 256 == 0 && K >= 256 && nb01 % 16 == 0 && K * ncols < ((int64_t) 1 << 31) && (int64_t) nb01 * 32 < ((int64_t) 1 << 31);
    }
    return (type == 12 || type == 13) && K % 256 == 0 && K >= 256 && ycol % 16 == 0 && K * ncols < ((int64_t) 1 << 31) &&
           (int64_t) nb01 * XBM < ((int64_t) 1 << 31);
}

// tiles of every member for a tile shape of tr rows x tc columns; returns the total
static int64_t mmx_deal(mi_mmx_group & g, int64_t tr, int64_t tc) {
    int64_t t = 0;
    for (int i = 0; i < g.n; i++) {
        g.m[i].tile_begin = t;
        t += ((g.m[i].N + tr - 1) / tr) * ((g.m[i].act.ncols + tc - 1) / tc);
    }
    return t;
}

void mi_mul_mat_mmqx_group(mi_mmx_group & g, hipStream_t s) {
    if (g.n <= 0) return;
    const int type = g.type;
    const int64_t K = g.K;
    const int64_t ncols = g.m[0].act.ncols;  // every member has the same column count
    if (type == 2 || type == 8) {  // Q4_0 / Q8_0: q8_0 activations (mi_act_mmx0_*), every column count
        // By workgroup count: 64 x 128 tiles of 4 waves, each 64 rows x 32 columns (k_mmq0x NR = 2)
        // when there are >= 256 of them; else 64 x 64 tiles of 4 waves (k_mmq0x half width) when
        // >= 256 (Q8_0: 128); else 32 x 32 tiles of 4 waves on one tile (k_mmq0p). Variant bits force one: 16 k_mmq0p, 128 k_mmq0x (8 waves, 64 x 128), 128 |
        // 65536 half width, 128 | 2^24 NR = 2, 128 | 2^25 NR = 2 with 8 waves (64 x 256). Every one
        // keeps the family's canonical combine: the same bits.
        const int var = g_mi_tuning.mmq_variant;
        int pick;
        if (var & 16) pick = 0;
        else if (var & 128) pick = (var & (1 << 25)) ? 4 : (var & (1 << 24)) ? 3 : (var & 65536) ? 2 : 1;
        else {
            int64_t t2 = 0, th = 0;
            for (int i = 0; i < g.n; i++) {
                const int64_t rt = (g.m[i].N + XBM - 1) / XBM, nc = g.m[i].act.ncols;
                t2 += rt * ((nc + 127) / 128);
                th += rt * ((nc + 63) / 64);
            }
            // (k_mmq0p's Q8_0 operands -- five dword loads per block and lane -- make it the
            // slower one for Q8_0 from 128 half-width tiles on)
            pick = t2 >= 256 && ncols > 64 ? 3 : th >= (type == 8 ? 128 : 256) ? 2 : 0;
        }
        const bool q8 = type == 8;
        switch (pick) {
            case 0: {  // (a deeper weight ring, RING 3, spills: 36-dword units)
                const dim3 grid((unsigned) mmx_deal(g, 32, 32));
                if (!q8) hipLaunchKernelGGL((k_mmq0p<false>), grid, dim3(256), 0, s, g);
                else hipLaunchKernelGGL((k_mmq0p<true>), grid, dim3(256), 0, s, g);
                return;
            }
            case 1: {
                const dim3 grid((unsigned) mmx_deal(g, XBM, XBN));
                if (!q8) hipLaunchKernelGGL((k_mmq0x<false, 8, 4>), grid, dim3(512), 0, s, g);
                else hipLaunchKernelGGL((k_mmq0x<true, 8, 4>), grid, dim3(512), 0, s, g);
                return;
            }
            case 2: {
                const dim3 grid((unsigned) mmx_deal(g, XBM, 64));
                if (!q8) hipLaunchKernelGGL((k_mmq0x<false, 4, 2>), grid, dim3(256), 0, s, g);
                else hipLaunchKernelGGL((k_mmq0x<true, 4, 2>), grid, dim3(256), 0, s, g);
                return;
            }
            case 3: {
                const dim3 grid((unsigned) mmx_deal(g, XBM, 128));
                if (!q8) hipLaunchKernelGGL((k_mmq0x<false, 4, 2, 2>), grid, dim3(256), 0, s, g);
                else hipLaunchKernelGGL((k_mmq0x<true, 4, 2, 2>), grid, dim3(256), 0, s, g);
                return;
            }
            default: {
                const dim3 grid((unsigned) mmx_deal(g, XBM, 256));
                if (!q8) hipLaunchKernelGGL((k_mmq0x<false, 8, 2, 2>), grid, dim3(512), 0, s, g);
                else hipLaunchKernelGGL((k_mmq0x<true, 8, 2, 2>), grid, dim3(512), 0, s, g);
                return;
            }
        }
    }
    // short prompts (<= 128 columns): pipelined 32 x 32 tiles of 4 waves (k_mmqp; variant bit
    // 2048: k_mmqd1, a wave per superblock) or, <= 16 columns, 16 x 16 tiles of a wave per
    // superblock (k_mmqd16); long ones: 64 x 128 tiles with the weights dequantized once per
    // workgroup into LDS (k_mmqx). All follow the same canonical combine order (cfold), so a
    // prompt's column shards give the whole prompt's bits whichever kernel runs them (variant bit
    // 128 forces k_mmqx, 16 the short-prompt kernels).
    const int var = g_mi_tuning.mmq_variant;
    // k_mmqx / k_mmqw park the low half of the canonical fold in their own output locations until
    // the end: only plain device memory of this device may be used that way. An output in pinned
    // host memory (host-staged logits) or on a peer device takes the pipelined 32 x 32 tiles, which
    // store each element once (the same bits: the family's canonical combine).
    bool dst_local = true;
    for (int i = 0; i < g.n && dst_local; i++) {
        hipPointerAttribute_t pa;
        int dev = 0;
        (void) hipGetDevice(&dev);
        if (hipPointerGetAttributes(&pa, g.m[i].dst) != hipSuccess) {
            (void) hipGetLastError();
            dst_local = false;  // unknown to HIP: plain host memory
        } else {
            dst_local = pa.type == hipMemoryTypeDevice && pa.device == dev;
        }
    }
    // long prompts on repacked planes (mmq_planes.hip) when every member carries them (each output
    // stored once: any destination); variant bits forcing a canonical kernel (16, 128) keep it
    if (ncols >= kMiPlanesMinCols && !(var & (16 | 128)) && mi_mul_mat_mmqr_group(g, s)) return;
    // Q4_K prompts of 33..128 columns whose launch (nearly) fills the chip with k_mmqt's 128 x 64
    // tiles (one workgroup per CU; mmqt_short, default 192 workgroups): k_mmqt instead of k_mmqp
    // (round 6, bit-identical). 32 rotated weights grouped 16 to a launch: B = 64 7.29 -> 5.36 us,
    // B = 128 13.39 -> 10.04 us per mul_mat (profiles/r06s2_pf_mmqt_short.txt); by group size
    // (r06s2b_mmqt_short_groups.txt, r06s2c_mmqt_short_threshold.txt) k_mmqt wins from 192 of its
    // workgroups (3 x B = 128: 13.99 -> 11.19 us; 6 x B = 64: 6.98 -> 5.72 us) and loses below (4 x
    // B = 64, 128 workgroups: 7.76 vs 7.86; a lone B = 64 member's 32: 12.4 vs 26.6 us); B = 32 stays
    // on k_mmqp (4.52 vs 4.85). Variant bits that ask for a particular kernel turn it off.
    constexpr int kShortTBlock = 16 | 128 | 2048 | 4096 | 8192 | (1 << 19) | (1 << 21) | (1 << 22) | (1 << 26) | (1 << 27);
    bool short_t = false;
    if (type == 12 && ncols > 32 && ncols <= 128 && dst_local && g_mi_tuning.mmqt_short > 0 && !(var & kShortTBlock)) {
        int64_t tt = 0;
        for (int i = 0; i < g.n; i++) tt += ((g.m[i].N + 127) / 128) * ((g.m[i].act.ncols + 63) / 64);
        short_t = tt >= g_mi_tuning.mmqt_short;
    }
    // k_mmqt plain, or (diagnostic builds, mmq_long 5) with the high half staggered (ST; measured
    // 3-9 % slower, profiles/r06s2h_mmqt_stagger_ab.txt)
    const bool st = MI_DIAG && g_mi_tuning.mmq_long == 5;
    if (short_t) {
        const dim3 gridt((unsigned) mmx_deal(g, 128, 64));
#if MI_DIAG
        if (st) hipLaunchKernelGGL((k_mmqt<12, 0, false, true>), gridt, dim3(512), 0, s, g);
        else
#endif
        hipLaunchKernelGGL((k_mmqt<12>), gridt, dim3(512), 0, s, g);
        return;
    }
    const bool direct = (var & 16) || (ncols <= 128 && !(var & 128)) || !dst_local;
    if (direct) {
        const int S = (int) (K / 256);
        // 16 x 16 tiles (k_mmqd16) only when asked: variant bit 2^21 up to 16 columns, 2^22 up to 128.
        // Round 6 (profiles/r06a_short_prefill.txt, Q4_K / Q5_K 4096^2, 8 rotated weights): k_mmqp's
        // 32 x 32 tiles are faster at B = 9 and 16 both grouped (Q4_K 3.98 / 4.07 vs 5.56 / 5.63 us per
        // mul_mat) and alone in a graph (11.5 / 11.4 vs 12.0 / 12.0 us)
        const int64_t lim16 = (var & (1 << 22)) ? 128 : (var & (1 << 21)) ? 16 : 0;
        if (S <= 16 && ncols <= lim16 && !(var & (2048 | 4096))) {
            const dim3 grid16((unsigned) mmx_deal(g, 16, 16));
            const size_t lds16 = (size_t) S * 64 * 4 * sizeof(float) + (size_t) S * 16 * sizeof(float);
            if (type == 12) hipLaunchKernelGGL((k_mmqd16<12>), grid16, dim3(64 * S), lds16, s, g);
            else hipLaunchKernelGGL((k_mmqd16<13>), grid16, dim3(64 * S), lds16, s, g);
            return;
        }
        const dim3 grid((unsigned) mmx_deal(g, 32, 32));
        if (S <= 16 && (var & 2048)) {  // one round: a wave per superblock (variant bit 2048: k_mmqd1)
            const size_t lds = (size_t) S * 64 * 16 * sizeof(float) + (size_t) S * 32 * sizeof(float);
            // ABL bits 1..8 from variant bits 12..15, 16 from bit 23
#if MI_DIAG  // timing ablations (results invalid): diagnostic builds only (make DIAG=1)
            const int abl = ((var >> 12) & 15) | (((var >> 23) & 1) << 4);
            if (abl && type == 12) {
#define MI_MMQD1A(A) hipLaunchKernelGGL((k_mmqd1<12, A>), grid, dim3(64 * S), lds, s, g)
                switch (abl) {
                case 1: MI_MMQD1A(1); break;
                case 2: MI_MMQD1A(2); break;
                case 4: MI_MMQD1A(4); break;
                case 8: MI_MMQD1A(8); break;
                case 10: MI_MMQD1A(10); break;
                case 16: MI_MMQD1A(16); break;
                default: MI_MMQD1A(15); break;
                }
#undef MI_MMQD1A
                return;
            }
#endif
            if (type == 12) hipLaunchKernelGGL((k_mmqd1<12>), grid, dim3(64 * S), lds, s, g);
            else hipLaunchKernelGGL((k_mmqd1<13>), grid, dim3(64 * S), lds, s, g);
            return;
        }
        // pipelined 32 x 32 tiles, 8 waves each (k_mmqp; variant bit 2^26: 32 x 64 tiles)
        const int64_t t64 = mmx_deal(g, 32, 64);
        const int nc = (MI_DIAG && (var & (1 << 26))) ? 2 : 1;  // 64-column tiles spill: diagnostic builds only
        const dim3 gridp((unsigned) (nc == 2 ? t64 : mmx_deal(g, 32, 32)));
        // 4 waves per tile (two workgroups per CU) unless variant bit 2^27 (8 waves, one per CU);
        // weight ring of 2 (variant bit 2^19: 4 -- slower, profiles/r03w_mmqp_ring.txt: vmcnt retires
        // in issue order, so a step waiting for its activations also waits for every weight request
        // issued before them; a deeper weight lead alone only adds outstanding loads)
        const bool w8 = (var & (1 << 27)) != 0;
        const bool r2 = !MI_DIAG || (var & (1 << 19)) == 0;  // (ring 4: diagnostic builds only)
#define MI_MMQP(TY, NCC, NWW, RG) hipLaunchKernelGGL((k_mmqp<TY, NCC, NWW, 0, RG>), gridp, dim3(64 * NWW), 0, s, g)
#if MI_DIAG
#define MI_MMQP1(TY, NWW) do { if (r2) MI_MMQP(TY, 1, NWW, 2); else MI_MMQP(TY, 1, NWW, 4); } while (0)
        if (type == 12) {
            if (nc == 2) { if (w8) MI_MMQP(12, 2, 8, 2); else MI_MMQP(12, 2, 4, 2); }
            else { if (w8) MI_MMQP1(12, 8); else MI_MMQP1(12, 4); }
        } else {
            if (nc == 2) { if (w8) MI_MMQP(13, 2, 8, 2); else MI_MMQP(13, 2, 4, 2); }
            else { if (w8) MI_MMQP1(13, 8); else MI_MMQP1(13, 4); }
        }
#undef MI_MMQP1
#else
        (void) nc;
        (void) r2;
        if (type == 12) { if (w8) MI_MMQP(12, 1, 8, 2); else MI_MMQP(12, 1, 4, 2); }
        else { if (w8) MI_MMQP(13, 1, 8, 2); else MI_MMQP(13, 1, 4, 2); }
#endif
#undef MI_MMQP
        return;
    }
    // half-width workgroups (two per CU) when full-width tiles would leave CUs idle: Q4_K B=256
    // 27.8 -> 26.4 us (B=512 41.7 vs 34.7 us: the per-workgroup dequantization then doubles)
    int64_t full_tiles = 0;
    for (int i = 0; i < g.n; i++) full_tiles += ((g.m[i].N + XBM - 1) / XBM) * ((g.m[i].act.ncols + XBN - 1) / XBN);
    const bool half = (var & 65536) || (type == 12 && full_tiles < 256 && !(var & 131072));
    if (half) {
        const dim3 grid4((unsigned) mmx_deal(g, XBM, 64));
        if (type == 12) hipLaunchKernelGGL((k_mmqx<12, false, 0, 2, 0, 4>), grid4, dim3(256), 0, s, g);
        else hipLaunchKernelGGL((k_mmqx<13, false, 0, 2, 0, 4>), grid4, dim3(256), 0, s, g);
        return;
    }
    // Q4_K: K split over wave pairs, 128 x 64 tiles (k_mmqt, the default; B=512 33.4 vs 36.6 us for
    // k_mmqw, B=256 18.5 vs 19.7, profiles/r04i_pf_long_mmqt.txt; its DMAs all at the step start
    // instead of one behind each MFMA step: 37.1 us; the high half folding one step late from a
    // 3-slot LDS ring, so the two waves of a SIMD alternate MFMA and VALU phases: 38.7 us,
    // profiles/r04k_mmqt_skew_ab.txt, r04m_mmqt_skew_stamps.txt; DMAs through buffer descriptors:
    // no change, r04p_mmqt_buf_ab.txt; the two column tiles in two passes over held planes with
    // tile 0's combine under tile 1's MFMAs: 36.4 vs 35.5 us, r04r_mmqt_split_ab.txt, and tile 1's
    // combine deferred into the next step too: 36.9 vs 35.4 us, r04t_mmqt_split2_ab.txt -- all
    // removed)
    const int lng = g_mi_tuning.mmq_long;
    if ((!MI_DIAG || lng == 0 || lng == 2 || lng == 3 || lng == 4 || lng == 5) && type == 12 && !(var & ((1 << 28) | 64 | 1024))) {
        const dim3 gridt((unsigned) mmx_deal(g, 128, 64));
#if MI_DIAG  // measured slower (round 6, profiles/r06e_mmqv_prefill.txt): diagnostic builds only
        if (lng == 3) hipLaunchKernelGGL((k_mmqt<12, 0, true>), gridt, dim3(512), 0, s, g);  // per-half stage sync
        else if (lng == 4) hipLaunchKernelGGL((k_mmqv<12>), gridt, dim3(256), 0, s, g);  // one wave per SIMD, pipelined
        else
#endif
#if MI_DIAG
        if (st) hipLaunchKernelGGL((k_mmqt<12, 0, false, true>), gridt, dim3(512), 0, s, g);
        else
#endif
        hipLaunchKernelGGL((k_mmqt<12>), gridt, dim3(512), 0, s, g);
        (void) st;
        return;
    }
#if MI_DIAG
    if (lng >= 16 && lng < 24 && type == 12) {  // k_mmqt stamps (+ ablation bits lng - 16; results invalid)
        const dim3 gridt((unsigned) mmx_deal(g, 128, 64));
        switch (lng - 16) {
            case 1: hipLaunchKernelGGL((k_mmqt<12, 9>), gridt, dim3(512), 0, s, g); break;
            case 2: hipLaunchKernelGGL((k_mmqt<12, 10>), gridt, dim3(512), 0, s, g); break;
            case 4: hipLaunchKernelGGL((k_mmqt<12, 12>), gridt, dim3(512), 0, s, g); break;
            case 6: hipLaunchKernelGGL((k_mmqt<12, 14>), gridt, dim3(512), 0, s, g); break;
            case 7: hipLaunchKernelGGL((k_mmqt<12, 8, true>), gridt, dim3(512), 0, s, g); break;  // per-half sync, stamps
            default: hipLaunchKernelGGL((k_mmqt<12, 8>), gridt, dim3(512), 0, s, g); break;
        }
        return;
    }
#endif
    const dim3 grid((unsigned) mmx_deal(g, XBM, XBN));
    // warp-specialized k_mmqw (4 loader + 8 MFMA waves; Q4_K B=512 32.1 -> 31.2 us, Q5_K 46.2 ->
    // 43.8 us grouped, profiles/r03r_prefill_mmqw.txt) unless variant bit 2^28 asks for k_mmqx
#if MI_DIAG
    if ((var & 1024) && (var & (1 << 29)) && type == 12) {  // k_mmqw timing stamps (results invalid)
        hipLaunchKernelGGL((k_mmqw<12, 4, 8>), grid, dim3(768), 0, s, g);
        return;
    }
#endif
    if (!(var & ((1 << 28) | 64 | 1024)) && (K / 256) % 4 == 0) {
#if MI_DIAG  // (Q4_K on k_mmqw: mmq_long 1, diagnostic builds only)
        if (type == 12) hipLaunchKernelGGL((k_mmqw<12, 4>), grid, dim3(768), 0, s, g);
        else
#endif
        hipLaunchKernelGGL((k_mmqw<13, 4>), grid, dim3(768), 0, s, g);
        return;
    }
    // weight ring depth LEAD (variant bits: 64 -> 1, default 4). (Fully unrolling the stage loop
    // for K = 4096, SCT = 16, spills: the compiler hoists loads across stages.)
#define MI_MMQX_T(TY, LD) hipLaunchKernelGGL((k_mmqx<TY, false, 0, LD, 0>), grid, dim3(512), 0, s, g)
    const int lead = (var & 64) ? 1 : 4;
#if MI_DIAG
    if (var & 1024) {  // timing stamps (results invalid)
        if (type == 12) hipLaunchKernelGGL((k_mmqx<12, false, 8, 4, 0>), grid, dim3(512), 0, s, g);
        return;
    }
#endif
    if (type == 12) {
        if (lead == 1) MI_MMQX_T(12, 1); else MI_MMQX_T(12, 4);
    } else {
        if (lead == 1) MI_MMQX_T(13, 1); else MI_MMQX_T(13, 4);
    }
#undef MI_MMQX_T
}

void mi_mul_mat_mmqx(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_mmx & act, float * dst,
                     size_t ycol, hipStream_t s, const char * planes) {
    mi_mmx_group g;
    g.type = type;
    g.n = 1;
    g.K = K;
    g.m[0] = mi_mmx_member{W, nb01, N, act, dst, ycol, 0, planes};
    mi_mul_mat_mmqx_group(g, s);
}
