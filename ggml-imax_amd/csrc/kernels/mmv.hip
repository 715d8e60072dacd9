// mmv.hip -- GGML_OP_MUL_MAT for few activation columns (decode / GEMV regime) on gfx950.
//
// Memory-bound: every weight byte is read once from HBM, activations (a few KB per column)
// come from L1/L2. One wave64 owns one weight row; its lanes split the row into
// (superblock, 64-element group) items so that a K=4096 Q4_K row (16 superblocks x 4 groups)
// is exactly one item per lane, loaded with three aligned 16-byte loads per lane
// (header + 32 B of nibbles). Integer dot products use v_dot4_i32_i8 on the reference's own
// quantized activations, so each superblock's integer sum is bit-identical to
// ggml_vec_dot_q4_K_q8_K (src/ggml-quants.c:7007-7502); only the f32 combination order across
// superblocks differs from the CPU.
//
// Reference per-type dot products mirrored here:
//   Q4_0 x Q8_0  ggml_vec_dot_q4_0_q8_0  src/ggml-quants.c:3469-3874
//   Q8_0 x Q8_0  ggml_vec_dot_q8_0_q8_0  src/ggml-quants.c:4819+
//   Q4_K x Q8_K  ggml_vec_dot_q4_K_q8_K  src/ggml-quants.c:7007-7502
//   Q5_K x Q8_K  ggml_vec_dot_q5_K_q8_K  src/ggml-quants.c:7833-8378
// (F16 and F32 live in mmv_ordered.hip: bit-exact CPU summation order.)

#include "mi355x_common.h"
#include "mi355x_kernels.h"

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves x 1 row
constexpr int kMaxCols = 8;

struct mmv_geom {
    int64_t K, N;
    int64_t ne11, ne12, ne13;
    int64_t r2, r3;          // broadcast ratios ne12/ne02, ne13/ne03
    size_t nb01, nb02, nb03;
    size_t nb1, nb2, nb3;
    int64_t col_chunks;      // ceil(ne11 / NC)
};

// Decode blockIdx.y into (first column i11, i12, i13) and return the weight row pointer base.
__device__ __forceinline__ void mmv_coords(const mmv_geom & g, int NC, int64_t & i11, int64_t & i12, int64_t & i13,
                                           int64_t & i02, int64_t & i03) {
    const int64_t y = blockIdx.y;
    const int64_t chunk = y % g.col_chunks;
    const int64_t z = y / g.col_chunks;
    i12 = z % g.ne12;
    i13 = z / g.ne12;
    i11 = chunk * NC;
    i02 = i12 / g.r2;
    i03 = i13 / g.r3;
}

template <int NC>
__device__ __forceinline__ void mmv_store(const mmv_geom & g, float * dst, int64_t row, int64_t i11, int64_t i12, int64_t i13,
                                          float (&acc)[NC], int lane) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float v = mi_wave_sum(acc[c]);
        if (lane == 0 && i11 + c < g.ne11) {
            *(float *) ((char *) dst + (i11 + c) * g.nb1 + i12 * g.nb2 + i13 * g.nb3 + row * sizeof(float)) = v;
        }
    }
}

// ---------------------------------------------------------------- Q4_K / Q5_K x Q8_K

template <int NC, bool Q5>
__global__ __launch_bounds__(256) void k_mmv_kq(const uint8_t * __restrict__ W, mi_act_q8 act, float * __restrict__ dst, mmv_geom g) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
    if (row >= g.N) return;
    int64_t i11, i12, i13, i02, i03;
    mmv_coords(g, NC, i11, i12, i13, i02, i03);
    constexpr int BS = Q5 ? 176 : 144;
    const uint8_t * wrow = W + i02 * g.nb02 + i03 * g.nb03 + row * g.nb01;
    const int nsb = (int) (g.K / 256);
    const int64_t col0 = i11 + g.ne11 * (i12 + g.ne12 * i13);

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = 0.0f;

    for (int it = lane; it < 4 * nsb; it += 64) {
        const int s = it >> 2;
        const int j = it & 3;
        const uint8_t * blk = wrow + (size_t) s * BS;
        const uint4 hdr = *(const uint4 *) blk;
        const uint8_t * qp = blk + (Q5 ? 48 : 16) + 32 * j;
        const uint4 qa = *(const uint4 *) qp;
        const uint4 qb = *(const uint4 *) (qp + 16);
        uint32_t q[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        uint32_t qlo[8], qhi[8];
        if constexpr (Q5) {
            const uint4 ha = *(const uint4 *) (blk + 16);
            const uint4 hb = *(const uint4 *) (blk + 32);
            const uint32_t h[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
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
        const float dw = mi_h2f((uint16_t) (hdr.x & 0xFFFF));
        const float dmw = mi_h2f((uint16_t) (hdr.x >> 16));
        int sc0, m0, sc1, m1;
        mi_scale_min_k4(2 * j, hdr.y, hdr.z, hdr.w, sc0, m0);
        mi_scale_min_k4(2 * j + 1, hdr.y, hdr.z, hdr.w, sc1, m1);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && i11 + c >= g.ne11) break;
            const int64_t col = col0 + c;
            const int4 * a = (const int4 *) (act.qs + col * g.K + (int64_t) s * 256 + 64 * j);
            const int4 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
            const int alo[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const int ahi[8] = {a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            int lo = 0, hi = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                lo = mi_dot4((int) qlo[i], alo[i], lo);
                hi = mi_dot4((int) qhi[i], ahi[i], hi);
            }
            const int sumi = sc0 * lo + sc1 * hi;
            const int ss = *(const int *) (act.s32 + col * (g.K / 32) + s * 8 + 2 * j);
            const int summ = m0 * (int) (int16_t) (ss & 0xFFFF) + m1 * (ss >> 16);
            const float dy = act.d[col * nsb + s];
            acc[c] += dy * (dw * (float) sumi - dmw * (float) summ);
        }
    }
    mmv_store<NC>(g, dst, row, i11, i12, i13, acc, lane);
}

// ---------------------------------------------------------------- Q4_0 / Q8_0 x Q8_0

// 32 quants of a block starting at a 2-byte aligned address, gathered from aligned dwords.
template <int NBYTES>
__device__ __forceinline__ void load_qs_unaligned(const uint8_t * p, uint32_t (&out)[NBYTES / 4]) {
    const uintptr_t addr = (uintptr_t) p;
    const uint32_t * w = (const uint32_t *) (addr & ~(uintptr_t) 3);
    const int shift = (int) (addr & 3);  // 0 or 2 here
    uint32_t raw[NBYTES / 4 + 1];
#pragma unroll
    for (int i = 0; i < NBYTES / 4; i++) raw[i] = w[i];
    raw[NBYTES / 4] = shift ? w[NBYTES / 4] : 0u;  // buffers carry 256 B of tail slack
#pragma unroll
    for (int i = 0; i < NBYTES / 4; i++) out[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], shift);
}

template <int NC, bool Q8>
__global__ __launch_bounds__(256) void k_mmv_q0(const uint8_t * __restrict__ W, mi_act_q8 act, float * __restrict__ dst, mmv_geom g) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
    if (row >= g.N) return;
    int64_t i11, i12, i13, i02, i03;
    mmv_coords(g, NC, i11, i12, i13, i02, i03);
    constexpr int BS = Q8 ? 34 : 18;
    const uint8_t * wrow = W + i02 * g.nb02 + i03 * g.nb03 + row * g.nb01;
    const int nb = (int) (g.K / 32);
    const int64_t col0 = i11 + g.ne11 * (i12 + g.ne12 * i13);

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = 0.0f;

    for (int b = lane; b < nb; b += 64) {
        const uint8_t * blk = wrow + (size_t) b * BS;
        const float dw = mi_h2f(*(const uint16_t *) blk);
        int wq[8];
        if constexpr (Q8) {
            uint32_t t[8];
            load_qs_unaligned<32>(blk + 2, t);
#pragma unroll
            for (int i = 0; i < 8; i++) wq[i] = (int) t[i];
        } else {
            uint32_t t[4];
            load_qs_unaligned<16>(blk + 2, t);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                wq[i] = (int) (t[i] & 0x0F0F0F0Fu);          // elements 4i..4i+3
                wq[i + 4] = (int) ((t[i] >> 4) & 0x0F0F0F0Fu);  // elements 16+4i..
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && i11 + c >= g.ne11) break;
            const int64_t col = col0 + c;
            const int4 * a = (const int4 *) (act.qs + col * g.K + (int64_t) b * 32);
            const int4 a0 = a[0], a1 = a[1];
            const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            int sumi = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) sumi = mi_dot4(wq[i], av[i], sumi);
            if constexpr (!Q8) {
                // (q - 8) * y summed = q*y - 8 * sum(y)
                int sy = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) sy = mi_dot4(0x01010101, av[i], sy);
                sumi -= 8 * sy;
            }
            acc[c] += (float) sumi * (dw * act.d[col * nb + b]);
        }
    }
    mmv_store<NC>(g, dst, row, i11, i12, i13, acc, lane);
}

// Reference CPU order (mmv_order 1) for the Q4_0 / Q8_0 rows this generic path serves -- K % 256
// != 0 (rows of any block count, so only 2-byte aligned) and 3-D weight batches, where the fused
// reference-order kernel (mmv_fused_impl.h) does not apply. The reference's AVX2 dot
// (ggml_vec_dot_q8_0_q8_0 src/ggml-quants.c:4819+, ggml_vec_dot_q4_0_q8_0 :3469+) keeps eight
// float lanes: lane l gets the exact int32 sum of elements 4l..4l+3 of each block
// (mul_sum_i8_pairs_float; Q4_0 after bytes_from_nibbles_32 - 8: low nibbles of bytes 4l.. for
// l < 4, high nibbles of bytes 4(l-4).. for l >= 4) in acc[l] = fma(x.d * y.d, q, acc[l]) over the
// blocks in order, then hsum_float_8. Here eight lanes are those eight CPU lanes of one row (8 rows
// per wave): each runs its own chain, the hsum is three xor shuffles in the same pairing.
template <int NC, bool Q8>
__global__ __launch_bounds__(256) void k_mmv_q0_ord(const uint8_t * __restrict__ W, mi_act_q8 act, float * __restrict__ dst, mmv_geom g) {
    const int l = threadIdx.x & 7;
    const int64_t row = (int64_t) blockIdx.x * 32 + (threadIdx.x >> 3);
    const bool live = row < g.N;
    const int64_t rc = live ? row : g.N - 1;  // (dead groups run a valid row: no early exit before the shuffles)
    int64_t i11, i12, i13, i02, i03;
    mmv_coords(g, NC, i11, i12, i13, i02, i03);
    constexpr int BS = Q8 ? 34 : 18;
    const uint8_t * wrow = W + i02 * g.nb02 + i03 * g.nb03 + rc * g.nb01;
    const int nb = (int) (g.K / 32);
    const int64_t col0 = i11 + g.ne11 * (i12 + g.ne12 * i13);
    // the lane's 4 quant bytes: block byte 2 + 4 l (Q4_0: 2 + 4 (l & 3), nibble half l >> 2)
    const int qoff = 2 + 4 * (Q8 ? l : (l & 3));

    float A[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) A[c] = 0.0f;

#pragma unroll 4
    for (int b = 0; b < nb; b++) {
        const uintptr_t blk = (uintptr_t) (wrow + (size_t) b * BS);
        // blocks are 2-byte aligned: d and the quants from the aligned dwords covering them
        // (buffers carry 256 B of tail slack)
        const uint32_t dw0 = *(const uint32_t *) (blk & ~(uintptr_t) 3);
        const float dw = mi_h2f((uint16_t) ((blk & 2) ? dw0 >> 16 : dw0 & 0xFFFF));
        const uintptr_t qa = blk + qoff;
        const uint32_t * qp = (const uint32_t *) (qa & ~(uintptr_t) 3);
        uint32_t q = __builtin_amdgcn_alignbyte(qp[1], qp[0], (uint32_t) (qa & 3));
        if constexpr (!Q8) q = (l < 4 ? q : q >> 4) & 0x0F0F0F0Fu;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && i11 + c >= g.ne11) break;
            const int64_t col = col0 + c;
            const int av = *(const int *) (act.qs + col * g.K + (int64_t) b * 32 + 4 * l);
            // Q4_0: (q - 8) . y, exact (0xF8 = -8 per byte)
            const int sumi = Q8 ? mi_dot4((int) q, av, 0) : mi_dot4((int) q, av, mi_dot4((int) 0xF8F8F8F8u, av, 0));
            A[c] = fmaf(dw * act.d[col * nb + b], (float) sumi, A[c]);  // _mm256_fmadd_ps, exact int -> float
        }
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        // hsum_float_8: ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
        float z = A[c] + __shfl_xor(A[c], 4, 8);
        z = z + __shfl_xor(z, 2, 8);
        z = z + __shfl_xor(z, 1, 8);
        if (l == 0 && live && i11 + c < g.ne11)
            *(float *) ((char *) dst + (i11 + c) * g.nb1 + i12 * g.nb2 + i13 * g.nb3 + row * sizeof(float)) = z;
    }
}

// Reference-order Q4_K / Q5_K mul_mat for the shapes the fused stream kernel does not take (3-D
// weight batches broadcast over r2 / r3, strided src1): the reference's AVX2 vec_dot
// (ggml-quants.c:7089-7152 Q4_K, :7920-8002 Q5_K) keeps eight int32 lanes `sumi` per superblock,
// lane l = sum over the four 64-element chunks j of sc[2j] * (4 low-nibble products at 4l..4l+3) +
// sc[2j+1] * (4 high-nibble products), then acc[l] = fma(d, (float) sumi[l], acc[l]) with
// d = y.d * fp16(x.d); the mins go to four f32 lanes acc_m[k] = fma(dmin, (float) (m[2k] S[2k] +
// m[2k+1] S[2k+1]), acc_m[k]) (Q4_K; dmin = -y.d * fp16(x.dmin)), or to one scalar the -mfma build
// contracts, summs = fma(dmin, (float) sum_k prod[k], summs) (Q5_K). Result hsum_float_8(acc) +
// ((acc_m0 + acc_m2) + (acc_m1 + acc_m3)), resp. + summs. Here eight lanes are the eight CPU lanes
// of one row (8 rows per wave), lanes 0..3 also the four acc_m lanes.
template <int NC, bool Q5>
__global__ __launch_bounds__(256) void k_mmv_kq_ord(const uint8_t * __restrict__ W, mi_act_q8 act, float * __restrict__ dst, mmv_geom g) {
    const int l = threadIdx.x & 7;
    const int64_t row = (int64_t) blockIdx.x * 32 + (threadIdx.x >> 3);
    const bool live = row < g.N;
    const int64_t rc = live ? row : g.N - 1;  // (dead groups run a valid row: no early exit before the shuffles)
    int64_t i11, i12, i13, i02, i03;
    mmv_coords(g, NC, i11, i12, i13, i02, i03);
    constexpr int BS = Q5 ? 176 : 144;
    const uint8_t * wrow = W + i02 * g.nb02 + i03 * g.nb03 + rc * g.nb01;
    const int nsb = (int) (g.K / 256);
    const int64_t col0 = i11 + g.ne11 * (i12 + g.ne12 * i13);

    float A[NC], M[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) A[c] = M[c] = 0.0f;

    for (int s = 0; s < nsb; s++) {
        const uint8_t * blk = wrow + (size_t) s * BS;
        const uint4 hdr = *(const uint4 *) blk;
        const float dw = mi_h2f((uint16_t) (hdr.x & 0xFFFF));
        const float dmw = mi_h2f((uint16_t) (hdr.x >> 16));
        uint32_t qlo[4], qhi[4];
        int sc[8], mn[8];
#pragma unroll
        for (int j = 0; j < 8; j++) mi_scale_min_k4(j, hdr.y, hdr.z, hdr.w, sc[j], mn[j]);
        const uint32_t hb = Q5 ? *(const uint32_t *) (blk + 16 + 4 * l) : 0u;  // qh bytes 4l..4l+3
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t q = *(const uint32_t *) (blk + (Q5 ? 48 : 16) + 32 * j + 4 * l);
            qlo[j] = q & 0x0F0F0F0Fu;
            qhi[j] = (q >> 4) & 0x0F0F0F0Fu;
            if constexpr (Q5) {
                qlo[j] |= ((hb >> (2 * j)) & 0x01010101u) << 4;
                qhi[j] |= ((hb >> (2 * j + 1)) & 0x01010101u) << 4;
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && i11 + c >= g.ne11) break;
            const int64_t col = col0 + c;
            const int8_t * aq = act.qs + col * g.K + (int64_t) s * 256 + 4 * l;
            int sumi = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int lo = mi_dot4((int) qlo[j], *(const int *) (aq + 64 * j), 0);
                const int hi = mi_dot4((int) qhi[j], *(const int *) (aq + 64 * j + 32), 0);
                sumi += sc[2 * j] * lo + sc[2 * j + 1] * hi;  // madd(scale_l, p16l) + madd(scale_h, p16h)
            }
            const float ya = act.d[col * nsb + s];
            A[c] = fmaf(ya * dw, (float) sumi, A[c]);  // _mm256_fmadd_ps(d, cvt(sumi), acc)
            const float dmin = -ya * dmw;
            const int16_t * S = act.s32 + col * (g.K / 32) + (int64_t) s * 8;
            if constexpr (!Q5) {
                if (l < 4) {
                    const int prod = mn[2 * l] * (int) S[2 * l] + mn[2 * l + 1] * (int) S[2 * l + 1];
                    M[c] = fmaf(dmin, (float) prod, M[c]);  // _mm_fmadd_ps(dmin, cvt(prod), acc_m)
                }
            } else {
                int tot = 0;
#pragma unroll
                for (int j = 0; j < 8; j++) tot += mn[j] * (int) S[j];
                M[c] = fmaf(dmin, (float) tot, M[c]);  // summs += dmin * hsum(prod), contracted
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        // hsum_float_8: ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
        float z = A[c] + __shfl_xor(A[c], 4, 8);
        z = z + __shfl_xor(z, 2, 8);
        z = z + __shfl_xor(z, 1, 8);
        float m = M[c];
        if constexpr (!Q5) {
            // acc_m + movehl(acc_m), then lane 0 + lane 1: (m0 + m2) + (m1 + m3)
            m = m + __shfl_xor(m, 2, 8);
            m = m + __shfl_xor(m, 1, 8);
        }
        if (l == 0 && live && i11 + c < g.ne11)
            *(float *) ((char *) dst + (i11 + c) * g.nb1 + i12 * g.nb2 + i13 * g.nb3 + row * sizeof(float)) = z + m;
    }
}

mmv_geom make_geom(const mi_mm_desc & m, int NC) {
    mmv_geom g;
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

} // namespace

#define MI_MMV_LAUNCH(KERNEL, NC, ...)                                                          \
    do {                                                                                         \
        const mmv_geom g = make_geom(m, NC);                                                     \
        const dim3 grid((unsigned) ((m.N + kRowsPerBlock - 1) / kRowsPerBlock),                  \
                        (unsigned) (g.col_chunks * m.ne12 * m.ne13));                            \
        hipLaunchKernelGGL((KERNEL<NC, ##__VA_ARGS__>), grid, dim3(256), 0, s, (const uint8_t *) m.W, \
                           act_or_x, m.dst, g);                                                  \
    } while (0)

#define MI_MMV_SWITCH(KERNEL, ...)                                  \
    switch (nc) {                                                   \
        case 1: MI_MMV_LAUNCH(KERNEL, 1, ##__VA_ARGS__); break;     \
        case 2: MI_MMV_LAUNCH(KERNEL, 2, ##__VA_ARGS__); break;     \
        case 3: MI_MMV_LAUNCH(KERNEL, 3, ##__VA_ARGS__); break;     \
        case 4: MI_MMV_LAUNCH(KERNEL, 4, ##__VA_ARGS__); break;     \
        default: MI_MMV_LAUNCH(KERNEL, 8, ##__VA_ARGS__); break;    \
    }

void mi_mul_mat_q(const mi_mm_desc & m, const mi_act_q8 & act, hipStream_t s) {
    const int nc = m.ne11 >= 5 ? 8 : (int) m.ne11;
    const mi_act_q8 act_or_x = act;
    if (mi_mmv_order() == 1 && (m.type == 2 || m.type == 8)) {  // reference CPU order: 8 rows per wave (mode 2 is a timing ablation of the fused kernel only)
        const bool q8 = m.type == 8;
#define MI_MMV_ORD_LAUNCH(NC)                                                                               \
        do {                                                                                                 \
            const mmv_geom g = make_geom(m, NC);                                                             \
            const dim3 grid((unsigned) ((m.N + 31) / 32), (unsigned) (g.col_chunks * m.ne12 * m.ne13));     \
            if (q8) hipLaunchKernelGGL((k_mmv_q0_ord<NC, true>), grid, dim3(256), 0, s, (const uint8_t *) m.W, act, m.dst, g); \
            else hipLaunchKernelGGL((k_mmv_q0_ord<NC, false>), grid, dim3(256), 0, s, (const uint8_t *) m.W, act, m.dst, g); \
        } while (0)
        switch (nc) {
            case 1: MI_MMV_ORD_LAUNCH(1); break;
            case 2: MI_MMV_ORD_LAUNCH(2); break;
            case 3: case 4: MI_MMV_ORD_LAUNCH(4); break;
            default: MI_MMV_ORD_LAUNCH(8); break;
        }
#undef MI_MMV_ORD_LAUNCH
        return;
    }
    if (mi_mmv_order() == 1 && (m.type == 12 || m.type == 13)) {  // reference CPU order, K-quants: 8 rows per wave
        const bool q5 = m.type == 13;
#define MI_MMV_KORD_LAUNCH(NC)                                                                               \
        do {                                                                                                  \
            const mmv_geom g = make_geom(m, NC);                                                              \
            const dim3 grid((unsigned) ((m.N + 31) / 32), (unsigned) (g.col_chunks * m.ne12 * m.ne13));      \
            if (q5) hipLaunchKernelGGL((k_mmv_kq_ord<NC, true>), grid, dim3(256), 0, s, (const uint8_t *) m.W, act, m.dst, g); \
            else hipLaunchKernelGGL((k_mmv_kq_ord<NC, false>), grid, dim3(256), 0, s, (const uint8_t *) m.W, act, m.dst, g); \
        } while (0)
        switch (nc) {
            case 1: MI_MMV_KORD_LAUNCH(1); break;
            case 2: MI_MMV_KORD_LAUNCH(2); break;
            case 3: case 4: MI_MMV_KORD_LAUNCH(4); break;
            default: MI_MMV_KORD_LAUNCH(8); break;
        }
#undef MI_MMV_KORD_LAUNCH
        return;
    }
    switch (m.type) {
        case 12: MI_MMV_SWITCH(k_mmv_kq, false); break;  // Q4_K
        case 13: MI_MMV_SWITCH(k_mmv_kq, true); break;   // Q5_K
        case 2:  MI_MMV_SWITCH(k_mmv_q0, false); break;  // Q4_0
        case 8:  MI_MMV_SWITCH(k_mmv_q0, true); break;   // Q8_0
        default: break;
    }
}
