// mmv_fused.hip -- decode-regime GGML_OP_MUL_MAT with the activation quantizer fused in, and
// several independent mul_mat nodes of one graph served by a single launch.
//
// Per workgroup (256 threads = 4 wave64s, RPW weight rows per wave):
//   1. every lane issues its weight loads for the first K-item of each of its RPW rows
//      (aligned 16-byte global loads straight to VGPRs; nothing else is waited on yet),
//   2. the workgroup quantizes the NC f32 activation columns of its group member into LDS with
//      the reference's exact Q8_K rounding (see quantize.hip) -- X is a few KB, L2-resident,
//   3. barrier, then integer dot products (v_dot4_i32_i8) of the prefetched weights against the
//      LDS activations; activations are read from LDS once per lane and reused for RPW rows.
// A launch covers up to kMaxMembers independent mul_mats with the same weight type and shape
// (blockIdx.x -> member, row block), so a decode graph's independent projections stream their
// weights back to back without launch gaps.
//
// Numerics are identical to mmv.hip (bit-exact activation quants, exact per-superblock int
// sums, f32 combination); reference dot products: ggml_vec_dot_q4_K_q8_K
// (src/ggml-quants.c:7007-7502), ggml_vec_dot_q5_K_q8_K (:7833-8378).

#include "mi355x_common.h"
#include "mi355x_kernels.h"

namespace {

// Q8_K quantization of one 256-superblock from registers (four floats per lane) into LDS.
// Same rounding sequence as k_quantize_q8_K / quantize_row_q8_K_reference.
__device__ __forceinline__ void quantize_sb_to_lds(float4 v4, int lane, int8_t * qs, float * d, int16_t * s32) {
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
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
    float dd = 0.0f;
    if (amax != 0.0f) {
        const float iscale = -127.f / vmax;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float t = __builtin_fmaf(iscale, v[i], 12582912.f);
            int q = (__float_as_int(t) & 0x007fffff) - 0x00400000;
            q = q < 127 ? q : 127;
            sum += q;
            packed |= ((uint32_t) (q & 0xFF)) << (8 * i);
        }
        dd = 1.0f / iscale;
    }
    *(uint32_t *) (qs + lane * 4) = packed;
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    if ((lane & 7) == 0) s32[lane >> 3] = (int16_t) sum;
    if (lane == 0) *d = dd;
}

struct kq_regs {
    uint4 hdr, qa, qb, ha, hb;
};

template <bool Q5>
__device__ __forceinline__ kq_regs kq_load(const uint8_t * blk, int j) {
    kq_regs r;
    r.hdr = *(const uint4 *) blk;
    const uint8_t * qp = blk + (Q5 ? 48 : 16) + 32 * j;
    r.qa = *(const uint4 *) qp;
    r.qb = *(const uint4 *) (qp + 16);
    if constexpr (Q5) {
        r.ha = *(const uint4 *) (blk + 16);
        r.hb = *(const uint4 *) (blk + 32);
    }
    return r;
}

// One K-item (superblock s, 64-element group j) of one row against NC LDS columns.
template <int NC, bool Q5>
__device__ __forceinline__ void kq_item(const kq_regs & r, int s, int j, int ncols, const int8_t * lqs, const float * ld,
                                        const int16_t * ls32, int64_t K, float (&acc)[NC]) {
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
    int sc0, m0, sc1, m1;
    mi_scale_min_k4(2 * j, r.hdr.y, r.hdr.z, r.hdr.w, sc0, m0);
    mi_scale_min_k4(2 * j + 1, r.hdr.y, r.hdr.z, r.hdr.w, sc1, m1);
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if (NC > 1 && c >= ncols) break;
        const int4 * a = (const int4 *) (lqs + c * K + (int64_t) s * 256 + 64 * j);
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
        const int ss = *(const int *) (ls32 + c * (K / 32) + s * 8 + 2 * j);
        const int summ = m0 * (int) (int16_t) (ss & 0xFFFF) + m1 * (ss >> 16);
        const float dy = ld[c * (K / 256) + s];
        acc[c] += dy * (dw * (float) sumi - dmw * (float) summ);
    }
}

template <int NC, bool Q5, int RPW>
__global__ __launch_bounds__(256) void k_mmv_kq_fused(mi_mmv_group g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int BS = Q5 ? 176 : 144;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int member = blockIdx.x / g.blocks_per_member;
    const int rb = blockIdx.x - member * g.blocks_per_member;
    const uint8_t * W = (const uint8_t *) g.m[member].W;
    const char * X = g.m[member].X;
    float * dst = g.m[member].dst;
    const int64_t K = g.K;
    const int nsb = (int) (K / 256);
    const int nitems = 4 * nsb;
    const int ncols = g.ncols;

    int8_t * lqs = (int8_t *) lds;
    float * ld = (float *) (lds + NC * K);
    int16_t * ls32 = (int16_t *) (lds + NC * K + NC * (K / 256) * 4);

    const int64_t row0 = ((int64_t) rb * 4 + wave) * RPW;

    // 1) weight prefetch for the first K-item of every row of this wave
    kq_regs pre[RPW];
    const bool have_first = lane < nitems;
    const int s0 = lane >> 2, j0 = lane & 3;
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        const int64_t row = row0 + r;
        if (have_first && row < g.N) pre[r] = kq_load<Q5>(W + row * g.nb01 + (size_t) s0 * BS, j0);
    }

    // 2) quantize X (NC columns) into LDS: wave w takes superblocks w, w+4, ...
    for (int p = wave; p < nsb * ncols; p += 4) {
        const int c = p / nsb, s = p - c * nsb;
        const float4 v4 = *(const float4 *) (X + c * g.xcol + ((size_t) s * 256 + lane * 4) * sizeof(float));
        quantize_sb_to_lds(v4, lane, lqs + c * K + s * 256, ld + c * nsb + s, ls32 + c * (K / 32) + s * 8);
    }
    __syncthreads();

    // 3) dot products
#pragma unroll
    for (int r = 0; r < RPW; r++) {
        const int64_t row = row0 + r;
        if (row >= g.N) break;  // wave-uniform
        float acc[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) acc[c] = 0.0f;
        if (have_first) kq_item<NC, Q5>(pre[r], s0, j0, ncols, lqs, ld, ls32, K, acc);
        for (int it = lane + 64; it < nitems; it += 64) {
            const int s = it >> 2, j = it & 3;
            const kq_regs rr = kq_load<Q5>(W + row * g.nb01 + (size_t) s * BS, j);
            kq_item<NC, Q5>(rr, s, j, ncols, lqs, ld, ls32, K, acc);
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const float v = mi_wave_sum(acc[c]);
            if (lane == 0 && c < ncols) *(float *) ((char *) dst + c * g.ycol + row * sizeof(float)) = v;
        }
    }
}

template <int NC, bool Q5>
void launch_kq(const mi_mmv_group & g, int rpw, hipStream_t s) {
    const size_t lds = (size_t) NC * (g.K + (g.K / 256) * 4 + (g.K / 32) * 2);
    const dim3 grid((unsigned) (g.blocks_per_member * g.n));
    switch (rpw) {
        case 1: hipLaunchKernelGGL((k_mmv_kq_fused<NC, Q5, 1>), grid, dim3(256), lds, s, g); break;
        case 2: hipLaunchKernelGGL((k_mmv_kq_fused<NC, Q5, 2>), grid, dim3(256), lds, s, g); break;
        default: hipLaunchKernelGGL((k_mmv_kq_fused<NC, Q5, 4>), grid, dim3(256), lds, s, g); break;
    }
}

template <bool Q5>
void launch_kq_nc(const mi_mmv_group & g, int rpw, hipStream_t s) {
    switch (g.ncols) {
        case 1: launch_kq<1, Q5>(g, rpw, s); break;
        case 2: launch_kq<2, Q5>(g, rpw, s); break;
        case 3: case 4: launch_kq<4, Q5>(g, rpw, s); break;
        default: launch_kq<8, Q5>(g, rpw, s); break;
    }
}

} // namespace

size_t mi_mmv_fused_lds_bytes(int type, int64_t K, int64_t ncols) {
    const int64_t nc = ncols <= 2 ? ncols : (ncols <= 4 ? 4 : 8);
    if (type == 12 || type == 13) return (size_t) nc * (K + (K / 256) * 4 + (K / 32) * 2);
    return SIZE_MAX;
}

bool mi_mmv_fused_supported(int type, int64_t K, int64_t ncols) {
    if (type != 12 && type != 13) return false;
    if (ncols < 1 || ncols > 8) return false;
    return mi_mmv_fused_lds_bytes(type, K, ncols) <= 64 * 1024;
}

void mi_mul_mat_q_fused(mi_mmv_group & g, hipStream_t s) {
    // rows per wave: amortize the per-workgroup activation quantization when there is enough
    // work to fill the chip (256 CUs x 4+ workgroups), otherwise maximize parallelism
    const int64_t total_rows = g.N * g.n;
    int rpw = 1;
    if (total_rows >= 256 * 16 * 4) rpw = 4;
    else if (total_rows >= 256 * 16 * 2) rpw = 2;
    g.blocks_per_member = (int) ((g.N + 4 * rpw - 1) / (4 * rpw));
    if (g.type == 12) launch_kq_nc<false>(g, rpw, s);
    else launch_kq_nc<true>(g, rpw, s);
}
