// mmv_fused.hip -- decode-regime GGML_OP_MUL_MAT with the activation quantizer fused in, and
// several independent mul_mat nodes of one graph served by a single streaming launch.
//
// Structure (HBM-bound weight stream; MI355X_MICROARCH.md: 8 TB/s, ~6.3 TB/s achievable):
//   * grid = ~4 workgroups per CU; each workgroup owns a contiguous row range of ONE group
//     member (blockIdx.x -> member, row range), so the activation quantization below is paid
//     once per ~16-128 rows instead of once per row;
//   * per workgroup: issue the weight loads of the first row chunk (aligned 16-byte global loads
//     straight to VGPRs), quantize the member's NC f32 activation columns into LDS with the
//     reference's exact Q8_K rounding (quantize.hip), barrier;
//   * then each wave streams its chunks of RPW rows with one chunk of loads always in flight
//     (prefetch chunk k+1, then v_dot4_i32_i8 on chunk k); for K <= 4096 a lane's K-item is the
//     same for every row, so its activation slice is read from LDS once and kept in VGPRs.
// One K-item = (superblock s, 64-element group j): 16 B header + 32 B nibbles (+ 32 B qh for
// Q5_K), so a K=4096 Q4_K row is exactly one item per lane, three 16-byte loads.
//
// Numerics: bit-exact activation quants, exact per-item integer sums, f32 combination per
// superblock, i.e. ggml_vec_dot_q4_K_q8_K (src/ggml-quants.c:7007-7502) /
// ggml_vec_dot_q5_K_q8_K (:7833-8378) up to f32 summation order.

#include "mi355x_common.h"
#include "mi355x_kernels.h"

#include <stdlib.h>

namespace {

// Q8_K quantization of one 256-superblock (four floats per lane) into LDS; rounding identical
// to k_quantize_q8_K / quantize_row_q8_K_reference (mi_q8K_superblock).
__device__ __forceinline__ void quantize_sb_to_lds(float4 v4, int lane, int8_t * qs, float * d, int16_t * s32) {
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    uint32_t packed;
    int sum32;
    float dd;
    mi_q8K_superblock(v, lane, packed, sum32, dd);
    *(uint32_t *) (qs + lane * 4) = packed;
    if ((lane & 7) == 0) s32[lane >> 3] = (int16_t) sum32;
    if (lane == 0) *d = dd;
}

template <bool Q5>
struct kq_regs {
    uint4 hdr, qa, qb;
    uint4 ha, hb;  // Q5 only (dead for Q4)
};

template <bool Q5>
__device__ __forceinline__ void kq_load(kq_regs<Q5> & r, const uint8_t * blk, int j) {
    r.hdr = *(const uint4 *) blk;
    const uint8_t * qp = blk + (Q5 ? 48 : 16) + 32 * j;
    r.qa = *(const uint4 *) qp;
    r.qb = *(const uint4 *) (qp + 16);
    if constexpr (Q5) {
        r.ha = *(const uint4 *) (blk + 16);
        r.hb = *(const uint4 *) (blk + 32);
    }
}

// activation slice of one K-item for one column: 64 int8 (32 pair with low nibbles, 32 with
// high), the superblock scale and the two sums of 32 the item's sub-blocks need
struct act_item {
    int lo[8], hi[8];
    float d;
    int s0, s1;
};

__device__ __forceinline__ void act_load(act_item & a, const int8_t * lqs, const float * ld, const int16_t * ls32,
                                         int64_t K, int c, int s, int j) {
    const int4 * p = (const int4 *) (lqs + c * K + (int64_t) s * 256 + 64 * j);
    const int4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
    a.lo[0] = a0.x; a.lo[1] = a0.y; a.lo[2] = a0.z; a.lo[3] = a0.w;
    a.lo[4] = a1.x; a.lo[5] = a1.y; a.lo[6] = a1.z; a.lo[7] = a1.w;
    a.hi[0] = a2.x; a.hi[1] = a2.y; a.hi[2] = a2.z; a.hi[3] = a2.w;
    a.hi[4] = a3.x; a.hi[5] = a3.y; a.hi[6] = a3.z; a.hi[7] = a3.w;
    a.d = ld[c * (K / 256) + s];
    const int ss = *(const int *) (ls32 + c * (K / 32) + s * 8 + 2 * j);
    a.s0 = (int) (int16_t) (ss & 0xFFFF);
    a.s1 = ss >> 16;
}

// contribution of one K-item of one weight row to NC columns
template <int NC, bool Q5>
__device__ __forceinline__ void kq_dot(const kq_regs<Q5> & r, int j, const act_item (&a)[NC], int ncols, float (&acc)[NC]) {
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
        int lo = 0, hi = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            lo = mi_dot4((int) qlo[i], a[c].lo[i], lo);
            hi = mi_dot4((int) qhi[i], a[c].hi[i], hi);
        }
        const int sumi = sc0 * lo + sc1 * hi;
        const int summ = m0 * a[c].s0 + m1 * a[c].s1;
        acc[c] += a[c].d * (dw * (float) sumi - dmw * (float) summ);
    }
}

// One weight row of the stream: dot products of its K-items against the LDS / VGPR activations,
// wave reduction, store.
template <int NC, bool Q5, bool KEEP>
__device__ __forceinline__ void kq_row(const kq_regs<Q5> & first, const uint8_t * wrow, int64_t row, const mi_mmv_group & g,
                                       bool have_first, bool single_item, int s0, int j0, int lane, int nitems, int ncols,
                                       const act_item (&a0)[KEEP ? NC : 1], const int8_t * lqs, const float * ld,
                                       const int16_t * ls32, float * dst) {
    constexpr int BS = Q5 ? 176 : 144;
    const int64_t K = g.K;
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = 0.0f;
    if (have_first) {
        if constexpr (KEEP) {
            if (single_item) kq_dot<NC, Q5>(first, j0, *(const act_item(*)[NC]) a0, ncols, acc);
        }
        if (!KEEP || !single_item) {
            act_item a[NC];
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (NC > 1 && c >= ncols) break;
                act_load(a[c], lqs, ld, ls32, K, c, s0, j0);
            }
            kq_dot<NC, Q5>(first, j0, a, ncols, acc);
        }
    }
    for (int it = lane + 64; it < nitems; it += 64) {
        const int s = it >> 2, j = it & 3;
        kq_regs<Q5> rr;
        kq_load<Q5>(rr, wrow + (size_t) s * BS, j);
        act_item a[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            act_load(a[c], lqs, ld, ls32, K, c, s, j);
        }
        kq_dot<NC, Q5>(rr, j, a, ncols, acc);
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float v = mi_wave_sum_u(acc[c]);
        if (lane == 0 && c < ncols) *(float *) ((char *) dst + c * g.ycol + row * sizeof(float)) = v;
    }
}

// PD = rows of weight loads a wave keeps in flight ahead of the row it is computing.
template <int NC, bool Q5, int PD, bool KEEP_ACT, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_mmv_kq_stream(mi_mmv_group g) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int BS = Q5 ? 176 : 144;
    constexpr int NB = PD + 1;  // ring slots
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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

    const int64_t row_begin = (int64_t) rb * g.rows_per_block;
    const int64_t row_end = row_begin + g.rows_per_block < g.N ? row_begin + g.rows_per_block : g.N;
    // wave w streams rows row_begin + w, row_begin + w + 4, ...
    const int64_t nrows = row_end - row_begin > wave ? (row_end - row_begin - wave + 3) / 4 : 0;

    const bool single_item = nitems <= 64;
    const bool have_first = lane < nitems;
    const int s0 = lane >> 2, j0 = lane & 3;
    const size_t item_off = (size_t) s0 * BS;
    auto wrow_of = [&](int64_t k) { return W + (row_begin + 4 * k + wave) * g.nb01; };

    // 1) the first PD rows' weights in flight
    kq_regs<Q5> ring[NB];
#pragma unroll
    for (int u = 0; u < PD; u++) {
        if (have_first && u < nrows) kq_load<Q5>(ring[u], wrow_of(u) + item_off, j0);
    }

    // 2) quantize the member's activation columns into LDS (wave w: superblocks w, w+4, ...)
    {
        const int total = nsb * ncols;
        for (int p0 = wave; p0 < total; p0 += 16) {
            // unconditional loads (clamped index): a predicated load makes hipcc wait vmcnt(0)
            // per element instead of once for the batch
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = min(p0 + 4 * u, total - 1);
                const int c = p / nsb, sb = p - c * nsb;
                v[u] = *(const float4 *) (X + c * g.xcol + ((size_t) sb * 256 + lane * 4) * sizeof(float));
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = p0 + 4 * u;
                if (p < total) {
                    const int c = p / nsb, sb = p - c * nsb;
                    quantize_sb_to_lds(v[u], lane, lqs + c * K + sb * 256, ld + c * nsb + sb, ls32 + c * (K / 32) + sb * 8);
                }
            }
        }
    }
    __syncthreads();

    // few columns: the lane's activation slice may live in VGPRs for the whole stream
    constexpr bool KEEP = KEEP_ACT && NC <= 2;
    act_item a0[KEEP ? NC : 1];
    if (KEEP && single_item && have_first) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if (NC > 1 && c >= ncols) break;
            act_load(a0[c], lqs, ld, ls32, K, c, s0, j0);
        }
    }

    // 3) stream: ring slot u holds row k0+u; refill it with row k0+u+PD right before using it
    for (int64_t k0 = 0; k0 < nrows; k0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int64_t k = k0 + u;
            if (k >= nrows) break;  // wave-uniform
            if (have_first && k + PD < nrows) kq_load<Q5>(ring[(u + PD) % NB], wrow_of(k + PD) + item_off, j0);
            kq_row<NC, Q5, KEEP>(ring[u], wrow_of(k), row_begin + 4 * k + wave, g, have_first, single_item, s0, j0, lane,
                                 nitems, ncols, a0, lqs, ld, ls32, dst);
        }
    }
}

template <int NC, bool Q5>
void launch_kq(const mi_mmv_group & g, int pd, hipStream_t s) {
    const size_t lds = (size_t) NC * (g.K + (g.K / 256) * 4 + (g.K / 32) * 2);
    const dim3 grid((unsigned) (g.blocks_per_member * g.n));
    // variant codes (tuning): 10*PD + v, v: 0 = act in VGPRs, 1 = act from LDS, 2 = LDS + 5 waves/EU
    switch (pd) {
        case 10: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 1, true, 1>), grid, dim3(256), lds, s, g); break;
        case 11: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 1, false, 1>), grid, dim3(256), lds, s, g); break;
        case 12: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 1, false, 5>), grid, dim3(256), lds, s, g); break;
        case 20: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 2, true, 1>), grid, dim3(256), lds, s, g); break;
        case 21: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 2, false, 1>), grid, dim3(256), lds, s, g); break;
        case 22: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 2, false, 4>), grid, dim3(256), lds, s, g); break;
        case 31: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 3, false, 1>), grid, dim3(256), lds, s, g); break;
        case 32: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 3, false, 4>), grid, dim3(256), lds, s, g); break;
        case 41: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 4, false, 1>), grid, dim3(256), lds, s, g); break;
        default: hipLaunchKernelGGL((k_mmv_kq_stream<NC, Q5, 1, true, 1>), grid, dim3(256), lds, s, g); break;
    }
}

template <bool Q5>
void launch_kq_nc(const mi_mmv_group & g, int pd, hipStream_t s) {
    switch (g.ncols) {
        case 1: launch_kq<1, Q5>(g, pd, s); break;
        case 2: launch_kq<2, Q5>(g, pd, s); break;
        case 3: case 4: launch_kq<4, Q5>(g, pd, s); break;
        default: launch_kq<8, Q5>(g, pd, s); break;
    }
}

} // namespace

static int env_int(const char * name, int def) {
    const char * v = getenv(name);
    return v ? atoi(v) : def;
}

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

mi_tuning g_mi_tuning = {env_int("GGML_MI355X_MMV_BLOCKS", 1024), env_int("GGML_MI355X_MMV_VARIANT", 21)};

void mi_mul_mat_q_fused(mi_mmv_group & g, hipStream_t s) {
    // ~4 resident workgroups per CU over all members; each workgroup streams a row range
    const int target_blocks = g_mi_tuning.mmv_blocks;
    const int variant = g_mi_tuning.mmv_variant;
    int bpm = target_blocks / g.n;
    if (bpm < 1) bpm = 1;
    int64_t rows = (g.N + bpm - 1) / bpm;
    rows = (rows + 3) / 4 * 4;
    g.rows_per_block = rows;
    g.blocks_per_member = (int) ((g.N + rows - 1) / rows);
    if (g.type == 12) launch_kq_nc<false>(g, variant, s);
    else launch_kq_nc<true>(g, variant, s);
}
