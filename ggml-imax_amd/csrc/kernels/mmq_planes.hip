// mmq_planes.hip -- long-prompt Q4_K / Q5_K GEMM on weights repacked once into MFMA-ready int8
// planes, and the repack cache that keeps those planes next to the canonical blocks.
//
// The exact-integer formulation is mmq_exact.hip's (ggml-quants.c:7089-7152 vec_dot_q4_K_q8_K,
// :7920-8003 q5_K): per superblock T = sum_j sc_j sum_k q_k q8_k from NP int8 planes
// P_p = q * (bit field p of sc_j) on v_mfma_i32_32x32x32_i8, U = sum_j m_j S_j on one f16 MFMA,
// then the family's canonical combine (mmqx_pre, cfold) -- so this kernel's outputs are bit-identical
// to k_mmqt / k_mmqx / k_mmqp on the same inputs, and column shards stay bit-equal.
// What changes is where the dequantization happens: the canonical kernels expand the 4/5-bit
// quants and multiply by the sub-block scale fields inside the MFMA loop (13.9 VALU per MFMA for
// k_mmqt, profiles/r04x_mmqt_pmc.txt); here that runs once per weight upload (k_planes_repack) and
// the GEMM's VALU is the per-superblock combine alone.
//
// Repacked layout, per 32-row tile rt and superblock s (rows past N replicate row N-1), RB bytes at
// (rt * S + s) * RB:
//   [kk = 0..7][p = 0..NP-1] 1 KB: lane l's 16 bytes = rows rt*32 + (l & 31), K 32 kk + 16 (l >> 5)
//                                  .. + 15 of plane p (the MFMA B operand, one dwordx4 per lane)
//   U 1 KB: lane l's 8 halves [m_j, 64 m_j], j = 4 (l >> 5) .. + 3 of row l & 31
//   256 B: (d, dmin) of the 32 rows as f32 pairs
// Q4_K: NP = 2 (P0 = q (sc & 7), P1 = q (sc >> 3); T = (P1 << 3) + P0), RB = 17.25 KB per 8 KB of
// weights (2.16 B per weight); Q5_K: NP = 3 (q (sc >> 2p & 3)), RB = 25.25 KB.
//
// k_mmqr: 8 waves (two per SIMD), tile 64 weight rows x 128 prompt columns; wave (rw, cw) owns the
// 32 x 32 output tile of row tile rw and column group cw (NP int8 accumulators). A stage is one
// superblock: the activation quants, their U halves and d_a (36.5 KB) and the two row tiles' planes,
// U operands and (d, dmin) (34.5 KB for Q4_K) land in LDS by DMA, double-buffered, the next stage's
// pieces issued behind the current stage's MFMA steps (as k_mmqt). Per superblock and wave: NP x 8
// int8 MFMAs + one U MFMA, 3 ds_read_b128 per 32-deep step and the 16-element combine -- no
// dequantization VALU. Q4_K only: Q5_K's three planes (two 25 KB row tiles) do not fit two stages.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <atomic>
#include <iterator>
#include <map>
#include <mutex>

#include "mmq_exact_common.h"

namespace {

template <int TYPE>
struct PFmt {
    static constexpr int NP = XFmt<TYPE>::NP;
    static constexpr int PB = NP * 8 * 1024;  // plane bytes of one (tile, superblock)
    static constexpr int RB = PB + 1024 + 256;
};

// 6-bit scale and min of sub-block j from the 12 packed bytes (get_scale_min_k4, ggml-quants.c)
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t * q, int & sc, int & m) {
    if (j < 4) {
        sc = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

// one wave per (32-row tile, superblock): grid (S, tiles)
template <int TYPE>
__global__ __launch_bounds__(64) void k_planes_repack(const uint8_t * __restrict__ W, size_t nb01, int64_t N, int S, int64_t rt0,
                                                      char * __restrict__ planes) {
    using P = PFmt<TYPE>;
    constexpr int NP = P::NP;
    constexpr bool Q5 = TYPE == 13;
    constexpr int BS = XFmt<TYPE>::BS;
    const int lane = (int) threadIdx.x;
    const int r = lane & 31, h = lane >> 5;
    const int s = (int) blockIdx.x;
    const int64_t rt = rt0 + (int64_t) blockIdx.y;
    const int64_t n = std::min<int64_t>(rt * 32 + r, N - 1);
    const uint8_t * blk = W + (size_t) n * nb01 + (size_t) s * BS;
    const uint8_t * scales = blk + 4;
    const uint8_t * qh = blk + 16;                   // Q5_K high bits
    const uint8_t * qs = blk + (Q5 ? 48 : 16);
    char * out = planes + ((size_t) rt * S + s) * P::RB;
    for (int kk = 0; kk < 8; kk++) {
        int sc, m;
        scale_min_k4(kk, scales, sc, m);
        uint8_t v[NP][16];
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int idx = 16 * h + e;  // element of sub-block kk
            const uint8_t b = qs[32 * (kk >> 1) + idx];
            int q = (kk & 1) ? (b >> 4) : (b & 15);
            if constexpr (Q5) q |= ((qh[idx] >> kk) & 1) << 4;
#pragma unroll
            for (int p = 0; p < NP; p++) v[p][e] = (uint8_t) (q * (int) XFmt<TYPE>::factor(sc, p));
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            uint4 w;
            memcpy(&w, v[p], 16);
            *(uint4 *) (out + (kk * NP + p) * 1024 + lane * 16) = w;
        }
    }
    uint16_t u[8];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int sc, m;
        scale_min_k4(4 * h + q, scales, sc, m);
        u[2 * q] = mi_f2h((float) m);
        u[2 * q + 1] = mi_f2h((float) (64 * m));
    }
    uint4 uw;
    memcpy(&uw, u, 16);
    *(uint4 *) (out + P::PB + lane * 16) = uw;
    if (h == 0) {
        const uint16_t d = *(const uint16_t *) blk, dm = *(const uint16_t *) (blk + 2);
        *(float2 *) (out + P::PB + 1024 + r * 8) = make_float2(mi_h2f(d), mi_h2f(dm));
    }
}

// STAMP (diagnostic builds, mmq_long 24): wave 0 of every workgroup records s_memrealtime at entry
// (slot 0), after the prologue (1) and per superblock sb at 2 + 4 sb + {0 step start, 1 MFMAs
// issued, 2 combine done, 3 past the end-of-step wait and barrier}; ns slots per workgroup
template <int TYPE, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void k_mmqr(mi_mmx_group grp, uint64_t * st = nullptr, int ns = 0) {
    MI_MMX_MEMBER(grp);
    using P = PFmt<TYPE>;
    using F = XFmt<TYPE>;
    constexpr int NP = P::NP;
    constexpr int BM = 64, BN = 128;
    // one stage (a superblock) in LDS: [X 32 KB | XU 4 KB | D 512 B | W rt0 | W rt1 | dwdm 2 x 256 B]
    constexpr int XB = 8 * BN * 32;          // activation quants [kk][128 cols][32]
    constexpr int UB = BN * 32;              // U halves of the activations
    constexpr int DB = BN * 4;               // d_a
    constexpr int WT = P::PB + 1024;         // one row tile's planes + weight U operand
    constexpr int OW = XB + UB + DB;         // W region
    constexpr int OM = OW + 2 * WT;          // (d, dmin) of the two row tiles
    constexpr int SB = OM + 2 * 256;
    constexpr int NX = (XB + UB) / 1024;     // activation pieces (36)
    constexpr int NW1 = WT / 1024;           // weight pieces per row tile (17 / 25)
    constexpr int NPIECE = NX + 2 * NW1;     // 1-KB DMA pieces per stage (70 for Q4_K)
    constexpr int NI = (NPIECE + 7) / 8;     // pieces per wave (the last waves may have one fewer)
    __shared__ __attribute__((aligned(16))) char lds[2 * SB];

    const char * __restrict__ planes = grp.m[mmx_i_].planes;
    auto stamp = [&](int slot) {
        if constexpr (STAMP) {
            if (threadIdx.x == 0) st[(size_t) blockIdx.x * ns + slot] = __builtin_amdgcn_s_memrealtime();
        }
    };
    stamp(0);
    const int tid = (int) threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int rw = w & 1, cw = w >> 1;  // wave: row tile rw (32 rows) x column group cw (32 columns)
    const int64_t ncols = act.ncols;
    const int S = (int) (K / 256);
    const int gs = cfold_gs(S);
    const int64_t nrt = (N + BM - 1) / BM;
    const int64_t n0 = (mmx_tile % nrt) * BM, c0 = (mmx_tile / nrt) * BN;
    const int64_t rt_last = (N + 31) / 32 - 1;
    auto col_of = [&](int c) { return (uint32_t) std::min<int64_t>(c0 + c, ncols - 1); };

    // ---- staging: piece q = w + 8 i: q < 32 activation step kk = q >> 2, 32-column group q & 3
    // (16-byte halves swapped for columns 16-31 of a group: conflict-free ds_read_b128); q < 36 the
    // activation U halves of group q - 32; else weight piece (q - 36) % NW1 of row tile (q - 36) / NW1
    // (planes then U, lane-linear as stored). Small DMAs (4 bytes per lane): waves 0, 1 d_a, waves
    // 2, 3 the (d, dmin) pairs of row tile w - 2.
    const char * pbase[NI];
    uint32_t pstride[NI], poff[NI], pdst[NI];
    bool pvalid[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int q = w + 8 * i;
        pvalid[i] = q < NPIECE;
        const uint32_t half = 16 * ((lane & 1) ^ ((lane >> 5) & 1));
        if (q < 32) {
            pdst[i] = (uint32_t) ((q >> 2) * (BN * 32) + (q & 3) * 1024);
            pbase[i] = (const char *) act.xq + (size_t) (q >> 2) * ncols * 32;
            pstride[i] = 8 * (uint32_t) ncols * 32;
            poff[i] = col_of(32 * (q & 3) + (lane >> 1)) * 32 + half;
        } else if (q < NX) {
            pdst[i] = (uint32_t) (XB + (q - 32) * 1024);
            pbase[i] = (const char *) act.xu;
            pstride[i] = (uint32_t) ncols * 32;
            poff[i] = col_of(32 * (q - 32) + (lane >> 1)) * 32 + half;
        } else {
            const int t = (q - NX) / NW1, j = (q - NX) % NW1;
            const int64_t rt = std::min<int64_t>(n0 / 32 + t, rt_last);
            pdst[i] = (uint32_t) (OW + t * WT + j * 1024);
            pbase[i] = planes + (size_t) rt * S * P::RB;
            pstride[i] = (uint32_t) P::RB;
            poff[i] = (uint32_t) (j * 1024 + lane * 16);
        }
    }
    const char * sbase;
    uint32_t sstride, soff, sdst;
    if (w < 2) {
        sbase = (const char *) act.xd;
        sstride = (uint32_t) ncols * 4;
        soff = col_of(64 * w + lane) * 4;
        sdst = (uint32_t) (XB + UB + 256 * w);
    } else {
        const int64_t rt = std::min<int64_t>(n0 / 32 + (w & 1), rt_last);
        sbase = planes + (size_t) rt * S * P::RB + P::PB + 1024;
        sstride = (uint32_t) P::RB;
        soff = (uint32_t) lane * 4;
        sdst = (uint32_t) (OM + 256 * (w & 1));
    }
    auto stage_piece = [&](int sb, int i) {  // (sb wave-uniform; past the end: nothing)
        if (sb >= S) return;
        char * sbuf = lds + (sb & 1) * SB;
        if (i < NI) {
            if (pvalid[i]) mi_glds16(pbase[i] + (size_t) sb * pstride[i] + poff[i], mi_lds_addr(sbuf + pdst[i]));
        } else if (w < 4) {
            mi_glds4(sbase + (size_t) sb * sstride + soff, mi_lds_addr(sbuf + sdst));
        }
    };

    const uint32_t xoff = (uint32_t) (cw * 1024 + r * 32 + 16 * (h ^ ((r >> 4) & 1)));
    const uint32_t woff = (uint32_t) (OW + rw * WT + lane * 16);
    f32x16 y = f32x16(-0.0f), lo = f32x16(-0.0f), gsum = {};
    i32x16 acc[NP];

    auto step = [&](int sb) {
        const char * base = lds + (sb & 1) * SB;
        stamp(2 + 4 * sb);
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const i32x4 xa = *(const i32x4 *) (base + kk * (BN * 32) + xoff);
            i32x4 b[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) b[p] = *(const i32x4 *) (base + woff + (kk * NP + p) * 1024);
            stage_piece(sb + 1, kk);  // the next stage, one DMA piece per step
#pragma unroll
            for (int p = 0; p < NP; p++) acc[p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa, b[p], kk == 0 ? i32x16{} : acc[p], 0, 0, 0);
        }
#pragma unroll
        for (int i = 8; i <= NI; i++) stage_piece(sb + 1, i);
        stamp(3 + 4 * sb);
        // combine: U on the f16 MFMA, mmqx_pre per element, canonical fold
        const half8 mu = *(const half8 *) (base + woff + P::PB);
        const float2 dd = *(const float2 *) (base + OM + rw * 256 + r * 8);
        const half8 xu = *(const half8 *) (base + XB + xoff);
        const f32x16 Uv = __builtin_amdgcn_mfma_f32_32x32x16_f16(xu, mu, f32x16{}, 0, 0, 0);
        const float * dal = (const float *) (base + XB + UB) + 32 * cw;
        f32x16 tv, dv;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float2 d2 = *(const float2 *) &dal[8 * (j >> 1) + 4 * h + 2 * (j & 1)];
            dv[2 * j] = d2.x;
            dv[2 * j + 1] = d2.y;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int el = 2 * j + e;
                int T = acc[NP - 1][el];
#pragma unroll
                for (int p = NP - 2; p >= 0; p--) T = (T << F::SHIFT) + acc[p][el];
                tv[el] = mmqx_pre(T, Uv[el], dd.x, dd.y);
            }
        }
        cfold_vec(gsum, y, lo, tv, dv, sb, gs, S);
        stamp(4 + 4 * sb);
    };

#pragma unroll
    for (int i = 0; i <= NI; i++) stage_piece(0, i);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    stamp(1);
    for (int sb = 0; sb < S; sb++) {
        step(sb);
        // the next stage has landed (every global load of this kernel is a DMA), every wave is done
        // with this stage's buffer
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        stamp(5 + 4 * sb);
    }

    const int64_t n = n0 + 32 * rw + r;
    if (n >= N) return;
    const f32x16 yv = lo + y;  // cfold_end
#pragma unroll
    for (int el = 0; el < 16; el++) {
        const int64_t c = c0 + 32 * cw + (el & 3) + 8 * (el >> 2) + 4 * h;
        if (c < ncols) *(float *) ((char *) dst + c * ycol + n * sizeof(float)) = yv[el];
    }
}

// ---- Q4_0 decode weights, 16-byte aligned (round 6) -------------------------------------------------
// The canonical Q4_0 block (d f16, 16 bytes of nibbles; 18 bytes, ggml-common.h block_q4_0) leaves
// the quants 2-byte aligned, so the tree-order GEMV (FmtQ0Pair) loads each 36-byte block pair with
// dword loads that straddle 16-byte and cache-line boundaries. The repacked copy of row n (the same
// bytes, K / 32 * 18 per row, rows packed) puts the quants first and the scales after them:
//   [b * 16 .. b * 16 + 15]   block b's 16 quant bytes        (pair p = 32 bytes at 32 p)
//   [nblk * 16 + 2 b]        block b's d                     (pair p = one dword at nblk * 16 + 4 p)
// so a lane's pair is two aligned dwordx4 loads plus one dword, and consecutive lanes read
// consecutive bytes (FmtQ0R, mmv_fused_impl.h). One thread per block, grid (N, row chunks).
__global__ __launch_bounds__(256) void k_q40_repack(const uint8_t * __restrict__ W, size_t nb01, int64_t nblk, uint8_t * __restrict__ out) {
    const int64_t n = blockIdx.x;
    const int64_t b = (int64_t) blockIdx.y * 256 + threadIdx.x;
    if (b >= nblk) return;
    const uint16_t * src = (const uint16_t *) (W + (size_t) n * nb01 + (size_t) b * 18);  // 2-byte aligned
    uint16_t h[9];
#pragma unroll
    for (int i = 0; i < 9; i++) h[i] = src[i];
    uint8_t * row = out + (size_t) n * (size_t) nblk * 18;
    uint4 q;
    q.x = h[1] | ((uint32_t) h[2] << 16);
    q.y = h[3] | ((uint32_t) h[4] << 16);
    q.z = h[5] | ((uint32_t) h[6] << 16);
    q.w = h[7] | ((uint32_t) h[8] << 16);
    *(uint4 *) (row + (size_t) b * 16) = q;
    *(uint16_t *) (row + (size_t) nblk * 16 + (size_t) b * 2) = h[0];
}

// Q8_0 (d f16 + 32 quant bytes = 34 B, block_q8_0): the same reordering -- per row the blocks' 32
// quant bytes (block b at 32 b), then their scales (at K + 2 b) -- read by FmtQ8R.
__global__ __launch_bounds__(256) void k_q80_repack(const uint8_t * __restrict__ W, size_t nb01, int64_t nblk, uint8_t * __restrict__ out) {
    const int64_t n = blockIdx.x;
    const int64_t b = (int64_t) blockIdx.y * 256 + threadIdx.x;
    if (b >= nblk) return;
    const uint16_t * src = (const uint16_t *) (W + (size_t) n * nb01 + (size_t) b * 34);  // 2-byte aligned
    uint16_t h[17];
#pragma unroll
    for (int i = 0; i < 17; i++) h[i] = src[i];
    uint8_t * row = out + (size_t) n * (size_t) nblk * 34;
#pragma unroll
    for (int v = 0; v < 2; v++) {
        uint4 q;
        q.x = h[1 + 8 * v] | ((uint32_t) h[2 + 8 * v] << 16);
        q.y = h[3 + 8 * v] | ((uint32_t) h[4 + 8 * v] << 16);
        q.z = h[5 + 8 * v] | ((uint32_t) h[6 + 8 * v] << 16);
        q.w = h[7 + 8 * v] | ((uint32_t) h[8 + 8 * v] << 16);
        *(uint4 *) (row + (size_t) b * 32 + 16 * v) = q;
    }
    *(uint16_t *) (row + (size_t) nblk * 32 + (size_t) b * 2) = h[0];
}

// ---- the cache ------------------------------------------------------------------------------------
struct PlanesEntry {
    int type;
    size_t nb01;
    int64_t K, N;
    size_t span;   // bytes of W covered: (N - 1) nb01 + S * BS
    char * planes;
    size_t bytes;
    int device;
};
std::mutex g_planes_mu;
std::map<uintptr_t, PlanesEntry> g_planes;  // keyed by W
std::atomic<size_t> g_planes_n{0};           // g_planes.size(), readable without the lock
std::atomic<uint64_t> g_planes_gen{0};       // bumped whenever an entry is created or dropped

int planes_enabled() { return g_mi_tuning.planes; }

void launch_repack(const PlanesEntry & e, const void * W, hipStream_t s) {
    if (e.type == 2 || e.type == 8) {
        const int64_t nblk = e.K / 32;
        const dim3 grid((unsigned) e.N, (unsigned) ((nblk + 255) / 256));
        if (e.type == 2) hipLaunchKernelGGL(k_q40_repack, grid, dim3(256), 0, s, (const uint8_t *) W, e.nb01, nblk, (uint8_t *) e.planes);
        else hipLaunchKernelGGL(k_q80_repack, grid, dim3(256), 0, s, (const uint8_t *) W, e.nb01, nblk, (uint8_t *) e.planes);
        return;
    }
    const int S = (int) (e.K / 256);
    const int64_t nt = (e.N + 31) / 32;
    const dim3 grid((unsigned) S, (unsigned) nt);
    if (e.type == 12) hipLaunchKernelGGL((k_planes_repack<12>), grid, dim3(64), 0, s, (const uint8_t *) W, e.nb01, e.N, S, (int64_t) 0, e.planes);
    else hipLaunchKernelGGL((k_planes_repack<13>), grid, dim3(64), 0, s, (const uint8_t *) W, e.nb01, e.N, S, (int64_t) 0, e.planes);
}

} // namespace

const char * mi_planes_get(int type, const void * W, size_t nb01, int64_t K, int64_t N, hipStream_t s) {
    // (Q4_K: the planes kernel beats the canonical one; Q5_K's 3 planes do not fit its LDS stages.
    // Q4_0 / Q8_0: the 16-byte-aligned decode copies, g_mi_tuning.q40r / q80r)
    const bool q0 = type == 2 || type == 8;  // the aligned decode copies (Q4_0 / Q8_0)
    if (type == 2 ? !g_mi_tuning.q40r : type == 8 ? !g_mi_tuning.q80r : (!planes_enabled() || type != 12)) return nullptr;
    if (K % 256 != 0 || N <= 0 || !W) return nullptr;
    const int64_t row_min = q0 ? K / 32 * (type == 2 ? 18 : 34) : K / 256 * (type == 12 ? 144 : 176);
    if (nb01 % (q0 ? 2 : 4) != 0 || (int64_t) nb01 < row_min) return nullptr;
    std::lock_guard<std::mutex> lk(g_planes_mu);
    auto it = g_planes.find((uintptr_t) W);
    if (it != g_planes.end()) {
        const PlanesEntry & e = it->second;
        if (e.type == type && e.nb01 == nb01 && e.K == K && e.N >= N) return e.planes;
        return nullptr;  // the same address seen with another shape: the canonical kernels
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        (void) hipGetLastError();
        return nullptr;  // no allocation inside a capture: this launch takes the canonical kernels
    }
    // entries never overlap one another (mi_planes_refresh relies on it): a W inside another
    // entry's span, or one whose span reaches the next entry, keeps the canonical kernels
    const uintptr_t wa = (uintptr_t) W, wb = wa + (size_t) (N - 1) * nb01 + (size_t) row_min;
    {
        auto nx = g_planes.lower_bound(wa);
        if (nx != g_planes.end() && nx->first < wb) return nullptr;
        if (nx != g_planes.begin() && std::prev(nx)->first + std::prev(nx)->second.span > wa) return nullptr;
    }
    PlanesEntry e;
    e.type = type;
    e.nb01 = nb01;
    e.K = K;
    e.N = N;
    e.span = (size_t) (N - 1) * nb01 + (size_t) row_min;
    e.bytes = q0 ? (size_t) N * (size_t) row_min : (size_t) ((N + 31) / 32) * (K / 256) * (type == 12 ? PFmt<12>::RB : PFmt<13>::RB);
    (void) hipGetDevice(&e.device);
    void * p = nullptr;
    if (hipMalloc(&p, e.bytes) != hipSuccess) {
        (void) hipGetLastError();
        return nullptr;  // out of memory: the canonical kernels
    }
    e.planes = (char *) p;
    launch_repack(e, W, s);
    g_planes[(uintptr_t) W] = e;
    g_planes_n = g_planes.size();
    g_planes_gen++;
    return e.planes;
}

void mi_planes_refresh(const void * lo, size_t bytes, hipStream_t s) {
    if (bytes == 0 || mi_planes_count() == 0) return;
    std::lock_guard<std::mutex> lk(g_planes_mu);
    if (g_planes.empty()) return;
    const uintptr_t a = (uintptr_t) lo, b = a + bytes;
    int dev = -1;
    (void) hipGetDevice(&dev);
    // entries do not overlap one another: the only one that can start below a is the last such
    auto it = g_planes.lower_bound(a);
    if (it != g_planes.begin()) --it;
    for (; it != g_planes.end() && it->first < b; ++it) {
        const PlanesEntry & e = it->second;
        if (it->first + e.span <= a || e.device != dev) continue;
        launch_repack(e, (const void *) it->first, s);
    }
}

void mi_planes_drop(const void * lo, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_planes_mu);
    const uintptr_t a = (uintptr_t) lo, b = a + bytes;
    for (auto it = g_planes.begin(); it != g_planes.end();) {
        if (it->first >= a && it->first < b) {
            (void) hipFree(it->second.planes);
            it = g_planes.erase(it);
            g_planes_gen++;
        } else {
            ++it;
        }
    }
    g_planes_n = g_planes.size();
}

size_t mi_planes_count() { return g_planes_n.load(std::memory_order_relaxed); }

uint64_t mi_planes_generation() { return g_planes_gen.load(std::memory_order_relaxed); }

size_t mi_planes_bytes() {
    std::lock_guard<std::mutex> lk(g_planes_mu);
    size_t t = 0;
    for (const auto & kv : g_planes) t += kv.second.bytes;
    return t;
}

bool mi_mul_mat_mmqr_group(mi_mmx_group & g, hipStream_t s) {
    if (g.n <= 0 || g.type != 12 || g.K % 256 != 0) return false;
    int64_t tiles = 0;
    for (int i = 0; i < g.n; i++) {
        if (!g.m[i].planes) return false;
        g.m[i].tile_begin = tiles;
        tiles += ((g.m[i].N + 63) / 64) * ((g.m[i].act.ncols + 127) / 128);
    }
    const int var = g_mi_tuning.mmq_variant;
#if MI_DIAG
    if (g_mi_tuning.mmq_long == 24) {  // per-step stamps (tools/mmqr_stamps.py)
        const int ns = ((4 * (int) (g.K / 256) + 2 + 7) / 8) * 8;
        uint64_t * st = mi_stamp_take("k_mmqr", (unsigned) (tiles * ns / 8));
        if (st) {
            hipLaunchKernelGGL((k_mmqr<12, true>), dim3((unsigned) tiles), dim3(512), 0, s, g, st, ns);
            return true;
        }
    }
#endif
    (void) var;
    hipLaunchKernelGGL((k_mmqr<12>), dim3((unsigned) tiles), dim3(512), 0, s, g);
    return true;
}
