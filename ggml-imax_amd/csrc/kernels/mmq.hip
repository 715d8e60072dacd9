// mmq.hip -- batched GGML_OP_MUL_MAT (prompt / prefill regime, many activation columns) on the
// gfx950 matrix cores.
//
// Activations: the columns are first quantized exactly as the CPU path quantizes them
// (quantize.hip: q8_0 / q8_K, bit-identical) and then expanded once to f16(d * q) in a
// [ncols][K] buffer (k_act_to_f16) -- every column tile of the GEMM reads them from there
// instead of re-converting per tile. F16 weights use the f16-rounded activations of
// ggml_fp32_to_fp16_row, as the CPU does.
//
// GEMM (default k_mmq3, below): the same tiles and weight staging as k_mmq2, but each wave owns
// all 64 rows x 32 columns and takes its f16 activation fragments straight from a K-blocked copy
// of the activations ([K/16][ncols][16], written by the quantizer) into a register ring; only the
// dequantized weight slab passes through LDS. Measured on MI355X, Q4_K 4096x4096 B=512 (whole
// mul_mat incl. activation quantization): k_mmq2 53 us -> k_mmq3 43 us (395 TFLOP/s).
//
// GEMM (k_mmq2): workgroup = 4 wave64s, output tile 64 weight rows x 128 activation columns,
// each wave 32 rows x 64 columns = two v_mfma_f32_32x32x16_f16 per 16-deep K step sharing one
// A fragment. Per 64-deep K stage the workgroup dequantizes its 64 x 64 weight slab into LDS
// (16 consecutive weights per lane, the reference dequantize_row_* arithmetic:
// src/ggml-quants.c:980-998 q4_0, :1074-1088 q8_0, :2181-2218 q4_K, :2464-2507 q5_K) and copies
// the 128 x 64 activation slab; LDS is double-buffered, so the next stage's global loads are in
// flight while the MFMAs of the current one run, and the dequantization of the next stage
// follows the MFMAs (one barrier per stage).
//
// Relative to the CPU the only extra rounding is the f16 representation of the two operands
// (<= 2^-11 each) and the f32 MFMA accumulation order.
// Roofline: 2*N*K*B flops against weight bytes + 2*K*B (f16 activations) + 4*N*B -- at B=512,
// N=K=4096 ~17.2 GFLOP over ~17 MB: MFMA-bound (f16 dense ~2.5 PF/s).

#include <algorithm>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

namespace {

constexpr int BM = 64;          // weight rows per tile
constexpr int BN = 128;         // activation columns per tile
constexpr int BK = 64;          // K per LDS stage
constexpr int LDS_STRIDE = BK + 8;  // padded f16 row stride (144 B)
constexpr int kPF = 4;          // stages of global loads in flight (register ring)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t pack2h(float a, float b) {
    return (uint32_t) mi_f2h(a) | ((uint32_t) mi_f2h(b) << 16);
}

// ---- activations: q8 (+ scales) -> f16(d * q), [ncols][K] ----------------------------------
template <int QKA>
__global__ __launch_bounds__(256) void k_act_to_f16(mi_act_q8 act, int64_t K, uint16_t * __restrict__ out, int64_t total8) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < total8; i += (int64_t) gridDim.x * blockDim.x) {
        const int64_t e0 = i * 8;                 // 8 consecutive elements of one column
        const int64_t c = e0 / K, k = e0 - c * K;
        const float d = act.d[c * (K / QKA) + k / QKA];
        const int2 q = *(const int2 *) (act.qs + e0);
        const int qq[2] = {q.x, q.y};
        uint32_t h[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int w = qq[j >> 1];
            const int sh = 16 * (j & 1);
            h[j] = pack2h(d * (float) (int8_t) (w >> sh), d * (float) (int8_t) (w >> (sh + 8)));
        }
        *(uint4 *) (out + e0) = make_uint4(h[0], h[1], h[2], h[3]);
    }
}

// ---- weights: raw loads for 16 consecutive elements of one row, then dequantization ----------
// The raw registers are loaded before a stage's MFMAs and dequantized after them.
template <int TYPE>
struct WRaw;

// Q4_K / Q5_K: header (d, dmin, 12 scale bytes) + 16 quant bytes (+ 16 qh bytes)
template <int TYPE>
struct WRaw {
    static constexpr bool Q5 = TYPE == 13;
    static constexpr int BS = Q5 ? 176 : 144;
    uint4 hdr, qs, qh;
    __device__ __forceinline__ void load(const uint8_t * row, int64_t k) {
        // k: first of the 16 elements; within superblock s = k/256, 64-group j, part p = 0..3
        const uint8_t * blk = row + (k >> 8) * BS;
        const int p = (int) (k & 63) >> 4;  // 16-element part of the 64-group
        const int j = (int) (k & 255) >> 6;
        hdr = *(const uint4 *) blk;
        qs = *(const uint4 *) (blk + (Q5 ? 48 : 16) + 32 * j + 16 * (p & 1));
        if constexpr (Q5) qh = *(const uint4 *) (blk + 16 + 16 * (p & 1));
    }
    __device__ __forceinline__ void dequant(int64_t k, float (&v)[16]) const {
        const int p = (int) (k & 63) >> 4;
        const int j = (int) (k & 255) >> 6;
        const bool high = p >= 2;  // elements 32..63 of the group: high nibbles, subblock 2j+1
        const float d = mi_h2f((uint16_t) (hdr.x & 0xFFFF));
        const float dmin = mi_h2f((uint16_t) (hdr.x >> 16));
        int sc, m;
        mi_scale_min_k4(2 * j + (high ? 1 : 0), hdr.y, hdr.z, hdr.w, sc, m);
        const float d1 = d * sc, m1 = dmin * m;
        const uint32_t q[4] = {qs.x, qs.y, qs.z, qs.w};
        const uint32_t h[4] = {qh.x, qh.y, qh.z, qh.w};
        const int hbit = 2 * j + (high ? 1 : 0);
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t byte = (q[e >> 2] >> (8 * (e & 3))) & 0xFF;
            int val = high ? (int) (byte >> 4) : (int) (byte & 0xF);
            if constexpr (Q5) val += ((h[e >> 2] >> (8 * (e & 3) + hbit)) & 1) ? 16 : 0;
            v[e] = d1 * (float) val - m1;
        }
    }
};

// Q4_0 (18 B) / Q8_0 (34 B): 2-byte aligned blocks; dword loads re-aligned with v_alignbyte
template <bool Q8>
struct WRawQ0 {
    static constexpr int BS = Q8 ? 34 : 18;
    static constexpr int NW = Q8 ? 5 : 5;  // dwords covering the 16 quant bytes + misalignment
    uint32_t w[NW];
    uint32_t shift;
    uint32_t dbits;
    __device__ __forceinline__ void load(const uint8_t * row, int64_t k) {
        const uint8_t * blk = row + (k >> 5) * BS;
        const int half = (int) (k & 31) >> 4;  // Q8_0: bytes 16*half..; Q4_0: nibble half
        const uint8_t * qp = blk + 2 + (Q8 ? 16 * half : 0);
        const uintptr_t a = (uintptr_t) qp;
        const uint32_t * wp = (const uint32_t *) (a & ~(uintptr_t) 3);
        shift = (uint32_t) (a & 3);
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = wp[i];  // buffers carry 256 B of tail slack
        dbits = *(const uint16_t *) blk;
    }
    __device__ __forceinline__ void dequant(int64_t k, float (&v)[16]) const {
        const int half = (int) (k & 31) >> 4;
        const float d = mi_h2f((uint16_t) dbits);
        uint32_t t[4];
#pragma unroll
        for (int i = 0; i < 4; i++) t[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], shift);
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t byte = (t[e >> 2] >> (8 * (e & 3))) & 0xFF;
            if constexpr (Q8) {
                v[e] = (float) (int8_t) byte * d;
            } else {
                const int q = half ? (int) (byte >> 4) : (int) (byte & 0xF);
                v[e] = (float) (q - 8) * d;
            }
        }
    }
};

struct WRawF16 {
    uint4 a, b;
    __device__ __forceinline__ void load(const uint8_t * row, int64_t k) {
        a = *(const uint4 *) (row + k * 2);
        b = *(const uint4 *) (row + k * 2 + 16);
    }
};

template <int TYPE> struct raw_of { using T = WRaw<TYPE>; };
template <> struct raw_of<2> { using T = WRawQ0<false>; };
template <> struct raw_of<8> { using T = WRawQ0<true>; };
template <> struct raw_of<1> { using T = WRawF16; };

// ---- the GEMM ---------------------------------------------------------------------------------
template <int TYPE, int SK>
__global__ __launch_bounds__(256 * SK) void k_mmq2(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                              const uint16_t * __restrict__ xh, int64_t ncols, float * __restrict__ dst,
                                              size_t ycol) {
    // SK K-split groups of 4 waves each, every group with its own double-buffered LDS slabs
    __shared__ __attribute__((aligned(16))) _Float16 lds_a[SK][2][BM * LDS_STRIDE];
    __shared__ __attribute__((aligned(16))) _Float16 lds_b[SK][2][BN * LDS_STRIDE];
    using Raw = typename raw_of<TYPE>::T;
    const int grp = (int) threadIdx.x >> 8;
    const int tid = (int) threadIdx.x & 255;
    _Float16 (&la)[2][BM * LDS_STRIDE] = lds_a[grp];
    _Float16 (&lb)[2][BN * LDS_STRIDE] = lds_b[grp];
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t n0 = (int64_t) blockIdx.x * BM;
    const int64_t b0 = (int64_t) blockIdx.y * BN;
    const int wm = wave & 1, wb = wave >> 1;  // wave sub-tile: rows wm*32.., columns wb*64..

    // staging roles: weights -- thread t: row t/4, 16 elements at (t%4)*16;
    //                activations -- thread t: column t/2, 32 elements at (t%2)*32
    const int ar = tid >> 2, ak = (tid & 3) * 16;
    const int bc = tid >> 1, bk = (tid & 1) * 32;
    const int64_t arow = n0 + ar;
    const bool alive = arow < N;
    const uint8_t * wrow = W + (alive ? arow : 0) * nb01;
    const int64_t bcol = b0 + bc;
    const bool blive = bcol < ncols;
    const uint16_t * xcol = xh + (blive ? bcol : 0) * K;

    // register ring: the raw weights and activations of the next kPF stages are in flight while
    // the current stage's MFMAs run (a memory round trip is ~1 us = several stages of MFMA work)
    Raw raw[kPF];
    uint4 xb[kPF][4];
    auto load_stage = [&](int slot_unused, Raw & rw, uint4 (&xv)[4], int64_t k0) {
        (void) slot_unused;
        rw.load(wrow, k0 + ak);
#pragma unroll
        for (int i = 0; i < 4; i++) xv[i] = *(const uint4 *) (xcol + k0 + bk + 8 * i);
    };
    auto store_stage = [&](int buf, const Raw & rw, const uint4 (&xv)[4], int64_t k0) {
        _Float16 * pa = la[buf] + ar * LDS_STRIDE + ak;
        if constexpr (TYPE == 1) {
            *(uint4 *) pa = alive ? rw.a : make_uint4(0, 0, 0, 0);
            *(uint4 *) (pa + 8) = alive ? rw.b : make_uint4(0, 0, 0, 0);
        } else {
            float v[16];
            rw.dequant(k0 + ak, v);
            uint4 u0, u1;
            u0.x = pack2h(v[0], v[1]);   u0.y = pack2h(v[2], v[3]);   u0.z = pack2h(v[4], v[5]);   u0.w = pack2h(v[6], v[7]);
            u1.x = pack2h(v[8], v[9]);   u1.y = pack2h(v[10], v[11]); u1.z = pack2h(v[12], v[13]); u1.w = pack2h(v[14], v[15]);
            if (!alive) u0 = u1 = make_uint4(0, 0, 0, 0);
            *(uint4 *) pa = u0;
            *(uint4 *) (pa + 8) = u1;
        }
        _Float16 * pb = lb[buf] + bc * LDS_STRIDE + bk;
#pragma unroll
        for (int i = 0; i < 4; i++) *(uint4 *) (pb + 8 * i) = blive ? xv[i] : make_uint4(0, 0, 0, 0);
    };

    float16v acc0 = {}, acc1 = {};
    const int r = lane & 31, h = lane >> 5;
    const int64_t nst = K / BK / SK;  // stages of this group
    const int64_t kg = (int64_t) grp * nst * BK;  // first K of this group
    // K % 256 == 0 (mi_mmq_supported) -> nst is a multiple of kPF. Loads are unconditional
    // (clamped to the last stage): a predicated load makes the compiler drain vmcnt to 0.
#pragma unroll
    for (int u = 0; u < kPF; u++) load_stage(u, raw[u], xb[u], kg + (int64_t) (u < nst ? u : nst - 1) * BK);
    store_stage(0, raw[0], xb[0], kg);
    mi_lds_barrier();
    for (int64_t s0 = 0; s0 < nst; s0 += kPF) {
#pragma unroll
        for (int u = 0; u < kPF; u++) {
            const int64_t st = s0 + u;
            const int cur = (int) (st & 1);
            // slot u held stage st, already in LDS: refill it with stage st + kPF
            const int64_t nxt = st + kPF < nst ? st + kPF : nst - 1;
            load_stage(u, raw[u], xb[u], kg + nxt * BK);
            const _Float16 * pa = la[cur] + (wm * 32 + r) * LDS_STRIDE + 8 * h;
            const _Float16 * pb0 = lb[cur] + (wb * 64 + r) * LDS_STRIDE + 8 * h;
            const _Float16 * pb1 = pb0 + 32 * LDS_STRIDE;
#pragma unroll
            for (int kk = 0; kk < BK; kk += 16) {
                const half8 a = *(const half8 *) (pa + kk);
                const half8 x0 = *(const half8 *) (pb0 + kk);
                const half8 x1 = *(const half8 *) (pb1 + kk);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, x0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, x1, acc1, 0, 0, 0);
            }
            const int un = (u + 1) % kPF;
            store_stage(cur ^ 1, raw[un], xb[un], kg + (st + 1 < nst ? st + 1 : st) * BK);  // last: harmless rewrite
            mi_lds_barrier();  // keeps the ring's global loads in flight
        }
    }

    if constexpr (SK == 2) {
        // group 1 hands its partial sums to group 0 through its own activation slabs (36 KB, idle
        // once every wave is past its last MFMA); the sum is group0 + group1 in that fixed order
        float * red = (float *) &lds_b[1][0][0];
        mi_lds_barrier();
        if (grp == 1) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                red[(i * 2 + 0) * 256 + tid] = acc0[i];
                red[(i * 2 + 1) * 256 + tid] = acc1[i];
            }
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            acc0[i] += red[(i * 2 + 0) * 256 + tid];
            acc1[i] += red[(i * 2 + 1) * 256 + tid];
        }
    }

    // D[n][b]: column b = lane & 31, rows n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
    for (int half = 0; half < 2; half++) {
        const float16v & acc = half ? acc1 : acc0;
        const int64_t b = b0 + wb * 64 + 32 * half + (lane & 31);
        if (b >= ncols) continue;
        float * out = (float *) ((char *) dst + b * ycol);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int64_t n = n0 + wm * 32 + 8 * g + 4 * (lane >> 5);
            if (n + 3 < N) {
                *(float4 *) (out + n) = make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = acc[4 * g + e];
            }
        }
    }
}

// ---- k_mmq3: activations straight into MFMA operand registers ------------------------------------
// Same 64 x 128 workgroup tile and K split (SK groups of 4 waves) as k_mmq2, but each wave owns
// all 64 weight rows x its own 32 activation columns: the f16 activation fragment of a 16-deep
// K step is one 16-byte load per lane straight from xh (lane l: column l & 31, k + 8 (l >> 5)),
// held in a register ring kPF stages deep, so activations never pass through LDS (k_mmq2 wrote
// 16 KB and re-read it per stage and group, which left the LDS array, not the MFMAs, as the
// busiest unit). Only the dequantized 64 x 64 weight slab of a stage goes through LDS, written
// once per group and read by its four waves (two A fragments per K step each).
template <int TYPE, int SK, int NST, bool XCD, int ABL = 0>
__global__ __launch_bounds__(256 * SK) void k_mmq3(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                              const uint16_t * __restrict__ xh, int64_t ncols, float * __restrict__ dst,
                                              size_t ycol) {
    constexpr int kSlab = 2 * BM * LDS_STRIDE;  // halves per group: double-buffered weight slab
    constexpr int kRedBytes = 256 * 32 * 4;     // one group's partial tile (SK == 2 hand-off)
    constexpr int kSlabBytes = SK * kSlab * 2;
    __shared__ __attribute__((aligned(16))) char lds_raw[SK == 2 && kRedBytes > kSlabBytes ? kRedBytes : kSlabBytes];
    using Raw = typename raw_of<TYPE>::T;
    const int grp = (int) threadIdx.x >> 8;
    const int tid = (int) threadIdx.x & 255;
    _Float16 * la0 = (_Float16 *) lds_raw + grp * kSlab;
    const int wave = tid >> 6, lane = tid & 63;
    int64_t n0 = (int64_t) blockIdx.x * BM;
    int64_t b0 = (int64_t) blockIdx.y * BN;
    if constexpr (XCD) {
        // 1-D grid: workgroup i runs on XCD i % 8; give each XCD a contiguous run of tiles in
        // column-tile-major order, so an XCD's L2 holds few activation column tiles
        const int64_t nrt = (N + BM - 1) / BM, nct = (ncols + BN - 1) / BN, T = nrt * nct;
        const int64_t per = (T + 7) / 8;
        const int64_t t = (int64_t) (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (t >= T) return;
        n0 = (t % nrt) * BM;
        b0 = (t / nrt) * BN;
    }

    // weight staging: thread t dequantizes row t/4, 16 elements at (t%4)*16 (as k_mmq2)
    const int ar = tid >> 2, ak = (tid & 3) * 16;
    const int64_t arow = n0 + ar;
    const bool alive = arow < N;
    const uint8_t * wrow = W + (alive ? arow : 0) * nb01;
    // activation fragment: column b0 + 32 wave + (lane & 31), 8 halves at k + 8 (lane >> 5), from
    // the K-blocked layout xh[k / 16][ncols][16]: one K step of 32 columns = 1 KB contiguous
    const int64_t bcol = std::min<int64_t>(b0 + 32 * wave + (lane & 31), ncols - 1);
    const uint16_t * xcol = xh + bcol * 16 + 8 * (lane >> 5);
    const int64_t kstep = ncols * 16;  // halves per 16-deep K step

    Raw raw[kPF];
    half8 xb[kPF][BK / 16];
    auto load_stage = [&](Raw & rw, half8 (&xv)[BK / 16], int64_t k0) {
        if constexpr (ABL == 2) k0 = 0;  // ablation (timing only): every stage reads the first slab
        rw.load(wrow, k0 + ak);
#pragma unroll
        for (int i = 0; i < BK / 16; i++) xv[i] = *(const half8 *) (xcol + (k0 / 16 + i) * kstep);
    };
    auto store_stage = [&](int buf, const Raw & rw, int64_t k0) {
        _Float16 * pa = la0 + buf * (BM * LDS_STRIDE) + ar * LDS_STRIDE + ak;
        if constexpr (TYPE == 1) {
            *(uint4 *) pa = alive ? rw.a : make_uint4(0, 0, 0, 0);
            *(uint4 *) (pa + 8) = alive ? rw.b : make_uint4(0, 0, 0, 0);
        } else {
            float v[16];
            rw.dequant(k0 + ak, v);
            uint4 u0, u1;
            u0.x = pack2h(v[0], v[1]);   u0.y = pack2h(v[2], v[3]);   u0.z = pack2h(v[4], v[5]);   u0.w = pack2h(v[6], v[7]);
            u1.x = pack2h(v[8], v[9]);   u1.y = pack2h(v[10], v[11]); u1.z = pack2h(v[12], v[13]); u1.w = pack2h(v[14], v[15]);
            if (!alive) u0 = u1 = make_uint4(0, 0, 0, 0);
            *(uint4 *) pa = u0;
            *(uint4 *) (pa + 8) = u1;
        }
    };

    float16v acc0 = {}, acc1 = {};  // rows 0..31 / 32..63 of the tile, this wave's 32 columns
    const int r = lane & 31, h = lane >> 5;
    const int64_t nst = NST ? NST : K / BK / SK;
    const int64_t kg = (int64_t) grp * nst * BK;
#pragma unroll
    for (int u = 0; u < kPF; u++) load_stage(raw[u], xb[u], kg + (int64_t) (u < nst ? u : nst - 1) * BK);
    store_stage(0, raw[0], kg);
    mi_lds_barrier();
#pragma unroll (NST ? NST / kPF : 1)
    for (int64_t s0 = 0; s0 < nst; s0 += kPF) {
#pragma unroll
        for (int u = 0; u < kPF; u++) {
            const int64_t st = s0 + u;
            const int cur = (int) (st & 1);
            const _Float16 * pa0 = la0 + cur * (BM * LDS_STRIDE) + r * LDS_STRIDE + 8 * h;
            const _Float16 * pa1 = pa0 + 32 * LDS_STRIDE;
            // all of the stage's A fragments are requested before the first MFMA, so the LDS
            // latency is exposed once per stage rather than once per K step
            half8 a0[BK / 16], a1[BK / 16];
#pragma unroll
            for (int kk = 0; kk < BK / 16; kk++) {
                a0[kk] = *(const half8 *) (pa0 + 16 * kk);
                a1[kk] = *(const half8 *) (pa1 + 16 * kk);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < BK / 16; kk++) {
                if constexpr (ABL == 1) {  // ablation (timing only): no MFMAs
                    acc0[kk] += (float) a0[kk][0] * (float) xb[u][kk][0];
                    acc1[kk] += (float) a1[kk][1] * (float) xb[u][kk][1];
                } else {
                    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[kk], xb[u][kk], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[kk], xb[u][kk], acc1, 0, 0, 0);
                }
            }
            const int un = (u + 1) % kPF;
            store_stage(cur ^ 1, raw[un], kg + (st + 1 < nst ? st + 1 : st) * BK);  // last: harmless rewrite
            // slot u's activations are consumed and its weights are in LDS: refill with st + kPF
            const int64_t nxt = st + kPF < nst ? st + kPF : nst - 1;
            load_stage(raw[u], xb[u], kg + nxt * BK);
            mi_lds_barrier();  // keeps the ring's global loads in flight
        }
    }

    if constexpr (SK == 2) {
        // group 1 hands its partial tile to group 0 through LDS (the slabs are idle once every
        // wave is past its last MFMA); the sum is group0 + group1 in that fixed order
        float * red = (float *) lds_raw;
        __syncthreads();
        if (grp == 1) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                red[(i * 2 + 0) * 256 + tid] = acc0[i];
                red[(i * 2 + 1) * 256 + tid] = acc1[i];
            }
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            acc0[i] += red[(i * 2 + 0) * 256 + tid];
            acc1[i] += red[(i * 2 + 1) * 256 + tid];
        }
    }

    // D[n][b]: column b = lane & 31 of this wave's 32, rows n = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    const int64_t b = b0 + 32 * wave + (lane & 31);
    if (b >= ncols) return;
    float * out = (float *) ((char *) dst + b * ycol);
#pragma unroll
    for (int half = 0; half < 2; half++) {
        const float16v & acc = half ? acc1 : acc0;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int64_t n = n0 + 32 * half + 8 * g + 4 * (lane >> 5);
            if (n + 3 < N) {
                *(float4 *) (out + n) = make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = acc[4 * g + e];
            }
        }
    }
}

// ---- F16 weights, short prompts (<= 128 columns): 32 x 32 tiles, K split over the 4 waves -------
// k_mmq3's 64 x 128 tiles give N / 64 workgroups at B <= 128 (64 of the 256 CUs at N = 4096). Here
// a workgroup computes 32 weight rows x 32 prompt columns and wave w the K range [w K/4, (w+1) K/4)
// on v_mfma_f32_32x32x16_f16, 64 K per chunk, a register ring PF chunks deep:
//  * weights: coalesced loads (8 lanes per 128-byte row segment, 8 rows per instruction) into a
//    wave-private LDS tile (row stride 144 B: the MFMA fragment reads of 16 rows hit 16 distinct
//    bank quads), then one ds_read_b128 per lane and K step (row lane % 32, halves 8 (lane / 32));
//    LDS operations of one wave execute in order, so one buffer suffices;
//  * activations: the K-blocked f16 layout [K/16][ncols][16] -- a 16-deep step of 32 columns is 1 KB
//    contiguous, one 16-byte load per lane.
// (A first version loaded both operands row-per-lane straight from global memory: every lane
// touched its own cache line, TCP_TOTAL_CACHE_ACCESSES = 64 per load instruction, 19.5 us at B = 64,
// profiles/r03z_f16_pmc.txt.) The four partial tiles meet in LDS and are added in wave order.
// Products of fp16 values are exact in f32; only the summation order differs from the reference's
// ggml_vec_dot_f16 (~1e-7 relative).
// F32X: the activations are the f32 src1 itself (columns of K contiguous floats, xcs floats apart),
// rounded to f16 in the kernel as ggml_fp32_to_fp16_row does (RNE; ggml.c:605-616) right before
// their MFMA -- no separate conversion launch (each column tile's activations are converted by every
// row tile that reads them: VALU the memory-bound kernel has to spare)
template <int PF, int NW, bool F32X = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void k_mmf16p(const uint8_t * __restrict__ W, size_t nb01, int64_t K, int64_t N,
                                                   const uint16_t * __restrict__ xh, int64_t ncols, float * __restrict__ dst,
                                                   size_t ycol, const float * __restrict__ xf = nullptr, int64_t xcs = 0) {
    constexpr int kRow = 72;  // halves per LDS row (64 + 8 pad)
    __shared__ __attribute__((aligned(16))) _Float16 lw[NW][32 * kRow];
    __shared__ __attribute__((aligned(16))) float red[NW][16][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int lr = lane >> 3, lp = lane & 7;  // weight staging: row lr + 8 q, 16-byte piece lp
    const int64_t nrt = (N + 31) / 32;
    const int64_t n0 = ((int64_t) blockIdx.x % nrt) * 32, c0 = ((int64_t) blockIdx.x / nrt) * 32;
    const int64_t kw = K / NW;       // this wave's K range (K % (64 NW) == 0)
    const int nch = (int) (kw / 64);  // 64-deep chunks
    const uint8_t * wq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) wq[q] = W + std::min<int64_t>(n0 + lr + 8 * q, N - 1) * nb01 + (size_t) (w * kw) * 2 + 16 * lp;
    const int64_t col = std::min<int64_t>(c0 + r, ncols - 1);
    const uint16_t * xc = F32X ? nullptr : xh + ((size_t) (w * kw / 16) * ncols + col) * 16 + 8 * h;
    const float * xfc = F32X ? xf + col * xcs + w * kw + 8 * h : nullptr;
    const size_t xstep = (size_t) ncols * 16;  // halves per 16-deep K step
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // (a HIP uint4 array is not promoted to registers)
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    struct Chunk {
        u32x4 wv[4];
        u32x4 xv[F32X ? 0 : 4];
        f32x4 xw[F32X ? 8 : 0];  // F32X: the 8 floats of each 16-deep step's lane half
    };
    auto load = [&](Chunk & c, int i) {
        i = i < nch ? i : nch - 1;  // past the end: a harmless re-read of the last chunk
#pragma unroll
        for (int q = 0; q < 4; q++) c.wv[q] = *(const u32x4 *) (wq[q] + (size_t) i * 128);
        if constexpr (F32X) {
#pragma unroll
            for (int st = 0; st < 4; st++) {
                c.xw[2 * st] = *(const f32x4 *) (xfc + (size_t) i * 64 + 16 * st);
                c.xw[2 * st + 1] = *(const f32x4 *) (xfc + (size_t) i * 64 + 16 * st + 4);
            }
        } else {
#pragma unroll
            for (int st = 0; st < 4; st++) c.xv[st] = *(const u32x4 *) (xc + ((size_t) i * 4 + st) * xstep);
        }
    };
    auto xop = [&](const Chunk & c, int st) -> half8 {
        if constexpr (F32X) {
            half8 v;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                v[e] = (_Float16) c.xw[2 * st][e];
                v[4 + e] = (_Float16) c.xw[2 * st + 1][e];
            }
            return v;
        } else {
            return __builtin_bit_cast(half8, c.xv[st]);
        }
    };
    _Float16 * tile = lw[w];
    Chunk ring[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) load(ring[u], u);
    float16v acc = {};
    auto step = [&](Chunk & c, int i) {
        if (i >= nch) return;  // uniform
#pragma unroll
        for (int q = 0; q < 4; q++) *(u32x4 *) (tile + (lr + 8 * q) * kRow + 8 * lp) = c.wv[q];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const half8 a = *(const half8 *) (tile + r * kRow + 16 * st + 8 * h);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, xop(c, st), acc, 0, 0, 0);
        }
        load(c, i + PF);
    };
    static_assert(PF == 2 || PF == 3, "the ring below is written out for 2 or 3 chunks");
    for (int i0 = 0; i0 < nch; i0 += PF) {  // ring slots named statically (no private-array indexing)
        step(ring[0], i0);
        step(ring[1], i0 + 1);
        if constexpr (PF == 3) step(ring[PF - 1], i0 + 2);
    }
#pragma unroll
    for (int el = 0; el < 16; el++) red[w][el][lane] = acc[el];
    __syncthreads();
    // wave w < 4 stores accumulator elements 4w .. 4w + 3 (rows n0 + 8 w + 4 (l / 32) + e) of column
    // c0 + l % 32, the NW partial tiles added in wave order
    if (w >= 4) return;
    const int64_t b = c0 + r;
    const int64_t n = n0 + 8 * w + 4 * h;
    float y[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int el = 4 * w + e;
        y[e] = red[0][el][lane] + red[1][el][lane];
#pragma unroll
        for (int v = 2; v < NW; v++) y[e] = y[e] + red[v][el][lane];
    }
    if (b >= ncols) return;
    float * out = (float *) ((char *) dst + b * ycol);
    if (n + 3 < N) {
        *(float4 *) (out + n) = make_float4(y[0], y[1], y[2], y[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; e++) if (n + e < N) out[n + e] = y[e];
    }
}

} // namespace

bool mi_mmf16p_supported(int64_t K, int64_t N, size_t nb01, int64_t ncols, size_t ycol) {
    return mi_mmq_wants_blocked() && (g_mi_tuning.mmq_variant & (1 << 18)) == 0 && ncols > 8 && ncols <= 128 && K % 256 == 0 && N >= 1 &&
           nb01 % 16 == 0 && ycol % 16 == 0;
}

void mi_mul_mat_f16p(const void * W, size_t nb01, int64_t K, int64_t N, const uint16_t * xh, int64_t ncols, float * dst, size_t ycol,
                     hipStream_t s) {
    const int64_t tiles = ((N + 31) / 32) * ((ncols + 31) / 32);
    // variant bit 2^20: 8 waves per tile (K in eighths: twice the loads in flight per CU when the
    // tiles do not fill the chip twice over); K % 512 == 0
    const bool w8 = K % 512 == 0 && tiles < 512 && (g_mi_tuning.mmq_variant & (1 << 20)) != 0;
    if (w8) hipLaunchKernelGGL((k_mmf16p<3, 8>), dim3((unsigned) tiles), dim3(512), 0, s, (const uint8_t *) W, nb01, K, N, xh, ncols, dst, ycol);
    else hipLaunchKernelGGL((k_mmf16p<3, 4>), dim3((unsigned) tiles), dim3(256), 0, s, (const uint8_t *) W, nb01, K, N, xh, ncols, dst, ycol);
}

bool mi_mmf16p_f32_supported(int64_t K, int64_t N, size_t nb01, int64_t ncols, size_t ycol, const void * x, size_t xnb1) {
    // opt-in (variant bit 2^17): measured SLOWER than the separate conversion launch + k_mmf16p
    // (profiles/r04c_pf_f16.txt, 16 rotated weights: B=64 23.3 vs 17.3 us, B=32 22.9 vs 17.2 us) --
    // every row tile re-reads and re-converts its columns' f32 (twice the bytes of f16, 128 row tiles)
    // (diagnostic builds only)
    return MI_DIAG && mi_mmf16p_supported(K, N, nb01, ncols, ycol) && ((uintptr_t) x % 16) == 0 && xnb1 % 16 == 0 &&
           (g_mi_tuning.mmq_variant & (1 << 17)) != 0;
}

void mi_mul_mat_f16p_f32(const void * W, size_t nb01, int64_t K, int64_t N, const float * x, size_t xnb1, int64_t ncols, float * dst,
                         size_t ycol, hipStream_t s) {
#if MI_DIAG
    const int64_t tiles = ((N + 31) / 32) * ((ncols + 31) / 32);
    hipLaunchKernelGGL((k_mmf16p<2, 4, true>), dim3((unsigned) tiles), dim3(256), 0, s, (const uint8_t *) W, nb01, K, N, nullptr, ncols,
                       dst, ycol, x, (int64_t) (xnb1 / sizeof(float)));
#else
    (void) W; (void) nb01; (void) K; (void) N; (void) x; (void) xnb1; (void) ncols; (void) dst; (void) ycol; (void) s;
#endif
}

bool mi_mmq_wants_blocked() { return (g_mi_tuning.mmq_variant & 1) == 0; }

bool mi_mmq_supported(int type, int64_t K, size_t nb01, size_t ycol) {
    if (type != 12 && type != 13 && type != 2 && type != 8 && type != 1) return false;
    if (K % 256 != 0) return false;
    if (type == 1 && nb01 % 16 != 0) return false;
    return ycol % 16 == 0;
}

size_t mi_mmq_scratch_bytes(int type, int64_t K, int64_t ncols) {
    return type == 1 ? 0 : (size_t) K * ncols * sizeof(uint16_t);
}

void mi_mul_mat_mmq(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_q8 & act, const uint16_t * xh,
                    int64_t ncols, float * dst, size_t ycol, uint16_t * scratch, hipStream_t s) {
    if (type != 1 && xh == nullptr) {
        // quantized activations -> f16(d * q) once for all column tiles
        const int64_t total8 = K * ncols / 8;
        const unsigned grid = (unsigned) std::min<int64_t>((total8 + 255) / 256, 8192);
        if (type == 12 || type == 13) hipLaunchKernelGGL(k_act_to_f16<256>, dim3(grid), dim3(256), 0, s, act, K, scratch, total8);
        else hipLaunchKernelGGL(k_act_to_f16<32>, dim3(grid), dim3(256), 0, s, act, K, scratch, total8);
        xh = scratch;
    }
    const dim3 grid((unsigned) ((N + BM - 1) / BM), (unsigned) ((ncols + BN - 1) / BN));
    const uint8_t * w = (const uint8_t *) W;
    // split K over two 4-wave groups when each group keeps a whole number of ring turns: with
    // one 64x128 tile per CU (grid <= 256) a single 4-wave group leaves one wave per SIMD
    const bool sk2 = K % (2 * BK * kPF) == 0;
    // variant bits: 1 = k_mmq2 (activations via LDS), 2 = XCD-contiguous tile order, 8/16 = timing
    // ablations; k_mmq3 is fully unrolled over the K stages for the common K (the loop back-edge
    // of the runtime-K loop makes the compiler drain the load ring: measured 47 -> 43 us at 4096)
    const int var = g_mi_tuning.mmq_variant;
    const bool v3 = (var & 1) == 0;
    const bool xcd = (var & 2) != 0;
    const int abl = MI_DIAG ? (var >> 3) & 3 : 0;  // timing ablations (results invalid): make DIAG=1 only
    const int nst2 = sk2 ? (int) (K / BK / 2) : 0;
    const dim3 grid1((unsigned) (((grid.x * grid.y) + 7) / 8 * 8));
#define MI_MMQ3(T, NST) hipLaunchKernelGGL((k_mmq3<T, 2, NST, false>), grid, dim3(512), 0, s, w, nb01, K, N, xh, ncols, dst, ycol)
#define MI_MMQ_LAUNCH(T)                                                                                             \
    if (v3 && abl == 1 && nst2 == 32) hipLaunchKernelGGL((k_mmq3<T, 2, 32, false, 1>), grid, dim3(512), 0, s, w, nb01, K, N, xh, ncols, dst, ycol); \
    else if (v3 && abl == 2 && nst2 == 32) hipLaunchKernelGGL((k_mmq3<T, 2, 32, false, 2>), grid, dim3(512), 0, s, w, nb01, K, N, xh, ncols, dst, ycol); \
    else if (v3 && sk2 && xcd) hipLaunchKernelGGL((k_mmq3<T, 2, 0, true>), grid1, dim3(512), 0, s, w, nb01, K, N, xh, ncols, dst, ycol); \
    else if (v3 && nst2 == 32) MI_MMQ3(T, 32);                                                                       \
    else if (v3 && nst2 == 24) MI_MMQ3(T, 24);                                                                       \
    else if (v3 && nst2 == 16) MI_MMQ3(T, 16);                                                                       \
    else if (v3 && sk2) MI_MMQ3(T, 0);                                                                               \
    else if (v3) hipLaunchKernelGGL((k_mmq3<T, 1, 0, false>), grid, dim3(256), 0, s, w, nb01, K, N, xh, ncols, dst, ycol);       \
    else if (sk2) hipLaunchKernelGGL((k_mmq2<T, 2>), grid, dim3(512), 0, s, w, nb01, K, N, xh, ncols, dst, ycol);      \
    else hipLaunchKernelGGL((k_mmq2<T, 1>), grid, dim3(256), 0, s, w, nb01, K, N, xh, ncols, dst, ycol);
    switch (type) {
        case 12: MI_MMQ_LAUNCH(12) break;
        case 13: MI_MMQ_LAUNCH(13) break;
        case 2: MI_MMQ_LAUNCH(2) break;
        case 8: MI_MMQ_LAUNCH(8) break;
        case 1: MI_MMQ_LAUNCH(1) break;
        default: break;
    }
#undef MI_MMQ_LAUNCH
#undef MI_MMQ3
}
