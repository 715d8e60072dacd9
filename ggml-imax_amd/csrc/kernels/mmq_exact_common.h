// mmq_exact_common.h -- device helpers shared by the exact-integer Q4_K / Q5_K prefill GEMMs
// (mmq_exact.hip: the kernels on canonical weight blocks; mmq_planes.hip: the kernel on repacked
// MFMA planes). The canonical combine (mmqx_pre + cfold) lives here so every kernel of the family
// produces the same bits for the same output.
#pragma once

#include <algorithm>
#include <type_traits>
#include <utility>

#include "mi355x_common.h"
#include "mi355x_kernels.h"

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

// the canonical per-superblock value t = d_w T - dmin_w U (every kernel of the family computes
// exactly this); the group sums then take da * t fused: g = fma(da, t, g) (cfold below)
__device__ __forceinline__ float mmqx_pre(int T, float U, float dw, float dm) {
    return __builtin_fmaf(-dm, U, dw * (float) T);
}
__device__ __forceinline__ f32x16 fma_vec(const f32x16 & a, const f32x16 & b, const f32x16 & c) {
    f32x16 r;
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = __builtin_fmaf(a[i], b[i], c[i]);
    return r;
}

// The canonical combine order of an output's superblock terms, shared by every kernel of this
// file (so any column shard of a prompt gives the same bits whichever kernel computes it): the S
// superblocks form kCfoldGroups contiguous groups of gs = ceil(S / kCfoldGroups) (the last ones
// shorter or empty), each group's terms are accumulated in superblock order from -0 with the
// activation scale fused in (g = -0; g = fma(d_a, t, g); ...: round-4 form, one VALU op per
// element and superblock fewer than a separate product and sum); the sums
// of groups 0..3 and of groups 4..7 are left-folded separately from -0 (lo = lo + g_0 ...; hi = hi +
// g_4 ...) and y = lo + hi. (-0 + x == x for every float x, signed zeros and NaNs included, so an
// empty half changes nothing.) The pipelined kernel (k_mmqp) gives each group to one of its waves,
// the split-K kernel (k_mmqt) each half to one wave of a pair.
constexpr int kCfoldGroups = 8;
constexpr int kCfoldHalf = kCfoldGroups / 2;  // first group of the high half
__host__ __device__ constexpr int cfold_gs(int S) { return (S + kCfoldGroups - 1) / kCfoldGroups; }
// first superblock of the high half
__host__ __device__ constexpr int cfold_split(int S) { return kCfoldHalf * cfold_gs(S) < S ? kCfoldHalf * cfold_gs(S) : S; }
// Sequential form: value t and activation scale da of superblock sb (in superblock order); g, y,
// lo updated in place, y and lo starting at -0: y folds the current half, lo receives the low
// half's sum when the high half's first group ends. The result is cfold_end(lo, y).
__device__ __forceinline__ void cfold(float & g, float & y, float & lo, float t, float da, int sb, int gs, int S) {
    const int pos = sb % gs;
    g = __builtin_fmaf(da, t, pos == 0 ? -0.0f : g);
    if (pos == gs - 1 || sb == S - 1) {
        if (sb / gs == kCfoldHalf) {
            lo = y;
            y = g;
        } else {
            y = y + g;
        }
    }
}
__device__ __forceinline__ float cfold_end(float lo, float y) { return lo + y; }
__device__ __forceinline__ f32x16 cfold_end_vec(const f32x16 & lo, const f32x16 & y) { return lo + y; }
// the same for a whole accumulator (sb wave-uniform) without per-element selects; the resets are
// uniform branches kept as branches (the empty asm stops their if-conversion into 16 v_cndmask
// per superblock)
__device__ __forceinline__ void cfold_vec(f32x16 & g, f32x16 & y, f32x16 & lo, const f32x16 & t, const f32x16 & da, int sb, int gs, int S) {
    const int pos = sb % gs;
    if (pos == 0) {  // a group's first value: da * t (bitwise fma(da, t, -0))
        asm volatile("" ::: "memory");
        g = da * t;
    } else {
        g = fma_vec(da, t, g);
    }
    if (pos == gs - 1 || sb == S - 1) {
        asm volatile("" ::: "memory");
        if (sb / gs == kCfoldHalf) {
            lo = y;
            y = g;
        } else {
            y = y + g;
        }
    }
}
// cfold_vec for kernels without 16 registers to spare: the low half's sum is parked by `park(y)`
// (e.g. in the thread's own output locations) when the high half's first group ends; the result is
// then unpark() + y if cfold_split(S) < S, else y
template <typename Park>
__device__ __forceinline__ void cfold_vec_park(f32x16 & g, f32x16 & y, const f32x16 & t, const f32x16 & da, int sb, int gs, int S, Park && park) {
    const int pos = sb % gs;
    if (pos == 0) {  // a group's first value: da * t (bitwise fma(da, t, -0))
        asm volatile("" ::: "memory");
        g = da * t;
    } else {
        g = fma_vec(da, t, g);
    }
    if (pos == gs - 1 || sb == S - 1) {
        asm volatile("" ::: "memory");
        if (sb / gs == kCfoldHalf) {
            park(y);
            y = g;
        } else {
            y = y + g;
        }
    }
}
// group sums v = 0 .. ngroups - 1 read by `at(v)`, folded canonically
template <typename At>
__device__ __forceinline__ float cfold_groups(int ngroups, At && at) {
    float lo = -0.0f, hi = -0.0f;
    for (int v = 0; v < ngroups && v < kCfoldHalf; v++) lo = lo + at(v);
    for (int v = kCfoldHalf; v < ngroups; v++) hi = hi + at(v);
    return lo + hi;
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

// The member of a grouped launch that workgroup blockIdx.x belongs to (members' tiles are dealt
// consecutively: tile_begin ascending), and the workgroup's tile inside it. blockIdx.x is
// wave-uniform, so the scan is scalar; the member's fields are scalar loads from the kernel
// arguments. Defines W, nb01, K, N, act, dst, ycol and mmx_tile.
#define MI_MMX_MEMBER(g)                                                                   \
    int mmx_i_ = 0;                                                                        \
    while (mmx_i_ + 1 < (g).n && (int64_t) blockIdx.x >= (g).m[mmx_i_ + 1].tile_begin) mmx_i_++; \
    const int64_t mmx_tile = (int64_t) blockIdx.x - (g).m[mmx_i_].tile_begin;               \
    const uint8_t * __restrict__ W = (const uint8_t *) (g).m[mmx_i_].W;                    \
    const size_t nb01 = (g).m[mmx_i_].nb01;                                                \
    const int64_t K = (g).K;                                                               \
    const int64_t N = (g).m[mmx_i_].N;                                                     \
    const mi_act_mmx act = (g).m[mmx_i_].act;                                              \
    float * __restrict__ dst = (g).m[mmx_i_].dst;                                          \
    const size_t ycol = (g).m[mmx_i_].ycol;                                                \
    (void) nb01; (void) N; (void) dst; (void) ycol

// LDS-DMA of 16 (4) bytes per lane: lane l's bytes land at LDS byte address lds + 16 l (4 l). As
// inline asm, outside the compiler's wait bookkeeping: with the builtin, hipcc treats the DMA as a
// pending write to any LDS address and waits vmcnt(0) before the next LDS read -- the current
// stage's fragment reads -- which serializes the next stage's DMA with the current stage's
// compute. The caller waits for the DMAs itself (vmcnt(0) before the stage barrier, an asm
// statement with a memory clobber, which also keeps the DMAs of a stage ahead of it). No memory
// clobber here: the compiler may move the current stage's LDS reads across a DMA (it writes the
// other buffer). M0 is saved and restored within the statement (the compiler owns it).
__device__ __forceinline__ void mi_glds16(const void * gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds));
}
__device__ __forceinline__ void mi_glds4(const void * gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds));
}
// LDS byte address of a __shared__ location (the low 32 bits of its flat address), wave-uniform
__device__ __forceinline__ uint32_t mi_lds_addr(const void * p) {
    return (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (uintptr_t) p);
}


} // namespace
