// cpu_order.h -- device helpers that reproduce the reference CPU's floating-point rounding
// sequence (shared by ops.hip and mmv_ordered.hip). Including this header turns off FMA
// contraction for the rest of the translation unit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi355x_common.h"

// Bit-exactness with the CPU needs every multiply and add rounded separately unless written as
// __fmaf_rn: HIP's __fmul_rn/__fadd_rn are plain operators defined in a header (so this file's
// pragma does not reach them) that -ffp-contract=fast would fuse; mul_rn/add_rn below are
// written under the pragma instead. (__fsqrt_rn is the approximate native sqrt; sqrtf and '/'
// are correctly rounded under hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt.)
#pragma clang fp contract(off)

namespace mi_cpu {
__device__ __forceinline__ float mul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float add_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float sub_rn(float a, float b) { return a - b; }


// The CPU accumulates row sums one element at a time in double (ggml_float) and then rounds
// sum/n to float. A parallel double sum S differs from that sequential sum by at most
// 2 n 2^-53 A (A = sum |term|; both are within n 2^-53 A of the exact sum), so whenever
// (S - B)/n and (S + B)/n (B = 4 n 2^-53 A) round to the same float -- all but ~1e-5 of rows --
// that float IS the CPU's result (division and rounding are monotonic). Otherwise one lane
// replays the CPU's sequential chain. Rows are staged in a float buffer (LDS when they fit, else
// the dst row).
template <bool SQ> __device__ __forceinline__ float sum_term(float v) { return SQ ? mul_rn(v, v) : v; }

template <bool SQ>
__device__ float row_mean_cpu_order(const float * buf, int64_t n, double * shd) {
    double s = 0.0, a = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const double t = (double) sum_term<SQ>(buf[i]);
        s += t;
        a += fabs(t);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off, 64);
        a += __shfl_xor(a, off, 64);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = (int) (blockDim.x >> 6);
    if (lane == 0) {
        shd[wave] = s;
        shd[4 + wave] = a;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0, A = 0.0;
        for (int w = 0; w < nw; w++) {
            S += shd[w];
            A += shd[4 + w];
        }
        const double B = 4.0 * (double) n * A * 0x1p-53 + 0x1p-1074;
        const float lo = (float) ((S - B) / (double) n);
        const float hi = (float) ((S + B) / (double) n);
        float r;
        if (lo == hi) {
            r = lo == 0.0f ? 0.0f : lo;  // the CPU's chain starts at +0.0
        } else {
            double q = 0.0;
            int64_t i = 0;
            for (; i + 8 <= n; i += 8) {
                float v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) v[k] = buf[i + k];
#pragma unroll
                for (int k = 0; k < 8; k++) q += (double) sum_term<SQ>(v[k]);
            }
            for (; i < n; i++) q += (double) sum_term<SQ>(buf[i]);
            r = (float) (q / (double) n);
        }
        shd[8] = (double) r;
    }
    __syncthreads();
    const float r = (float) shd[8];
    __syncthreads();  // shd is reused by the caller's next reduction
    return r;
}

// Wave-level variant for rows held in registers: lane l owns elements k = l + 64 j (j < J), so
// element order k is (j, lane). Every lane ends with the same float (no LDS, no barrier). The
// sequential fallback walks k in order with v_readlane.
template <bool SQ, int J>
__device__ float wave_mean_cpu_order(const float (&v)[J], int64_t n) {
    const int lane = threadIdx.x & 63;
    double s = 0.0, a = 0.0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        if ((int64_t) j * 64 + lane < n) {
            const double t = (double) sum_term<SQ>(v[j]);
            s += t;
            a += fabs(t);
        }
    }
    // DPP wave sums (any order: the bound below holds for every order)
    s = mi_wave_sum_u_f64(s);
    a = mi_wave_sum_u_f64(a);
    const double B = 4.0 * (double) n * a * 0x1p-53 + 0x1p-1074;
    const float lo = (float) ((s - B) / (double) n);
    const float hi = (float) ((s + B) / (double) n);
    if (lo == hi) return lo == 0.0f ? 0.0f : lo;  // the CPU's chain starts at +0.0
    double q = 0.0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const float t = sum_term<SQ>(v[j]);
        for (int l = 0; l < 64; l++) {
            if ((int64_t) j * 64 + l < n) q += (double) __shfl(t, l, 64);
        }
    }
    return (float) (q / (double) n);
}

// The same for rows held four consecutive elements per lane: lane l owns k = 256 j + 4 l + i
// (j < J, i < 4); the fallback walks k in order (j, lane, i).
template <bool SQ, int J>
__device__ float wave_mean_cpu_order4(const float4 (&v)[J], int64_t n) {
    const int lane = threadIdx.x & 63;
    double s = 0.0, a = 0.0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if ((int64_t) j * 256 + lane * 4 + i < n) {
                const double t = (double) sum_term<SQ>(e[i]);
                s += t;
                a += fabs(t);
            }
        }
    }
    s = mi_wave_sum_u_f64(s);
    a = mi_wave_sum_u_f64(a);
    const double B = 4.0 * (double) n * a * 0x1p-53 + 0x1p-1074;
    const float lo = (float) ((s - B) / (double) n);
    const float hi = (float) ((s + B) / (double) n);
    if (lo == hi) return lo == 0.0f ? 0.0f : lo;  // the CPU's chain starts at +0.0
    double q = 0.0;
#pragma unroll
    for (int j = 0; j < J; j++) {
        const float e[4] = {sum_term<SQ>(v[j].x), sum_term<SQ>(v[j].y), sum_term<SQ>(v[j].z), sum_term<SQ>(v[j].w)};
        for (int l = 0; l < 64; l++) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if ((int64_t) j * 256 + l * 4 + i < n) q += (double) __shfl(e[i], l, 64);
            }
        }
    }
    return (float) (q / (double) n);
}

} // namespace mi_cpu

using mi_cpu::wave_mean_cpu_order4;
using mi_cpu::add_rn;
using mi_cpu::mul_rn;
using mi_cpu::row_mean_cpu_order;
using mi_cpu::sub_rn;
using mi_cpu::wave_mean_cpu_order;
