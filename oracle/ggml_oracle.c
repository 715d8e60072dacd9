// ggml_oracle.c -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference ggml (NAIST-Archlab/ggml-imax @ v2) arithmetic on the
// GGML_OP_MUL_MAT hot path. It is the *checker* for the MI355X backend: only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
// (ggml-imax_amd/) never links or calls it.
//
// Pinning: every quantizer here is checked bit-exactly against fixtures produced by the real
// reference build (oracle/_ref, see oracle/Makefile + oracle/gen_fixtures.c) in
// tests/test_oracle.py. The reference is built with gcc 11 `-O3 -mavx -mavx2 -mfma -mf16c -msse3`
// (its CMake's own x86 flags, src/CMakeLists.txt:75-96). With -mfma gcc contracts a*b+c into
// FMA, and that changes quantizer bytes (e.g. quantize_row_q8_K_reference's
// nearest_int(iscale*x) becomes fma(iscale, x, 12582912.f) -- visible as vfmadd132ps in the
// reference object code). This file is therefore compiled with the SAME flags and keeps the
// reference's expression shapes wherever rounding matters, and spells out the FMA explicitly
// where the reference build emits one.
//
// Block layouts follow src/ggml-common.h:144-321; function citations are per function.

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <immintrin.h>

#include "ggml_oracle.h"

#define QK4_0 32
#define QK8_0 32
#define QK_K 256

typedef uint16_t half_t;

// src/ggml-common.h:144-149
typedef struct { half_t d; uint8_t qs[16]; } orc_q4_0;
// src/ggml-common.h:186-191
typedef struct { half_t d; int8_t qs[32]; } orc_q8_0;
// src/ggml-common.h:261-272
typedef struct { half_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } orc_q4_K;
// src/ggml-common.h:288-300
typedef struct { half_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; } orc_q5_K;
// src/ggml-common.h:316-321
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } orc_q8_K;

_Static_assert(sizeof(orc_q4_0) == 18, "q4_0");
_Static_assert(sizeof(orc_q8_0) == 34, "q8_0");
_Static_assert(sizeof(orc_q4_K) == 144, "q4_K");
_Static_assert(sizeof(orc_q5_K) == 176, "q5_K");
_Static_assert(sizeof(orc_q8_K) == 292, "q8_K");

// ---------------------------------------------------------------------------------------------
// fp16 <-> fp32.  The AVX2 reference uses F16C _cvtss_sh(x, 0) (round-to-nearest-even) and
// _cvtsh_ss (src/ggml-impl.h:446-462).
// ---------------------------------------------------------------------------------------------

uint16_t orc_fp32_to_fp16(float f) { return _cvtss_sh(f, 0); }
float orc_fp16_to_fp32(uint16_t h) { return _cvtsh_ss(h); }

// src/ggml-quants.c:1097-1102 -- round-to-nearest-even via the 1.5*2^23 magic constant.
static inline int orc_nearest_int(float v) {
    float t = v + 12582912.f;
    int32_t i;
    memcpy(&i, &t, sizeof(i));
    return (i & 0x007fffff) - 0x00400000;
}

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------------------------
// type table (src/ggml.c:564-918 type_traits: blck_size / type_size / vec_dot_type)
// ---------------------------------------------------------------------------------------------

int orc_block_size(int type) {
    switch (type) {
        case ORC_F32: case ORC_F16: return 1;
        case ORC_Q4_0: case ORC_Q8_0: return 32;
        case ORC_Q4_K: case ORC_Q5_K: case ORC_Q8_K: return 256;
        default: return 0;
    }
}

int orc_type_size(int type) {
    switch (type) {
        case ORC_F32: return 4;
        case ORC_F16: return 2;
        case ORC_Q4_0: return sizeof(orc_q4_0);
        case ORC_Q8_0: return sizeof(orc_q8_0);
        case ORC_Q4_K: return sizeof(orc_q4_K);
        case ORC_Q5_K: return sizeof(orc_q5_K);
        case ORC_Q8_K: return sizeof(orc_q8_K);
        default: return 0;
    }
}

size_t orc_row_size(int type, int64_t n) {
    return (size_t) (n / orc_block_size(type)) * (size_t) orc_type_size(type);
}

// src/ggml.c:596-770: F32->F32, F16->F16, Q4_0->Q8_0, Q8_0->Q8_0, Q4_K/Q5_K->Q8_K
int orc_vec_dot_type(int type) {
    switch (type) {
        case ORC_Q4_0: case ORC_Q8_0: return ORC_Q8_0;
        case ORC_Q4_K: case ORC_Q5_K: return ORC_Q8_K;
        default: return type;
    }
}

// ---------------------------------------------------------------------------------------------
// Weight quantizers (imatrix == NULL path of ggml_quantize_chunk, src/ggml.c:21594-21660)
// ---------------------------------------------------------------------------------------------

// src/ggml-quants.c:260-295 quantize_row_q4_0_reference
static void q4_0_quantize(const float * restrict x, orc_q4_0 * restrict y, int64_t k) {
    const int nb = (int) (k / QK4_0);
    for (int b = 0; b < nb; b++, x += QK4_0) {
        float amax = 0.0f, vmax = 0.0f;
        for (int j = 0; j < QK4_0; j++) {
            if (amax < fabsf(x[j])) { amax = fabsf(x[j]); vmax = x[j]; }
        }
        const float d  = vmax / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = orc_fp32_to_fp16(d);
        for (int j = 0; j < QK4_0 / 2; j++) {
            const float a0 = x[j] * id;
            const float a1 = x[QK4_0 / 2 + j] * id;
            const uint8_t lo = (uint8_t) imin(15, (int8_t) (a0 + 8.5f));
            const uint8_t hi = (uint8_t) imin(15, (int8_t) (a1 + 8.5f));
            y[b].qs[j] = (uint8_t) (lo | (hi << 4));
        }
    }
}

// src/ggml-quants.c:440-463 quantize_row_q8_0_reference (scalar: used for Q8_0 *weights*,
// quantize_q8_0 :3066-3071)
static void q8_0_quantize_ref(const float * restrict x, orc_q8_0 * restrict y, int64_t k) {
    const int nb = (int) (k / QK8_0);
    for (int b = 0; b < nb; b++, x += QK8_0) {
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; j++) amax = fmaxf(amax, fabsf(x[j]));
        const float d  = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = orc_fp32_to_fp16(d);
        for (int j = 0; j < QK8_0; j++) y[b].qs[j] = (int8_t) roundf(x[j] * id);
    }
}

// src/ggml-quants.c:535-618 quantize_row_q8_0, AVX2 branch (used for *activations*: the
// from_float of vec_dot_type Q8_0). Differs from the scalar reference: id = 127/amax and
// round-half-even (_mm256_round_ps(_MM_ROUND_NEAREST)) instead of 1/(amax/127) and roundf.
static void q8_0_quantize_act(const float * restrict x, orc_q8_0 * restrict y, int64_t k) {
    const int nb = (int) (k / QK8_0);
    for (int b = 0; b < nb; b++, x += QK8_0) {
        float amax = 0.0f;
        for (int j = 0; j < QK8_0; j++) {
            const float a = fabsf(x[j]);
            amax = a > amax ? a : amax;
        }
        const float d = amax / 127.f;
        y[b].d = orc_fp32_to_fp16(d);
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        for (int j = 0; j < QK8_0; j++) {
            const float v = x[j] * id;           // vmulps
            y[b].qs[j] = (int8_t) nearbyintf(v); // vroundps nearest-even, then cvtps_epi32
        }
    }
}

// src/ggml-quants.c:1275-1354 make_qkx2_quants (expression shapes kept: see file header)
static float make_qkx2_quants(int n, int nmax, const float * restrict x, const float * restrict weights,
        uint8_t * restrict L, float * restrict the_min, uint8_t * restrict Laux,
        float rmin, float rdelta, int nstep, bool use_mad) {
    float min = x[0];
    float max = x[0];
    float sum_w = weights[0];
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < min) min = x[i];
        if (x[i] > max) max = x[i];
        float w = weights[i];
        sum_w += w;
        sum_x += w * x[i];
    }
    if (min > 0) min = 0;
    if (max == min) {
        for (int i = 0; i < n; ++i) L[i] = 0;
        *the_min = -min;
        return 0.f;
    }
    float iscale = nmax / (max - min);
    float scale = 1 / iscale;
    float best_mad = 0;
    for (int i = 0; i < n; ++i) {
        int l = orc_nearest_int(iscale * (x[i] - min));
        L[i] = (uint8_t) imax(0, imin(nmax, l));
        float diff = scale * L[i] + min - x[i];
        diff = use_mad ? fabsf(diff) : diff * diff;
        float w = weights[i];
        best_mad += w * diff;
    }
    if (nstep < 1) {
        *the_min = -min;
        return scale;
    }
    for (int is = 0; is <= nstep; ++is) {
        iscale = (rmin + rdelta * is + nmax) / (max - min);
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < n; ++i) {
            int l = orc_nearest_int(iscale * (x[i] - min));
            l = imax(0, imin(nmax, l));
            Laux[i] = (uint8_t) l;
            float w = weights[i];
            sum_l += w * l;
            sum_l2 += w * l * l;
            sum_xl += w * l * x[i];
        }
        float D = sum_w * sum_l2 - sum_l * sum_l;
        if (D > 0) {
            float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
            float this_min   = (sum_l2 * sum_x - sum_l * sum_xl) / D;
            if (this_min > 0) {
                this_min = 0;
                this_scale = sum_xl / sum_l2;
            }
            float mad = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = use_mad ? fabsf(diff) : diff * diff;
                float w = weights[i];
                mad += w * diff;
            }
            if (mad < best_mad) {
                for (int i = 0; i < n; ++i) L[i] = Laux[i];
                best_mad = mad;
                scale = this_scale;
                min = this_min;
            }
        }
    }
    *the_min = -min;
    return scale;
}

// src/ggml-quants.c:1357-1364 get_scale_min_k4: 6-bit scale/min j of the 12-byte packed array
static inline void scale_min_k4(int j, const uint8_t * restrict q, uint8_t * restrict sc, uint8_t * restrict mn) {
    if (j < 4) {
        *sc = q[j] & 63;
        *mn = q[j + 4] & 63;
    } else {
        *sc = (uint8_t) ((q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4));
        *mn = (uint8_t) ((q[j + 4] >> 4) | ((q[j] >> 6) << 4));
    }
}

// Shared first half of the Q4_K / Q5_K reference quantizers: per-32 (scale, min) search and
// 6-bit packing (src/ggml-quants.c:2085-2141 for Q4_K, :2339-2390 for Q5_K).
static void kquant_scales(const float * restrict x, int nmax, float rmin, int nstep,
                          uint8_t * restrict scales12, half_t * d_out, half_t * dmin_out, uint8_t * restrict L) {
    uint8_t Laux[32];
    float weights[32];
    float mins[QK_K / 32];
    float scales[QK_K / 32];
    float max_scale = 0, max_min = 0;
    for (int j = 0; j < QK_K / 32; ++j) {
        float sum_x2 = 0;
        for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
        float av_x = sqrtf(sum_x2 / 32);
        for (int l = 0; l < 32; ++l) weights[l] = av_x + fabsf(x[32 * j + l]);
        scales[j] = make_qkx2_quants(32, nmax, x + 32 * j, weights, L + 32 * j, &mins[j], Laux, rmin, 0.1f, nstep, false);
        if (scales[j] > max_scale) max_scale = scales[j];
        if (mins[j] > max_min) max_min = mins[j];
    }
    float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
    float inv_min   = max_min   > 0 ? 63.f / max_min   : 0.f;
    memset(scales12, 0, 12);
    for (int j = 0; j < QK_K / 32; ++j) {
        uint8_t ls = (uint8_t) orc_nearest_int(inv_scale * scales[j]);
        uint8_t lm = (uint8_t) orc_nearest_int(inv_min * mins[j]);
        ls = ls < 63 ? ls : 63;
        lm = lm < 63 ? lm : 63;
        if (j < 4) {
            scales12[j] = ls;
            scales12[j + 4] = lm;
        } else {
            scales12[j + 4] = (uint8_t) ((ls & 0xF) | ((lm & 0xF) << 4));
            scales12[j - 4] |= (uint8_t) ((ls >> 4) << 6);
            scales12[j - 0] |= (uint8_t) ((lm >> 4) << 6);
        }
    }
    *d_out = orc_fp32_to_fp16(max_scale / 63.f);
    *dmin_out = orc_fp32_to_fp16(max_min / 63.f);
    uint8_t sc, mn;
    for (int j = 0; j < QK_K / 32; ++j) {
        scale_min_k4(j, scales12, &sc, &mn);
        const float d = orc_fp16_to_fp32(*d_out) * sc;
        if (!d) continue;
        const float dm = orc_fp16_to_fp32(*dmin_out) * mn;
        for (int ii = 0; ii < 32; ++ii) {
            int l = orc_nearest_int((x[32 * j + ii] + dm) / d);
            L[32 * j + ii] = (uint8_t) imax(0, imin(nmax, l));
        }
    }
}

// src/ggml-quants.c:2074-2179 quantize_row_q4_K_reference
static void q4_K_quantize(const float * restrict x, orc_q4_K * restrict y, int64_t k) {
    uint8_t L[QK_K];
    const int64_t nb = k / QK_K;
    for (int64_t b = 0; b < nb; b++, x += QK_K) {
        kquant_scales(x, 15, -1.f, 20, y[b].scales, &y[b].d, &y[b].dmin, L);
        // nibble packing: low = element l, high = element l+32 of each 64-chunk (:2170-2174)
        for (int c = 0; c < 4; c++) {
            for (int l = 0; l < 32; ++l) {
                y[b].qs[32 * c + l] = (uint8_t) (L[64 * c + l] | (L[64 * c + l + 32] << 4));
            }
        }
    }
}

// src/ggml-quants.c:2322-2411 quantize_row_q5_K_reference
static void q5_K_quantize(const float * restrict x, orc_q5_K * restrict y, int64_t k) {
    uint8_t L[QK_K];
    const int64_t nb = k / QK_K;
    for (int64_t b = 0; b < nb; b++, x += QK_K) {
        kquant_scales(x, 31, -0.5f, 15, y[b].scales, &y[b].d, &y[b].dmin, L);
        memset(y[b].qh, 0, 32);
        // 5th bit goes to a bit-plane: chunk c uses qh bits 2c (low half) and 2c+1 (high half)
        for (int c = 0; c < 4; c++) {
            for (int j = 0; j < 32; ++j) {
                int l1 = L[64 * c + j];
                int l2 = L[64 * c + j + 32];
                if (l1 > 15) { l1 -= 16; y[b].qh[j] |= (uint8_t) (1u << (2 * c)); }
                if (l2 > 15) { l2 -= 16; y[b].qh[j] |= (uint8_t) (2u << (2 * c)); }
                y[b].qs[32 * c + j] = (uint8_t) (l1 | (l2 << 4));
            }
        }
    }
}

// src/ggml-quants.c:3370-3407 quantize_row_q8_K_reference (activation quantizer for Q4_K/Q5_K).
// The reference AVX2 build contracts nearest_int(iscale*x) into fma(iscale, x, 1.5*2^23).
static void q8_K_quantize(const float * restrict x, orc_q8_K * restrict y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t b = 0; b < nb; b++, x += QK_K) {
        float vmax = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            const float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; vmax = x[j]; }
        }
        if (!amax) {
            memset(&y[b], 0, sizeof(y[b]));
            continue;
        }
        const float iscale = -127.f / vmax;
        for (int j = 0; j < QK_K; ++j) {
            const float t = fmaf(iscale, x[j], 12582912.f);
            int32_t bits;
            memcpy(&bits, &t, 4);
            const int v = (bits & 0x007fffff) - 0x00400000;
            y[b].qs[j] = (int8_t) imin(127, v);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int s = 0;
            for (int ii = 0; ii < 16; ++ii) s += y[b].qs[16 * j + ii];
            y[b].bsums[j] = (int16_t) s;
        }
        y[b].d = 1 / iscale;
    }
}

// src/ggml.c:365-382 ggml_fp32_to_fp16_row (F16C, round-to-nearest-even)
static void f16_from_f32(const float * x, half_t * y, int64_t n) {
    for (int64_t i = 0; i < n; i++) y[i] = orc_fp32_to_fp16(x[i]);
}

size_t orc_quantize_chunk(int type, const float * src, void * dst, int64_t nrows, int64_t n_per_row) {
    const int64_t n = nrows * n_per_row;
    switch (type) {
        case ORC_Q4_0: q4_0_quantize(src, dst, n); break;
        case ORC_Q8_0: q8_0_quantize_ref(src, dst, n); break;
        case ORC_Q4_K: q4_K_quantize(src, dst, n); break;
        case ORC_Q5_K: q5_K_quantize(src, dst, n); break;
        case ORC_F16:  f16_from_f32(src, dst, n); break;
        case ORC_F32:  memcpy(dst, src, (size_t) n * 4); break;
        default: return 0;
    }
    return (size_t) nrows * orc_row_size(type, n_per_row);
}

// Activation conversion = type_traits[vec_dot_type].from_float on the AVX2 build.
void orc_quantize_act(int vec_dot_type, const float * x, void * dst, int64_t n) {
    switch (vec_dot_type) {
        case ORC_Q8_0: q8_0_quantize_act(x, dst, n); break;
        case ORC_Q8_K: q8_K_quantize(x, dst, n); break;
        case ORC_F16:  f16_from_f32(x, dst, n); break;
        case ORC_F32:  memcpy(dst, x, (size_t) n * 4); break;
        default: abort();
    }
}

// ---------------------------------------------------------------------------------------------
// Dequantizers (to_float)
// ---------------------------------------------------------------------------------------------

void orc_dequantize_row(int type, const void * src, float * y, int64_t k) {
    switch (type) {
        case ORC_Q4_0: {  // src/ggml-quants.c:980-998
            const orc_q4_0 * x = src;
            for (int64_t b = 0; b < k / QK4_0; b++) {
                const float d = orc_fp16_to_fp32(x[b].d);
                for (int j = 0; j < 16; ++j) {
                    y[b * 32 + j]      = ((x[b].qs[j] & 0x0F) - 8) * d;
                    y[b * 32 + j + 16] = ((x[b].qs[j] >> 4) - 8) * d;
                }
            }
        } break;
        case ORC_Q8_0: {  // src/ggml-quants.c:1074-1088
            const orc_q8_0 * x = src;
            for (int64_t b = 0; b < k / QK8_0; b++) {
                const float d = orc_fp16_to_fp32(x[b].d);
                for (int j = 0; j < 32; ++j) y[b * 32 + j] = x[b].qs[j] * d;
            }
        } break;
        case ORC_Q4_K: {  // src/ggml-quants.c:2181-2218
            const orc_q4_K * x = src;
            for (int64_t b = 0; b < k / QK_K; b++) {
                const float d = orc_fp16_to_fp32(x[b].d), mn = orc_fp16_to_fp32(x[b].dmin);
                for (int c = 0; c < 4; c++) {
                    uint8_t sc, m;
                    scale_min_k4(2 * c, x[b].scales, &sc, &m);
                    const float d1 = d * sc, m1 = mn * m;
                    scale_min_k4(2 * c + 1, x[b].scales, &sc, &m);
                    const float d2 = d * sc, m2 = mn * m;
                    const uint8_t * q = x[b].qs + 32 * c;
                    for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
                    for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
                }
            }
        } break;
        case ORC_Q5_K: {  // src/ggml-quants.c:2464-2507
            const orc_q5_K * x = src;
            for (int64_t b = 0; b < k / QK_K; b++) {
                const float d = orc_fp16_to_fp32(x[b].d), mn = orc_fp16_to_fp32(x[b].dmin);
                for (int c = 0; c < 4; c++) {
                    uint8_t sc, m;
                    scale_min_k4(2 * c, x[b].scales, &sc, &m);
                    const float d1 = d * sc, m1 = mn * m;
                    scale_min_k4(2 * c + 1, x[b].scales, &sc, &m);
                    const float d2 = d * sc, m2 = mn * m;
                    const uint8_t * ql = x[b].qs + 32 * c;
                    const uint8_t u1 = (uint8_t) (1u << (2 * c)), u2 = (uint8_t) (2u << (2 * c));
                    for (int l = 0; l < 32; ++l) *y++ = d1 * ((ql[l] & 0xF) + (x[b].qh[l] & u1 ? 16 : 0)) - m1;
                    for (int l = 0; l < 32; ++l) *y++ = d2 * ((ql[l] >> 4) + (x[b].qh[l] & u2 ? 16 : 0)) - m2;
                }
            }
        } break;
        case ORC_Q8_K: {  // src/ggml-quants.c:3409-3418
            const orc_q8_K * x = src;
            for (int64_t b = 0; b < k / QK_K; b++)
                for (int j = 0; j < QK_K; ++j) *y++ = x[b].d * x[b].qs[j];
        } break;
        case ORC_F16: {
            const half_t * x = src;
            for (int64_t i = 0; i < k; i++) y[i] = orc_fp16_to_fp32(x[i]);
        } break;
        case ORC_F32: memcpy(y, src, (size_t) k * 4); break;
        default: abort();
    }
}

// ---------------------------------------------------------------------------------------------
// Dot products. Integer parts are exact; float combination follows the reference's scalar
// branches (which differ from its AVX2 lane order only by float summation order).
// ---------------------------------------------------------------------------------------------

// src/ggml-quants.c:3855-3872 (scalar branch of ggml_vec_dot_q4_0_q8_0)
static float dot_q4_0_q8_0(int n, const orc_q4_0 * x, const orc_q8_0 * y) {
    float sumf = 0;
    for (int b = 0; b < n / QK8_0; b++) {
        int sumi = 0;
        for (int j = 0; j < 16; ++j) {
            sumi += ((x[b].qs[j] & 0x0F) - 8) * y[b].qs[j] + ((x[b].qs[j] >> 4) - 8) * y[b].qs[j + 16];
        }
        sumf += sumi * orc_fp16_to_fp32(x[b].d) * orc_fp16_to_fp32(y[b].d);
    }
    return sumf;
}

// src/ggml-quants.c:4819+ (ggml_vec_dot_q8_0_q8_0)
static float dot_q8_0_q8_0(int n, const orc_q8_0 * x, const orc_q8_0 * y) {
    float sumf = 0;
    for (int b = 0; b < n / QK8_0; b++) {
        int sumi = 0;
        for (int j = 0; j < 32; ++j) sumi += x[b].qs[j] * y[b].qs[j];
        sumf += sumi * (orc_fp16_to_fp32(x[b].d) * orc_fp16_to_fp32(y[b].d));
    }
    return sumf;
}

// src/ggml-quants.c:7007-7502 ggml_vec_dot_q4_K_q8_K: per superblock
//   d*sum_j sc_j*<q4,q8>_j - dmin*sum_j m_j*bsum_j  with d = y.d*fp16(x.d), dmin = y.d*fp16(x.dmin)
static float dot_q4_K_q8_K(int n, const orc_q4_K * x, const orc_q8_K * y) {
    float sumf = 0;
    for (int b = 0; b < n / QK_K; b++) {
        int sumi = 0, summ = 0;
        for (int j = 0; j < 8; j++) {
            uint8_t sc, m;
            scale_min_k4(j, x[b].scales, &sc, &m);
            const uint8_t * q = x[b].qs + 32 * (j / 2);
            const int8_t * a = y[b].qs + 32 * j;
            int s = 0;
            for (int l = 0; l < 32; l++) s += ((j & 1) ? (q[l] >> 4) : (q[l] & 0xF)) * a[l];
            sumi += sc * s;
            summ += m * (y[b].bsums[2 * j] + y[b].bsums[2 * j + 1]);
        }
        const float d = y[b].d * orc_fp16_to_fp32(x[b].d);
        const float dmin = y[b].d * orc_fp16_to_fp32(x[b].dmin);
        sumf += d * sumi - dmin * summ;
    }
    return sumf;
}

// src/ggml-quants.c:7833-8378 ggml_vec_dot_q5_K_q8_K (q5 = low nibble + 16 * qh bit)
static float dot_q5_K_q8_K(int n, const orc_q5_K * x, const orc_q8_K * y) {
    float sumf = 0;
    for (int b = 0; b < n / QK_K; b++) {
        int sumi = 0, summ = 0;
        for (int j = 0; j < 8; j++) {
            uint8_t sc, m;
            scale_min_k4(j, x[b].scales, &sc, &m);
            const uint8_t * q = x[b].qs + 32 * (j / 2);
            const int8_t * a = y[b].qs + 32 * j;
            int s = 0;
            for (int l = 0; l < 32; l++) {
                int v = (j & 1) ? (q[l] >> 4) : (q[l] & 0xF);
                v += (x[b].qh[l] >> j) & 1 ? 16 : 0;
                s += v * a[l];
            }
            sumi += sc * s;
            summ += m * (y[b].bsums[2 * j] + y[b].bsums[2 * j + 1]);
        }
        const float d = y[b].d * orc_fp16_to_fp32(x[b].d);
        const float dmin = y[b].d * orc_fp16_to_fp32(x[b].dmin);
        sumf += d * sumi - dmin * summ;
    }
    return sumf;
}

// src/ggml.c:1674-1714 ggml_vec_dot_f16 (products in f32, sum in ggml_float = double)
static float dot_f16(int n, const half_t * x, const half_t * y) {
    double s = 0;
    for (int i = 0; i < n; i++) s += (double) (orc_fp16_to_fp32(x[i]) * orc_fp16_to_fp32(y[i]));
    return (float) s;
}

// src/ggml.c:1567-1608 ggml_vec_dot_f32
static float dot_f32(int n, const float * x, const float * y) {
    double s = 0;
    for (int i = 0; i < n; i++) s += (double) (x[i] * y[i]);
    return (float) s;
}

float orc_vec_dot(int type, int n, const void * x, const void * y) {
    switch (type) {
        case ORC_Q4_0: return dot_q4_0_q8_0(n, x, y);
        case ORC_Q8_0: return dot_q8_0_q8_0(n, x, y);
        case ORC_Q4_K: return dot_q4_K_q8_K(n, x, y);
        case ORC_Q5_K: return dot_q5_K_q8_K(n, x, y);
        case ORC_F16:  return dot_f16(n, x, y);
        case ORC_F32:  return dot_f32(n, x, y);
        default: abort();
    }
}

// ---------------------------------------------------------------------------------------------
// mul_mat driver: src/ggml.c:11808-12097 ggml_compute_forward_mul_mat for contiguous 2-D
// W [K, N] (rows of K), X [K, B] f32 -> Y [N, B] f32.  INIT: X columns -> vec_dot_type
// (:11952-11974); COMPUTE: rows split across threads (:12010-12033), vec_dot per (row, col).
// ---------------------------------------------------------------------------------------------

struct mm_job {
    int type;
    const uint8_t * W;
    const uint8_t * Xq;
    float * Y;
    int64_t K, N, B;
    size_t wrow, xrow;
    int64_t r0, r1;
};

static void * mm_worker(void * arg) {
    struct mm_job * j = arg;
    for (int64_t c = 0; c < j->B; c++) {
        for (int64_t r = j->r0; r < j->r1; r++) {
            j->Y[c * j->N + r] = orc_vec_dot(j->type, (int) j->K, j->W + r * j->wrow, j->Xq + c * j->xrow);
        }
    }
    return NULL;
}

void orc_mul_mat(int type, const void * W, int64_t K, int64_t N, const float * X, int64_t B, float * Y, int nthreads) {
    const int vdt = orc_vec_dot_type(type);
    const size_t xrow = orc_row_size(vdt, K);
    uint8_t * Xq = malloc(xrow * (size_t) B);
    for (int64_t c = 0; c < B; c++) orc_quantize_act(vdt, X + c * K, Xq + c * xrow, K);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    struct mm_job jobs[256];
    const int64_t per = (N + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct mm_job) { type, W, Xq, Y, K, N, B, orc_row_size(type, K), xrow,
                                    t * per < N ? t * per : N, (t + 1) * per < N ? (t + 1) * per : N };
        if (t > 0) pthread_create(&th[t], NULL, mm_worker, &jobs[t]);
    }
    mm_worker(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    free(Xq);
}
