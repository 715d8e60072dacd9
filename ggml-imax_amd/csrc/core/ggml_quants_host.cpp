// ggml_quants_host.cpp -- ggml_quantize_chunk (include/ggml/ggml.h:2240-2254) for the weight
// formats on the hot path: Q4_0, Q8_0, Q4_K, Q5_K (+ F16 / F32 passthrough).
//
// These produce the bytes the MI355X kernels consume. They must be bit-identical to the
// reference's imatrix == NULL path (src/ggml.c:21594-21660 -> src/ggml-quants.c reference
// quantizers), which its x86 build compiles with -mfma and gcc's default FP contraction.
// This file is compiled with the same flags and keeps the reference's expression shapes
// where the rounding depends on them; tests/test_core.py checks it against the golden vectors.

#include "ggml_abi.h"

#include <cmath>
#include <cstring>

namespace {

constexpr int kQK4_0 = 32;
constexpr int kQK8_0 = 32;
constexpr int kQKK = 256;

struct blk_q4_0 { ggml_fp16_t d; uint8_t qs[16]; };
struct blk_q8_0 { ggml_fp16_t d; int8_t qs[32]; };
struct blk_q4_K { ggml_fp16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; };
struct blk_q5_K { ggml_fp16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; };
static_assert(sizeof(blk_q4_0) == 18 && sizeof(blk_q8_0) == 34 && sizeof(blk_q4_K) == 144 && sizeof(blk_q5_K) == 176, "blocks");

// src/ggml-quants.c:1097-1102: round half to even through the 1.5*2^23 bias
inline int rne_int(float v) {
    float t = v + 12582912.f;
    int32_t bits;
    memcpy(&bits, &t, 4);
    return (bits & 0x007fffff) - 0x00400000;
}

template <typename T> inline T clampv(T v, T lo, T hi) { return v < lo ? lo : (v > hi ? hi : v); }

// src/ggml-quants.c:260-295
void quantize_q4_0_rows(const float * x, blk_q4_0 * y, int64_t n) {
    for (int64_t b = 0; b < n / kQK4_0; ++b, x += kQK4_0) {
        float amax = 0.0f, extreme = 0.0f;
        for (int j = 0; j < kQK4_0; ++j) {
            if (amax < fabsf(x[j])) {
                amax = fabsf(x[j]);
                extreme = x[j];
            }
        }
        const float d = extreme / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = ggml_fp32_to_fp16(d);
        for (int j = 0; j < kQK4_0 / 2; ++j) {
            const float v0 = x[j] * id;
            const float v1 = x[kQK4_0 / 2 + j] * id;
            const int q0 = std::min(15, (int) (int8_t) (v0 + 8.5f));
            const int q1 = std::min(15, (int) (int8_t) (v1 + 8.5f));
            y[b].qs[j] = (uint8_t) (q0 | (q1 << 4));
        }
    }
}

// src/ggml-quants.c:440-463 (scalar reference; the weight path uses it, :3066-3071)
void quantize_q8_0_rows(const float * x, blk_q8_0 * y, int64_t n) {
    for (int64_t b = 0; b < n / kQK8_0; ++b, x += kQK8_0) {
        float amax = 0.0f;
        for (int j = 0; j < kQK8_0; ++j) amax = std::max(amax, fabsf(x[j]));
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = ggml_fp32_to_fp16(d);
        for (int j = 0; j < kQK8_0; ++j) y[b].qs[j] = (int8_t) roundf(x[j] * id);
    }
}

// src/ggml-quants.c:1275-1354 make_qkx2_quants: weighted (scale, min) search for one 32-group
float search_scale_min(int nmax, const float * x, const float * w, uint8_t * L, float * out_min,
                       float rmin, float rdelta, int nstep) {
    constexpr int n = 32;
    uint8_t Laux[n];
    float lo = x[0], hi = x[0];
    float sum_w = w[0];
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < lo) lo = x[i];
        if (x[i] > hi) hi = x[i];
        float wi = w[i];
        sum_w += wi;
        sum_x += wi * x[i];
    }
    if (lo > 0) lo = 0;
    if (hi == lo) {
        memset(L, 0, n);
        *out_min = -lo;
        return 0.f;
    }
    float iscale = nmax / (hi - lo);
    float scale = 1 / iscale;
    float best = 0;
    for (int i = 0; i < n; ++i) {
        int l = rne_int(iscale * (x[i] - lo));
        L[i] = (uint8_t) clampv(l, 0, nmax);
        float diff = scale * L[i] + lo - x[i];
        diff = diff * diff;
        float wi = w[i];
        best += wi * diff;
    }
    for (int is = 0; is <= nstep; ++is) {
        iscale = (rmin + rdelta * is + nmax) / (hi - lo);
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < n; ++i) {
            int l = rne_int(iscale * (x[i] - lo));
            l = clampv(l, 0, nmax);
            Laux[i] = (uint8_t) l;
            float wi = w[i];
            sum_l += wi * l;
            sum_l2 += wi * l * l;
            sum_xl += wi * l * x[i];
        }
        float D = sum_w * sum_l2 - sum_l * sum_l;
        if (D > 0) {
            float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
            float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
            if (this_min > 0) {
                this_min = 0;
                this_scale = sum_xl / sum_l2;
            }
            float mad = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = diff * diff;
                float wi = w[i];
                mad += wi * diff;
            }
            if (mad < best) {
                memcpy(L, Laux, n);
                best = mad;
                scale = this_scale;
                lo = this_min;
            }
        }
    }
    *out_min = -lo;
    return scale;
}

// src/ggml-quants.c:1357-1364
inline void unpack_scale_min(int j, const uint8_t * q, uint8_t & sc, uint8_t & m) {
    if (j < 4) {
        sc = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        sc = (uint8_t) ((q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4));
        m = (uint8_t) ((q[j + 4] >> 4) | ((q[j] >> 6) << 4));
    }
}

// Per-superblock scale search + 6-bit packing + final levels, shared by Q4_K (nmax 15) and
// Q5_K (nmax 31): src/ggml-quants.c:2085-2160 / :2339-2390.
template <int NMAX>
void kquant_superblock(const float * x, ggml_fp16_t & d_out, ggml_fp16_t & dmin_out, uint8_t * scales, uint8_t * L) {
    constexpr float rmin = NMAX == 15 ? -1.f : -0.5f;
    constexpr int nstep = NMAX == 15 ? 20 : 15;
    float w[32], mins[8], scl[8];
    float max_scale = 0, max_min = 0;
    for (int j = 0; j < 8; ++j) {
        float sum_x2 = 0;
        for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
        float av_x = sqrtf(sum_x2 / 32);
        for (int l = 0; l < 32; ++l) w[l] = av_x + fabsf(x[32 * j + l]);
        scl[j] = search_scale_min(NMAX, x + 32 * j, w, L + 32 * j, &mins[j], rmin, 0.1f, nstep);
        if (scl[j] > max_scale) max_scale = scl[j];
        if (mins[j] > max_min) max_min = mins[j];
    }
    float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
    float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
    memset(scales, 0, 12);
    for (int j = 0; j < 8; ++j) {
        uint8_t ls = (uint8_t) rne_int(inv_scale * scl[j]);
        uint8_t lm = (uint8_t) rne_int(inv_min * mins[j]);
        ls = std::min<uint8_t>(63, ls);
        lm = std::min<uint8_t>(63, lm);
        if (j < 4) {
            scales[j] = ls;
            scales[j + 4] = lm;
        } else {
            scales[j + 4] = (uint8_t) ((ls & 0xF) | ((lm & 0xF) << 4));
            scales[j - 4] |= (uint8_t) ((ls >> 4) << 6);
            scales[j] |= (uint8_t) ((lm >> 4) << 6);
        }
    }
    d_out = ggml_fp32_to_fp16(max_scale / 63.f);
    dmin_out = ggml_fp32_to_fp16(max_min / 63.f);
    for (int j = 0; j < 8; ++j) {
        uint8_t sc, m;
        unpack_scale_min(j, scales, sc, m);
        const float d = ggml_fp16_to_fp32(d_out) * sc;
        if (!d) continue;
        const float dm = ggml_fp16_to_fp32(dmin_out) * m;
        for (int ii = 0; ii < 32; ++ii) {
            int l = rne_int((x[32 * j + ii] + dm) / d);
            L[32 * j + ii] = (uint8_t) clampv(l, 0, NMAX);
        }
    }
}

void quantize_q4_K_rows(const float * x, blk_q4_K * y, int64_t n) {
    uint8_t L[kQKK];
    for (int64_t b = 0; b < n / kQKK; ++b, x += kQKK) {
        kquant_superblock<15>(x, y[b].d, y[b].dmin, y[b].scales, L);
        for (int c = 0; c < 4; ++c)
            for (int l = 0; l < 32; ++l) y[b].qs[32 * c + l] = (uint8_t) (L[64 * c + l] | (L[64 * c + 32 + l] << 4));
    }
}

void quantize_q5_K_rows(const float * x, blk_q5_K * y, int64_t n) {
    uint8_t L[kQKK];
    for (int64_t b = 0; b < n / kQKK; ++b, x += kQKK) {
        kquant_superblock<31>(x, y[b].d, y[b].dmin, y[b].scales, L);
        memset(y[b].qh, 0, 32);
        for (int c = 0; c < 4; ++c) {
            for (int l = 0; l < 32; ++l) {
                int lo = L[64 * c + l], hi = L[64 * c + 32 + l];
                if (lo > 15) { lo -= 16; y[b].qh[l] |= (uint8_t) (1u << (2 * c)); }
                if (hi > 15) { hi -= 16; y[b].qh[l] |= (uint8_t) (2u << (2 * c)); }
                y[b].qs[32 * c + l] = (uint8_t) (lo | (hi << 4));
            }
        }
    }
}

} // namespace

extern "C" {

void ggml_quantize_init(enum ggml_type) {}
void ggml_quantize_free(void) {}

bool ggml_quantize_requires_imatrix(enum ggml_type type) {
    return type == GGML_TYPE_IQ2_XXS || type == GGML_TYPE_IQ2_XS || type == GGML_TYPE_IQ1_S;
}

size_t ggml_quantize_chunk(enum ggml_type type, const float * src, void * dst, int64_t start, int64_t nrows,
                           int64_t n_per_row, const float * imatrix) {
    GGML_ASSERT(start % ggml_blck_size(type) == 0);
    GGML_ASSERT(start % n_per_row == 0);
    const int64_t n = nrows * n_per_row;
    const size_t row_size = ggml_row_size(type, n_per_row);
    char * out = (char *) dst + (start / n_per_row) * row_size;
    const float * in = src + start;
    if (imatrix != NULL && type != GGML_TYPE_Q8_0 && type != GGML_TYPE_F16 && type != GGML_TYPE_F32) {
        GGML_ASSERT(!"importance-matrix quantization is not supported by this runtime");
    }
    switch (type) {
        case GGML_TYPE_Q4_0: quantize_q4_0_rows(in, (blk_q4_0 *) out, n); break;
        case GGML_TYPE_Q8_0: quantize_q8_0_rows(in, (blk_q8_0 *) out, n); break;
        case GGML_TYPE_Q4_K: quantize_q4_K_rows(in, (blk_q4_K *) out, n); break;
        case GGML_TYPE_Q5_K: quantize_q5_K_rows(in, (blk_q5_K *) out, n); break;
        case GGML_TYPE_F16: ggml_fp32_to_fp16_row(in, (ggml_fp16_t *) out, n); break;
        case GGML_TYPE_F32: memcpy(out, in, (size_t) n * sizeof(float)); break;
        default: GGML_ASSERT(!"ggml_quantize_chunk: type not supported by this runtime");
    }
    return (size_t) nrows * row_size;
}

} // extern "C"
