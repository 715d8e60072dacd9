// gen_fixtures.c -- TEST INFRASTRUCTURE ONLY.
//
// Golden-vector generator. Links the REAL reference ggml (oracle/_ref/libggml_ref.so, built by
// oracle/Makefile from /root/reference/src with the reference CMake's x86 flags) and writes the
// reference's own outputs for the mul_mat hot path: quantized weights (ggml_quantize_chunk,
// src/ggml.c:21594), dequantized weights (type_traits.to_float), quantized activations
// (type_traits[vec_dot_type].from_float -- the AVX2 code path the CPU mul_mat uses,
// src/ggml.c:11952-11974) and mul_mat outputs computed by ggml_graph_compute on the CPU
// (src/ggml.c:11808-12097).
//
// Inputs are drawn from a *specified* generator (splitmix64, value = (u>>40)*2^-24*2-1), not
// std::uniform_real_distribution, so Python can regenerate them bit-for-bit
// (ggml-imax_amd/ggml_mi355x/synth.py implements the same stream).
//
// Usage: gen_fixtures <outdir>   (driven by tests/golden/make_golden.py)

#include "ggml.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t splitmix64_next(uint64_t * s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void fill_uniform(float * x, size_t n, uint64_t seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; i++) {
        const uint64_t u = splitmix64_next(&s);
        x[i] = (float) (u >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    }
}

static const char * g_out;
static FILE * g_manifest;
static int g_first = 1;

static void put_blob(const char * name, const void * data, size_t n) {
    char path[1024];
    snprintf(path, sizeof(path), "%s/%s", g_out, name);
    FILE * f = fopen(path, "wb");
    if (!f) { perror(path); exit(1); }
    fwrite(data, 1, n, f);
    fclose(f);
}

static void manifest_case(const char * name, int type, int64_t K, int64_t N, int64_t B,
                          uint64_t wseed, uint64_t xseed, int large) {
    fprintf(g_manifest, "%s\n  {\"name\": \"%s\", \"type\": %d, \"type_name\": \"%s\", \"K\": %lld, \"N\": %lld, \"B\": %lld,"
            " \"wseed\": %llu, \"xseed\": %llu, \"large\": %d}",
            g_first ? "" : ",", name, type, ggml_type_name((enum ggml_type) type), (long long) K, (long long) N,
            (long long) B, (unsigned long long) wseed, (unsigned long long) xseed, large);
    g_first = 0;
}

// One mul_mat case: W [K, N] of `type`, X [K, B] f32.
static void run_case(const char * name, enum ggml_type type, int64_t K, int64_t N, int64_t B,
                     uint64_t wseed, uint64_t xseed, int large, int nthreads) {
    const ggml_type_traits_t tt = ggml_internal_get_type_traits(type);
    const ggml_type_traits_t vt = ggml_internal_get_type_traits(tt.vec_dot_type);

    float * wf = malloc(sizeof(float) * K * N);
    float * xf = malloc(sizeof(float) * K * B);
    fill_uniform(wf, (size_t) (K * N), wseed);
    fill_uniform(xf, (size_t) (K * B), xseed);

    const size_t wrow = ggml_row_size(type, K);
    uint8_t * wq = malloc(wrow * N);
    ggml_quantize_chunk(type, wf, wq, 0, N, K, NULL);

    // mul_mat on the reference CPU executor
    const size_t ctx_size = wrow * N + sizeof(float) * (K * B + N * B) + 16 * 1024 * 1024;
    struct ggml_init_params ip = { ctx_size, NULL, false };
    struct ggml_context * ctx = ggml_init(ip);
    struct ggml_tensor * tw = ggml_new_tensor_2d(ctx, type, K, N);
    struct ggml_tensor * tx = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, B);
    memcpy(tw->data, wq, wrow * N);
    memcpy(tx->data, xf, sizeof(float) * K * B);
    struct ggml_tensor * ty = ggml_mul_mat(ctx, tw, tx);
    struct ggml_cgraph * gf = ggml_new_graph(ctx);
    ggml_build_forward_expand(gf, ty);
    ggml_graph_compute_with_ctx(ctx, gf, nthreads);

    char fn[512];
    snprintf(fn, sizeof(fn), "%s.y.f32", name);
    put_blob(fn, ty->data, sizeof(float) * N * B);

    snprintf(fn, sizeof(fn), "%s.wq.bin", name);
    put_blob(fn, wq, wrow * N);

    if (!large) {
        // dequantized weights (to_float) and quantized activations (from_float of vec_dot_type)
        if (type != GGML_TYPE_F32 && K * N <= 16384) {
            float * wd = malloc(sizeof(float) * K * N);
            for (int64_t r = 0; r < N; r++) tt.to_float(wq + r * wrow, wd + r * K, K);
            snprintf(fn, sizeof(fn), "%s.wdq.f32", name);
            put_blob(fn, wd, sizeof(float) * K * N);
            free(wd);
        }
        if (tt.vec_dot_type != GGML_TYPE_F32) {
            const size_t xrow = ggml_row_size(tt.vec_dot_type, K);
            uint8_t * xq = malloc(xrow * B);
            for (int64_t c = 0; c < B; c++) vt.from_float(xf + c * K, xq + c * xrow, K);
            snprintf(fn, sizeof(fn), "%s.xq.bin", name);
            put_blob(fn, xq, xrow * B);
            free(xq);
        }
    }
    manifest_case(name, type, K, N, B, wseed, xseed, large);

    ggml_free(ctx);
    free(wq);
    free(wf);
    free(xf);
}

// tests/test-quantize-fns.cpp:28-32 synthetic data: 0.1 + 2*cos(i + offset)
static void run_cos_case(enum ggml_type type) {
    const int n = 4096;
    float x[4096];
    for (int i = 0; i < n; i++) x[i] = 0.1f + 2.0f * cosf((float) i + 0.0f);
    const size_t rs = ggml_row_size(type, n);
    uint8_t * q = malloc(rs);
    ggml_quantize_chunk(type, x, q, 0, 1, n, NULL);
    char fn[256];
    snprintf(fn, sizeof(fn), "cos_%s.wq.bin", ggml_type_name(type));
    put_blob(fn, q, rs);
    put_blob("cos_input.f32", x, sizeof(x));
    free(q);
}

int main(int argc, char ** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s outdir\n", argv[0]); return 1; }
    g_out = argv[1];
    char mpath[1024];
    snprintf(mpath, sizeof(mpath), "%s/cases.json", g_out);
    g_manifest = fopen(mpath, "w");
    fprintf(g_manifest, "[");

    const enum ggml_type types[] = { GGML_TYPE_F32, GGML_TYPE_F16, GGML_TYPE_Q4_0, GGML_TYPE_Q8_0, GGML_TYPE_Q4_K, GGML_TYPE_Q5_K };
    for (size_t t = 0; t < sizeof(types) / sizeof(types[0]); t++) {
        const enum ggml_type ty = types[t];
        char name[128];
        // small: ragged batch, N not a multiple of any tile
        snprintf(name, sizeof(name), "s_%s", ggml_type_name(ty));
        run_case(name, ty, 256, 48, 5, 1000 + ty, 2000 + ty, 0, 4);
        // medium: K of the 4096 configs, a few rows
        snprintf(name, sizeof(name), "m_%s", ggml_type_name(ty));
        run_case(name, ty, ty == GGML_TYPE_F32 || ty == GGML_TYPE_F16 ? 1024 : 4096, 40, 3, 3000 + ty, 4000 + ty, 0, 4);
        // batched: enough columns to exercise the MFMA prefill path
        snprintf(name, sizeof(name), "b_%s", ggml_type_name(ty));
        run_case(name, ty, 512, 96, 72, 5000 + ty, 6000 + ty, 0, 8);
        if (ty != GGML_TYPE_F32) run_cos_case(ty);
    }
    // BASELINE.json configs (large: weights hashed, outputs kept)
    run_case("L_q4_0_4096x4096", GGML_TYPE_Q4_0, 4096, 4096, 1, 42, 43, 1, 8);
    run_case("L_q4_K_4096x4096", GGML_TYPE_Q4_K, 4096, 4096, 1, 42, 43, 1, 8);
    run_case("L_q4_K_4096x11008", GGML_TYPE_Q4_K, 4096, 11008, 1, 42, 43, 1, 8);
    run_case("L_q5_K_4096x11008", GGML_TYPE_Q5_K, 4096, 11008, 1, 42, 43, 1, 8);
    run_case("L_q8_0_4096x11008", GGML_TYPE_Q8_0, 4096, 11008, 1, 42, 43, 1, 8);
    run_case("L_f32_256x256", GGML_TYPE_F32, 256, 256, 256, 42, 43, 1, 8);
    run_case("L_q4_K_4096x4096_b8", GGML_TYPE_Q4_K, 4096, 4096, 8, 42, 43, 1, 8);
    // prefill (configs[4], B=512) and the mid-batch sizes: Y is kept as its SHA-256 plus sampled
    // columns (tests/golden/make_golden.py); X = the first B columns of the seed-43 stream
    run_case("P_q4_K_4096x4096_b512", GGML_TYPE_Q4_K, 4096, 4096, 512, 42, 43, 1, 8);
    run_case("P_q4_K_4096x4096_b64", GGML_TYPE_Q4_K, 4096, 4096, 64, 42, 43, 1, 8);
    run_case("P_q4_K_4096x4096_b32", GGML_TYPE_Q4_K, 4096, 4096, 32, 42, 43, 1, 8);
    run_case("P_q4_K_4096x4096_b16", GGML_TYPE_Q4_K, 4096, 4096, 16, 42, 43, 1, 8);
    run_case("P_q4_K_4096x4096_b9", GGML_TYPE_Q4_K, 4096, 4096, 9, 42, 43, 1, 8);
    run_case("P_q5_K_4096x11008_b64", GGML_TYPE_Q5_K, 4096, 11008, 64, 42, 43, 1, 8);

    fprintf(g_manifest, "\n]\n");
    fclose(g_manifest);
    return 0;
}
