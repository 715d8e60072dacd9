// mmv_fused.hip -- decode-regime GGML_OP_MUL_MAT with the activation quantizer fused in, and
// several independent mul_mat nodes of one graph served by a single streaming launch.
//
// Structure (HBM-bound weight stream; MI355X_MICROARCH.md: 8 TB/s, ~6.3 TB/s achievable):
//   * grid = ~4 workgroups per CU (all resident); each workgroup owns a contiguous row range of
//     ONE group member (blockIdx.x -> member, row range), so the activation quantization is paid
//     once per workgroup, not per row;
//   * prologue: issue the weight loads of the first rows (global loads straight to VGPRs), then
//     quantize the member's NC f32 activation columns into LDS with the reference's exact
//     rounding (Q8_K for Q4_K/Q5_K, AVX2-path Q8_0 for Q4_0/Q8_0), barrier;
//   * stream: wave w walks rows w, w+4, ... keeping PD rows of loads in flight in a register ring
//     ahead of the row being computed; v_dot4_i32_i8 against the LDS activations; DPP wave
//     reduction; one store per row.
// A lane's K-items are the same for every row: item = lane + 64*i. Items:
//   Q4_K / Q5_K: (superblock s, 64-element group j): 16 B header + 32 B nibbles (+32 B qh),
//                aligned dwordx4 loads; a K=4096 row is one item per lane.
//   Q4_0 / Q8_0: one 32-element block (18 / 34 B, only 2-byte aligned): aligned dword loads
//                re-aligned with v_alignbyte; a K=4096 row is two items per lane.
//
// Numerics: bit-exact activation quants, exact integer sums per item, f32 combination, i.e.
// ggml_vec_dot_q4_K_q8_K (src/ggml-quants.c:7007-7502), ggml_vec_dot_q5_K_q8_K (:7833-8378),
// ggml_vec_dot_q4_0_q8_0 (:3469-3874), ggml_vec_dot_q8_0_q8_0 (:4819+) up to summation order.


#include "mi355x_common.h"
#include "mi355x_kernels.h"


#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

static int env_int(const char * name, int def) {
    const char * v = getenv(name);
    return v ? atoi(v) : def;
}

// mmv_blocks == 0: size the grid from the kernel's residency (hipOccupancy...) per instance
mi_tuning g_mi_tuning = {env_int("GGML_MI355X_MMV_BLOCKS", 0), env_int("GGML_MI355X_MMV_VARIANT", 0), env_int("GGML_MI355X_F16_VARIANT", 0), 0, env_int("GGML_MI355X_MMQ_VARIANT", 0), env_int("GGML_MI355X_ATTN_VARIANT", 0), env_int("GGML_MI355X_ATTN_ABL", 0), env_int("GGML_MI355X_MMV_ORDER", -1), env_int("GGML_MI355X_F16_WAVES", 0), env_int("GGML_MI355X_F16_RGS", 0), env_int("GGML_MI355X_F16_PS_WAVES", 0), env_int("GGML_MI355X_MMQ_LONG", 0), env_int("GGML_MI355X_XFIRST", -1), env_int("GGML_MI355X_F16_NORM_WAVES", 0), env_int("GGML_MI355X_PLANES", 0), env_int("GGML_MI355X_F16_NC", 10), env_int("GGML_MI355X_MMV_DMA", 0), env_int("GGML_MI355X_F16_BN", 5), env_int("GGML_MI355X_F16_BP", 0), env_int("GGML_MI355X_Q40R", 1), env_int("GGML_MI355X_Q80R", 1), env_int("GGML_MI355X_MMV_PRO4", 1), env_int("GGML_MI355X_F16_MT", 1), env_int("GGML_MI355X_F16_M8", 0), env_int("GGML_MI355X_MMQT_SHORT", 192)};
thread_local int tl_mi_graph_order = 0;

// ---- diagnostic phase stamps (make DIAG=1 builds; MI_STAMP in mi355x_common.h) ----
// A device buffer of kMiStampSlots words per workgroup and launch; each instrumented launch takes
// the next range (mi_stamp_take) and the host log records (kernel, workgroups, offset) so a tool
// can rebuild the device timeline: per-launch first-start / last-end and per-workgroup phases.
uint64_t * g_mi_stamp_dev = nullptr;
static size_t g_mi_stamp_cap = 0, g_mi_stamp_cur = 0;
static std::string g_mi_stamp_log;

bool mi_stamps_enable(size_t slots) {
#if MI_DIAG
    if (g_mi_stamp_dev) (void) hipFree(g_mi_stamp_dev);
    g_mi_stamp_dev = nullptr;
    g_mi_stamp_cap = g_mi_stamp_cur = 0;
    g_mi_stamp_log.clear();
    if (slots == 0) return true;
    if (hipMalloc(&g_mi_stamp_dev, slots * sizeof(uint64_t)) != hipSuccess) {
        g_mi_stamp_dev = nullptr;
        return false;
    }
    (void) hipMemset(g_mi_stamp_dev, 0, slots * sizeof(uint64_t));
    g_mi_stamp_cap = slots;
    return true;
#else
    (void) slots;
    return false;  // release build: the kernels carry no stamps
#endif
}

bool mi_diag_build() { return MI_DIAG != 0; }

void mi_stamps_reset() {
    g_mi_stamp_cur = 0;
    g_mi_stamp_log.clear();
}

uint64_t * mi_stamp_take(const char * name, unsigned nblocks) {
    if (!g_mi_stamp_dev) return nullptr;
    const size_t need = (size_t) nblocks * kMiStampSlots;
    if (g_mi_stamp_cur + need > g_mi_stamp_cap) return nullptr;
    uint64_t * p = g_mi_stamp_dev + g_mi_stamp_cur;
    char line[160];
    snprintf(line, sizeof line, "%s %u %zu\n", name, nblocks, g_mi_stamp_cur);
    g_mi_stamp_log += line;
    g_mi_stamp_cur += need;
    return p;
}

size_t mi_stamps_read(uint64_t * host, size_t n, char * log, size_t log_size) {
    if (!g_mi_stamp_dev) return 0;
    const size_t m = n < g_mi_stamp_cur ? n : g_mi_stamp_cur;
    if (host && m) (void) hipMemcpy(host, g_mi_stamp_dev, m * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (log && log_size) {
        const size_t k = g_mi_stamp_log.size() < log_size - 1 ? g_mi_stamp_log.size() : log_size - 1;
        memcpy(log, g_mi_stamp_log.data(), k);
        log[k] = 0;
    }
    return g_mi_stamp_cur;
}


// per-format launchers (mmv_fused_q4k.hip, _q5k, _q40, _q80: one translation unit each)
void mi_mmv_launch_q4k(const mi_mmv_group & g, int variant, hipStream_t s);
void mi_mmv_launch_q5k(const mi_mmv_group & g, int variant, hipStream_t s);
void mi_mmv_launch_q40(const mi_mmv_group & g, int variant, hipStream_t s);
void mi_mmv_launch_q80(const mi_mmv_group & g, int variant, hipStream_t s);

// LDS of the quantized activations: qs [NC][K] int8 | d [NC][K/QKA] f32 | s32 [NC][K/32] int16
// (lds_bytes in mmv_fused_impl.h)
size_t mi_mmv_fused_lds_bytes(int type, int64_t K, int64_t ncols) {
    const int nc = ncols <= 2 ? (int) ncols : (ncols <= 4 ? 4 : 8);
    const int64_t qka = (type == 12 || type == 13) ? 256 : 32;
    return (size_t) nc * (K + (K / qka) * 4 + (K / 32) * 2);
}

bool mi_mmv_fused_supported(int type, int64_t K, int64_t ncols) {
    if (type != 12 && type != 13 && type != 2 && type != 8) return false;
    if (ncols < 1 || ncols > 8 || K % 256 != 0) return false;
    // more than 4 columns whose activations do not fit run as two launches of <= 4 columns
    return mi_mmv_fused_lds_bytes(type, K, ncols < 4 ? ncols : 4) <= 64 * 1024;  // + <= 36 KB of order scratch
}



static void mi_mul_mat_q_fused_launch(mi_mmv_group & g, hipStream_t s);

void mi_mul_mat_q_fused(mi_mmv_group & g, hipStream_t s) {
    if (g.ncols > 4 && mi_mmv_fused_lds_bytes(g.type, g.K, g.ncols) > 64 * 1024) {
        for (int c0 = 0; c0 < g.ncols; c0 += 4) {
            mi_mmv_group h = g;
            h.ncols = g.ncols - c0 < 4 ? g.ncols - c0 : 4;
            for (int m = 0; m < g.n; m++) {
                h.m[m].X = g.m[m].X + (size_t) c0 * g.xcol;
                h.m[m].dst = (float *) ((char *) g.m[m].dst + (size_t) c0 * g.ycol);
            }
            if (h.epi.resid) h.epi.resid += (size_t) c0 * h.epi.resid_nb1;
            for (auto & cp : h.epi.copy)
                if (cp.ptr) cp.ptr += (size_t) c0 * cp.col_stride;
            mi_mul_mat_q_fused_launch(h, s);
        }
        return;
    }
    mi_mul_mat_q_fused_launch(g, s);
}

static void mi_mul_mat_q_fused_launch(mi_mmv_group & g, hipStream_t s) {
    // variant 0 = per-type default, from interleaved A/B runs on MI355X (tools/mmv_tune.py):
    // prefetch depth 2 for Q4_K / Q8_0 / Q4_0 (Q4_0 in block pairs: 4096 x 11008 5.34 -> 5.58
    // TB/s), depth 1 for Q5_K (fewer VGPRs, more waves)
    // (Nontemporal weight loads -- the guide's nt-weights -- measured 30-37 % SLOWER on every
    // shape, profiles/r04g_nt_ab.txt: removed.) Round-4 defaults from two interleaved sweeps on two
    // boxes (profiles/r04p_gemv_sweep.txt, r04r_gemv_sweep.txt): Q4_K depth 3 (4096^2 +2..4 %,
    // 4096 x 11008 +2..4 %), Q5_K depth 2 (+2 %), Q4_0 pairs depth 3 (+1..4 %), Q8_0 depth 1 (+1 %)
    int variant = g_mi_tuning.mmv_variant;
    if (variant == 0) variant = g.type == 12 ? 31 : g.type == 13 ? 21 : g.type == 2 ? 32 : 11;
    switch (g.type) {
        case 12: mi_mmv_launch_q4k(g, variant, s); break;
        case 13: mi_mmv_launch_q5k(g, variant, s); break;
        case 2: mi_mmv_launch_q40(g, variant, s); break;
        case 8: mi_mmv_launch_q80(g, variant, s); break;
        default: break;
    }
}
