// mi355x_kernels.h -- host-side launchers of the gfx950 kernels (internal to the backend).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Activation columns of one mul_mat, quantized exactly as the reference CPU path quantizes
// them (vec_dot_type from_float, src/ggml.c:11952-11974), stored structure-of-arrays in HBM:
//   qs  [ncols][K]      int8 quants
//   d   [ncols][K/QK]   f32 block scale (Q8_0: the fp16-rounded d; Q8_K: f32 d)
//   s32 [ncols][K/32]   int16 sums of 32 quants (Q8_K only; = bsums[2j] + bsums[2j+1])
struct mi_act_q8 {
    int8_t * qs;
    float * d;
    int16_t * s32;
    int64_t K;
    int64_t ncols;
};

// Strided f32 activation source: column c = i1 + ne1*(i2 + ne2*i3) starts at
// base + i1*nb1 + i2*nb2 + i3*nb3 (elements along K contiguous).
struct mi_src_cols {
    const char * base;
    int64_t ne1, ne2, ne3;
    size_t nb1, nb2, nb3;
};

// Weight matrix / output description shared by the mul_mat launchers.
struct mi_mm_desc {
    const void * W;        // src0 data
    int type;              // ggml_type of src0
    int64_t K, N;          // ne00, ne01
    int64_t ne02, ne03;    // src0 batch dims (broadcast into src1's)
    size_t nb01, nb02, nb03;
    int64_t ne11, ne12, ne13;  // src1 columns / batch dims
    float * dst;
    size_t nb1, nb2, nb3;  // dst strides in bytes (nb0 == 4)
};

size_t mi_act_q8_bytes(int64_t K, int64_t ncols, bool is_q8K);
mi_act_q8 mi_act_q8_carve(void * base, int64_t K, int64_t ncols, bool is_q8K);

void mi_quantize_q8_0(const mi_src_cols & x, int64_t K, const mi_act_q8 & act, hipStream_t s);
void mi_quantize_q8_K(const mi_src_cols & x, int64_t K, const mi_act_q8 & act, hipStream_t s);
// blocked: write the GEMM's K-blocked layout [K/16][ncols][16] instead of [ncols][K];
// src_f16: the columns are f16 already (copied, not rounded)
void mi_convert_f16(const mi_src_cols & x, int64_t K, uint16_t * out, hipStream_t s, bool blocked = false, bool src_f16 = false);
// quantize to q8_K / q8_0 exactly as above and store f16(d * q) as [ncols][K] (no q8 blocks):
// the activation operand of mi_mul_mat_mmq for quantized weights
void mi_quantize_expand_f16(const mi_src_cols & x, int64_t K, int64_t ncols, bool is_q8K, uint16_t * xh, hipStream_t s,
                            bool blocked = false);
// the layout mi_mul_mat_mmq expects for xh under the current tuning (true: K-blocked)
bool mi_mmq_wants_blocked();

// quantized weights x quantized activations (integer dot products), any number of columns
void mi_mul_mat_q(const mi_mm_desc & m, const mi_act_q8 & act, hipStream_t s);

// Decode-regime mul_mat with the activation quantizer fused in; one launch serves up to
// kMiMaxMembers independent mul_mats of identical weight type / shape (2-D weights, 2-D f32 src1
// with 16-byte aligned columns, contiguous f32 dst columns).
constexpr int kMiMaxMembers = 64;
struct mi_mmv_member {
    const void * W;
    const char * X;
    float * dst;
};
struct mi_mmv_group {
    int type;
    int n;                  // members in this launch
    int ncols;              // src1 columns (ne11), 1..8
    int blocks_per_member;  // set by the launcher
    int64_t rows_per_block; // set by the launcher
    int64_t K, N;
    size_t nb01;            // weight row stride (bytes)
    size_t xcol;            // src1 column stride (bytes)
    size_t ycol;            // dst column stride (bytes)
    int abl = 0;            // timing ablation of the reference-order chain (mmv_order 2: no chain; results invalid)
    int ord_rows = 0;       // reference order: rows per chain pass (0: one pass per 64-item chunk of a row)
    int ord_cs = 0;         // reference order: scratch words per (row, column)
    int ord_s = 0;          // reference order: Q4_0/Q8_0 lane-row stride in the scratch
    // the graph's following bias / residual / GELU and K/V row copies (one-member groups; same
    // fields and rounding as mi_f16_epilogue)
    struct epilogue {
        const float * bias = nullptr;
        const char * resid = nullptr;
        size_t resid_nb1 = 0;
        const uint16_t * gelu_table = nullptr;
        struct row_copy {
            int64_t row0 = 0, row1 = 0;
            char * ptr = nullptr;
            size_t col_stride = 0;
        } copy[2];
    } epi;
    // the graph's norm|rms_norm -> mul(g) -> add(b) producing src1, computed by the kernel from X
    // (one-member groups, K <= 768; same semantics as mi_norm_prologue)
    struct prologue {
        const float * g = nullptr;
        const float * b = nullptr;
        float eps = 0.0f;
        int mode = 0;  // 0 none, 1 norm, 2 rms_norm
    } pro;
    int pro_off = 0;   // set by the launcher: LDS byte offset of the normalized columns
    uint64_t * stamps = nullptr;  // diagnostic builds: per-workgroup phase stamps (g_mi_stamp_dev)
    int q0r = 0;       // Q4_0 / Q8_0: every member's W is its 16-byte-aligned repacked copy (mi_planes_get type 2 / 8), nb01 = K / 32 * 18 / 34
    int pro_q = 0;     // set by the launcher (g_mi_tuning.mmv_pro4): one Q8_K column's norm prologue quantizes from registers
    mi_mmv_member m[kMiMaxMembers];
};
// Diagnostic builds (make DIAG=1): when non-null, the decode kernels write s_memrealtime phase
// stamps of wave 0 of every workgroup here (kMiStampSlots per workgroup); release builds never do
extern uint64_t * g_mi_stamp_dev;
constexpr int kMiStampSlots = 8;
bool mi_stamps_enable(size_t slots);  // 0: off; false in release builds
void mi_stamps_reset();
bool mi_diag_build();  // this library's kernels were built with MI_DIAG (make diaglib)
// the next launch's stamp range (nullptr when off or full); logs "name nblocks offset"
uint64_t * mi_stamp_take(const char * name, unsigned nblocks);
// copies up to n stamp words and the log; returns the words written so far
size_t mi_stamps_read(uint64_t * host, size_t n, char * log, size_t log_size);
bool mi_mmv_fused_supported(int type, int64_t K, int64_t ncols);
constexpr int64_t kMiMmvProMaxK = 768;  // norm prologue: the column is held in one wave's registers

// launch-shape knobs of the streaming kernels (defaults tuned on MI355X; settable for A/B runs)
struct mi_tuning {
    int mmv_blocks;   // target resident workgroups for the fused GEMV (all members)
    int mmv_variant;  // 10*prefetch_depth + {0: activations in VGPRs, 1: from LDS, 2: LDS + waves/EU cap}
    int f16_variant;  // decode F16 GEMV: 0 = 16 lanes per row (k_mmv_f16_w16), 1 = quad per row (k_mmv_f16_x)
    int f16_threads;  // k_mmv_f16_w16 workgroup size override (0 = automatic)
    int mmq_variant;  // prefill GEMM: 0 = k_mmq3 (activations in registers), 1 = k_mmq2 (activations via LDS)
    int attn_variant; // attention block: 0 = k_attn_fast where it fits, 1 = k_attn_ordered
    int attn_abl;     // timing ablations of k_attn_fast (0 = none; results invalid otherwise)
    int mmv_order;    // decode GEMVs (quantized and F16) and attention: 1 = the reference CPU's summation order (bit-identical,
                      // slower), 0 = tree sums, -1 (default) = per graph: 1 where a quantized MUL_MAT consumes a value the
                      // graph computes (its activation re-quantization would carry order differences forward), else 0
    int f16_waves;    // fast F16 decode GEMV: target waves on the chip (0 = automatic)
    int f16_rgs;      // fast F16 decode GEMV: row groups (4 rows) per workgroup (0 = automatic)
    int f16_ps_waves; // k_gemv_f16_ps (GEMV over summed partials): waves per workgroup, 2 / 4 / 8 (0 = automatic)
    int mmq_long;     // Q4_K / Q5_K prefill past 128 columns: 0 = automatic (Q4_K k_mmqt, Q5_K k_mmqw), 1 = k_mmqw, 2 = k_mmqt; 16-23 k_mmqt stamps (diagnostic builds)
    int xfirst;       // lone decode GEMVs: activation loads issued and landed before the weight loads: 1 always, 0 / -1 never (-1: the default)
    int f16_norm_waves; // F16 GEMV, several columns with the norm prologue: waves per workgroup (0 = automatic)
    int planes;       // long Q4_K prompts on repacked MFMA planes (mmq_planes.hip k_mmqr): 1 on, 0 off (default: slower than k_mmqt with HBM-streamed weights)
    int f16_nc;       // F16 decode GEMVs: columns per workgroup at most (ones digit: plain, tens: norm prologue; 0: up to 8)
    int mmv_dma;      // grouped tree-order Q4_K GEMVs on the LDS-DMA weight stream (k_mmv_dma): 0 off, 1-3 shapes, +10 default load policy
    int f16_bn;       // F16 decode GEMVs, 2..8 columns with the norm prologue (K <= 1024) on k_gemv_f16_bn: 0 off, 1-5 shapes (default 5), +10 one column too
    int f16_bp;       // F16 decode GEMVs, 2..8 plain columns (K <= 3072) on k_gemv_f16_bn's staging form: 0 off, 1 on
    int q40r;         // tree-order Q4_0 decode GEMVs on the 16-byte-aligned repacked copy (mmq_planes.hip k_q40_repack, FmtQ0R): 1 on (default), 0 off
    int q80r;         // tree-order Q8_0 decode GEMVs on the 16-byte-aligned repacked copy (k_q80_repack, FmtQ8R): 1 on (default), 0 off
    int mmv_pro4;     // decode GEMVs with the norm prologue, one Q8_K column: normalize and quantize in registers (norm_quant_prologue1): 1 (default), 0 through LDS
    int f16_mt;       // tall F16 GEMVs (lm_head) of 2..8 columns, K <= 768, on the matrix cores (k_gemv_f16_mt): 1 on (default), 0 k_gemv_f16_tall
    int f16_m8;       // plain F16 GEMVs of 2..8 columns (K <= 4096, K % 32 == 0) on the matrix cores (k_gemv_f16_m8): 0 off (default), 1 on (diagnostic builds: measured slower)
    int mmqt_short;   // Q4_K prompts of 33..128 columns on k_mmqt (128 x 64 tiles) when a launch has at least this many of its workgroups (default 192; 0: never)
};
extern mi_tuning g_mi_tuning;
// the order of the graph being launched when mmv_order is -1 (set by the backend per graph)
extern thread_local int tl_mi_graph_order;
inline int mi_mmv_order() { return g_mi_tuning.mmv_order >= 0 ? g_mi_tuning.mmv_order : tl_mi_graph_order; }
size_t mi_mmv_fused_lds_bytes(int type, int64_t K, int64_t ncols);
void mi_mul_mat_q_fused(mi_mmv_group & g, hipStream_t s);
// Batched (prefill) mul_mat on MFMA: 2-D weights [K, N] of type Q4_0/Q8_0/Q4_K/Q5_K/F16,
// `ncols` activation columns already converted: xh = f16 [ncols][K] (F16 weights: the f16
// activations; quantized weights: f16(d * q) from mi_quantize_expand_f16), or, for quantized
// weights with xh == nullptr, the q8 blocks in act expanded into `scratch` first.
// dst columns of ycol bytes. Requires K % 256 == 0.
bool mi_mmq_supported(int type, int64_t K, size_t nb01, size_t ycol);
// F16 weights, 9..128 columns (mmq.hip k_mmf16p): xh = f16 activations in the K-blocked layout
// [K/16][ncols][16]; K % 256 == 0, 16-byte aligned rows (mmq_variant bits 1 / 2^18 turn it off)
bool mi_mmf16p_supported(int64_t K, int64_t N, size_t nb01, int64_t ncols, size_t ycol);
void mi_mul_mat_f16p(const void * W, size_t nb01, int64_t K, int64_t N, const uint16_t * xh, int64_t ncols, float * dst, size_t ycol,
                     hipStream_t s);
// the same reading the f32 src1 columns (xnb1 bytes apart) and rounding them to f16 in the kernel
// (one launch, no conversion pass); 16-byte aligned columns
bool mi_mmf16p_f32_supported(int64_t K, int64_t N, size_t nb01, int64_t ncols, size_t ycol, const void * x, size_t xnb1);
void mi_mul_mat_f16p_f32(const void * W, size_t nb01, int64_t K, int64_t N, const float * x, size_t xnb1, int64_t ncols, float * dst,
                         size_t ycol, hipStream_t s);
// scratch for the f16 expansion of quantized activations when xh == nullptr (0 for F16 weights)
size_t mi_mmq_scratch_bytes(int type, int64_t K, int64_t ncols);
void mi_mul_mat_mmq(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_q8 & act, const uint16_t * xh,
                    int64_t ncols, float * dst, size_t ycol, uint16_t * scratch, hipStream_t s);

// ---- exact-integer prefill GEMM for Q4_K / Q5_K (mmq_exact.hip) ----
// q8_K activation quants in the int8-MFMA layouts: xq [K/64][ncols][64] int8, xd [K/256][ncols]
// f32 scale, xu [K/256][ncols][16] f16 (S_j & 63, S_j >> 6; S_j = sum of the 32 quants of
// sub-block j) -- the bytes of quantize_row_q8_K_reference, rearranged
struct mi_act_mmx {
    int8_t * xq;
    float * xd;
    uint16_t * xu;
    int64_t K;
    int64_t ncols;
};
size_t mi_act_mmx_bytes(int64_t K, int64_t ncols);
mi_act_mmx mi_act_mmx_carve(void * base, int64_t K, int64_t ncols);
void mi_quantize_q8_K_mmx(const mi_src_cols & x, int64_t K, const mi_act_mmx & act, hipStream_t s);
// several activation sources (same K) quantized by one launch
constexpr int kMiMaxPrefillMembers = 16;
struct mi_mmx_qgroup {
    int n = 0;
    int64_t K = 0;
    struct member {
        mi_src_cols x;
        mi_act_mmx act;
        int64_t col_begin;  // set by the launcher
    } m[kMiMaxPrefillMembers];
};
void mi_quantize_q8_K_mmx_group(mi_mmx_qgroup & q, hipStream_t s);
// q8_0 activations (Q4_0 / Q8_0 weights) in the MFMA layout: xq [K/32][ncols][32] int8, xd
// [K/32][ncols] f32 (xu unused) -- the bytes of the AVX2 quantize_row_q8_0, rearranged
size_t mi_act_mmx0_bytes(int64_t K, int64_t ncols);
mi_act_mmx mi_act_mmx0_carve(void * base, int64_t K, int64_t ncols);
void mi_quantize_q8_0_mmx_group(mi_mmx_qgroup & q, hipStream_t s);
// src1 of the weight's vec_dot type (quantize.hip): GGML_OP_CPY F32 -> Q8_K / Q8_0 rows in the
// reference block layouts (dst columns addressed like src1's), and such rows -> the GEMV's q8 SoA
// (act) or the prefill GEMMs' MFMA layout (mx); exactly one of act / mx non-null
void mi_quantize_rows_q8(const mi_src_cols & x, int64_t K, bool is_q8K, const mi_src_cols & dst, hipStream_t s);
void mi_q8_rows_to_act(const mi_src_cols & xs, int64_t K, bool is_q8K, const mi_act_q8 * act, const mi_act_mmx * mx, hipStream_t s);
bool mi_mmqx_supported(int type, int64_t K, size_t ycol, int64_t ncols, size_t nb01);
// Independent Q4_K / Q5_K (q8_K activations) or Q4_0 / Q8_0 (q8_0 activations, mi_act_mmx0_*)
// mul_mats (same type, K and activation column count) in one launch:
// member i = 2-D weights [K, N_i] x act_i.ncols columns -> dst_i (column stride ycol_i bytes)
struct mi_mmx_member {
    const void * W;
    size_t nb01;
    int64_t N;
    mi_act_mmx act;
    float * dst;
    size_t ycol;
    int64_t tile_begin;  // set by the launcher
    const char * planes;  // Q4_K / Q5_K: the weights' repacked MFMA planes (mi_planes_get) or null
};
struct mi_mmx_group {
    int type = 0;
    int n = 0;
    int64_t K = 0;
    mi_mmx_member m[kMiMaxPrefillMembers];
};
void mi_mul_mat_mmqx_group(mi_mmx_group & g, hipStream_t s);
// one member
void mi_mul_mat_mmqx(int type, const void * W, size_t nb01, int64_t K, int64_t N, const mi_act_mmx & act, float * dst,
                     size_t ycol, hipStream_t s, const char * planes = nullptr);
// Repacked MFMA planes of Q4_K / Q5_K weights for long prompts (mmq_planes.hip): per 32-row tile
// and superblock the int8 planes q * (sc_j bit field) in v_mfma_i32_32x32x32_i8 operand order, the
// U operand [m_j, 64 m_j] and (d, dmin) -- a device-side copy kept next to the canonical blocks,
// which stay untouched (get_tensor, views, GET_ROWS, cpy see the reference bytes). mi_planes_get
// returns the planes of W (creating them with one repack launch on s when missing and s is not
// capturing), or null (disabled: GGML_MI355X_PLANES=0, unsupported shape, capture). Any write to
// weight memory must be followed by mi_planes_refresh over the written bytes (a repack launch on
// s for every overlapping entry; capturable); freeing the memory by mi_planes_drop.
// mmq_variant bits of opt-in kernel forms measured slower than the defaults: diagnostic builds only
constexpr int kMiMmqDiagBits = (1 << 19) | (1 << 26);  // (bit 2^17 doubles as k_mmqx's full-width bit)
constexpr int64_t kMiPlanesMinCols = 129;  // prompts of more columns take the planes kernel
// Types 2 / 8 (Q4_0 / Q8_0, g_mi_tuning.q40r / q80r): the tree-order decode GEMV's 16-byte-aligned
// copy instead (k_q40_repack / k_q80_repack: per row the quants of every block, then their f16
// scales; K / 32 * 18 / 34 bytes a row).
const char * mi_planes_get(int type, const void * W, size_t nb01, int64_t K, int64_t N, hipStream_t s);
void mi_planes_refresh(const void * lo, size_t bytes, hipStream_t s);
void mi_planes_drop(const void * lo, size_t bytes);
size_t mi_planes_count();
uint64_t mi_planes_generation();  // changes whenever a planes entry is created or dropped (graph keys)
size_t mi_planes_bytes();
// the planes kernel over a group whose members all carry planes (false: not applicable)
bool mi_mul_mat_mmqr_group(mi_mmx_group & g, hipStream_t s);

// ---- companion ops (ops.hip) ----
// a tensor view as the element-wise kernels see it: f32 (type 0), f16 (1) or i32 (26) elements
struct mi_tensor_desc {
    char * data;
    int type;
    int64_t ne[4];
    size_t nb[4];
};
enum mi_elt_op { MI_OP_ADD, MI_OP_MUL, MI_OP_SUB, MI_OP_DIV, MI_OP_SCALE, MI_OP_GELU, MI_OP_SILU, MI_OP_CPY };
void mi_op_binary(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & b, int op, hipStream_t s);
void mi_op_unary(const mi_tensor_desc & d, const mi_tensor_desc & a, int op, float p0, const uint16_t * table, hipStream_t s);
void mi_op_cpy(const mi_tensor_desc & d, const mi_tensor_desc & a, hipStream_t s);
// several independent copies (element i of a[c] -> element i of d[c]) in one launch
constexpr int kMiMaxCopies = 4;
void mi_op_cpy_multi(const mi_tensor_desc * d, const mi_tensor_desc * a, int count, hipStream_t s);
void mi_op_get_rows(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & idx, hipStream_t s);
// d = get_rows(a, ia) + get_rows(b, ib) (1-D index vectors, f32 dst): the graph's two GET_ROWS and
// their ADD in one launch, each value as the separate nodes compute it
void mi_op_get_rows_add(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & ia, const mi_tensor_desc & b,
                        const mi_tensor_desc & ib, hipStream_t s);
void mi_op_diag_mask(const mi_tensor_desc & d, const mi_tensor_desc & a, int n_past, float value, hipStream_t s);
// norm / rms_norm; g, b (optional, 1-D over ne0): the graph's following mul(., g) and add(., b)
void mi_op_norm(const mi_tensor_desc & d, const mi_tensor_desc & a, float eps, bool rms, const float * g, const float * b,
                hipStream_t s);
// rope f32 forward, modes 0/2; corr = ggml_rope_yarn_corr_dims() computed on the host; tab: the
// backend's host-built {cos, sin} table [tab_p][pairs] for positions < tab_p (or null)
void mi_op_rope(const mi_tensor_desc & d, const mi_tensor_desc & a, const int32_t * pos, int n_dims, int mode, float freq_base,
                float freq_scale, float ext_factor, float attn_factor, float corr0, float corr1, const float * tab, int tab_p,
                hipStream_t s);
// soft_max (max_bias 0); n_past >= 0 fuses the preceding scale(pre_scale) + diag_mask_inf(n_past)
void mi_op_soft_max(const mi_tensor_desc & d, const mi_tensor_desc & a, const mi_tensor_desc & mask, float scale,
                    const uint16_t * exp_table, float pre_scale, int n_past, hipStream_t s);

// Decode-regime F16 mul_mat (2-D weights, few f32 src1 columns of contiguous K) that converts the
// activations itself and applies the graph's following bias add / residual add / GELU.
struct mi_f16_epilogue {
    const float * bias = nullptr;        // [N] f32, or null
    const char * resid = nullptr;        // [N, ncols] f32 (row stride resid_nb1), or null
    size_t resid_nb1 = 0;
    const uint16_t * gelu_table = nullptr;  // fp16 GELU table (applied after bias), or null
    // up to two extra destinations of output row ranges (the graph's following CPY of a row view of
    // the output, e.g. GPT-2's K/V cache writes): element (row, col) with row0 <= row < row1 is
    // also stored at ptr + col * col_stride + (row - row0) * 4
    struct row_copy {
        int64_t row0 = 0, row1 = 0;
        char * ptr = nullptr;
        size_t col_stride = 0;
    } copy[2];
    uint64_t * stamps = nullptr;  // diagnostic builds: phase stamps (g_mi_stamp_dev)
    int xfirst = 0;               // set by the launcher (g_mi_tuning.xfirst): activations landed before the weight loads
};
// optional prologue: src1 = add(mul(norm|rms_norm(x, eps), g), b) computed in the kernel from x
struct mi_norm_prologue {
    const float * g = nullptr;  // [K] or null
    const float * b = nullptr;  // [K] or null
    float eps = 0.0f;
    int mode = 0;               // 0 none, 1 norm, 2 rms_norm
    // the norm's input as partial sums (mi_attn_proj's output; fast F16 path, one column only):
    // x = sum_{p < nparts} parts[p][0 .. K), and the first workgroup stores x to `store`
    const float * parts = nullptr;
    int nparts = 0;
    float * store = nullptr;
};
bool mi_mul_mat_f16_fused_supported(int64_t K, int64_t ncols);
// xh: optional f16 [ncols][K] activations already converted (then x is not read)
void mi_mul_mat_f16_fused(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh,
                          int64_t ncols, float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro,
                          hipStream_t s);

// the same in tree order (mmv_f16.hip; the fast F16 decode mode, mmv_order 0): 1..8 columns,
// K % 8 == 0, 16-byte aligned activation columns (or xh), norm prologue for K <= 3072
bool mi_mul_mat_f16_fast_supported(int64_t K, int64_t ncols, const mi_src_cols & x, const uint16_t * xh, const mi_norm_prologue & pro);
void mi_mul_mat_f16_fast(const void * W, size_t nb01, int64_t K, int64_t N, const mi_src_cols & x, const uint16_t * xh, int64_t ncols,
                         float * dst, size_t ycol, const mi_f16_epilogue & e, const mi_norm_prologue & pro, hipStream_t s);

// attention of the GPT-2 graph (KQ, scale, causal mask, soft_max, KQV, merge) in one launch,
// bit-identical to the separate nodes. Strides in bytes; element (i0, i1, i2) at base + sum i*nb.
struct mi_attn_desc {
    const char * q;   // Q [D, N, H]
    size_t q_nb[3];
    const char * k;   // K [D, n_kv, Hk]
    size_t k_nb[3];
    const char * v;   // V_trans [n_kv, D, Hk]
    size_t v_nb[3];
    char * out;       // KQV (d, t, h) destination
    size_t o_nb[3];
    int D, N, H, n_kv, r2;  // r2 = H / Hk
    int n_past;             // diag_mask_inf n_past
    float pre_scale;        // ggml_scale factor
    float sm_scale;         // soft_max scale (op_params[0])
    const char * mask = nullptr;  // ADD(scale(KQ), mask) form: F32 mask [n_kv, N] added after the
    size_t mask_nb1 = 0;          // pre-scale (n_past then disables the causal mask)
};
bool mi_attn_supported(int D, int n_kv);
// mmv_order 1 (or attn_variant 1): the reference's summation order, bit-identical; otherwise the
// tree-order kernel of attn_fast.hip where it applies (mi_attn_tree_supported)
void mi_attn_ordered(const mi_attn_desc & a, const uint16_t * exp_table, hipStream_t s);
bool mi_attn_tree_supported(const mi_attn_desc & a);
void mi_attn_tree(const mi_attn_desc & a, hipStream_t s);
// one decode token's attention fused with the F16 output projection W [K = D H, N] that consumes
// it, plus the projection's bias and residual ADDs: parts[h][i] = W[i, hD .. hD + D) . o_h (head 0
// also + bias[i] + resid[i]); sum_h parts[h] (head order) is the projection's output
struct mi_attn_proj_desc {
    const uint8_t * W;
    size_t nb01;
    int64_t N;
    const float * bias;   // [N]
    const float * resid;  // [N]
    float * parts;        // [H][N]
    uint64_t * stamps = nullptr;  // diagnostic builds: phase stamps (g_mi_stamp_dev)
};
bool mi_attn_proj_supported(const mi_attn_desc & a, int64_t K, int64_t N, size_t nb01, const void * W);
void mi_attn_proj(const mi_attn_desc & a, const mi_attn_proj_desc & p, hipStream_t s);
// out[i] = sum_{h < nparts} parts[h][i], in h order
void mi_sum_parts(float * out, const float * parts, int nparts, int64_t n, hipStream_t s);

// f16 weights x f16-rounded activations
void mi_mul_mat_f16(const mi_mm_desc & m, const uint16_t * xh, hipStream_t s);
// f32 x f32, both operands arbitrarily strided (src1 described by x, src0 by m.nb0x)
void mi_mul_mat_f32(const mi_mm_desc & m, const mi_src_cols & x, hipStream_t s);
