// ggml_abi.h -- ABI-identical re-declaration of the reference ggml data model and plugin API
// for the MI355X backend (NAIST-Archlab/ggml-imax @ v2).
//
// Everything the GGML_OP_MUL_MAT path crosses is declared here with the reference layout:
//   * struct ggml_tensor / ggml_object / ggml_cgraph / ggml_init_params  (include/ggml/ggml.h:542-666)
//   * enum ggml_type / ggml_op / ggml_unary_op / ggml_status               (ggml.h:319-481)
//   * quant block layouts                                                    (src/ggml-common.h:144-321)
//   * the backend vtables ggml_backend_buffer_type_i / ggml_backend_buffer_i / ggml_backend_i,
//     struct ggml_backend / ggml_backend_event / registry init fn           (src/ggml-backend-impl.h:18-137)
//   * the public backend / allocator functions                              (include/ggml/ggml-backend.h, ggml-alloc.h)
// Layout is pinned by static_asserts against the reference build (sizeof(ggml_tensor)=368, ...),
// so a backend compiled against this header loads into the reference libggml unchanged, and
// code written against the reference headers links against our runtime unchanged.
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_API __attribute__((visibility("default")))
#define GGML_CALL

#define GGML_FILE_MAGIC   0x67676d6c
#define GGML_FILE_VERSION 1
#define GGML_QNT_VERSION        2
#define GGML_QNT_VERSION_FACTOR 1000

#define GGML_MAX_DIMS           4
#define GGML_MAX_PARAMS         2048
#define GGML_MAX_CONTEXTS       64
#define GGML_MAX_SRC            10
#define GGML_MAX_NAME           64
#define GGML_MAX_OP_PARAMS      64
#define GGML_DEFAULT_N_THREADS  4
#define GGML_DEFAULT_GRAPH_SIZE 2048
#define GGML_MEM_ALIGN          16

#define GGML_EXIT_SUCCESS 0
#define GGML_EXIT_ABORTED 1

#define GGML_UNUSED(x) (void)(x)
#define GGML_PAD(x, n) (((x) + (n) - 1) & ~((n) - 1))

GGML_API void ggml_print_backtrace(void);

// reference semantics (ggml.h:257-265): print, backtrace, abort
#define GGML_ASSERT(x) \
    do { \
        if (!(x)) { \
            fflush(stdout); \
            fprintf(stderr, "GGML_ASSERT: %s:%d: %s\n", __FILE__, __LINE__, #x); \
            ggml_print_backtrace(); \
            abort(); \
        } \
    } while (0)

enum ggml_status {
    GGML_STATUS_ALLOC_FAILED = -2,
    GGML_STATUS_FAILED       = -1,
    GGML_STATUS_SUCCESS      =  0,
    GGML_STATUS_ABORTED      =  1,
};

typedef uint16_t ggml_fp16_t;
typedef struct { uint16_t bits; } ggml_bf16_t;

struct ggml_object;
struct ggml_context;

enum ggml_type {
    GGML_TYPE_F32 = 0, GGML_TYPE_F16 = 1, GGML_TYPE_Q4_0 = 2, GGML_TYPE_Q4_1 = 3,
    GGML_TYPE_Q5_0 = 6, GGML_TYPE_Q5_1 = 7, GGML_TYPE_Q8_0 = 8, GGML_TYPE_Q8_1 = 9,
    GGML_TYPE_Q2_K = 10, GGML_TYPE_Q3_K = 11, GGML_TYPE_Q4_K = 12, GGML_TYPE_Q5_K = 13,
    GGML_TYPE_Q6_K = 14, GGML_TYPE_Q8_K = 15, GGML_TYPE_IQ2_XXS = 16, GGML_TYPE_IQ2_XS = 17,
    GGML_TYPE_IQ3_XXS = 18, GGML_TYPE_IQ1_S = 19, GGML_TYPE_IQ4_NL = 20, GGML_TYPE_IQ3_S = 21,
    GGML_TYPE_IQ2_S = 22, GGML_TYPE_IQ4_XS = 23, GGML_TYPE_I8 = 24, GGML_TYPE_I16 = 25,
    GGML_TYPE_I32 = 26, GGML_TYPE_I64 = 27, GGML_TYPE_F64 = 28, GGML_TYPE_IQ1_M = 29,
    GGML_TYPE_BF16 = 30,
    GGML_TYPE_COUNT,
};

enum ggml_prec { GGML_PREC_DEFAULT, GGML_PREC_F32 };

enum ggml_backend_type {
    GGML_BACKEND_TYPE_CPU = 0,
    GGML_BACKEND_TYPE_GPU = 10,
    GGML_BACKEND_TYPE_GPU_SPLIT = 20,
};

enum ggml_ftype {
    GGML_FTYPE_UNKNOWN = -1, GGML_FTYPE_ALL_F32 = 0, GGML_FTYPE_MOSTLY_F16 = 1,
    GGML_FTYPE_MOSTLY_Q4_0 = 2, GGML_FTYPE_MOSTLY_Q4_1 = 3, GGML_FTYPE_MOSTLY_Q4_1_SOME_F16 = 4,
    GGML_FTYPE_MOSTLY_Q8_0 = 7, GGML_FTYPE_MOSTLY_Q5_0 = 8, GGML_FTYPE_MOSTLY_Q5_1 = 9,
    GGML_FTYPE_MOSTLY_Q2_K = 10, GGML_FTYPE_MOSTLY_Q3_K = 11, GGML_FTYPE_MOSTLY_Q4_K = 12,
    GGML_FTYPE_MOSTLY_Q5_K = 13, GGML_FTYPE_MOSTLY_Q6_K = 14, GGML_FTYPE_MOSTLY_BF16 = 24,
};

// Operation codes: values are ABI (GGML_OP_MUL_MAT == 23, GGML_OP_COUNT == 76).
enum ggml_op {
    GGML_OP_NONE = 0,
    GGML_OP_DUP, GGML_OP_ADD, GGML_OP_ADD1, GGML_OP_ACC, GGML_OP_SUB, GGML_OP_MUL, GGML_OP_DIV,
    GGML_OP_SQR, GGML_OP_SQRT, GGML_OP_LOG, GGML_OP_SUM, GGML_OP_SUM_ROWS, GGML_OP_MEAN,
    GGML_OP_ARGMAX, GGML_OP_REPEAT, GGML_OP_REPEAT_BACK, GGML_OP_CONCAT, GGML_OP_SILU_BACK,
    GGML_OP_NORM, GGML_OP_RMS_NORM, GGML_OP_RMS_NORM_BACK, GGML_OP_GROUP_NORM,
    GGML_OP_MUL_MAT, GGML_OP_MUL_MAT_ID, GGML_OP_OUT_PROD,
    GGML_OP_SCALE, GGML_OP_SET, GGML_OP_CPY, GGML_OP_CONT, GGML_OP_RESHAPE, GGML_OP_VIEW,
    GGML_OP_PERMUTE, GGML_OP_TRANSPOSE, GGML_OP_GET_ROWS, GGML_OP_GET_ROWS_BACK, GGML_OP_DIAG,
    GGML_OP_DIAG_MASK_INF, GGML_OP_DIAG_MASK_ZERO, GGML_OP_SOFT_MAX, GGML_OP_SOFT_MAX_BACK,
    GGML_OP_ROPE, GGML_OP_ROPE_BACK, GGML_OP_CLAMP, GGML_OP_CONV_TRANSPOSE_1D, GGML_OP_IM2COL,
    GGML_OP_CONV_TRANSPOSE_2D, GGML_OP_POOL_1D, GGML_OP_POOL_2D, GGML_OP_UPSCALE, GGML_OP_PAD,
    GGML_OP_ARANGE, GGML_OP_TIMESTEP_EMBEDDING, GGML_OP_ARGSORT, GGML_OP_LEAKY_RELU,
    GGML_OP_FLASH_ATTN, GGML_OP_FLASH_ATTN_EXT, GGML_OP_FLASH_FF, GGML_OP_FLASH_ATTN_BACK,
    GGML_OP_SSM_CONV, GGML_OP_SSM_SCAN, GGML_OP_WIN_PART, GGML_OP_WIN_UNPART,
    GGML_OP_GET_REL_POS, GGML_OP_ADD_REL_POS, GGML_OP_UNARY, GGML_OP_MAP_UNARY,
    GGML_OP_MAP_BINARY, GGML_OP_MAP_CUSTOM1_F32, GGML_OP_MAP_CUSTOM2_F32, GGML_OP_MAP_CUSTOM3_F32,
    GGML_OP_MAP_CUSTOM1, GGML_OP_MAP_CUSTOM2, GGML_OP_MAP_CUSTOM3, GGML_OP_CROSS_ENTROPY_LOSS,
    GGML_OP_CROSS_ENTROPY_LOSS_BACK,
    GGML_OP_COUNT,
};

enum ggml_unary_op {
    GGML_UNARY_OP_ABS, GGML_UNARY_OP_SGN, GGML_UNARY_OP_NEG, GGML_UNARY_OP_STEP,
    GGML_UNARY_OP_TANH, GGML_UNARY_OP_ELU, GGML_UNARY_OP_RELU, GGML_UNARY_OP_SIGMOID,
    GGML_UNARY_OP_GELU, GGML_UNARY_OP_GELU_QUICK, GGML_UNARY_OP_SILU, GGML_UNARY_OP_HARDSWISH,
    GGML_UNARY_OP_HARDSIGMOID,
    GGML_UNARY_OP_COUNT,
};

enum ggml_object_type { GGML_OBJECT_TYPE_TENSOR, GGML_OBJECT_TYPE_GRAPH, GGML_OBJECT_TYPE_WORK_BUFFER };

enum ggml_tensor_flag {
    GGML_TENSOR_FLAG_INPUT  = 1,
    GGML_TENSOR_FLAG_OUTPUT = 2,
    GGML_TENSOR_FLAG_PARAM  = 4,
};

struct ggml_object {
    size_t offs;
    size_t size;
    struct ggml_object * next;
    enum ggml_object_type type;
    char padding[4];
};

struct ggml_tensor {
    enum ggml_type type;
    enum ggml_backend_type backend;
    struct ggml_backend_buffer * buffer;
    int64_t ne[GGML_MAX_DIMS];
    size_t  nb[GGML_MAX_DIMS];
    enum ggml_op op;
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor * grad;
    struct ggml_tensor * src[GGML_MAX_SRC];
    int     perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;
    struct ggml_tensor * view_src;
    size_t view_offs;
    void * data;
    char name[GGML_MAX_NAME];
    void * extra;
    char padding[8];
};

static const size_t GGML_OBJECT_SIZE = sizeof(struct ggml_object);
static const size_t GGML_TENSOR_SIZE = sizeof(struct ggml_tensor);

typedef bool (*ggml_abort_callback)(void * data);

enum ggml_cgraph_eval_order {
    GGML_CGRAPH_EVAL_ORDER_LEFT_TO_RIGHT = 0,
    GGML_CGRAPH_EVAL_ORDER_RIGHT_TO_LEFT,
    GGML_CGRAPH_EVAL_ORDER_COUNT
};

struct ggml_hash_set {
    size_t size;
    struct ggml_tensor ** keys;
};

struct ggml_cgraph {
    int size;
    int n_nodes;
    int n_leafs;
    struct ggml_tensor ** nodes;
    struct ggml_tensor ** grads;
    struct ggml_tensor ** leafs;
    struct ggml_hash_set visited_hash_table;
    enum ggml_cgraph_eval_order order;
    int     perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;
};

struct ggml_init_params {
    size_t mem_size;
    void * mem_buffer;
    bool   no_alloc;
};

typedef uint8_t ggml_guid[16];
typedef ggml_guid * ggml_guid_t;

#ifndef __cplusplus
_Static_assert(sizeof(struct ggml_tensor) == 368, "ggml_tensor ABI");
_Static_assert(offsetof(struct ggml_tensor, ne) == 16, "ne");
_Static_assert(offsetof(struct ggml_tensor, nb) == 48, "nb");
_Static_assert(offsetof(struct ggml_tensor, op) == 80, "op");
_Static_assert(offsetof(struct ggml_tensor, op_params) == 84, "op_params");
_Static_assert(offsetof(struct ggml_tensor, src) == 160, "src");
_Static_assert(offsetof(struct ggml_tensor, view_src) == 264, "view_src");
_Static_assert(offsetof(struct ggml_tensor, view_offs) == 272, "view_offs");
_Static_assert(offsetof(struct ggml_tensor, data) == 280, "data");
_Static_assert(offsetof(struct ggml_tensor, extra) == 352, "extra");
_Static_assert(sizeof(struct ggml_object) == 32, "ggml_object ABI");
_Static_assert(GGML_OP_MUL_MAT == 23 && GGML_OP_COUNT == 76, "ggml_op ABI");
#else
static_assert(sizeof(struct ggml_tensor) == 368, "ggml_tensor ABI");
static_assert(offsetof(struct ggml_tensor, ne) == 16, "ne");
static_assert(offsetof(struct ggml_tensor, nb) == 48, "nb");
static_assert(offsetof(struct ggml_tensor, op) == 80, "op");
static_assert(offsetof(struct ggml_tensor, op_params) == 84, "op_params");
static_assert(offsetof(struct ggml_tensor, src) == 160, "src");
static_assert(offsetof(struct ggml_tensor, view_src) == 264, "view_src");
static_assert(offsetof(struct ggml_tensor, view_offs) == 272, "view_offs");
static_assert(offsetof(struct ggml_tensor, data) == 280, "data");
static_assert(offsetof(struct ggml_tensor, extra) == 352, "extra");
static_assert(sizeof(struct ggml_object) == 32, "ggml_object ABI");
static_assert(GGML_OP_MUL_MAT == 23 && GGML_OP_COUNT == 76, "ggml_op ABI");
#endif

// ------------------------------------------------------------------------------------------
// core API (ggml.h) -- the subset the runtime implements
// ------------------------------------------------------------------------------------------

GGML_API const char * ggml_status_to_string(enum ggml_status status);
GGML_API float        ggml_fp16_to_fp32(ggml_fp16_t x);
GGML_API ggml_fp16_t  ggml_fp32_to_fp16(float x);
GGML_API void         ggml_fp16_to_fp32_row(const ggml_fp16_t * x, float * y, int64_t n);
GGML_API void         ggml_fp32_to_fp16_row(const float * x, ggml_fp16_t * y, int64_t n);
GGML_API bool         ggml_guid_matches(ggml_guid_t a, ggml_guid_t b);
GGML_API void         ggml_time_init(void);
GGML_API int64_t      ggml_time_ms(void);
GGML_API int64_t      ggml_time_us(void);

GGML_API int64_t ggml_nelements(const struct ggml_tensor * t);
GGML_API int64_t ggml_nrows(const struct ggml_tensor * t);
GGML_API size_t  ggml_nbytes(const struct ggml_tensor * t);
GGML_API size_t  ggml_nbytes_pad(const struct ggml_tensor * t);
GGML_API int     ggml_blck_size(enum ggml_type type);
GGML_API size_t  ggml_type_size(enum ggml_type type);
GGML_API size_t  ggml_row_size(enum ggml_type type, int64_t ne);
GGML_API const char * ggml_type_name(enum ggml_type type);
GGML_API const char * ggml_op_name(enum ggml_op op);
GGML_API const char * ggml_op_symbol(enum ggml_op op);
GGML_API const char * ggml_unary_op_name(enum ggml_unary_op op);
GGML_API const char * ggml_op_desc(const struct ggml_tensor * t);
GGML_API size_t  ggml_element_size(const struct ggml_tensor * t);
GGML_API bool    ggml_is_quantized(enum ggml_type type);
GGML_API enum ggml_type ggml_ftype_to_ggml_type(enum ggml_ftype ftype);
GGML_API bool    ggml_is_transposed(const struct ggml_tensor * t);
GGML_API bool    ggml_is_contiguous(const struct ggml_tensor * t);
GGML_API bool    ggml_is_permuted(const struct ggml_tensor * t);
GGML_API bool    ggml_is_empty(const struct ggml_tensor * t);
GGML_API bool    ggml_is_scalar(const struct ggml_tensor * t);
GGML_API bool    ggml_is_vector(const struct ggml_tensor * t);
GGML_API bool    ggml_is_matrix(const struct ggml_tensor * t);
GGML_API bool    ggml_is_3d(const struct ggml_tensor * t);
GGML_API int     ggml_n_dims(const struct ggml_tensor * t);
GGML_API bool    ggml_are_same_shape(const struct ggml_tensor * a, const struct ggml_tensor * b);
GGML_API size_t  ggml_tensor_overhead(void);

GGML_API struct ggml_context * ggml_init(struct ggml_init_params params);
GGML_API void   ggml_free(struct ggml_context * ctx);
GGML_API size_t ggml_used_mem(const struct ggml_context * ctx);
GGML_API bool   ggml_get_no_alloc(struct ggml_context * ctx);
GGML_API void   ggml_set_no_alloc(struct ggml_context * ctx, bool no_alloc);
GGML_API void * ggml_get_mem_buffer(const struct ggml_context * ctx);
GGML_API size_t ggml_get_mem_size(const struct ggml_context * ctx);
GGML_API size_t ggml_get_max_tensor_size(const struct ggml_context * ctx);

GGML_API struct ggml_tensor * ggml_new_tensor(struct ggml_context * ctx, enum ggml_type type, int n_dims, const int64_t * ne);
GGML_API struct ggml_tensor * ggml_new_tensor_1d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0);
GGML_API struct ggml_tensor * ggml_new_tensor_2d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1);
GGML_API struct ggml_tensor * ggml_new_tensor_3d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2);
GGML_API struct ggml_tensor * ggml_new_tensor_4d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
GGML_API struct ggml_tensor * ggml_dup_tensor(struct ggml_context * ctx, const struct ggml_tensor * src);
GGML_API struct ggml_tensor * ggml_view_tensor(struct ggml_context * ctx, struct ggml_tensor * src);
GGML_API struct ggml_tensor * ggml_get_first_tensor(const struct ggml_context * ctx);
GGML_API struct ggml_tensor * ggml_get_next_tensor(const struct ggml_context * ctx, struct ggml_tensor * tensor);
GGML_API struct ggml_tensor * ggml_get_tensor(struct ggml_context * ctx, const char * name);
GGML_API const char *         ggml_get_name(const struct ggml_tensor * t);
GGML_API struct ggml_tensor * ggml_set_name(struct ggml_tensor * t, const char * name);
GGML_API struct ggml_tensor * ggml_format_name(struct ggml_tensor * t, const char * fmt, ...);
GGML_API void ggml_set_input(struct ggml_tensor * t);
GGML_API void ggml_set_output(struct ggml_tensor * t);
GGML_API void * ggml_get_data(const struct ggml_tensor * t);
GGML_API float * ggml_get_data_f32(const struct ggml_tensor * t);

// ops
GGML_API struct ggml_tensor * ggml_mul_mat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API void ggml_mul_mat_set_prec(struct ggml_tensor * a, enum ggml_prec prec);
GGML_API struct ggml_tensor * ggml_dup(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_add(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_add_inplace(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_mul(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_mul_inplace(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_scale(struct ggml_context * ctx, struct ggml_tensor * a, float s);
GGML_API struct ggml_tensor * ggml_scale_inplace(struct ggml_context * ctx, struct ggml_tensor * a, float s);
GGML_API struct ggml_tensor * ggml_norm(struct ggml_context * ctx, struct ggml_tensor * a, float eps);
GGML_API struct ggml_tensor * ggml_rms_norm(struct ggml_context * ctx, struct ggml_tensor * a, float eps);
GGML_API struct ggml_tensor * ggml_gelu(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_gelu_inplace(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_silu(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_unary(struct ggml_context * ctx, struct ggml_tensor * a, enum ggml_unary_op op);
GGML_API enum ggml_unary_op   ggml_get_unary_op(const struct ggml_tensor * t);
GGML_API struct ggml_tensor * ggml_soft_max(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_soft_max_inplace(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_soft_max_ext(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * mask, float scale, float max_bias);
GGML_API struct ggml_tensor * ggml_diag_mask_inf(struct ggml_context * ctx, struct ggml_tensor * a, int n_past);
GGML_API struct ggml_tensor * ggml_diag_mask_inf_inplace(struct ggml_context * ctx, struct ggml_tensor * a, int n_past);
GGML_API struct ggml_tensor * ggml_get_rows(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_rope(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b, int n_dims, int mode, int n_ctx);
GGML_API struct ggml_tensor * ggml_cpy(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_cont(struct ggml_context * ctx, struct ggml_tensor * a);
GGML_API struct ggml_tensor * ggml_cont_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1);
GGML_API struct ggml_tensor * ggml_cont_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2);
GGML_API struct ggml_tensor * ggml_cont_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
GGML_API struct ggml_tensor * ggml_reshape(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
GGML_API struct ggml_tensor * ggml_reshape_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0);
GGML_API struct ggml_tensor * ggml_reshape_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1);
GGML_API struct ggml_tensor * ggml_reshape_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2);
GGML_API struct ggml_tensor * ggml_reshape_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3);
GGML_API struct ggml_tensor * ggml_view_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, size_t offset);
GGML_API struct ggml_tensor * ggml_view_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, size_t nb1, size_t offset);
GGML_API struct ggml_tensor * ggml_view_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, size_t nb1, size_t nb2, size_t offset);
GGML_API struct ggml_tensor * ggml_view_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3, size_t nb1, size_t nb2, size_t nb3, size_t offset);
GGML_API struct ggml_tensor * ggml_permute(struct ggml_context * ctx, struct ggml_tensor * a, int axis0, int axis1, int axis2, int axis3);
GGML_API struct ggml_tensor * ggml_transpose(struct ggml_context * ctx, struct ggml_tensor * a);

// graphs
GGML_API struct ggml_cgraph * ggml_new_graph(struct ggml_context * ctx);
GGML_API struct ggml_cgraph * ggml_new_graph_custom(struct ggml_context * ctx, size_t size, bool grads);
GGML_API size_t ggml_graph_overhead(void);
GGML_API size_t ggml_graph_overhead_custom(size_t size, bool grads);
GGML_API void   ggml_build_forward_expand(struct ggml_cgraph * cgraph, struct ggml_tensor * tensor);
GGML_API struct ggml_tensor * ggml_graph_get_tensor(struct ggml_cgraph * cgraph, const char * name);
GGML_API struct ggml_cgraph ggml_graph_view(struct ggml_cgraph * cgraph, int i0, int i1);
GGML_API void   ggml_graph_clear(struct ggml_cgraph * cgraph);
GGML_API void   ggml_graph_print(const struct ggml_cgraph * cgraph);  // ggml.h:2030

// quantization (ggml.h:2233-2254): imatrix == NULL reference path for the path's types
GGML_API void   ggml_quantize_init(enum ggml_type type);
GGML_API void   ggml_quantize_free(void);
GGML_API bool   ggml_quantize_requires_imatrix(enum ggml_type type);
GGML_API size_t ggml_quantize_chunk(enum ggml_type type, const float * src, void * dst,
                                    int64_t start, int64_t nrows, int64_t n_per_row, const float * imatrix);

// ------------------------------------------------------------------------------------------
// backend API (ggml-backend.h / ggml-backend-impl.h)
// ------------------------------------------------------------------------------------------

typedef struct ggml_backend_buffer_type * ggml_backend_buffer_type_t;
typedef struct ggml_backend_buffer * ggml_backend_buffer_t;
typedef struct ggml_backend_event * ggml_backend_event_t;
typedef struct ggml_backend * ggml_backend_t;
typedef void * ggml_backend_graph_plan_t;

enum ggml_backend_buffer_usage {
    GGML_BACKEND_BUFFER_USAGE_ANY = 0,
    GGML_BACKEND_BUFFER_USAGE_WEIGHTS = 1,
};

typedef void * ggml_backend_buffer_type_context_t;

struct ggml_backend_buffer_type_i {
    const char *          (*get_name)        (ggml_backend_buffer_type_t buft);
    ggml_backend_buffer_t (*alloc_buffer)    (ggml_backend_buffer_type_t buft, size_t size);
    size_t                (*get_alignment)   (ggml_backend_buffer_type_t buft);
    size_t                (*get_max_size)    (ggml_backend_buffer_type_t buft);
    size_t                (*get_alloc_size)  (ggml_backend_buffer_type_t buft, const struct ggml_tensor * tensor);
    bool                  (*supports_backend)(ggml_backend_buffer_type_t buft, ggml_backend_t backend);
    bool                  (*is_host)         (ggml_backend_buffer_type_t buft);
};

struct ggml_backend_buffer_type {
    struct ggml_backend_buffer_type_i iface;
    ggml_backend_buffer_type_context_t context;
};

typedef void * ggml_backend_buffer_context_t;

struct ggml_backend_buffer_i {
    const char * (*get_name)   (ggml_backend_buffer_t buffer);
    void         (*free_buffer)(ggml_backend_buffer_t buffer);
    void *       (*get_base)   (ggml_backend_buffer_t buffer);
    void         (*init_tensor)(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor);
    void         (*set_tensor) (ggml_backend_buffer_t buffer, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
    void         (*get_tensor) (ggml_backend_buffer_t buffer, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
    bool         (*cpy_tensor) (ggml_backend_buffer_t buffer, const struct ggml_tensor * src, struct ggml_tensor * dst);
    void         (*clear)      (ggml_backend_buffer_t buffer, uint8_t value);
    void         (*reset)      (ggml_backend_buffer_t buffer);
};

struct ggml_backend_buffer {
    struct ggml_backend_buffer_i iface;
    ggml_backend_buffer_type_t buft;
    ggml_backend_buffer_context_t context;
    size_t size;
    enum ggml_backend_buffer_usage usage;
};

typedef void * ggml_backend_context_t;

struct ggml_backend_i {
    const char * (*get_name)(ggml_backend_t backend);
    void (*free)(ggml_backend_t backend);
    ggml_backend_buffer_type_t (*get_default_buffer_type)(ggml_backend_t backend);
    void (*set_tensor_async)(ggml_backend_t backend, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
    void (*get_tensor_async)(ggml_backend_t backend, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
    bool (*cpy_tensor_async)(ggml_backend_t backend_src, ggml_backend_t backend_dst, const struct ggml_tensor * src, struct ggml_tensor * dst);
    void (*synchronize)(ggml_backend_t backend);
    ggml_backend_graph_plan_t (*graph_plan_create)(ggml_backend_t backend, const struct ggml_cgraph * cgraph);
    void (*graph_plan_free)(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    enum ggml_status (*graph_plan_compute)(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    enum ggml_status (*graph_compute)(ggml_backend_t backend, struct ggml_cgraph * cgraph);
    bool (*supports_op)(ggml_backend_t backend, const struct ggml_tensor * op);
    bool (*offload_op)(ggml_backend_t backend, const struct ggml_tensor * op);
    ggml_backend_event_t (*event_new)(ggml_backend_t backend);
    void (*event_free)(ggml_backend_event_t event);
    void (*event_record)(ggml_backend_event_t event);
    void (*event_wait)(ggml_backend_t backend, ggml_backend_event_t event);
    void (*event_synchronize)(ggml_backend_event_t event);
};

struct ggml_backend {
    ggml_guid_t guid;
    struct ggml_backend_i iface;
    ggml_backend_context_t context;
};

struct ggml_backend_event {
    ggml_backend_t backend;
    void * context;
};

typedef ggml_backend_t (*ggml_backend_init_fn)(const char * params, void * user_data);

#ifndef __cplusplus
_Static_assert(sizeof(struct ggml_backend_i) == 144, "ggml_backend_i ABI");
_Static_assert(sizeof(struct ggml_backend_buffer_i) == 72, "ggml_backend_buffer_i ABI");
_Static_assert(sizeof(struct ggml_backend_buffer_type_i) == 56, "ggml_backend_buffer_type_i ABI");
#else
static_assert(sizeof(struct ggml_backend_i) == 144, "ggml_backend_i ABI");
static_assert(sizeof(struct ggml_backend_buffer_i) == 72, "ggml_backend_buffer_i ABI");
static_assert(sizeof(struct ggml_backend_buffer_type_i) == 56, "ggml_backend_buffer_type_i ABI");
#endif

// buffer type / buffer
GGML_API const char *          ggml_backend_buft_name(ggml_backend_buffer_type_t buft);
GGML_API ggml_backend_buffer_t ggml_backend_buft_alloc_buffer(ggml_backend_buffer_type_t buft, size_t size);
GGML_API size_t                ggml_backend_buft_get_alignment(ggml_backend_buffer_type_t buft);
GGML_API size_t                ggml_backend_buft_get_max_size(ggml_backend_buffer_type_t buft);
GGML_API size_t                ggml_backend_buft_get_alloc_size(ggml_backend_buffer_type_t buft, struct ggml_tensor * tensor);
GGML_API bool                  ggml_backend_buft_supports_backend(ggml_backend_buffer_type_t buft, ggml_backend_t backend);
GGML_API bool                  ggml_backend_buft_is_host(ggml_backend_buffer_type_t buft);

GGML_API ggml_backend_buffer_t ggml_backend_buffer_init(ggml_backend_buffer_type_t buft, struct ggml_backend_buffer_i iface,
                                                        ggml_backend_buffer_context_t context, size_t size);
GGML_API const char * ggml_backend_buffer_name(ggml_backend_buffer_t buffer);
GGML_API void         ggml_backend_buffer_free(ggml_backend_buffer_t buffer);
GGML_API void *       ggml_backend_buffer_get_base(ggml_backend_buffer_t buffer);
GGML_API size_t       ggml_backend_buffer_get_size(ggml_backend_buffer_t buffer);
GGML_API void         ggml_backend_buffer_init_tensor(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor);
GGML_API size_t       ggml_backend_buffer_get_alignment(ggml_backend_buffer_t buffer);
GGML_API size_t       ggml_backend_buffer_get_max_size(ggml_backend_buffer_t buffer);
GGML_API size_t       ggml_backend_buffer_get_alloc_size(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor);
GGML_API void         ggml_backend_buffer_clear(ggml_backend_buffer_t buffer, uint8_t value);
GGML_API bool         ggml_backend_buffer_is_host(ggml_backend_buffer_t buffer);
GGML_API void         ggml_backend_buffer_set_usage(ggml_backend_buffer_t buffer, enum ggml_backend_buffer_usage usage);
GGML_API ggml_backend_buffer_type_t ggml_backend_buffer_get_type(ggml_backend_buffer_t buffer);
GGML_API void         ggml_backend_buffer_reset(ggml_backend_buffer_t buffer);
GGML_API bool         ggml_backend_buffer_copy_tensor(const struct ggml_tensor * src, struct ggml_tensor * dst);

// backend
GGML_API ggml_guid_t  ggml_backend_guid(ggml_backend_t backend);
GGML_API const char * ggml_backend_name(ggml_backend_t backend);
GGML_API void         ggml_backend_free(ggml_backend_t backend);
GGML_API ggml_backend_buffer_type_t ggml_backend_get_default_buffer_type(ggml_backend_t backend);
GGML_API ggml_backend_buffer_t      ggml_backend_alloc_buffer(ggml_backend_t backend, size_t size);
GGML_API size_t ggml_backend_get_alignment(ggml_backend_t backend);
GGML_API size_t ggml_backend_get_max_size(ggml_backend_t backend);
GGML_API void ggml_backend_tensor_set_async(ggml_backend_t backend, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
GGML_API void ggml_backend_tensor_get_async(ggml_backend_t backend, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
GGML_API void ggml_backend_tensor_set(struct ggml_tensor * tensor, const void * data, size_t offset, size_t size);
GGML_API void ggml_backend_tensor_get(const struct ggml_tensor * tensor, void * data, size_t offset, size_t size);
GGML_API void ggml_backend_synchronize(ggml_backend_t backend);
GGML_API ggml_backend_graph_plan_t ggml_backend_graph_plan_create(ggml_backend_t backend, struct ggml_cgraph * cgraph);
GGML_API void             ggml_backend_graph_plan_free(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
GGML_API enum ggml_status ggml_backend_graph_plan_compute(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
GGML_API enum ggml_status ggml_backend_graph_compute(ggml_backend_t backend, struct ggml_cgraph * cgraph);
GGML_API enum ggml_status ggml_backend_graph_compute_async(ggml_backend_t backend, struct ggml_cgraph * cgraph);
GGML_API bool ggml_backend_supports_op(ggml_backend_t backend, const struct ggml_tensor * op);
GGML_API bool ggml_backend_offload_op(ggml_backend_t backend, const struct ggml_tensor * op);
GGML_API void ggml_backend_tensor_copy(struct ggml_tensor * src, struct ggml_tensor * dst);
GGML_API void ggml_backend_tensor_copy_async(ggml_backend_t backend_src, ggml_backend_t backend_dst, struct ggml_tensor * src, struct ggml_tensor * dst);
GGML_API ggml_backend_event_t ggml_backend_event_new(ggml_backend_t backend);
GGML_API void ggml_backend_event_free(ggml_backend_event_t event);
GGML_API void ggml_backend_event_record(ggml_backend_event_t event);
GGML_API void ggml_backend_event_synchronize(ggml_backend_event_t event);
GGML_API void ggml_backend_event_wait(ggml_backend_t backend, ggml_backend_event_t event);
GGML_API void ggml_backend_tensor_alloc(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor, void * addr);
GGML_API void ggml_backend_view_init(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor);

// registry (ggml-backend.c:395-541; at most 16 entries)
GGML_API void   ggml_backend_register(const char * name, ggml_backend_init_fn init_fn, ggml_backend_buffer_type_t default_buffer_type, void * user_data);
GGML_API size_t ggml_backend_reg_get_count(void);
GGML_API size_t ggml_backend_reg_find_by_name(const char * name);
GGML_API ggml_backend_t ggml_backend_reg_init_backend_from_str(const char * backend_str);
GGML_API const char * ggml_backend_reg_get_name(size_t i);
GGML_API ggml_backend_t ggml_backend_reg_init_backend(size_t i, const char * params);
GGML_API ggml_backend_buffer_type_t ggml_backend_reg_get_default_buffer_type(size_t i);
GGML_API ggml_backend_buffer_t ggml_backend_reg_alloc_buffer(size_t i, size_t size);

// host (pageable) buffer type of the runtime: holds CPU-side tensors (no CPU compute backend)
GGML_API ggml_backend_buffer_type_t ggml_backend_cpu_buffer_type(void);
GGML_API ggml_backend_buffer_t      ggml_backend_cpu_buffer_from_ptr(void * ptr, size_t size);

// multi-buffer (ggml-backend-impl.h:58-61)
GGML_API ggml_backend_buffer_t ggml_backend_multi_buffer_alloc_buffer(ggml_backend_buffer_t * buffers, size_t n_buffers);
GGML_API bool ggml_backend_buffer_is_multi_buffer(ggml_backend_buffer_t buffer);
GGML_API void ggml_backend_multi_buffer_set_usage(ggml_backend_buffer_t buffer, enum ggml_backend_buffer_usage usage);

// ------------------------------------------------------------------------------------------
// allocator (ggml-alloc.h)
// ------------------------------------------------------------------------------------------

struct ggml_tallocr {
    ggml_backend_buffer_t buffer;
    void * base;
    size_t alignment;
    size_t offset;
};

GGML_API struct ggml_tallocr ggml_tallocr_new(ggml_backend_buffer_t buffer);
GGML_API void ggml_tallocr_alloc(struct ggml_tallocr * talloc, struct ggml_tensor * tensor);

typedef struct ggml_gallocr * ggml_gallocr_t;
GGML_API ggml_gallocr_t ggml_gallocr_new(ggml_backend_buffer_type_t buft);
GGML_API ggml_gallocr_t ggml_gallocr_new_n(ggml_backend_buffer_type_t * bufts, int n_bufs);
GGML_API void   ggml_gallocr_free(ggml_gallocr_t galloc);
GGML_API bool   ggml_gallocr_reserve(ggml_gallocr_t galloc, struct ggml_cgraph * graph);
GGML_API bool   ggml_gallocr_reserve_n(ggml_gallocr_t galloc, struct ggml_cgraph * graph, const int * node_buffer_ids, const int * leaf_buffer_ids);
GGML_API bool   ggml_gallocr_alloc_graph(ggml_gallocr_t galloc, struct ggml_cgraph * graph);
GGML_API size_t ggml_gallocr_get_buffer_size(ggml_gallocr_t galloc, int buffer_id);

GGML_API ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors_from_buft(struct ggml_context * ctx, ggml_backend_buffer_type_t buft);
GGML_API ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors(struct ggml_context * ctx, ggml_backend_t backend);

// ------------------------------------------------------------------------------------------
// GGUF model files (include/ggml/ggml.h:2247-2380; csrc/core/gguf.cpp). Same names, argument
// meaning and on-disk layout (v3: magic, version, n_tensors, n_kv, key/values, tensor infos,
// aligned data section).
// ------------------------------------------------------------------------------------------

#define GGUF_MAGIC "GGUF"
#define GGUF_VERSION 3
#define GGUF_DEFAULT_ALIGNMENT 32

enum gguf_type {
    GGUF_TYPE_UINT8 = 0,
    GGUF_TYPE_INT8 = 1,
    GGUF_TYPE_UINT16 = 2,
    GGUF_TYPE_INT16 = 3,
    GGUF_TYPE_UINT32 = 4,
    GGUF_TYPE_INT32 = 5,
    GGUF_TYPE_FLOAT32 = 6,
    GGUF_TYPE_BOOL = 7,
    GGUF_TYPE_STRING = 8,
    GGUF_TYPE_ARRAY = 9,
    GGUF_TYPE_UINT64 = 10,
    GGUF_TYPE_INT64 = 11,
    GGUF_TYPE_FLOAT64 = 12,
    GGUF_TYPE_COUNT,
};

struct gguf_context;

struct gguf_init_params {
    bool no_alloc;
    struct ggml_context ** ctx;  // if not NULL, create a ggml_context holding the tensors
};

GGML_API struct gguf_context * gguf_init_empty(void);
GGML_API struct gguf_context * gguf_init_from_file(const char * fname, struct gguf_init_params params);
GGML_API void gguf_free(struct gguf_context * ctx);
GGML_API const char * gguf_type_name(enum gguf_type type);
GGML_API int    gguf_get_version    (const struct gguf_context * ctx);
GGML_API size_t gguf_get_alignment  (const struct gguf_context * ctx);
GGML_API size_t gguf_get_data_offset(const struct gguf_context * ctx);
GGML_API void * gguf_get_data       (const struct gguf_context * ctx);
GGML_API int          gguf_get_n_kv(const struct gguf_context * ctx);
GGML_API int          gguf_find_key(const struct gguf_context * ctx, const char * key);
GGML_API const char * gguf_get_key (const struct gguf_context * ctx, int key_id);
GGML_API enum gguf_type gguf_get_kv_type (const struct gguf_context * ctx, int key_id);
GGML_API enum gguf_type gguf_get_arr_type(const struct gguf_context * ctx, int key_id);
GGML_API uint8_t      gguf_get_val_u8  (const struct gguf_context * ctx, int key_id);
GGML_API int8_t       gguf_get_val_i8  (const struct gguf_context * ctx, int key_id);
GGML_API uint16_t     gguf_get_val_u16 (const struct gguf_context * ctx, int key_id);
GGML_API int16_t      gguf_get_val_i16 (const struct gguf_context * ctx, int key_id);
GGML_API uint32_t     gguf_get_val_u32 (const struct gguf_context * ctx, int key_id);
GGML_API int32_t      gguf_get_val_i32 (const struct gguf_context * ctx, int key_id);
GGML_API float        gguf_get_val_f32 (const struct gguf_context * ctx, int key_id);
GGML_API uint64_t     gguf_get_val_u64 (const struct gguf_context * ctx, int key_id);
GGML_API int64_t      gguf_get_val_i64 (const struct gguf_context * ctx, int key_id);
GGML_API double       gguf_get_val_f64 (const struct gguf_context * ctx, int key_id);
GGML_API bool         gguf_get_val_bool(const struct gguf_context * ctx, int key_id);
GGML_API const char * gguf_get_val_str (const struct gguf_context * ctx, int key_id);
GGML_API const void * gguf_get_val_data(const struct gguf_context * ctx, int key_id);
GGML_API int          gguf_get_arr_n   (const struct gguf_context * ctx, int key_id);
GGML_API const void * gguf_get_arr_data(const struct gguf_context * ctx, int key_id);
GGML_API const char * gguf_get_arr_str (const struct gguf_context * ctx, int key_id, int i);
GGML_API int            gguf_get_n_tensors    (const struct gguf_context * ctx);
GGML_API int            gguf_find_tensor      (const struct gguf_context * ctx, const char * name);
GGML_API size_t         gguf_get_tensor_offset(const struct gguf_context * ctx, int i);
GGML_API char *         gguf_get_tensor_name  (const struct gguf_context * ctx, int i);
GGML_API enum ggml_type gguf_get_tensor_type  (const struct gguf_context * ctx, int i);
GGML_API void gguf_remove_key(struct gguf_context * ctx, const char * key);
GGML_API void gguf_set_val_u8  (struct gguf_context * ctx, const char * key, uint8_t  val);
GGML_API void gguf_set_val_i8  (struct gguf_context * ctx, const char * key, int8_t   val);
GGML_API void gguf_set_val_u16 (struct gguf_context * ctx, const char * key, uint16_t val);
GGML_API void gguf_set_val_i16 (struct gguf_context * ctx, const char * key, int16_t  val);
GGML_API void gguf_set_val_u32 (struct gguf_context * ctx, const char * key, uint32_t val);
GGML_API void gguf_set_val_i32 (struct gguf_context * ctx, const char * key, int32_t  val);
GGML_API void gguf_set_val_f32 (struct gguf_context * ctx, const char * key, float    val);
GGML_API void gguf_set_val_u64 (struct gguf_context * ctx, const char * key, uint64_t val);
GGML_API void gguf_set_val_i64 (struct gguf_context * ctx, const char * key, int64_t  val);
GGML_API void gguf_set_val_f64 (struct gguf_context * ctx, const char * key, double   val);
GGML_API void gguf_set_val_bool(struct gguf_context * ctx, const char * key, bool     val);
GGML_API void gguf_set_val_str (struct gguf_context * ctx, const char * key, const char * val);
GGML_API void gguf_set_arr_data(struct gguf_context * ctx, const char * key, enum gguf_type type, const void * data, int n);
GGML_API void gguf_set_arr_str (struct gguf_context * ctx, const char * key, const char ** data, int n);
GGML_API void gguf_set_kv(struct gguf_context * ctx, struct gguf_context * src);
GGML_API void gguf_add_tensor(struct gguf_context * ctx, const struct ggml_tensor * tensor);
GGML_API void gguf_set_tensor_type(struct gguf_context * ctx, const char * name, enum ggml_type type);
GGML_API void gguf_set_tensor_data(struct gguf_context * ctx, const char * name, const void * data, size_t size);
GGML_API void   gguf_write_to_file(const struct gguf_context * ctx, const char * fname, bool only_meta);
GGML_API size_t gguf_get_meta_size(const struct gguf_context * ctx);
GGML_API void   gguf_get_meta_data(const struct gguf_context * ctx, void * data);

#ifdef __cplusplus
}
#endif
