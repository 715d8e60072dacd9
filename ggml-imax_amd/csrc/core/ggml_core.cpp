// ggml_core.cpp -- host runtime: type table, contexts, tensors, op constructors, graphs.
//
// A from-scratch C++ implementation of the reference ggml data model (NAIST-Archlab/ggml-imax
// @ v2, src/ggml.c), ABI-compatible with it (include/ggml_abi.h). It owns no CPU compute
// kernels: graphs built here run on the MI355X backend (csrc/backend/). Semantics follow the
// reference function by function; citations are file:line into the reference.

#include "ggml_abi.h"

#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cinttypes>
#include <cstring>
#include <ctime>
#include <execinfo.h>
#include <mutex>

// ---------------------------------------------------------------------------------------------
// type table (src/ggml.c:564-918: type_name, blck_size, type_size, is_quantized)
// ---------------------------------------------------------------------------------------------

namespace {

struct type_info {
    const char * name;
    int blck;
    size_t size;
    bool quantized;
};

const type_info k_types[GGML_TYPE_COUNT] = {
    /* F32     */ {"f32", 1, 4, false},
    /* F16     */ {"f16", 1, 2, false},
    /* Q4_0    */ {"q4_0", 32, 18, true},
    /* Q4_1    */ {"q4_1", 32, 20, true},
    /* 4       */ {"DEPRECATED", 0, 0, false},
    /* 5       */ {"DEPRECATED", 0, 0, false},
    /* Q5_0    */ {"q5_0", 32, 22, true},
    /* Q5_1    */ {"q5_1", 32, 24, true},
    /* Q8_0    */ {"q8_0", 32, 34, true},
    /* Q8_1    */ {"q8_1", 32, 36, true},
    /* Q2_K    */ {"q2_K", 256, 84, true},
    /* Q3_K    */ {"q3_K", 256, 110, true},
    /* Q4_K    */ {"q4_K", 256, 144, true},
    /* Q5_K    */ {"q5_K", 256, 176, true},
    /* Q6_K    */ {"q6_K", 256, 210, true},
    /* Q8_K    */ {"q8_K", 256, 292, true},
    /* IQ2_XXS */ {"iq2_xxs", 256, 66, true},
    /* IQ2_XS  */ {"iq2_xs", 256, 74, true},
    /* IQ3_XXS */ {"iq3_xxs", 256, 98, true},
    /* IQ1_S   */ {"iq1_s", 256, 50, true},
    /* IQ4_NL  */ {"iq4_nl", 32, 18, true},
    /* IQ3_S   */ {"iq3_s", 256, 110, true},
    /* IQ2_S   */ {"iq2_s", 256, 82, true},
    /* IQ4_XS  */ {"iq4_xs", 256, 136, true},
    /* I8      */ {"i8", 1, 1, false},
    /* I16     */ {"i16", 1, 2, false},
    /* I32     */ {"i32", 1, 4, false},
    /* I64     */ {"i64", 1, 8, false},
    /* F64     */ {"f64", 1, 8, false},
    /* IQ1_M   */ {"iq1_m", 256, 56, true},
    /* BF16    */ {"bf16", 1, 2, false},
};

// GGML_OP_NAME / GGML_OP_SYMBOL (src/ggml.c:2517-2695)
const char * const k_op_names[GGML_OP_COUNT] = {
    "NONE", "DUP", "ADD", "ADD1", "ACC", "SUB", "MUL", "DIV", "SQR", "SQRT", "LOG", "SUM",
    "SUM_ROWS", "MEAN", "ARGMAX", "REPEAT", "REPEAT_BACK", "CONCAT", "SILU_BACK", "NORM",
    "RMS_NORM", "RMS_NORM_BACK", "GROUP_NORM", "MUL_MAT", "MUL_MAT_ID", "OUT_PROD", "SCALE",
    "SET", "CPY", "CONT", "RESHAPE", "VIEW", "PERMUTE", "TRANSPOSE", "GET_ROWS",
    "GET_ROWS_BACK", "DIAG", "DIAG_MASK_INF", "DIAG_MASK_ZERO", "SOFT_MAX", "SOFT_MAX_BACK",
    "ROPE", "ROPE_BACK", "CLAMP", "CONV_TRANSPOSE_1D", "IM2COL", "CONV_TRANSPOSE_2D",
    "POOL_1D", "POOL_2D", "UPSCALE", "PAD", "ARANGE", "TIMESTEP_EMBEDDING", "ARGSORT",
    "LEAKY_RELU", "FLASH_ATTN", "FLASH_ATTN_EXT", "FLASH_FF", "FLASH_ATTN_BACK", "SSM_CONV",
    "SSM_SCAN", "WIN_PART", "WIN_UNPART", "GET_REL_POS", "ADD_REL_POS", "UNARY", "MAP_UNARY",
    "MAP_BINARY", "MAP_CUSTOM1_F32", "MAP_CUSTOM2_F32", "MAP_CUSTOM3_F32", "MAP_CUSTOM1",
    "MAP_CUSTOM2", "MAP_CUSTOM3", "CROSS_ENTROPY_LOSS", "CROSS_ENTROPY_LOSS_BACK",
};

const char * const k_unary_names[GGML_UNARY_OP_COUNT] = {
    "ABS", "SGN", "NEG", "STEP", "TANH", "ELU", "RELU", "SIGMOID", "GELU", "GELU_QUICK", "SILU",
    "HARDSWISH", "HARDSIGMOID",
};

} // namespace

extern "C" {

void ggml_print_backtrace(void) {
    void * frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
}

const char * ggml_status_to_string(enum ggml_status status) {
    switch (status) {
        case GGML_STATUS_ALLOC_FAILED: return "GGML status: error (failed to allocate memory)";
        case GGML_STATUS_FAILED:       return "GGML status: error (operation failed)";
        case GGML_STATUS_SUCCESS:      return "GGML status: success";
        case GGML_STATUS_ABORTED:      return "GGML status: warning (operation aborted)";
    }
    return "GGML status: unknown";
}

// IEEE binary16 round-to-nearest-even, matching F16C _cvtss_sh(x, 0) used by the reference x86
// build (src/ggml-impl.h:446-462) bit for bit, NaN -> quiet NaN.
ggml_fp16_t ggml_fp32_to_fp16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u) return (ggml_fp16_t) (sign | 0x7e00u | ((ax >> 13) & 0x3ffu));  // NaN
    if (ax >= 0x477ff000u) return (ggml_fp16_t) (sign | 0x7c00u);                         // overflow -> inf
    if (ax < 0x38800000u) {                                                              // subnormal/zero
        if (ax < 0x33000000u) return (ggml_fp16_t) sign;                                 // < 2^-25: 0
        const uint32_t e = ax >> 23;
        const uint32_t m = (ax & 0x7fffffu) | 0x800000u;
        const uint32_t shift = 126u - e;  // value / 2^-24 = m * 2^(e - 126)
        const uint32_t rem = m & ((1u << shift) - 1u);
        const uint32_t half = 1u << (shift - 1);
        uint32_t q = m >> shift;
        if (rem > half || (rem == half && (q & 1u))) q++;  // carry into 0x400 = min normal
        return (ggml_fp16_t) (sign | q);
    }
    uint32_t h = ((ax - 0x38000000u) >> 13);
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (ggml_fp16_t) (sign | h);
}

float ggml_fp16_to_fp32(ggml_fp16_t h) {
    const uint32_t sign = (uint32_t) (h & 0x8000u) << 16;
    const uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    uint32_t x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else {
            int s = -1;
            do { s++; m <<= 1; } while (!(m & 0x400u));
            x = sign | ((uint32_t) (112 - s) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

void ggml_fp16_to_fp32_row(const ggml_fp16_t * x, float * y, int64_t n) {
    for (int64_t i = 0; i < n; i++) y[i] = ggml_fp16_to_fp32(x[i]);
}

void ggml_fp32_to_fp16_row(const float * x, ggml_fp16_t * y, int64_t n) {
    for (int64_t i = 0; i < n; i++) y[i] = ggml_fp32_to_fp16(x[i]);
}

bool ggml_guid_matches(ggml_guid_t a, ggml_guid_t b) { return memcmp(a, b, sizeof(ggml_guid)) == 0; }

static int64_t g_t0_us;

void ggml_time_init(void) {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    g_t0_us = (int64_t) ts.tv_sec * 1000000 + ts.tv_nsec / 1000;
}

int64_t ggml_time_us(void) {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t) ts.tv_sec * 1000000 + ts.tv_nsec / 1000 - g_t0_us;
}

int64_t ggml_time_ms(void) { return ggml_time_us() / 1000; }

// ---------------------------------------------------------------------------------------------
// tensor shape queries (src/ggml.c:2700-2870)
// ---------------------------------------------------------------------------------------------

int64_t ggml_nelements(const struct ggml_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
int64_t ggml_nrows(const struct ggml_tensor * t) { return t->ne[1] * t->ne[2] * t->ne[3]; }

size_t ggml_nbytes(const struct ggml_tensor * t) {
    size_t nbytes;
    const size_t blck = (size_t) ggml_blck_size(t->type);
    if (blck == 1) {
        nbytes = ggml_type_size(t->type);
        for (int i = 0; i < GGML_MAX_DIMS; ++i) nbytes += (size_t) (t->ne[i] - 1) * t->nb[i];
    } else {
        nbytes = (size_t) t->ne[0] * t->nb[0] / blck;
        for (int i = 1; i < GGML_MAX_DIMS; ++i) nbytes += (size_t) (t->ne[i] - 1) * t->nb[i];
    }
    return nbytes;
}

size_t ggml_nbytes_pad(const struct ggml_tensor * t) { return GGML_PAD(ggml_nbytes(t), GGML_MEM_ALIGN); }
int ggml_blck_size(enum ggml_type type) { return k_types[type].blck; }
size_t ggml_type_size(enum ggml_type type) { return k_types[type].size; }

size_t ggml_row_size(enum ggml_type type, int64_t ne) {
    GGML_ASSERT(ne % ggml_blck_size(type) == 0);
    return ggml_type_size(type) * (size_t) ne / (size_t) ggml_blck_size(type);
}

const char * ggml_type_name(enum ggml_type type) { return type < GGML_TYPE_COUNT ? k_types[type].name : "NONE"; }
const char * ggml_op_name(enum ggml_op op) { return k_op_names[op]; }
const char * ggml_op_symbol(enum ggml_op op) { return k_op_names[op]; }
const char * ggml_unary_op_name(enum ggml_unary_op op) { return k_unary_names[op]; }

enum ggml_unary_op ggml_get_unary_op(const struct ggml_tensor * t) {
    GGML_ASSERT(t->op == GGML_OP_UNARY);
    return (enum ggml_unary_op) t->op_params[0];
}

const char * ggml_op_desc(const struct ggml_tensor * t) {
    if (t->op == GGML_OP_UNARY) return ggml_unary_op_name(ggml_get_unary_op(t));
    return ggml_op_name(t->op);
}

size_t ggml_element_size(const struct ggml_tensor * t) { return ggml_type_size(t->type); }
bool ggml_is_quantized(enum ggml_type type) { return k_types[type].quantized; }

enum ggml_type ggml_ftype_to_ggml_type(enum ggml_ftype ftype) {
    switch (ftype) {
        case GGML_FTYPE_ALL_F32:      return GGML_TYPE_F32;
        case GGML_FTYPE_MOSTLY_F16:   return GGML_TYPE_F16;
        case GGML_FTYPE_MOSTLY_BF16:  return GGML_TYPE_BF16;
        case GGML_FTYPE_MOSTLY_Q4_0:  return GGML_TYPE_Q4_0;
        case GGML_FTYPE_MOSTLY_Q4_1:  return GGML_TYPE_Q4_1;
        case GGML_FTYPE_MOSTLY_Q5_0:  return GGML_TYPE_Q5_0;
        case GGML_FTYPE_MOSTLY_Q5_1:  return GGML_TYPE_Q5_1;
        case GGML_FTYPE_MOSTLY_Q8_0:  return GGML_TYPE_Q8_0;
        case GGML_FTYPE_MOSTLY_Q2_K:  return GGML_TYPE_Q2_K;
        case GGML_FTYPE_MOSTLY_Q3_K:  return GGML_TYPE_Q3_K;
        case GGML_FTYPE_MOSTLY_Q4_K:  return GGML_TYPE_Q4_K;
        case GGML_FTYPE_MOSTLY_Q5_K:  return GGML_TYPE_Q5_K;
        case GGML_FTYPE_MOSTLY_Q6_K:  return GGML_TYPE_Q6_K;
        default:                      return GGML_TYPE_COUNT;
    }
}

bool ggml_is_transposed(const struct ggml_tensor * t) { return t->nb[0] > t->nb[1]; }

bool ggml_is_contiguous(const struct ggml_tensor * t) {
    return t->nb[0] == ggml_type_size(t->type) &&
           t->nb[1] == (t->nb[0] * (size_t) t->ne[0]) / (size_t) ggml_blck_size(t->type) &&
           t->nb[2] == t->nb[1] * (size_t) t->ne[1] &&
           t->nb[3] == t->nb[2] * (size_t) t->ne[2];
}

bool ggml_is_permuted(const struct ggml_tensor * t) {
    return t->nb[0] > t->nb[1] || t->nb[1] > t->nb[2] || t->nb[2] > t->nb[3];
}

bool ggml_is_empty(const struct ggml_tensor * t) {
    for (int i = 0; i < GGML_MAX_DIMS; ++i) if (t->ne[i] == 0) return true;
    return false;
}

bool ggml_is_scalar(const struct ggml_tensor * t) { return t->ne[0] == 1 && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1; }
bool ggml_is_vector(const struct ggml_tensor * t) { return t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1; }
bool ggml_is_matrix(const struct ggml_tensor * t) { return t->ne[2] == 1 && t->ne[3] == 1; }
bool ggml_is_3d(const struct ggml_tensor * t) { return t->ne[3] == 1; }

int ggml_n_dims(const struct ggml_tensor * t) {
    for (int i = GGML_MAX_DIMS - 1; i >= 1; --i) if (t->ne[i] > 1) return i + 1;
    return 1;
}

bool ggml_are_same_shape(const struct ggml_tensor * a, const struct ggml_tensor * b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}

size_t ggml_tensor_overhead(void) { return GGML_OBJECT_SIZE + GGML_TENSOR_SIZE; }

} // extern "C"

// ---------------------------------------------------------------------------------------------
// contexts (src/ggml.c:2874-3125): a bump arena of ggml_object headers
// ---------------------------------------------------------------------------------------------

struct ggml_context {
    size_t mem_size;
    char * mem_buffer;
    bool mem_buffer_owned;
    bool no_alloc;
    int n_objects;
    ggml_object * objects_begin;
    ggml_object * objects_end;
};

static ggml_object * new_object(ggml_context * ctx, ggml_object_type type, size_t size) {
    ggml_object * cur = ctx->objects_end;
    const size_t cur_end = cur ? cur->offs + cur->size : 0;
    const size_t need = GGML_PAD(size, GGML_MEM_ALIGN);
    if (cur_end + need + GGML_OBJECT_SIZE > ctx->mem_size) {
        fprintf(stderr, "ggml: not enough space in the context's memory pool (needed %zu, available %zu)\n",
                cur_end + need + GGML_OBJECT_SIZE, ctx->mem_size);
        GGML_ASSERT(!"context memory pool exhausted");
    }
    ggml_object * obj = (ggml_object *) (ctx->mem_buffer + cur_end);
    obj->offs = cur_end + GGML_OBJECT_SIZE;
    obj->size = need;
    obj->next = nullptr;
    obj->type = type;
    memset(obj->padding, 0, sizeof(obj->padding));
    if (cur) cur->next = obj; else ctx->objects_begin = obj;
    ctx->objects_end = obj;
    ctx->n_objects++;
    return obj;
}

extern "C" {

struct ggml_context * ggml_init(struct ggml_init_params params) {
    static std::once_flag once;
    std::call_once(once, [] { ggml_time_init(); });
    if (params.mem_size == 0) params.mem_size = GGML_MEM_ALIGN;
    const size_t mem_size = params.mem_buffer ? params.mem_size : GGML_PAD(params.mem_size, GGML_MEM_ALIGN);
    auto * ctx = new ggml_context();
    ctx->mem_size = mem_size;
    if (params.mem_buffer) {
        ctx->mem_buffer = (char *) params.mem_buffer;
        ctx->mem_buffer_owned = false;
    } else {
        ctx->mem_buffer = (char *) aligned_alloc(GGML_MEM_ALIGN, mem_size);
        GGML_ASSERT(ctx->mem_buffer != nullptr);
        ctx->mem_buffer_owned = true;
    }
    ctx->no_alloc = params.no_alloc;
    ctx->n_objects = 0;
    ctx->objects_begin = ctx->objects_end = nullptr;
    return ctx;
}

void ggml_free(struct ggml_context * ctx) {
    if (!ctx) return;
    if (ctx->mem_buffer_owned) free(ctx->mem_buffer);
    delete ctx;
}

size_t ggml_used_mem(const struct ggml_context * ctx) {
    return ctx->objects_end ? ctx->objects_end->offs + ctx->objects_end->size : 0;
}

bool ggml_get_no_alloc(struct ggml_context * ctx) { return ctx->no_alloc; }
void ggml_set_no_alloc(struct ggml_context * ctx, bool no_alloc) { ctx->no_alloc = no_alloc; }
void * ggml_get_mem_buffer(const struct ggml_context * ctx) { return ctx->mem_buffer; }
size_t ggml_get_mem_size(const struct ggml_context * ctx) { return ctx->mem_size; }

size_t ggml_get_max_tensor_size(const struct ggml_context * ctx) {
    size_t m = 0;
    for (ggml_tensor * t = ggml_get_first_tensor(ctx); t; t = ggml_get_next_tensor(ctx, t)) {
        const size_t b = ggml_nbytes(t);
        if (b > m) m = b;
    }
    return m;
}

} // extern "C"

// src/ggml.c:3126-3210 ggml_new_tensor_impl
static ggml_tensor * new_tensor_impl(ggml_context * ctx, ggml_type type, int n_dims, const int64_t * ne,
                                     ggml_tensor * view_src, size_t view_offs) {
    GGML_ASSERT(n_dims >= 1 && n_dims <= GGML_MAX_DIMS);
    if (view_src && view_src->view_src) {
        view_offs += view_src->view_offs;
        view_src = view_src->view_src;
    }
    size_t data_size = ggml_row_size(type, ne[0]);
    for (int i = 1; i < n_dims; i++) data_size *= (size_t) ne[i];
    GGML_ASSERT(view_src == nullptr || data_size == 0 || data_size + view_offs <= ggml_nbytes(view_src));

    void * data = view_src ? view_src->data : nullptr;
    if (data) data = (char *) data + view_offs;
    const size_t obj_alloc = (!view_src && !ctx->no_alloc) ? data_size : 0;

    ggml_object * obj = new_object(ctx, GGML_OBJECT_TYPE_TENSOR, GGML_TENSOR_SIZE + obj_alloc);
    auto * t = (ggml_tensor *) (ctx->mem_buffer + obj->offs);
    memset(t, 0, sizeof(*t));
    t->type = type;
    t->backend = GGML_BACKEND_TYPE_CPU;
    t->view_src = view_src;
    t->view_offs = view_offs;
    t->data = obj_alloc > 0 ? (void *) (t + 1) : data;
    for (int i = 0; i < GGML_MAX_DIMS; i++) t->ne[i] = i < n_dims ? ne[i] : 1;
    t->nb[0] = ggml_type_size(type);
    t->nb[1] = t->nb[0] * (size_t) (t->ne[0] / ggml_blck_size(type));
    for (int i = 2; i < GGML_MAX_DIMS; i++) t->nb[i] = t->nb[i - 1] * (size_t) t->ne[i - 1];
    return t;
}

static void set_op_params(ggml_tensor * t, const void * params, size_t size) {
    GGML_ASSERT(size <= GGML_MAX_OP_PARAMS);
    memcpy(t->op_params, params, size);
}

extern "C" {

struct ggml_tensor * ggml_new_tensor(struct ggml_context * ctx, enum ggml_type type, int n_dims, const int64_t * ne) {
    return new_tensor_impl(ctx, type, n_dims, ne, nullptr, 0);
}

struct ggml_tensor * ggml_new_tensor_1d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0) {
    return ggml_new_tensor(ctx, type, 1, &ne0);
}

struct ggml_tensor * ggml_new_tensor_2d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    return ggml_new_tensor(ctx, type, 2, ne);
}

struct ggml_tensor * ggml_new_tensor_3d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    return ggml_new_tensor(ctx, type, 3, ne);
}

struct ggml_tensor * ggml_new_tensor_4d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return ggml_new_tensor(ctx, type, 4, ne);
}

struct ggml_tensor * ggml_dup_tensor(struct ggml_context * ctx, const struct ggml_tensor * src) {
    return ggml_new_tensor(ctx, src->type, GGML_MAX_DIMS, src->ne);
}

struct ggml_tensor * ggml_format_name(struct ggml_tensor * t, const char * fmt, ...) {
    va_list args;
    va_start(args, fmt);
    vsnprintf(t->name, sizeof(t->name), fmt, args);
    va_end(args);
    return t;
}

struct ggml_tensor * ggml_view_tensor(struct ggml_context * ctx, struct ggml_tensor * src) {
    ggml_tensor * r = new_tensor_impl(ctx, src->type, GGML_MAX_DIMS, src->ne, src, 0);
    ggml_format_name(r, "%s (view)", src->name);
    for (int i = 0; i < GGML_MAX_DIMS; i++) r->nb[i] = src->nb[i];
    return r;
}

struct ggml_tensor * ggml_get_first_tensor(const struct ggml_context * ctx) {
    for (ggml_object * o = ctx->objects_begin; o; o = o->next)
        if (o->type == GGML_OBJECT_TYPE_TENSOR) return (ggml_tensor *) (ctx->mem_buffer + o->offs);
    return nullptr;
}

struct ggml_tensor * ggml_get_next_tensor(const struct ggml_context * ctx, struct ggml_tensor * tensor) {
    ggml_object * o = (ggml_object *) ((char *) tensor - GGML_OBJECT_SIZE);
    for (o = o->next; o; o = o->next)
        if (o->type == GGML_OBJECT_TYPE_TENSOR) return (ggml_tensor *) (ctx->mem_buffer + o->offs);
    return nullptr;
}

struct ggml_tensor * ggml_get_tensor(struct ggml_context * ctx, const char * name) {
    for (ggml_tensor * t = ggml_get_first_tensor(ctx); t; t = ggml_get_next_tensor(ctx, t))
        if (strcmp(t->name, name) == 0) return t;
    return nullptr;
}

const char * ggml_get_name(const struct ggml_tensor * t) { return t->name; }

struct ggml_tensor * ggml_set_name(struct ggml_tensor * t, const char * name) {
    strncpy(t->name, name, sizeof(t->name) - 1);
    t->name[sizeof(t->name) - 1] = '\0';
    return t;
}

void ggml_set_input(struct ggml_tensor * t) { t->flags |= GGML_TENSOR_FLAG_INPUT; }
void ggml_set_output(struct ggml_tensor * t) { t->flags |= GGML_TENSOR_FLAG_OUTPUT; }
void * ggml_get_data(const struct ggml_tensor * t) { return t->data; }
float * ggml_get_data_f32(const struct ggml_tensor * t) {
    GGML_ASSERT(t->type == GGML_TYPE_F32);
    return (float *) t->data;
}

// ---------------------------------------------------------------------------------------------
// op constructors. Shapes / op_params follow the reference constructors cited per function.
// ---------------------------------------------------------------------------------------------

// src/ggml.c:4800-4840 ggml_can_mul_mat + ggml_mul_mat: dst f32 [a->ne1, b->ne1, b->ne2, b->ne3]
struct ggml_tensor * ggml_mul_mat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    GGML_ASSERT(a->ne[0] == b->ne[0] && b->ne[2] % a->ne[2] == 0 && b->ne[3] % a->ne[3] == 0);
    GGML_ASSERT(!ggml_is_transposed(a));
    const int64_t ne[4] = {a->ne[1], b->ne[1], b->ne[2], b->ne[3]};
    ggml_tensor * r = ggml_new_tensor(ctx, GGML_TYPE_F32, 4, ne);
    r->op = GGML_OP_MUL_MAT;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

// src/ggml.c:4842-4850
void ggml_mul_mat_set_prec(struct ggml_tensor * a, enum ggml_prec prec) {
    const int32_t p = (int32_t) prec;
    set_op_params(a, &p, sizeof(p));
}

static ggml_tensor * unary_like(ggml_context * ctx, ggml_tensor * a, ggml_op op, bool inplace) {
    ggml_tensor * r = inplace ? ggml_view_tensor(ctx, a) : ggml_dup_tensor(ctx, a);
    r->op = op;
    r->src[0] = a;
    return r;
}

struct ggml_tensor * ggml_dup(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_like(ctx, a, GGML_OP_DUP, false); }

// ggml_can_repeat_rows / ggml_can_repeat (src/ggml.c:2780-2800): b broadcasts into a
static bool can_repeat(const ggml_tensor * b, const ggml_tensor * a) {
    return ggml_is_empty(b) ? ggml_is_empty(a) :
        (a->ne[0] % b->ne[0] == 0) && (a->ne[1] % b->ne[1] == 0) && (a->ne[2] % b->ne[2] == 0) && (a->ne[3] % b->ne[3] == 0);
}

static ggml_tensor * binary_bcast(ggml_context * ctx, ggml_tensor * a, ggml_tensor * b, ggml_op op, bool inplace) {
    GGML_ASSERT(can_repeat(b, a));
    ggml_tensor * r = inplace ? ggml_view_tensor(ctx, a) : ggml_dup_tensor(ctx, a);
    r->op = op;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

// src/ggml.c:3934 ggml_add / :4158 ggml_mul (b broadcast over a)
struct ggml_tensor * ggml_add(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) { return binary_bcast(ctx, a, b, GGML_OP_ADD, false); }
struct ggml_tensor * ggml_add_inplace(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) { return binary_bcast(ctx, a, b, GGML_OP_ADD, true); }
struct ggml_tensor * ggml_mul(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) { return binary_bcast(ctx, a, b, GGML_OP_MUL, false); }
struct ggml_tensor * ggml_mul_inplace(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) { return binary_bcast(ctx, a, b, GGML_OP_MUL, true); }

// src/ggml.c:5092 ggml_scale_impl: op_params[0] = s
static ggml_tensor * scale_impl(ggml_context * ctx, ggml_tensor * a, float s, bool inplace) {
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_SCALE, inplace);
    set_op_params(r, &s, sizeof(s));
    return r;
}
struct ggml_tensor * ggml_scale(struct ggml_context * ctx, struct ggml_tensor * a, float s) { return scale_impl(ctx, a, s, false); }
struct ggml_tensor * ggml_scale_inplace(struct ggml_context * ctx, struct ggml_tensor * a, float s) { return scale_impl(ctx, a, s, true); }

// src/ggml.c:4632 ggml_norm_impl / :4672 ggml_rms_norm_impl: op_params[0] = eps
struct ggml_tensor * ggml_norm(struct ggml_context * ctx, struct ggml_tensor * a, float eps) {
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_NORM, false);
    set_op_params(r, &eps, sizeof(eps));
    return r;
}
struct ggml_tensor * ggml_rms_norm(struct ggml_context * ctx, struct ggml_tensor * a, float eps) {
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_RMS_NORM, false);
    set_op_params(r, &eps, sizeof(eps));
    return r;
}

// src/ggml.c:6250 ggml_unary_impl: op_params[0] = unary op
static ggml_tensor * unary_impl(ggml_context * ctx, ggml_tensor * a, ggml_unary_op op, bool inplace) {
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_UNARY, inplace);
    const int32_t p = (int32_t) op;
    set_op_params(r, &p, sizeof(p));
    return r;
}
struct ggml_tensor * ggml_unary(struct ggml_context * ctx, struct ggml_tensor * a, enum ggml_unary_op op) { return unary_impl(ctx, a, op, false); }
struct ggml_tensor * ggml_gelu(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_impl(ctx, a, GGML_UNARY_OP_GELU, false); }
struct ggml_tensor * ggml_gelu_inplace(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_impl(ctx, a, GGML_UNARY_OP_GELU, true); }
struct ggml_tensor * ggml_silu(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_impl(ctx, a, GGML_UNARY_OP_SILU, false); }

// src/ggml.c:5850 ggml_soft_max_impl: op_params = {scale, max_bias}, src[1] = mask (optional)
static ggml_tensor * soft_max_impl(ggml_context * ctx, ggml_tensor * a, ggml_tensor * mask, float scale, float max_bias, bool inplace) {
    GGML_ASSERT(ggml_is_contiguous(a));
    if (mask) {
        GGML_ASSERT(mask->type == GGML_TYPE_F16 || mask->type == GGML_TYPE_F32);
        GGML_ASSERT(ggml_is_contiguous(mask) && ggml_is_matrix(mask) && mask->ne[0] == a->ne[0] && mask->ne[1] >= a->ne[1]);
    }
    if (max_bias > 0.0f) GGML_ASSERT(mask);
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_SOFT_MAX, inplace);
    const float params[2] = {scale, max_bias};
    set_op_params(r, params, sizeof(params));
    r->src[1] = mask;
    return r;
}
struct ggml_tensor * ggml_soft_max(struct ggml_context * ctx, struct ggml_tensor * a) { return soft_max_impl(ctx, a, nullptr, 1.0f, 0.0f, false); }
struct ggml_tensor * ggml_soft_max_inplace(struct ggml_context * ctx, struct ggml_tensor * a) { return soft_max_impl(ctx, a, nullptr, 1.0f, 0.0f, true); }
struct ggml_tensor * ggml_soft_max_ext(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * mask, float scale, float max_bias) {
    return soft_max_impl(ctx, a, mask, scale, max_bias, false);
}

// src/ggml.c:5780 ggml_diag_mask_inf_impl: op_params[0] = n_past
static ggml_tensor * diag_mask_inf_impl(ggml_context * ctx, ggml_tensor * a, int n_past, bool inplace) {
    ggml_tensor * r = unary_like(ctx, a, GGML_OP_DIAG_MASK_INF, inplace);
    const int32_t p = n_past;
    set_op_params(r, &p, sizeof(p));
    return r;
}
struct ggml_tensor * ggml_diag_mask_inf(struct ggml_context * ctx, struct ggml_tensor * a, int n_past) { return diag_mask_inf_impl(ctx, a, n_past, false); }
struct ggml_tensor * ggml_diag_mask_inf_inplace(struct ggml_context * ctx, struct ggml_tensor * a, int n_past) { return diag_mask_inf_impl(ctx, a, n_past, true); }

// src/ggml.c:5654 ggml_get_rows: dst f32 [a->ne0, b->ne0, b->ne1, b->ne2] (i32 rows b)
struct ggml_tensor * ggml_get_rows(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    GGML_ASSERT(a->ne[2] == b->ne[1]);
    GGML_ASSERT(b->ne[3] == 1);
    GGML_ASSERT(b->type == GGML_TYPE_I32);
    const enum ggml_type type = a->type == GGML_TYPE_I32 ? GGML_TYPE_I32 : GGML_TYPE_F32;
    ggml_tensor * r = ggml_new_tensor_4d(ctx, type, a->ne[0], b->ne[0], b->ne[1], b->ne[2]);
    r->op = GGML_OP_GET_ROWS;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

// src/ggml.c:5960 ggml_rope_impl: op_params = {n_past(0), n_dims, mode, n_ctx, n_orig_ctx,
// freq_base, freq_scale, ext_factor, attn_factor, beta_fast, beta_slow, xpos_base, xpos_down}
struct ggml_tensor * ggml_rope(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b, int n_dims, int mode, int n_ctx) {
    GGML_ASSERT(ggml_is_vector(b) && b->type == GGML_TYPE_I32 && a->ne[2] == b->ne[0]);
    GGML_ASSERT((mode & 1) == 0 && "mode & 1 == 1 is no longer supported");
    ggml_tensor * r = ggml_dup_tensor(ctx, a);
    int32_t params[13] = {0, n_dims, mode, n_ctx, 0};
    const float freq_base = 10000.0f, freq_scale = 1.0f, ext_factor = 0.0f, attn_factor = 1.0f;
    const float beta_fast = 32.0f, beta_slow = 1.0f, xpos_base = 0.0f;
    const bool xpos_down = false;
    memcpy(params + 5, &freq_base, sizeof(float));
    memcpy(params + 6, &freq_scale, sizeof(float));
    memcpy(params + 7, &ext_factor, sizeof(float));
    memcpy(params + 8, &attn_factor, sizeof(float));
    memcpy(params + 9, &beta_fast, sizeof(float));
    memcpy(params + 10, &beta_slow, sizeof(float));
    memcpy(params + 11, &xpos_base, sizeof(float));
    memcpy(params + 12, &xpos_down, sizeof(bool));
    set_op_params(r, params, sizeof(params));
    r->op = GGML_OP_ROPE;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

// src/ggml.c:5220 ggml_cpy: result is a view of b
struct ggml_tensor * ggml_cpy(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    GGML_ASSERT(ggml_nelements(a) == ggml_nelements(b));
    ggml_tensor * r = ggml_view_tensor(ctx, b);
    if (strlen(b->name) > 0) ggml_format_name(r, "%s (copy of %s)", b->name, a->name);
    else ggml_format_name(r, "%s (copy)", a->name);
    r->op = GGML_OP_CPY;
    r->src[0] = a;
    r->src[1] = b;
    return r;
}

// src/ggml.c:5250 ggml_cont_impl / ggml_cont_4d
struct ggml_tensor * ggml_cont_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    GGML_ASSERT(ggml_nelements(a) == ne0 * ne1 * ne2 * ne3);
    ggml_tensor * r = ggml_new_tensor_4d(ctx, a->type, ne0, ne1, ne2, ne3);
    ggml_format_name(r, "%s (cont)", a->name);
    r->op = GGML_OP_CONT;
    r->src[0] = a;
    return r;
}
struct ggml_tensor * ggml_cont(struct ggml_context * ctx, struct ggml_tensor * a) {
    ggml_tensor * r = ggml_dup_tensor(ctx, a);
    ggml_format_name(r, "%s (cont)", a->name);
    r->op = GGML_OP_CONT;
    r->src[0] = a;
    return r;
}
struct ggml_tensor * ggml_cont_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1) { return ggml_cont_4d(ctx, a, ne0, ne1, 1, 1); }
struct ggml_tensor * ggml_cont_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2) { return ggml_cont_4d(ctx, a, ne0, ne1, ne2, 1); }

// src/ggml.c:5300-5400 ggml_reshape*: views of a contiguous tensor
static ggml_tensor * reshape_impl(ggml_context * ctx, ggml_tensor * a, int n_dims, const int64_t * ne) {
    GGML_ASSERT(ggml_is_contiguous(a));
    int64_t n = 1;
    for (int i = 0; i < n_dims; i++) n *= ne[i];
    GGML_ASSERT(ggml_nelements(a) == n);
    ggml_tensor * r = new_tensor_impl(ctx, a->type, n_dims, ne, a, 0);
    ggml_format_name(r, "%s (reshaped)", a->name);
    r->op = GGML_OP_RESHAPE;
    r->src[0] = a;
    return r;
}
struct ggml_tensor * ggml_reshape(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) { return reshape_impl(ctx, a, GGML_MAX_DIMS, b->ne); }
struct ggml_tensor * ggml_reshape_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0) { return reshape_impl(ctx, a, 1, &ne0); }
struct ggml_tensor * ggml_reshape_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    return reshape_impl(ctx, a, 2, ne);
}
struct ggml_tensor * ggml_reshape_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    return reshape_impl(ctx, a, 3, ne);
}
struct ggml_tensor * ggml_reshape_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return reshape_impl(ctx, a, 4, ne);
}

// src/ggml.c:5316-5424 ggml_view_impl / ggml_view_Nd: op_params[0..] = offset
static ggml_tensor * view_impl(ggml_context * ctx, ggml_tensor * a, int n_dims, const int64_t * ne, size_t offset) {
    ggml_tensor * r = new_tensor_impl(ctx, a->type, n_dims, ne, a, offset);
    ggml_format_name(r, "%s (view)", a->name);
    set_op_params(r, &offset, sizeof(offset));
    r->op = GGML_OP_VIEW;
    r->src[0] = a;
    return r;
}
struct ggml_tensor * ggml_view_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, size_t offset) { return view_impl(ctx, a, 1, &ne0, offset); }
struct ggml_tensor * ggml_view_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, size_t nb1, size_t offset) {
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor * r = view_impl(ctx, a, 2, ne, offset);
    r->nb[1] = nb1;
    r->nb[2] = r->nb[1] * (size_t) ne1;
    r->nb[3] = r->nb[2];
    return r;
}
struct ggml_tensor * ggml_view_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, size_t nb1, size_t nb2, size_t offset) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor * r = view_impl(ctx, a, 3, ne, offset);
    r->nb[1] = nb1;
    r->nb[2] = nb2;
    r->nb[3] = r->nb[2] * (size_t) ne2;
    return r;
}
struct ggml_tensor * ggml_view_4d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1, int64_t ne2, int64_t ne3,
                                  size_t nb1, size_t nb2, size_t nb3, size_t offset) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    ggml_tensor * r = view_impl(ctx, a, 4, ne, offset);
    r->nb[1] = nb1;
    r->nb[2] = nb2;
    r->nb[3] = nb3;
    return r;
}

// src/ggml.c:5425-5480 ggml_permute: op_params = {axis0..axis3}
struct ggml_tensor * ggml_permute(struct ggml_context * ctx, struct ggml_tensor * a, int axis0, int axis1, int axis2, int axis3) {
    GGML_ASSERT(axis0 >= 0 && axis0 < 4 && axis1 >= 0 && axis1 < 4 && axis2 >= 0 && axis2 < 4 && axis3 >= 0 && axis3 < 4);
    GGML_ASSERT(axis0 != axis1 && axis0 != axis2 && axis0 != axis3 && axis1 != axis2 && axis1 != axis3 && axis2 != axis3);
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    ggml_format_name(r, "%s (permuted)", a->name);
    int64_t ne[4];
    size_t nb[4];
    const int ax[4] = {axis0, axis1, axis2, axis3};
    for (int i = 0; i < 4; i++) {
        ne[ax[i]] = a->ne[i];
        nb[ax[i]] = a->nb[i];
    }
    for (int i = 0; i < 4; i++) {
        r->ne[i] = ne[i];
        r->nb[i] = nb[i];
    }
    r->op = GGML_OP_PERMUTE;
    r->src[0] = a;
    const int32_t params[4] = {axis0, axis1, axis2, axis3};
    set_op_params(r, params, sizeof(params));
    return r;
}

// src/ggml.c:5484 ggml_transpose
struct ggml_tensor * ggml_transpose(struct ggml_context * ctx, struct ggml_tensor * a) {
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    ggml_format_name(r, "%s (transposed)", a->name);
    r->ne[0] = a->ne[1];
    r->ne[1] = a->ne[0];
    r->nb[0] = a->nb[1];
    r->nb[1] = a->nb[0];
    r->op = GGML_OP_TRANSPOSE;
    r->src[0] = a;
    return r;
}

// ---------------------------------------------------------------------------------------------
// graphs (src/ggml.c:18787-18990): DFS post-order over src[], visited set = open-addressing
// hash of tensor pointers sized by the same prime table so ggml_graph_overhead() matches.
// ---------------------------------------------------------------------------------------------

static size_t hash_size_for(size_t min_sz) {
    static const size_t primes[] = {
        2, 3, 5, 11, 17, 37, 67, 131, 257, 521, 1031, 2053, 4099, 8209, 16411, 32771, 65537,
        131101, 262147, 524309, 1048583, 2097169, 4194319, 8388617, 16777259, 33554467,
        67108879, 134217757, 268435459, 536870923, 1073741827, 2147483659ull};
    for (size_t p : primes) if (p >= min_sz) return p;
    return min_sz | 1;
}

static size_t graph_nbytes(size_t size, bool grads) {
    size_t n = sizeof(ggml_cgraph) + size * sizeof(ggml_tensor *) * 2;
    if (grads) n += size * sizeof(ggml_tensor *);
    n += hash_size_for(size * 2) * sizeof(ggml_tensor *);
    return n;
}

size_t ggml_graph_overhead_custom(size_t size, bool grads) { return GGML_OBJECT_SIZE + GGML_PAD(graph_nbytes(size, grads), GGML_MEM_ALIGN); }
size_t ggml_graph_overhead(void) { return ggml_graph_overhead_custom(GGML_DEFAULT_GRAPH_SIZE, false); }

struct ggml_cgraph * ggml_new_graph_custom(struct ggml_context * ctx, size_t size, bool grads) {
    ggml_object * obj = new_object(ctx, GGML_OBJECT_TYPE_GRAPH, graph_nbytes(size, grads));
    auto * g = (ggml_cgraph *) (ctx->mem_buffer + obj->offs);
    auto ** base = (ggml_tensor **) (g + 1);
    const size_t hs = hash_size_for(size * 2);
    memset(g, 0, sizeof(*g));
    g->size = (int) size;
    g->nodes = base;
    g->leafs = base + size;
    g->visited_hash_table.size = hs;
    g->visited_hash_table.keys = base + 2 * size;
    g->grads = grads ? base + 2 * size + hs : nullptr;
    g->order = GGML_CGRAPH_EVAL_ORDER_LEFT_TO_RIGHT;
    memset(g->visited_hash_table.keys, 0, hs * sizeof(ggml_tensor *));
    return g;
}

struct ggml_cgraph * ggml_new_graph(struct ggml_context * ctx) { return ggml_new_graph_custom(ctx, GGML_DEFAULT_GRAPH_SIZE, false); }

// returns true when newly inserted
static bool visited_insert(ggml_hash_set & hs, ggml_tensor * t) {
    size_t h = ((uintptr_t) t >> 4) % hs.size;
    for (size_t probe = 0; probe < hs.size; probe++) {
        const size_t i = (h + probe) % hs.size;
        if (hs.keys[i] == t) return false;
        if (hs.keys[i] == nullptr) {
            hs.keys[i] = t;
            return true;
        }
    }
    GGML_ASSERT(!"graph hash table full");
    return false;
}

static void visit_parents(ggml_cgraph * g, ggml_tensor * node) {
    if (!visited_insert(g->visited_hash_table, node)) return;
    for (int i = 0; i < GGML_MAX_SRC; ++i) {
        const int k = g->order == GGML_CGRAPH_EVAL_ORDER_RIGHT_TO_LEFT ? GGML_MAX_SRC - 1 - i : i;
        if (node->src[k]) visit_parents(g, node->src[k]);
    }
    if (node->op == GGML_OP_NONE && node->grad == nullptr) {
        GGML_ASSERT(g->n_leafs < g->size);
        if (node->name[0] == '\0') ggml_format_name(node, "leaf_%d", g->n_leafs);
        g->leafs[g->n_leafs++] = node;
    } else {
        GGML_ASSERT(g->n_nodes < g->size);
        if (node->name[0] == '\0') ggml_format_name(node, "node_%d", g->n_nodes);
        g->nodes[g->n_nodes] = node;
        if (g->grads) g->grads[g->n_nodes] = node->grad;
        g->n_nodes++;
    }
}

void ggml_build_forward_expand(struct ggml_cgraph * cgraph, struct ggml_tensor * tensor) {
    const int n0 = cgraph->n_nodes;
    visit_parents(cgraph, tensor);
    if (cgraph->n_nodes > n0) GGML_ASSERT(cgraph->nodes[cgraph->n_nodes - 1] == tensor);
}

struct ggml_tensor * ggml_graph_get_tensor(struct ggml_cgraph * cgraph, const char * name) {
    for (int i = 0; i < cgraph->n_leafs; i++) if (strcmp(cgraph->leafs[i]->name, name) == 0) return cgraph->leafs[i];
    for (int i = 0; i < cgraph->n_nodes; i++) if (strcmp(cgraph->nodes[i]->name, name) == 0) return cgraph->nodes[i];
    return nullptr;
}

// src/ggml.c:18970 ggml_graph_view: nodes [i0, i1), no leafs, no hash table
struct ggml_cgraph ggml_graph_view(struct ggml_cgraph * cgraph, int i0, int i1) {
    ggml_cgraph v;
    memset(&v, 0, sizeof(v));
    v.size = i1 - i0;
    v.n_nodes = i1 - i0;
    v.n_leafs = 0;
    v.nodes = cgraph->nodes + i0;
    v.grads = cgraph->grads ? cgraph->grads + i0 : nullptr;
    v.leafs = nullptr;
    v.order = cgraph->order;
    return v;
}

void ggml_graph_clear(struct ggml_cgraph * cgraph) {
    cgraph->n_leafs = 0;
    cgraph->n_nodes = 0;
    memset(cgraph->visited_hash_table.keys, 0, cgraph->visited_hash_table.size * sizeof(ggml_tensor *));
}

// src/ggml.c:20421-20462: the nodes with their perf counters (filled by a backend's per-node timer,
// e.g. ggml_backend_mi355x_set_perf: perf_cycles then holds microseconds, so both columns read ms),
// the leafs, and the time per op
void ggml_graph_print(const struct ggml_cgraph * cgraph) {
    int64_t per_op_us[GGML_OP_COUNT] = {0};
    printf("=== GRAPH ===\n");
    printf("n_nodes = %d\n", cgraph->n_nodes);
    for (int i = 0; i < cgraph->n_nodes; i++) {
        const ggml_tensor * node = cgraph->nodes[i];
        per_op_us[node->op] += std::max<int64_t>(1, node->perf_time_us);
        const double runs = node->perf_runs ? (double) node->perf_runs : 1.0;
        printf(" - %3d: [ %5" PRId64 ", %5" PRId64 ", %5" PRId64 "] %16s %s (%3d) cpu = %7.3f / %7.3f ms, wall = %7.3f / %7.3f ms\n", i,
               node->ne[0], node->ne[1], node->ne[2], ggml_op_name(node->op), (node->flags & GGML_TENSOR_FLAG_PARAM) ? "x" : node->grad ? "g" : " ",
               node->perf_runs, (double) node->perf_cycles / 1000.0, (double) node->perf_cycles / 1000.0 / runs,
               (double) node->perf_time_us / 1000.0, (double) node->perf_time_us / 1000.0 / runs);
    }
    printf("n_leafs = %d\n", cgraph->n_leafs);
    for (int i = 0; i < cgraph->n_leafs; i++) {
        const ggml_tensor * node = cgraph->leafs[i];
        printf(" - %3d: [ %5" PRId64 ", %5" PRId64 "] %8s %16s\n", i, node->ne[0], node->ne[1], ggml_op_name(node->op), node->name);
    }
    for (int i = 0; i < GGML_OP_COUNT; i++) {
        if (per_op_us[i] == 0) continue;
        printf("perf_total_per_op_us[%16s] = %7.3f ms\n", ggml_op_name((ggml_op) i), (double) per_op_us[i] / 1000.0);
    }
    printf("========================================\n");
    fflush(stdout);
}

} // extern "C"
