// ggml-mi355x.cpp -- the MI355X (gfx950) ggml backend: buffer types, buffers, backend vtable
// and per-node dispatch into the hand-written HIP kernels of csrc/kernels/.
//
// Implements ggml_backend_buffer_type_i / ggml_backend_buffer_i / ggml_backend_i
// (src/ggml-backend-impl.h:18-117 of NAIST-Archlab/ggml-imax @ v2) the way the reference's
// device backends do (structural analogue: src/ggml-cuda.cu:366-576 buffers, :2156-2308
// dispatch, :2456-2713 graph_compute, :2715-2868 supports/offload, :2870-2942 events/vtable,
// :3024-3042 registration) -- but written for one process per GPU, HIP streams, wave64
// kernels and activation quantization on the device.
//
// This file only uses the generic ggml API (ggml_nbytes, ggml_backend_buffer_init, ...), so the
// same object loads into either the repo's runtime (csrc/core) or the reference libggml.

#include "ggml_abi.h"
#include "ggml-mi355x.h"
#include "../kernels/mi355x_kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#define MI_CHECK(call)                                                                                  \
    do {                                                                                                \
        const hipError_t err_ = (call);                                                                 \
        if (err_ != hipSuccess) {                                                                       \
            fprintf(stderr, "ggml-mi355x: %s failed at %s:%d: %s\n", #call, __FILE__, __LINE__,       \
                    hipGetErrorString(err_));                                                           \
            abort();                                                                                    \
        }                                                                                               \
    } while (0)

#define MI_ASSERT(x)                                                                                    \
    do {                                                                                                \
        if (!(x)) {                                                                                     \
            fflush(stdout);                                                                             \
            fprintf(stderr, "ggml-mi355x: assertion failed at %s:%d: %s\n", __FILE__, __LINE__, #x);  \
            abort();                                                                                    \
        }                                                                                               \
    } while (0)

static constexpr size_t kBufferAlign = 256;   // tensor alignment inside device buffers
static constexpr size_t kBufferSlack = 256;   // tail slack: kernels may over-read < 16 B past a row

// ---------------------------------------------------------------------------------------------
// devices
// ---------------------------------------------------------------------------------------------

static int device_count() {
    static int count = [] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        return std::min(n, GGML_MI355X_MAX_DEVICES);
    }();
    return count;
}

struct mi_device_guard {
    int prev = -1;
    explicit mi_device_guard(int dev) {
        MI_CHECK(hipGetDevice(&prev));
        if (prev != dev) MI_CHECK(hipSetDevice(dev));
    }
    ~mi_device_guard() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void) hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------------------------------------
// device buffer
// ---------------------------------------------------------------------------------------------

struct mi_buffer_ctx {
    int device;
    void * dev_ptr;
    std::string name;
};

static const char * mi_buffer_get_name(ggml_backend_buffer_t buffer) {
    return ((mi_buffer_ctx *) buffer->context)->name.c_str();
}

static bool buffer_is_mi355x(ggml_backend_buffer_t buffer) {
    return buffer && buffer->iface.get_name == mi_buffer_get_name;
}

static void mi_buffer_free(ggml_backend_buffer_t buffer) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    mi_device_guard g(ctx->device);
    mi_planes_drop(ctx->dev_ptr, buffer->size);
    MI_CHECK(hipFree(ctx->dev_ptr));
    delete ctx;
}

static void * mi_buffer_get_base(ggml_backend_buffer_t buffer) { return ((mi_buffer_ctx *) buffer->context)->dev_ptr; }

static void mi_buffer_set_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    mi_device_guard g(ctx->device);
    // null stream: ordered after any queued work on the (blocking) backend streams
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, nullptr));
    mi_planes_refresh((char *) tensor->data + offset, size, nullptr);  // repacked planes over these bytes
    MI_CHECK(hipStreamSynchronize(nullptr));
}

static void mi_buffer_get_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    mi_device_guard g(ctx->device);
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, nullptr));
    MI_CHECK(hipStreamSynchronize(nullptr));
}

static bool mi_buffer_cpy_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * src, ggml_tensor * dst) {
    ggml_backend_buffer_t src_buf = src->view_src ? src->view_src->buffer : src->buffer;
    if (!buffer_is_mi355x(src_buf)) return false;
    auto * sctx = (mi_buffer_ctx *) src_buf->context;
    auto * dctx = (mi_buffer_ctx *) buffer->context;
    mi_device_guard g(dctx->device);
    if (sctx->device == dctx->device) {
        MI_CHECK(hipMemcpyAsync(dst->data, src->data, ggml_nbytes(src), hipMemcpyDeviceToDevice, nullptr));
    } else {
        MI_CHECK(hipMemcpyPeerAsync(dst->data, dctx->device, src->data, sctx->device, ggml_nbytes(src), nullptr));
    }
    mi_planes_refresh(dst->data, ggml_nbytes(src), nullptr);
    MI_CHECK(hipStreamSynchronize(nullptr));
    return true;
}

static void mi_buffer_clear(ggml_backend_buffer_t buffer, uint8_t value) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    mi_device_guard g(ctx->device);
    MI_CHECK(hipMemset(ctx->dev_ptr, value, buffer->size));
    mi_planes_refresh(ctx->dev_ptr, buffer->size, nullptr);
    MI_CHECK(hipStreamSynchronize(nullptr));
}

static const ggml_backend_buffer_i k_mi_buffer_i = {
    /* get_name    */ mi_buffer_get_name,
    /* free_buffer */ mi_buffer_free,
    /* get_base    */ mi_buffer_get_base,
    /* init_tensor */ nullptr,
    /* set_tensor  */ mi_buffer_set_tensor,
    /* get_tensor  */ mi_buffer_get_tensor,
    /* cpy_tensor  */ mi_buffer_cpy_tensor,
    /* clear       */ mi_buffer_clear,
    /* reset       */ nullptr,
};

// ---------------------------------------------------------------------------------------------
// device buffer type (one static instance per device, ggml-cuda.cu:553-576)
// ---------------------------------------------------------------------------------------------

struct mi_buft_ctx {
    int device;
    std::string name;
};

static const char * mi_buft_get_name(ggml_backend_buffer_type_t buft) { return ((mi_buft_ctx *) buft->context)->name.c_str(); }

static ggml_backend_buffer_t mi_buft_alloc_buffer(ggml_backend_buffer_type_t buft, size_t size) {
    auto * bctx = (mi_buft_ctx *) buft->context;
    mi_device_guard g(bctx->device);
    size = std::max(size, (size_t) 1);
    void * ptr = nullptr;
    const hipError_t err = hipMalloc(&ptr, size + kBufferSlack);
    if (err != hipSuccess) {
        (void) hipGetLastError();
        fprintf(stderr, "%s: allocating %.2f MiB on device %d: hipMalloc failed: %s\n", __func__,
                size / 1024.0 / 1024.0, bctx->device, hipGetErrorString(err));
        return nullptr;
    }
    auto * ctx = new mi_buffer_ctx{bctx->device, ptr, "MI355X" + std::to_string(bctx->device)};
    return ggml_backend_buffer_init(buft, k_mi_buffer_i, ctx, size);
}

static size_t mi_buft_get_alignment(ggml_backend_buffer_type_t) { return kBufferAlign; }

static size_t mi_buft_get_max_size(ggml_backend_buffer_type_t) { return SIZE_MAX; }

static size_t mi_buft_get_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * tensor) { return ggml_nbytes(tensor); }

static bool mi_buft_supports_backend(ggml_backend_buffer_type_t buft, ggml_backend_t backend);

static const ggml_backend_buffer_type_i k_mi_buft_i = {
    /* get_name         */ mi_buft_get_name,
    /* alloc_buffer     */ mi_buft_alloc_buffer,
    /* get_alignment    */ mi_buft_get_alignment,
    /* get_max_size     */ mi_buft_get_max_size,
    /* get_alloc_size   */ mi_buft_get_alloc_size,
    /* supports_backend */ mi_buft_supports_backend,
    /* is_host          */ nullptr,
};

// ---------------------------------------------------------------------------------------------
// pinned host buffer type (ggml-cuda.cu:979-1050)
// ---------------------------------------------------------------------------------------------

static const char * mi_host_buffer_name(ggml_backend_buffer_t) { return "MI355X_Host"; }
static void mi_host_buffer_free(ggml_backend_buffer_t b) { MI_CHECK(hipHostFree(b->context)); }
static void * mi_host_buffer_base(ggml_backend_buffer_t b) { return b->context; }
static void mi_host_buffer_set(ggml_backend_buffer_t, ggml_tensor * t, const void * d, size_t o, size_t n) { memcpy((char *) t->data + o, d, n); }
static void mi_host_buffer_get(ggml_backend_buffer_t, const ggml_tensor * t, void * d, size_t o, size_t n) { memcpy(d, (const char *) t->data + o, n); }
static void mi_host_buffer_clear(ggml_backend_buffer_t b, uint8_t v) { memset(b->context, v, b->size); }

static const ggml_backend_buffer_i k_mi_host_buffer_i = {
    mi_host_buffer_name, mi_host_buffer_free, mi_host_buffer_base, nullptr, mi_host_buffer_set, mi_host_buffer_get,
    nullptr, mi_host_buffer_clear, nullptr,
};

static const char * mi_host_buft_name(ggml_backend_buffer_type_t) { return "MI355X_Host"; }

static ggml_backend_buffer_t mi_host_buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    void * ptr = nullptr;
    if (hipHostMalloc(&ptr, std::max(size, (size_t) 1), hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
        (void) hipGetLastError();
        // fall back to pageable host memory of the runtime's host buffer type
        return ggml_backend_buft_alloc_buffer(ggml_backend_cpu_buffer_type(), size);
    }
    return ggml_backend_buffer_init(buft, k_mi_host_buffer_i, ptr, size);
}

static size_t mi_host_buft_align(ggml_backend_buffer_type_t) { return 64; }
// pinned host memory is ordinary CPU memory to the scheduler: whatever backend can use a CPU
// buffer can use this one (ggml-cuda.cu:1037-1038 delegates the same way)
static bool mi_host_buft_supports(ggml_backend_buffer_type_t, ggml_backend_t backend) {
    ggml_backend_buffer_type_t cpu = ggml_backend_cpu_buffer_type();
    return cpu->iface.supports_backend(cpu, backend);
}
static bool mi_host_buft_is_host(ggml_backend_buffer_type_t) { return true; }

// ---------------------------------------------------------------------------------------------
// tensor-split row buffer type (ggml-cuda.cu:578-975 analogue)
// ---------------------------------------------------------------------------------------------
// The rows of each weight matrix are divided over "slots" by the cumulative fractions given to
// ggml_backend_mi355x_split_buffer_type(); slot s lives on device s. With the test setting
// GGML_MI355X_SPLIT_SLOTS=n on a machine with fewer devices, slot s lives on device s % count,
// still with its own allocation, stream and copies, so the whole multi-device path (activation
// copy in, per-slot GEMM, gather of the row slices) runs on one GPU. GGML_OP_MUL_MAT with such a
// weight is op_mul_mat_split below.

static int split_slots() {
    static int n = [] {
        const char * e = getenv("GGML_MI355X_SPLIT_SLOTS");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? std::min(v, GGML_MI355X_MAX_DEVICES) : std::max(device_count(), 1);
    }();
    return n;
}

static int slot_device(int slot) { return slot % std::max(device_count(), 1); }

struct mi_split_slice {
    int slot;
    int device;
    int64_t row_low, row_high;
    char * ptr;
};
struct mi_split_extra {
    std::vector<mi_split_slice> slices;
};
struct mi_split_buft_ctx {
    std::vector<float> split;  // cumulative start fraction of each slot
};
struct mi_split_buffer_ctx {
    std::vector<mi_split_extra *> extras;
};

// slices start on multiples of the GEMM's 64-row tile (any row count is valid for every kernel)
static constexpr int64_t kSplitRowRounding = 64;

static void split_rows(const ggml_tensor * t, const mi_split_buft_ctx * c, int slot, int64_t & lo, int64_t & hi) {
    const int64_t nrows = ggml_nrows(t);
    const int n = (int) c->split.size();
    lo = slot == 0 ? 0 : (int64_t) ((double) nrows * c->split[slot]);
    lo -= lo % kSplitRowRounding;
    if (slot == n - 1) {
        hi = nrows;
    } else {
        hi = (int64_t) ((double) nrows * c->split[slot + 1]);
        hi -= hi % kSplitRowRounding;
    }
    hi = std::max(hi, lo);
}

static const char * mi_split_buffer_name(ggml_backend_buffer_t) { return "MI355X_Split"; }

static bool buffer_is_split(ggml_backend_buffer_t buffer) {
    return buffer && buffer->iface.get_name == mi_split_buffer_name;
}

static bool is_split_tensor(const ggml_tensor * t) {
    const ggml_tensor * base = t->view_src ? t->view_src : t;
    return buffer_is_split(base->buffer);
}

static void mi_split_buffer_free(ggml_backend_buffer_t buffer) {
    auto * ctx = (mi_split_buffer_ctx *) buffer->context;
    for (mi_split_extra * e : ctx->extras) {
        for (const auto & sl : e->slices) {
            mi_device_guard g(sl.device);
            MI_CHECK(hipFree(sl.ptr));
        }
        delete e;
    }
    delete ctx;
}

static void * mi_split_buffer_base(ggml_backend_buffer_t) {
    return (void *) 0x1000;  // the slices' pointers live in tensor->extra; never dereferenced
}

static void mi_split_buffer_init_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor) {
    MI_ASSERT(tensor->view_src == nullptr && "views of split tensors are not supported");
    auto * ctx = (mi_split_buffer_ctx *) buffer->context;
    auto * bctx = (mi_split_buft_ctx *) buffer->buft->context;
    auto * extra = new mi_split_extra();
    ctx->extras.push_back(extra);
    const size_t nb1 = ggml_row_size(tensor->type, tensor->ne[0]);
    for (int s = 0; s < (int) bctx->split.size(); s++) {
        int64_t lo, hi;
        split_rows(tensor, bctx, s, lo, hi);
        if (hi == lo) continue;
        mi_split_slice sl{s, slot_device(s), lo, hi, nullptr};
        mi_device_guard g(sl.device);
        const size_t bytes = (size_t) (hi - lo) * nb1;
        MI_CHECK(hipMalloc((void **) &sl.ptr, bytes + kBufferSlack));  // init_tensor cannot fail (ggml-cuda.cu:755)
        MI_CHECK(hipMemset(sl.ptr + bytes, 0, kBufferSlack));
        extra->slices.push_back(sl);
    }
    tensor->extra = extra;
}

static void mi_split_buffer_set_tensor(ggml_backend_buffer_t, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    // split tensors are set whole (ggml-cuda.cu:781-782)
    MI_ASSERT(offset == 0 && size == ggml_nbytes(tensor));
    const auto * extra = (const mi_split_extra *) tensor->extra;
    for (const auto & sl : extra->slices) {
        mi_device_guard g(sl.device);
        MI_CHECK(hipMemcpy(sl.ptr, (const char *) data + sl.row_low * tensor->nb[1], (size_t) (sl.row_high - sl.row_low) * tensor->nb[1],
                           hipMemcpyHostToDevice));
    }
}

static void mi_split_buffer_get_tensor(ggml_backend_buffer_t, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    MI_ASSERT(offset == 0 && size == ggml_nbytes(tensor));
    const auto * extra = (const mi_split_extra *) tensor->extra;
    for (const auto & sl : extra->slices) {
        mi_device_guard g(sl.device);
        MI_CHECK(hipMemcpy((char *) data + sl.row_low * tensor->nb[1], sl.ptr, (size_t) (sl.row_high - sl.row_low) * tensor->nb[1],
                           hipMemcpyDeviceToHost));
    }
}

static void mi_split_buffer_clear(ggml_backend_buffer_t, uint8_t) {}  // as ggml-cuda.cu:856-859

static const ggml_backend_buffer_i k_mi_split_buffer_i = {
    /* get_name    */ mi_split_buffer_name,
    /* free_buffer */ mi_split_buffer_free,
    /* get_base    */ mi_split_buffer_base,
    /* init_tensor */ mi_split_buffer_init_tensor,
    /* set_tensor  */ mi_split_buffer_set_tensor,
    /* get_tensor  */ mi_split_buffer_get_tensor,
    /* cpy_tensor  */ nullptr,
    /* clear       */ mi_split_buffer_clear,
    /* reset       */ nullptr,
};

static const char * mi_split_buft_name(ggml_backend_buffer_type_t) { return "MI355X_Split"; }

static ggml_backend_buffer_t mi_split_buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    // the slices are allocated per tensor in init_tensor, once the rounded split is known; size is
    // the bound ggml-alloc enforces with get_alloc_size (ggml-cuda.cu:887-895)
    return ggml_backend_buffer_init(buft, k_mi_split_buffer_i, new mi_split_buffer_ctx(), size);
}

static size_t mi_split_buft_align(ggml_backend_buffer_type_t) { return kBufferAlign; }

static size_t mi_split_buft_alloc_size(ggml_backend_buffer_type_t buft, const ggml_tensor * tensor) {
    auto * c = (mi_split_buft_ctx *) buft->context;
    const size_t nb1 = ggml_row_size(tensor->type, tensor->ne[0]);
    size_t total = 0;
    for (int s = 0; s < (int) c->split.size(); s++) {
        int64_t lo, hi;
        split_rows(tensor, c, s, lo, hi);
        if (hi > lo) total += (size_t) (hi - lo) * nb1 + kBufferSlack;
    }
    return std::max(total, ggml_nbytes(tensor));
}

static bool mi_split_buft_supports(ggml_backend_buffer_type_t, ggml_backend_t backend) { return ggml_backend_is_mi355x(backend); }

static const ggml_backend_buffer_type_i k_mi_split_buft_i = {
    /* get_name         */ mi_split_buft_name,
    /* alloc_buffer     */ mi_split_buft_alloc,
    /* get_alignment    */ mi_split_buft_align,
    /* get_max_size     */ nullptr,
    /* get_alloc_size   */ mi_split_buft_alloc_size,
    /* supports_backend */ mi_split_buft_supports,
    /* is_host          */ nullptr,
};

// ---------------------------------------------------------------------------------------------
// backend context
// ---------------------------------------------------------------------------------------------

struct mi_act_cache_entry {
    const void * data;   // src1 data
    size_t nbytes;
    int kind;            // 0 = q8_0, 1 = q8_K, 2 = f16
    int64_t ne[4];
    size_t nb[4];
    void * dev;          // converted activations in scratch
};

struct mi_backend_ctx {
    int device;
    std::string name;
    hipStream_t stream = nullptr;
    void * scratch = nullptr;
    size_t scratch_size = 0;
    size_t scratch_used = 0;
    std::vector<mi_act_cache_entry> act_cache;
    int last_launches = 0;
    uint16_t * tables = nullptr;  // device: exp, gelu, silu fp16 tables (3 x 65536)
    hipEvent_t split_ready = nullptr;  // src1 of a split mul_mat is ready on `stream`
    hipEvent_t plan_marker = nullptr;  // recorded behind each plan launch (mi_graph_plan_compute)
    uint64_t scratch_gen = 0;     // bumped whenever `scratch` is reallocated (captures refer to it)
    // hipGraph plans (mi_graph_plan_create): captured launches of a whole ggml graph
    bool graphs = true;
    std::vector<hipGraphExec_t> exec_pool;  // executable graphs of freed plans, for in-place update
    int graph_fail_streak = 0;         // consecutive re-instantiations (update refused)
    // counters: [0] captures (plans and graph_compute), [1] instantiations, [2] in-place updates,
    // [3] direct (uncaptured) computes, [4] graph_compute replays of a cached capture,
    // [5] graph_compute captures
    int64_t graph_stats[6] = {};
    // graph_compute's own captures (ggml-cuda.cu:2456-2713 analogue): executable graphs keyed by
    // the exact launch-relevant content of the cgraph (mi_graph_key); an entry whose topology
    // matches a new graph is updated in place (hipGraphExecUpdate) before a new one is built
    struct gcache_entry {
        std::vector<uint64_t> key;
        uint64_t topo = 0;
        hipGraphExec_t exec = nullptr;
        hipEvent_t done = nullptr;  // recorded behind every launch of `exec`
        uint64_t last_use = 0;
        int launches = 0;
        bool no_update = false;  // hipGraphExecUpdate refused once: replay-only
    };
    // per-node timer (the reference's GGML_PERF, ggml.c:19195-19205): HIP events around every
    // dispatch unit of a directly launched graph; see ggml_backend_mi355x_set_perf
    bool perf = getenv("GGML_MI355X_PERF") != nullptr;
    std::vector<hipEvent_t> perf_ev;   // pool
    std::vector<int> perf_at;          // node index at which unit k starts
    std::vector<gcache_entry> gcache;
    uint64_t gclock = 0;
    std::unordered_map<uint64_t, int> topo_launches;  // kernel launches of a topology's last direct run
    std::unordered_map<uint64_t, int> topo_misses;    // consecutive captures of a topology without a replay
    // host-built RoPE {cos, sin} tables (rope_table_ensure), one per parameter set
    struct rope_table {
        int n_dims, ne0, mode, P;
        float freq_base, freq_scale, ext_factor, attn_factor, corr0, corr1;
        float * dev;
    };
    std::vector<rope_table> rope_tables;
    // a node value still held as partial sums (try_fuse_attn_proj): `out` = sum_h parts[h], to be
    // stored by its consumer's kernel (the next GEMV's norm prologue) or by mi_sum_parts
    struct {
        const ggml_tensor * out = nullptr;
        float * parts = nullptr;
        int nparts = 0;
        int64_t n = 0;
    } pend;
};

static ggml_guid_t mi_guid() {
    static ggml_guid guid = {0x4d, 0x49, 0x33, 0x35, 0x35, 0x58, 0x2d, 0x67, 0x66, 0x78, 0x39, 0x35, 0x30, 0x2d, 0x76, 0x31};
    return &guid;
}

static void * scratch_take(mi_backend_ctx * ctx, size_t bytes) {
    bytes = (bytes + kBufferAlign - 1) & ~(kBufferAlign - 1);
    MI_ASSERT(ctx->scratch_used + bytes <= ctx->scratch_size);
    void * p = (char *) ctx->scratch + ctx->scratch_used;
    ctx->scratch_used += bytes;
    return p;
}

static void scratch_reserve(mi_backend_ctx * ctx, size_t bytes) {
    if (bytes <= ctx->scratch_size) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    MI_CHECK(hipStreamIsCapturing(ctx->stream, &cs));
    MI_ASSERT(cs == hipStreamCaptureStatusNone && "scratch must be reserved before a graph capture");
    MI_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->scratch) MI_CHECK(hipFree(ctx->scratch));
    const size_t want = std::max(bytes + bytes / 2, (size_t) 16 << 20);
    MI_CHECK(hipMalloc(&ctx->scratch, want));
    ctx->scratch_size = want;
    ctx->scratch_gen++;  // executable graphs captured against the old buffer must not run again
}

// ---------------------------------------------------------------------------------------------
// op support (ggml-cuda.cu:2715-2859 analogue; the scheduler does not consult it, the
// conformance harness does)
// ---------------------------------------------------------------------------------------------

static bool mm_src0_supported(ggml_type t) {
    return t == GGML_TYPE_Q4_0 || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K ||
           t == GGML_TYPE_F16 || t == GGML_TYPE_F32;
}

static bool is_f32(const ggml_tensor * t) { return t && t->type == GGML_TYPE_F32; }
static bool is_f16_or_f32(const ggml_tensor * t) { return t && (t->type == GGML_TYPE_F32 || t->type == GGML_TYPE_F16); }

// the quantized vec_dot_type a src1 may already have for weight type t (GGML_TYPE_COUNT: none)
static ggml_type q8_src1_type(ggml_type t) {
    switch (t) {
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: return GGML_TYPE_Q8_K;
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q8_0: return GGML_TYPE_Q8_0;
        default: return GGML_TYPE_COUNT;
    }
}

static bool mi_supports_op(ggml_backend_t, const ggml_tensor * op) {
    const ggml_tensor * a = op->src[0];
    const ggml_tensor * b = op->src[1];
    switch (op->op) {
        case GGML_OP_NONE:
        case GGML_OP_RESHAPE:
        case GGML_OP_VIEW:
        case GGML_OP_PERMUTE:
        case GGML_OP_TRANSPOSE:
            return true;
        case GGML_OP_MUL_MAT: {
            if (!mm_src0_supported(a->type)) return false;
            if (a->nb[0] != ggml_type_size(a->type) || b->nb[0] != ggml_type_size(b->type)) return false;
            // src1 F32, or src1 already of the weight's vec_dot_type, which the reference CPU reads as
            // it lies (ggml.c:11952; F16 x F16, Q4_K/Q5_K x Q8_K, Q4_0/Q8_0 x Q8_0): the quantized
            // ones with whole superblocks, on the device's own weights
            // (the split-buffer path converts an F32 src1 on the main device: F16 src1 only unsplit)
            if (b->type == GGML_TYPE_F32 || (b->type == GGML_TYPE_F16 && a->type == GGML_TYPE_F16 && !is_split_tensor(a))) return true;
            return b->type == q8_src1_type(a->type) && a->ne[0] % 256 == 0 && !is_split_tensor(a);
        }
        case GGML_OP_ADD:
        case GGML_OP_SUB:
        case GGML_OP_MUL:
        case GGML_OP_DIV:
            return is_f16_or_f32(a) && is_f16_or_f32(b) && is_f16_or_f32(op);
        case GGML_OP_SCALE:
            return is_f32(a) && is_f32(op);
        case GGML_OP_NORM:
        case GGML_OP_RMS_NORM:
            // rows longer than the kernel's LDS staging (12288 floats) stage in a contiguous dst
            return is_f32(a) && is_f32(op) && a->nb[0] == sizeof(float) && (a->ne[0] <= 12288 || ggml_is_contiguous(op));
        case GGML_OP_SOFT_MAX: {
            float max_bias;
            memcpy(&max_bias, (const float *) op->op_params + 1, sizeof(float));
            return is_f32(a) && is_f32(op) && max_bias == 0.0f && (!b || is_f16_or_f32(b)) && ggml_is_contiguous(a);
        }
        case GGML_OP_DIAG_MASK_INF:
        case GGML_OP_DIAG_MASK_ZERO:
            return is_f32(a) && is_f32(op);
        case GGML_OP_UNARY:
            switch (ggml_get_unary_op(op)) {
                case GGML_UNARY_OP_GELU:
                case GGML_UNARY_OP_SILU:
                    return is_f32(a) && is_f32(op);
                default:
                    return false;
            }
        case GGML_OP_GET_ROWS:
            return (is_f16_or_f32(a) || a->type == GGML_TYPE_Q4_0 || a->type == GGML_TYPE_Q8_0 || a->type == GGML_TYPE_Q4_K ||
                    a->type == GGML_TYPE_Q5_K) &&
                   b->type == GGML_TYPE_I32 && is_f32(op);
        case GGML_OP_CPY:
        case GGML_OP_DUP:
        case GGML_OP_CONT:
            // F32 -> Q8_K / Q8_0 (from_float = quantize_row_q8_K / _q8_0): whole rows of blocks
            if (is_f32(a) && (op->type == GGML_TYPE_Q8_K || op->type == GGML_TYPE_Q8_0))
                return ggml_are_same_shape(a, op) && a->nb[0] == sizeof(float) && op->nb[0] == ggml_type_size(op->type) &&
                       op->ne[0] % (op->type == GGML_TYPE_Q8_K ? 256 : 32) == 0;
            return is_f16_or_f32(a) && is_f16_or_f32(op);
        case GGML_OP_ROPE: {
            const int32_t * pp = (const int32_t *) op->op_params;
            const int mode = pp[2];
            float xpos_base;
            memcpy(&xpos_base, pp + 11, sizeof(float));
            return is_f32(a) && is_f32(op) && (mode == 0 || mode == 2) && xpos_base == 0.0f && a->nb[0] == sizeof(float);
        }
        default:
            return false;
    }
}

static bool mi_offload_op(ggml_backend_t, const ggml_tensor * op) {
    // worth moving CPU-resident weights for batched work (ggml-cuda.cu:2861-2868 uses 32)
    return op->ne[1] >= 32 && op->op != GGML_OP_GET_ROWS;
}

// ---------------------------------------------------------------------------------------------
// GGML_OP_MUL_MAT
// ---------------------------------------------------------------------------------------------

static int act_kind(ggml_type wtype) {
    switch (wtype) {
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q8_0: return 0;
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: return 1;
        case GGML_TYPE_F16: return 2;
        default: return -1;
    }
}

// kinds: 0 q8_0, 1 q8_K, 2 f16, 3/4 q8_0/q8_K quants expanded to f16(d * q) (mmq.hip operand),
// 5/6/7 = 2/3/4 in the GEMM's K-blocked layout [K/16][ncols][16], 8 q8_K / 9 q8_0 in the int8-MFMA
// layouts of the exact prefill GEMMs (mmq_exact.hip)
static size_t act_bytes(int kind, int64_t K, int64_t ncols) {
    if (kind == 8) return mi_act_mmx_bytes(K, ncols);
    if (kind == 9) return mi_act_mmx0_bytes(K, ncols);
    if (kind >= 2) return (size_t) K * ncols * 2;
    return mi_act_q8_bytes(K, ncols, kind == 1);
}

static mi_src_cols src_cols(const ggml_tensor * t) {
    mi_src_cols x;
    x.base = (const char *) t->data;
    x.ne1 = t->ne[1];
    x.ne2 = t->ne[2];
    x.ne3 = t->ne[3];
    x.nb1 = t->nb[1];
    x.nb2 = t->nb[2];
    x.nb3 = t->nb[3];
    return x;
}

// Converted activations for (src1, kind), reused by later mul_mats of the same graph that read
// the same, unmodified src1 (Q/K/V or gate/up projections share their input).
static void * find_activations(const mi_backend_ctx * ctx, const ggml_tensor * src1, int kind) {
    for (const auto & e : ctx->act_cache) {
        if (e.data == src1->data && e.kind == kind && memcmp(e.ne, src1->ne, sizeof(e.ne)) == 0 &&
            memcmp(e.nb, src1->nb, sizeof(e.nb)) == 0) {
            return e.dev;
        }
    }
    return nullptr;
}

static void cache_activations(mi_backend_ctx * ctx, const ggml_tensor * src1, int kind, void * dev) {
    mi_act_cache_entry e;
    e.data = src1->data;
    e.nbytes = ggml_nbytes(src1);
    e.kind = kind;
    memcpy(e.ne, src1->ne, sizeof(e.ne));
    memcpy(e.nb, src1->nb, sizeof(e.nb));
    e.dev = dev;
    ctx->act_cache.push_back(e);
}

static void * get_activations(mi_backend_ctx * ctx, const ggml_tensor * src1, int kind, int64_t K) {
    if (void * hit = find_activations(ctx, src1, kind)) return hit;
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    void * dev = scratch_take(ctx, act_bytes(kind, K, ncols));
    const mi_src_cols x = src_cols(src1);
    if (src1->type == GGML_TYPE_Q8_K || src1->type == GGML_TYPE_Q8_0) {
        // already quantized by the reference's rules (e.g. a CPY F32 -> Q8_K): re-laid out only
        MI_ASSERT(kind == 0 || kind == 1 || kind == 8 || kind == 9);
        const bool q8K = src1->type == GGML_TYPE_Q8_K;
        MI_ASSERT(q8K == (kind == 1 || kind == 8));
        if (kind >= 8) {
            const mi_act_mmx mx = q8K ? mi_act_mmx_carve(dev, K, ncols) : mi_act_mmx0_carve(dev, K, ncols);
            mi_q8_rows_to_act(x, K, q8K, nullptr, &mx, ctx->stream);
        } else {
            const mi_act_q8 act = mi_act_q8_carve(dev, K, ncols, q8K);
            mi_q8_rows_to_act(x, K, q8K, &act, nullptr, ctx->stream);
        }
    } else if (kind == 8 || kind == 9) {
        mi_mmx_qgroup q;
        q.n = 1;
        q.K = K;
        q.m[0].x = x;
        q.m[0].act = kind == 8 ? mi_act_mmx_carve(dev, K, ncols) : mi_act_mmx0_carve(dev, K, ncols);
        if (kind == 8) mi_quantize_q8_K_mmx_group(q, ctx->stream);
        else mi_quantize_q8_0_mmx_group(q, ctx->stream);
    } else if (kind == 2 || kind == 5) {
        mi_convert_f16(x, K, (uint16_t *) dev, ctx->stream, kind == 5, src1->type == GGML_TYPE_F16);
    } else if (kind >= 3) {
        mi_quantize_expand_f16(x, K, ncols, kind == 4 || kind == 7, (uint16_t *) dev, ctx->stream, kind >= 6);
    } else {
        const mi_act_q8 act = mi_act_q8_carve(dev, K, ncols, kind == 1);
        if (kind == 1) mi_quantize_q8_K(x, K, act, ctx->stream);
        else mi_quantize_q8_0(x, K, act, ctx->stream);
    }
    ctx->last_launches++;
    cache_activations(ctx, src1, kind, dev);
    return dev;
}

static void invalidate_activations(mi_backend_ctx * ctx, const ggml_tensor * written) {
    const char * lo = (const char *) written->data;
    const char * hi = lo + ggml_nbytes(written);
    // a node writing into memory that repacked planes mirror (weights written through a view, or a
    // reused compute-buffer region that once held a Q4_K leaf) renews the planes over it
    if (mi_planes_count() > 0) mi_planes_refresh(lo, (size_t) (hi - lo), ctx->stream);
    auto & c = ctx->act_cache;
    c.erase(std::remove_if(c.begin(), c.end(), [&](const mi_act_cache_entry & e) {
                const char * elo = (const char *) e.data;
                return elo < hi && lo < elo + e.nbytes;
            }),
            c.end());
}

// the batched (prompt) GEMM applies: more than 8 columns of plain 2-D operands
static bool mm_batched(const mi_mm_desc & m, const ggml_tensor * src1) {
    static const bool no_mmq = getenv("GGML_MI355X_NO_MMQ") != nullptr;
    return !no_mmq && act_kind((ggml_type) m.type) >= 0 && src1->ne[1] > 8 && m.ne02 == 1 && m.ne03 == 1 && m.ne12 == 1 &&
           m.ne13 == 1 && mi_mmq_supported(m.type, m.K, m.nb01, m.nb1) && ((uintptr_t) m.W % 16) == 0;
}

// The activation format mul_mat_run converts src1 to for this mul_mat (act_bytes kinds), or -1
// (F32 weights: src1 is read as it lies). Q4_K / Q5_K prompts: the exact-integer int8 GEMM's
// q8_K layouts (8); Q4_0 / Q8_0 prompts: its q8_0 layouts (9); F16 prompts: f16 operands (2, or
// K-blocked 5); decode: q8 SoA (0 / 1) or f16 (2).
static int mm_act_kind(const mi_mm_desc & m, const ggml_tensor * src1) {
    const int kind = act_kind((ggml_type) m.type);
    if (kind < 0) return -1;
    const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
    if (src1->type != GGML_TYPE_F32 && src1->type != GGML_TYPE_F16) {
        // pre-quantized src1 (Q8_K / Q8_0 rows): the exact GEMMs' layouts, else the GEMV's
        return mm_batched(m, src1) && mi_mmqx_supported(m.type, m.K, m.nb1, ncols, m.nb01) ? (kind == 1 ? 8 : 9) : kind;
    }
    if (!mm_batched(m, src1)) return kind;
    // GGML_MI355X_MMQ_VARIANT bit 2^30 selects the f16 GEMM for the quantized types too (A/B
    // timing; the low bits are mmq_exact.hip's own kernel variants)
    if (kind <= 1 && (g_mi_tuning.mmq_variant & (1 << 30)) == 0 && mi_mmqx_supported(m.type, m.K, m.nb1, ncols, m.nb01)) return kind == 1 ? 8 : 9;
    return (kind == 2 ? 2 : kind + 3) + (mi_mmq_wants_blocked() ? 3 : 0);
}

// the repacked MFMA planes of the long Q4_K / Q5_K prompts' weights (before any capture: creating
// them allocates); only graph leaves (weights), never a tensor a node of the graph writes
static const char * planes_of(mi_backend_ctx * ctx, const ggml_tensor * a, const ggml_tensor * b) {
    if (!g_mi_tuning.planes || (a->type != GGML_TYPE_Q4_K && a->type != GGML_TYPE_Q5_K) || a->op != GGML_OP_NONE || a->ne[2] != 1 ||
        a->ne[3] != 1 || b->ne[1] * b->ne[2] * b->ne[3] < kMiPlanesMinCols || is_split_tensor(a))
        return nullptr;
    // only tensors of this backend's own device buffers: host and peer memory have write paths
    // (host-buffer set/clear, peer copies) that do not renew the planes. Within a device buffer every
    // write path renews them: set/get/cpy/clear (sync and async) and any graph node whose output
    // overlaps an entry (invalidate_activations), so a compute buffer's reused memory is covered too
    const ggml_backend_buffer_t buf = a->view_src ? a->view_src->buffer : a->buffer;
    if (!buffer_is_mi355x(buf) || ((mi_buffer_ctx *) buf->context)->device != ctx->device) return nullptr;
    return mi_planes_get(a->type, a->data, a->nb[1], a->ne[0], a->ne[1], ctx->stream);
}

// The 16-byte-aligned copy of a Q4_0 / Q8_0 weight for the tree-order decode GEMV (mmq_planes.hip
// k_q40_repack / k_q80_repack; created before any capture, renewed by the same write paths as the planes): the
// same conditions as planes_of -- a graph leaf in this backend's own device buffer
static const char * q40r_of(mi_backend_ctx * ctx, const ggml_tensor * a) {
    const bool on = a->type == GGML_TYPE_Q4_0 ? g_mi_tuning.q40r : a->type == GGML_TYPE_Q8_0 ? g_mi_tuning.q80r : 0;
    if (!on || a->op != GGML_OP_NONE || a->ne[2] != 1 || a->ne[3] != 1 || is_split_tensor(a))
        return nullptr;
    const ggml_backend_buffer_t buf = a->view_src ? a->view_src->buffer : a->buffer;
    if (!buffer_is_mi355x(buf) || ((mi_buffer_ctx *) buf->context)->device != ctx->device) return nullptr;
    return mi_planes_get(a->type, a->data, a->nb[1], a->ne[0], a->ne[1], ctx->stream);
}

// A Q4_0 / Q8_0 decode group in tree order on the repacked copies (FmtQ0R / FmtQ8R): every member's
// weight must have one, else the canonical blocks (FmtQ0Pair / FmtQ0<true>) -- the same bits
static void q40r_apply(mi_backend_ctx * ctx, mi_mmv_group & g, const ggml_tensor * const * w) {
    // (one column: with two, the aligned copy measured 2-3 % slower, profiles/r06s2_q40r_ab.txt)
    const bool q4 = g.type == GGML_TYPE_Q4_0;
    if ((!q4 && g.type != GGML_TYPE_Q8_0) || g.ncols != 1 || !(q4 ? g_mi_tuning.q40r : g_mi_tuning.q80r) || mi_mmv_order() != 0 ||
        (q4 && g_mi_tuning.mmv_variant % 10 == 1)) return;
    const void * p[kMiMaxMembers];
    for (int m = 0; m < g.n; m++) {
        p[m] = q40r_of(ctx, w[m]);
        if (!p[m]) return;
    }
    for (int m = 0; m < g.n; m++) g.m[m].W = p[m];
    g.nb01 = (size_t) (g.K / 32 * (q4 ? 18 : 34));
    g.q0r = 1;
}

// The mul_mat of (src0, src1) with src0's rows taken from (W, N) and the output written at out
// (column strides nb1..nb3): op_mul_mat runs the whole node through it, the split-buffer path
// (op_mul_mat_split) each device's row slice.
static void mul_mat_run(mi_backend_ctx * ctx, const ggml_tensor * src0, const void * W, int64_t N, const ggml_tensor * src1,
                        float * out, size_t nb1, size_t nb2, size_t nb3) {
    MI_ASSERT(src1->type == GGML_TYPE_F32 || (src1->type == GGML_TYPE_F16 && src0->type == GGML_TYPE_F16) ||
              src1->type == q8_src1_type(src0->type));
    MI_ASSERT(src0->nb[0] == ggml_type_size(src0->type));
    MI_ASSERT(src1->nb[0] == ggml_type_size(src1->type));
    MI_ASSERT(src0->ne[0] == src1->ne[0]);
    MI_ASSERT(src1->ne[2] % src0->ne[2] == 0 && src1->ne[3] % src0->ne[3] == 0);

    mi_mm_desc m;
    m.W = W;
    m.type = src0->type;
    m.K = src0->ne[0];
    m.N = N;
    m.ne02 = src0->ne[2];
    m.ne03 = src0->ne[3];
    m.nb01 = src0->nb[1];
    m.nb02 = src0->nb[2];
    m.nb03 = src0->nb[3];
    m.ne11 = src1->ne[1];
    m.ne12 = src1->ne[2];
    m.ne13 = src1->ne[3];
    m.dst = out;
    m.nb1 = nb1;
    m.nb2 = nb2;
    m.nb3 = nb3;

    const int xkind = mm_act_kind(m, src1);
    if (xkind == 5 && m.type == GGML_TYPE_F16 && src1->type == GGML_TYPE_F32 && src1->ne[2] == 1 && src1->ne[3] == 1 &&
        mi_mmf16p_f32_supported(m.K, m.N, m.nb01, src1->ne[1], m.nb1, src1->data, src1->nb[1])) {
        // F16 weights, a short prompt of plain f32 columns: one launch, activations rounded to f16
        // inside the GEMM (k_mmf16p<F32X>)
        mi_mul_mat_f16p_f32(m.W, m.nb01, m.K, m.N, (const float *) src1->data, src1->nb[1], src1->ne[1], m.dst, m.nb1, ctx->stream);
        ctx->last_launches++;
        return;
    }
    if (xkind < 0) {
        MI_ASSERT(src0->type == GGML_TYPE_F32);
        mi_mul_mat_f32(m, src_cols(src1), ctx->stream);
    } else {
        const int64_t ncols = src1->ne[1] * src1->ne[2] * src1->ne[3];
        void * xa = get_activations(ctx, src1, xkind, m.K);
        if (xkind == 8 || xkind == 9) {
            // Q4_K / Q5_K / Q4_0 / Q8_0: the exact-integer int8 MFMA GEMMs (mmq_exact.hip)
            const mi_act_mmx act = xkind == 8 ? mi_act_mmx_carve(xa, m.K, ncols) : mi_act_mmx0_carve(xa, m.K, ncols);
            mi_mul_mat_mmqx(m.type, m.W, m.nb01, m.K, m.N, act, m.dst, m.nb1, ctx->stream, W == src0->data && N == src0->ne[1] ? planes_of(ctx, src0, src1) : nullptr);
        } else if (xkind == 5 && m.type == GGML_TYPE_F16 && mi_mmf16p_supported(m.K, m.N, m.nb01, ncols, m.nb1)) {
            // F16 weights, a short prompt: 32 x 32 tiles with the K split over each tile's 4 waves
            mi_mul_mat_f16p(m.W, m.nb01, m.K, m.N, (const uint16_t *) xa, ncols, m.dst, m.nb1, ctx->stream);
        } else if (xkind >= 3 || (xkind == 2 && mm_batched(m, src1))) {
            // the GEMM's activation operand: f16 for F16 weights, else f16(d * q) of the q8 quants
            // written by the quantizer itself (kinds 3/4, K-blocked 5..7)
            mi_mul_mat_mmq(m.type, m.W, m.nb01, m.K, m.N, mi_act_q8{}, (const uint16_t *) xa, ncols, m.dst, m.nb1, nullptr, ctx->stream);
        } else if (xkind == 2) {
            mi_mul_mat_f16(m, (const uint16_t *) xa, ctx->stream);
        } else {
            mi_mul_mat_q(m, mi_act_q8_carve(xa, m.K, ncols, xkind == 1), ctx->stream);
        }
    }
    ctx->last_launches++;
}

// the mul_mat descriptor of a whole MUL_MAT node (as mul_mat_run builds it)
static mi_mm_desc mm_desc_of(const ggml_tensor * node) {
    const ggml_tensor * src0 = node->src[0], * src1 = node->src[1];
    mi_mm_desc m{};
    m.W = src0->data;
    m.type = src0->type;
    m.K = src0->ne[0];
    m.N = src0->ne[1];
    m.ne02 = src0->ne[2];
    m.ne03 = src0->ne[3];
    m.nb01 = src0->nb[1];
    m.nb02 = src0->nb[2];
    m.nb03 = src0->nb[3];
    m.ne11 = src1->ne[1];
    m.ne12 = src1->ne[2];
    m.ne13 = src1->ne[3];
    m.dst = (float *) node->data;
    m.nb1 = node->nb[1];
    m.nb2 = node->nb[2];
    m.nb3 = node->nb[3];
    return m;
}

static void op_mul_mat(mi_backend_ctx * ctx, ggml_tensor * dst) {
    MI_ASSERT(dst->nb[0] == sizeof(float));
    const ggml_tensor * src0 = dst->src[0];
    mul_mat_run(ctx, src0, src0->data, src0->ne[1], dst->src[1], (float *) dst->data, dst->nb[1], dst->nb[2], dst->nb[3]);
}

// Per-slot helper context of the split path: its own stream (on the slot's device), scratch and
// activation cache, plus the event that hands the slot's gathered rows back to the caller.
struct mi_split_aux {
    mi_backend_ctx ctx;
    hipEvent_t done = nullptr;
};

static mi_split_aux * split_aux(int slot, int main_device) {
    static std::mutex mutex;
    static mi_split_aux * aux[GGML_MI355X_MAX_DEVICES] = {};
    std::lock_guard<std::mutex> lock(mutex);
    if (!aux[slot]) {
        auto * a = new mi_split_aux();
        a->ctx.device = slot_device(slot);
        a->ctx.name = "MI355X_Split" + std::to_string(slot);
        mi_device_guard g(a->ctx.device);
        MI_CHECK(hipStreamCreateWithFlags(&a->ctx.stream, hipStreamNonBlocking));
        MI_CHECK(hipEventCreateWithFlags(&a->done, hipEventDisableTiming));
        aux[slot] = a;
    }
    if (aux[slot]->ctx.device != main_device) {
        // peer access both ways for the activation copy in and the row gather out (xGMI)
        for (const auto & pr : {std::make_pair(aux[slot]->ctx.device, main_device), std::make_pair(main_device, aux[slot]->ctx.device)}) {
            mi_device_guard g(pr.first);
            const hipError_t e = hipDeviceEnablePeerAccess(pr.second, 0);
            if (e != hipSuccess) (void) hipGetLastError();  // already enabled
        }
    }
    return aux[slot];
}

// GGML_OP_MUL_MAT with a weight in the split buffer type (ggml-cuda.cu:1360-1647 analogue): the
// slot on the backend's own device computes its rows in place into dst; every other slot gets the
// activations copied to its device (peer copy over xGMI), computes its rows on its own stream into
// local scratch, and copies them back into dst's row range (a pitched copy), ordered by events.
// As the reference quantizes src1 once and ships the q8_1 blocks (ggml-cuda.cu:1551-1565), the
// activations are converted ONCE on the main device, in the format the slots' kernels read (q8_K
// / q8_0 blocks, or f16), and those bytes travel -- for Q4_K at K = 4096 4.4 KB per column
// instead of the f32 column's 16 KB; only F32 weights ship f32.
static void op_mul_mat_split(mi_backend_ctx * ctx, ggml_tensor * dst) {
    const ggml_tensor * src0 = dst->src[0];
    const ggml_tensor * src1 = dst->src[1];
    MI_ASSERT(src0->view_src == nullptr && "views of split tensors are not supported");
    MI_ASSERT(src0->ne[2] == 1 && src0->ne[3] == 1 && src1->ne[2] == 1 && src1->ne[3] == 1);
    MI_ASSERT(src1->type == GGML_TYPE_F32 && ggml_is_contiguous(src1) && dst->nb[0] == sizeof(float));
    const auto * extra = (const mi_split_extra *) src0->extra;
    const int64_t K = src0->ne[0], ncols = src1->ne[1];
    // the backend's own slot (the first slot placed on its device) runs in place; further slots on
    // the same device (GGML_MI355X_SPLIT_SLOTS > device count) take the copy path
    auto is_local = [&](const mi_split_slice & sl) { return sl.device == ctx->device && sl.slot == ctx->device % split_slots(); };
    // the activation format of each remote slot's mul_mat, converted on the main stream first
    struct remote {
        const mi_split_slice * sl;
        int64_t ld;
        int xkind;        // act_bytes kind shipped, -1: the f32 columns
        const void * xa;  // converted activations on the main device
    };
    std::vector<remote> rem;
    for (const auto & sl : extra->slices) {
        if (is_local(sl)) continue;
        const int64_t rows = sl.row_high - sl.row_low;
        remote rm{&sl, (rows + 3) & ~(int64_t) 3, -1, src1->data};
        mi_mm_desc m{};
        m.W = sl.ptr;
        m.type = src0->type;
        m.K = K;
        m.N = rows;
        m.ne02 = m.ne03 = m.ne12 = m.ne13 = 1;
        m.nb01 = src0->nb[1];
        m.ne11 = ncols;
        m.nb1 = (size_t) rm.ld * sizeof(float);
        rm.xkind = mm_act_kind(m, src1);
        if (rm.xkind >= 0) rm.xa = get_activations(ctx, src1, rm.xkind, K);
        rem.push_back(rm);
    }
    if (!rem.empty()) {
        mi_device_guard g(ctx->device);
        if (!ctx->split_ready) MI_CHECK(hipEventCreateWithFlags(&ctx->split_ready, hipEventDisableTiming));
        MI_CHECK(hipEventRecord(ctx->split_ready, ctx->stream));  // src1 and its conversions are ready
    }
    for (const auto & sl : extra->slices) {
        if (!is_local(sl)) continue;
        mul_mat_run(ctx, src0, sl.ptr, sl.row_high - sl.row_low, src1, (float *) ((char *) dst->data + sl.row_low * sizeof(float)),
                    dst->nb[1], dst->nb[2], dst->nb[3]);
    }
    std::vector<mi_split_aux *> waits;
    for (const remote & rm : rem) {
        const mi_split_slice & sl = *rm.sl;
        const int64_t rows = sl.row_high - sl.row_low;
        float * out = (float *) ((char *) dst->data + sl.row_low * sizeof(float));
        mi_split_aux * a = split_aux(sl.slot, ctx->device);
        mi_device_guard g(a->ctx.device);
        MI_CHECK(hipStreamWaitEvent(a->ctx.stream, ctx->split_ready, 0));
        const size_t xbytes = rm.xkind >= 0 ? act_bytes(rm.xkind, K, ncols) : (size_t) K * ncols * sizeof(float);
        const size_t ybytes = (size_t) rm.ld * ncols * sizeof(float);
        scratch_reserve(&a->ctx, xbytes + ybytes + 4 * kBufferAlign);  // stream-ordered reuse: earlier users ran on the same stream
        a->ctx.scratch_used = 0;
        a->ctx.act_cache.clear();
        void * xl = scratch_take(&a->ctx, xbytes);
        float * yl = (float *) scratch_take(&a->ctx, ybytes);
        if (a->ctx.device == ctx->device) {
            MI_CHECK(hipMemcpyAsync(xl, rm.xa, xbytes, hipMemcpyDeviceToDevice, a->ctx.stream));
        } else {
            MI_CHECK(hipMemcpyPeerAsync(xl, a->ctx.device, rm.xa, ctx->device, xbytes, a->ctx.stream));
        }
        ggml_tensor x1 = *src1;  // src1 as the slot sees it (the f32 columns or their conversion)
        x1.data = xl;
        x1.view_src = nullptr;
        x1.view_offs = 0;
        if (rm.xkind >= 0) {
            // the slot's mul_mat finds its activations already converted
            mi_act_cache_entry e;
            e.data = xl;
            e.nbytes = ggml_nbytes(src1);
            e.kind = rm.xkind;
            memcpy(e.ne, x1.ne, sizeof(e.ne));
            memcpy(e.nb, x1.nb, sizeof(e.nb));
            e.dev = xl;
            a->ctx.act_cache.push_back(e);
        }
        a->ctx.last_launches = 0;
        mul_mat_run(&a->ctx, src0, sl.ptr, rows, &x1, yl, (size_t) rm.ld * sizeof(float), (size_t) rm.ld * ncols * sizeof(float),
                    (size_t) rm.ld * ncols * sizeof(float));
        ctx->last_launches += a->ctx.last_launches;
        MI_CHECK(hipMemcpy2DAsync(out, dst->nb[1], yl, (size_t) rm.ld * sizeof(float), (size_t) rows * sizeof(float), (size_t) ncols,
                                  hipMemcpyDeviceToDevice, a->ctx.stream));
        MI_CHECK(hipEventRecord(a->done, a->ctx.stream));
        waits.push_back(a);
    }
    mi_device_guard g(ctx->device);
    for (mi_split_aux * a : waits) MI_CHECK(hipStreamWaitEvent(ctx->stream, a->done, 0));
}

// ---------------------------------------------------------------------------------------------
// companion ops (GPT-2 / LLaMA-shaped graphs)
// ---------------------------------------------------------------------------------------------

static uint16_t host_f2h(float f) {  // round-to-nearest-even, as F16C _cvtss_sh(x, 0)
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u) return (uint16_t) (sign | 0x7e00u | ((ax >> 13) & 0x3ffu));
    if (ax >= 0x477ff000u) return (uint16_t) (sign | 0x7c00u);
    if (ax < 0x38800000u) {  // subnormal half
        const float v = fabsf(f) * 16777216.0f;  // exact scaling by 2^24
        return (uint16_t) (sign | (uint32_t) nearbyintf(v));
    }
    const uint32_t r = ax + 0xfffu + ((ax >> 13) & 1u) - 0x38000000u;
    return (uint16_t) (sign | (r >> 13));
}

static float host_h2f(uint16_t h) {
    const uint32_t sign = (uint32_t) (h & 0x8000u) << 16;
    const uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
    float r;
    if (e == 0) r = ldexpf((float) m, -24);
    else if (e == 31) r = m ? NAN : INFINITY;
    else r = ldexpf((float) (m | 0x400), (int) e - 25);
    uint32_t u;
    memcpy(&u, &r, 4);
    u |= sign;
    memcpy(&r, &u, 4);
    return r;
}

// the reference's fp16 lookup tables (src/ggml.c:2884-2898), same formulas and libm
static const float kGeluCoefA = 0.044715f;
static const float kSqrt2OverPi = 0.79788456080286535587989211986876f;
// ggml_gelu_f32 as the reference's gcc -O3 -mfma build evaluates it (read off its ggml_init):
// (0.5f*x) * (1 + tanhf((SQRT_2_OVER_PI*x) * fmaf(GELU_COEF_A*x, x, 1))) -- one contraction
static float gelu_ref(float x) {
    const float inner = fmaf(kGeluCoefA * x, x, 1.0f);
    const float arg = (kSqrt2OverPi * x) * inner;
    return (0.5f * x) * (1.0f + tanhf(arg));
}
static float silu_ref(float x) { return x / (1.0f + expf(-x)); }

static const uint16_t * op_tables(mi_backend_ctx * ctx) {
    if (!ctx->tables) {
        std::vector<uint16_t> h(3 * 65536);
        for (int i = 0; i < 65536; i++) {
            const float f = host_h2f((uint16_t) i);
            h[i] = host_f2h(expf(f));
            h[65536 + i] = host_f2h(gelu_ref(f));
            h[2 * 65536 + i] = host_f2h(silu_ref(f));
        }
        MI_CHECK(hipMalloc(&ctx->tables, h.size() * sizeof(uint16_t)));
        MI_CHECK(hipMemcpy(ctx->tables, h.data(), h.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    }
    return ctx->tables;
}

static mi_tensor_desc desc(const ggml_tensor * t) {
    mi_tensor_desc d;
    d.data = t ? (char *) t->data : nullptr;
    d.type = t ? (int) t->type : 0;
    for (int i = 0; i < 4; i++) {
        d.ne[i] = t ? t->ne[i] : 1;
        d.nb[i] = t ? t->nb[i] : 0;
    }
    return d;
}

static float op_param_f(const ggml_tensor * t, int i) {
    float v;
    memcpy(&v, (const int32_t *) t->op_params + i, sizeof(float));
    return v;
}

// ggml_rope_yarn_corr_dims (src/ggml.c:13746-13773)
static void rope_corr_dims(int n_dims, int n_orig_ctx, float freq_base, float beta_fast, float beta_slow, float dims[2]) {
    auto corr_dim = [&](float n_rot) {
        return n_dims * logf(n_orig_ctx / (n_rot * 2 * (float) M_PI)) / (2 * logf(freq_base));
    };
    const float start = floorf(corr_dim(beta_fast));
    const float end = ceilf(corr_dim(beta_slow));
    dims[0] = std::max(0.0f, start);
    dims[1] = std::min((float) (n_dims - 1), end);
}

// ---- RoPE {cos, sin} tables, built on the host exactly as the reference CPU computes them ----
// ggml_rope_cache_init / the NeoX loop of ggml_compute_forward_rope_f32 (src/ggml.c:13719-13948)
// and rope_yarn (:13680-13700) over positions 0 .. P-1, with the host libm's sincosf (the function
// the reference build calls) and the contractions its -mfma build makes (read off the object:
// theta = fma(theta_interp, 1 - ramp_mix, theta_extrap * ramp_mix); mscale *= fma(logf(1 /
// freq_scale), 0.1f, 1.0f)). Device positions outside [0, P) fall back to the kernel's own math.
#pragma clang fp contract(off)
static void rope_yarn_host(float theta_extrap, float freq_scale, const float corr[2], int64_t i0, float ext_factor, float mscale,
                           float * c, float * s) {
    const float theta_interp = freq_scale * theta_extrap;
    float theta = theta_interp;
    if (ext_factor != 0.0f) {
        const float y = ((float) (i0 / 2) - corr[0]) / std::max(0.001f, corr[1] - corr[0]);
        const float ramp_mix = (1.0f - std::min(1.0f, std::max(0.0f, y))) * ext_factor;
        theta = std::fma(theta_interp, 1.0f - ramp_mix, theta_extrap * ramp_mix);
        mscale *= std::fma(logf(1.0f / freq_scale), 0.1f, 1.0f);
    }
    float sv, cv;
    sincosf(theta, &sv, &cv);
    *c = cv * mscale;
    *s = sv * mscale;
}

static const mi_backend_ctx::rope_table * rope_table_find(mi_backend_ctx * ctx, int n_dims, int ne0, int mode, float fb, float fs,
                                                          float ef, float af, const float corr[2]) {
    for (const auto & t : ctx->rope_tables) {
        if (t.n_dims == n_dims && t.ne0 == ne0 && t.mode == mode && t.freq_base == fb && t.freq_scale == fs && t.ext_factor == ef &&
            t.attn_factor == af && t.corr0 == corr[0] && t.corr1 == corr[1]) return &t;
    }
    return nullptr;
}

// builds the table of a ROPE node if missing (synchronous upload: never while capturing)
static void rope_table_ensure(mi_backend_ctx * ctx, const ggml_tensor * node) {
    const int32_t * pp = (const int32_t *) node->op_params;
    const int n_dims = pp[1], mode = pp[2], n_ctx = pp[3], n_orig_ctx = pp[4];
    const float fb = op_param_f(node, 5), fs = op_param_f(node, 6), ef = op_param_f(node, 7), af = op_param_f(node, 8);
    float corr[2];
    rope_corr_dims(n_dims, n_orig_ctx, fb, op_param_f(node, 9), op_param_f(node, 10), corr);
    const int ne0 = (int) node->src[0]->ne[0];
    if ((mode != 0 && mode != 2) || n_dims <= 0 || n_dims % 2 || rope_table_find(ctx, n_dims, ne0, mode, fb, fs, ef, af, corr)) return;
    const int P = std::min(std::max({n_ctx, n_orig_ctx, 4096}), 1 << 16);
    const int pairs = mode == 0 ? ne0 / 2 : n_dims / 2;
    std::vector<float> h((size_t) P * pairs * 2);
    const float theta_scale = powf(fb, -2.0f / n_dims);
    const float inv_ndims = -1.f / n_dims;
    for (int p = 0; p < P; p++) {
        float * row = h.data() + (size_t) p * pairs * 2;
        if (mode == 0) {
            float theta = (float) p;
            for (int k = 0; k < pairs; k++) {
                rope_yarn_host(theta, fs, corr, 2 * k, ef, af, &row[2 * k], &row[2 * k + 1]);
                theta *= theta_scale;
            }
        } else {
            float theta = (float) p;
            theta *= fs;
            for (int k = 0; k < pairs; k++) {
                const float cur_rot = inv_ndims * (float) (2 * k) - 0.0f;
                rope_yarn_host(theta, fs, corr, (int64_t) cur_rot, ef, af, &row[2 * k], &row[2 * k + 1]);
                theta *= theta_scale;
            }
        }
    }
    mi_backend_ctx::rope_table t{n_dims, ne0, mode, P, fb, fs, ef, af, corr[0], corr[1], nullptr};
    mi_device_guard g(ctx->device);
    MI_CHECK(hipMalloc(&t.dev, h.size() * sizeof(float)));
    MI_CHECK(hipMemcpy(t.dev, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    ctx->rope_tables.push_back(t);
}
#pragma clang fp contract(on)

// builds the RoPE tables a graph needs (before any capture: the uploads are synchronous)
static void rope_tables_prepare(mi_backend_ctx * ctx, const ggml_cgraph * cgraph) {
    for (int i = 0; i < cgraph->n_nodes; i++) {
        const ggml_tensor * n = cgraph->nodes[i];
        if (n->op == GGML_OP_ROPE && n->src[0] && n->src[0]->type == GGML_TYPE_F32) rope_table_ensure(ctx, n);
        if (n->op == GGML_OP_MUL_MAT) (void) planes_of(ctx, n->src[0], n->src[1]);
        // (decode GEMVs of a tree-order graph: the Q4_0 weights' aligned copies)
        if (n->op == GGML_OP_MUL_MAT && n->src[1]->ne[1] == 1 && mi_mmv_order() == 0) (void) q40r_of(ctx, n->src[0]);
    }
}

static void op_companion(mi_backend_ctx * ctx, ggml_tensor * node) {
    const ggml_tensor * a = node->src[0];
    const ggml_tensor * b = node->src[1];
    hipStream_t st = ctx->stream;
    switch (node->op) {
        case GGML_OP_ADD: mi_op_binary(desc(node), desc(a), desc(b), MI_OP_ADD, st); break;
        case GGML_OP_SUB: mi_op_binary(desc(node), desc(a), desc(b), MI_OP_SUB, st); break;
        case GGML_OP_MUL: mi_op_binary(desc(node), desc(a), desc(b), MI_OP_MUL, st); break;
        case GGML_OP_DIV: mi_op_binary(desc(node), desc(a), desc(b), MI_OP_DIV, st); break;
        case GGML_OP_SCALE: mi_op_unary(desc(node), desc(a), MI_OP_SCALE, op_param_f(node, 0), nullptr, st); break;
        case GGML_OP_NORM: mi_op_norm(desc(node), desc(a), op_param_f(node, 0), false, nullptr, nullptr, st); break;
        case GGML_OP_RMS_NORM: mi_op_norm(desc(node), desc(a), op_param_f(node, 0), true, nullptr, nullptr, st); break;
        case GGML_OP_SOFT_MAX: mi_op_soft_max(desc(node), desc(a), desc(b), op_param_f(node, 0), op_tables(ctx), 1.0f, -1, st); break;
        case GGML_OP_DIAG_MASK_INF:
            mi_op_diag_mask(desc(node), desc(a), ((const int32_t *) node->op_params)[0], -INFINITY, st);
            break;
        case GGML_OP_DIAG_MASK_ZERO:
            mi_op_diag_mask(desc(node), desc(a), ((const int32_t *) node->op_params)[0], 0.0f, st);
            break;
        case GGML_OP_UNARY: {
            const ggml_unary_op u = ggml_get_unary_op(node);
            MI_ASSERT(u == GGML_UNARY_OP_GELU || u == GGML_UNARY_OP_SILU);
            const uint16_t * t = op_tables(ctx) + (u == GGML_UNARY_OP_GELU ? 65536 : 2 * 65536);
            mi_op_unary(desc(node), desc(a), u == GGML_UNARY_OP_GELU ? MI_OP_GELU : MI_OP_SILU, 0.0f, t, st);
            break;
        }
        case GGML_OP_GET_ROWS: mi_op_get_rows(desc(node), desc(a), desc(b), st); break;
        case GGML_OP_CPY:
        case GGML_OP_DUP:
        case GGML_OP_CONT:
            MI_ASSERT(ggml_nelements(node) == ggml_nelements(a));
            if (node->type == GGML_TYPE_Q8_K || node->type == GGML_TYPE_Q8_0) {
                mi_quantize_rows_q8(src_cols(a), a->ne[0], node->type == GGML_TYPE_Q8_K, src_cols(node), st);
                break;
            }
            mi_op_cpy(desc(node), desc(a), st);
            break;
        case GGML_OP_ROPE: {
            const int32_t * pp = (const int32_t *) node->op_params;
            const int n_dims = pp[1], mode = pp[2], n_orig_ctx = pp[4];
            const float freq_base = op_param_f(node, 5), freq_scale = op_param_f(node, 6), ext_factor = op_param_f(node, 7);
            const float attn_factor = op_param_f(node, 8), beta_fast = op_param_f(node, 9), beta_slow = op_param_f(node, 10);
            MI_ASSERT(n_dims <= a->ne[0] && n_dims % 2 == 0);
            float corr[2];
            rope_corr_dims(n_dims, n_orig_ctx, freq_base, beta_fast, beta_slow, corr);
            const auto * tab = rope_table_find(ctx, n_dims, (int) a->ne[0], mode, freq_base, freq_scale, ext_factor, attn_factor, corr);
            mi_op_rope(desc(node), desc(a), (const int32_t *) b->data, n_dims, mode, freq_base, freq_scale, ext_factor,
                       attn_factor, corr[0], corr[1], tab ? tab->dev : nullptr, tab ? tab->P : 0, st);
            break;
        }
        default:
            fprintf(stderr, "%s: error: op not supported %s (%s)\\n", __func__, node->name, ggml_op_desc(node));
            MI_ASSERT(!"unsupported op");
    }
    ctx->last_launches++;
}

// ---------------------------------------------------------------------------------------------
// graph execution
// ---------------------------------------------------------------------------------------------

static bool is_noop(const ggml_tensor * node) {
    return ggml_is_empty(node) || node->op == GGML_OP_NONE || node->op == GGML_OP_RESHAPE || node->op == GGML_OP_VIEW ||
           node->op == GGML_OP_PERMUTE || node->op == GGML_OP_TRANSPOSE;
}

static size_t graph_scratch_bytes(const ggml_cgraph * cgraph) {
    size_t total = 0;
    for (int i = 0; i < cgraph->n_nodes; i++) {
        const ggml_tensor * n = cgraph->nodes[i];
        if (n->op != GGML_OP_MUL_MAT) continue;
        if (n->src[0]->type == GGML_TYPE_F16 && n->src[1]->ne[1] == 1) {
            // a possible attention output projection (whatever op merged the heads -- ggml_cont as
            // main-backend.cpp:603 or ggml_cpy as main-ctx.cpp:566): room for its per-head partial
            // sums (try_fuse_attn_proj; head dim >= 64, so at most K / 64 heads)
            total += ((size_t) (n->src[0]->ne[0] / 64) * n->src[0]->ne[1] * sizeof(float) + kBufferAlign - 1) & ~(kBufferAlign - 1);
        }
        const int kind = act_kind(n->src[0]->type);
        if (kind < 0) continue;
        const ggml_tensor * b = n->src[1];
        const int64_t ncols = b->ne[1] * b->ne[2] * b->ne[3];
        // q8 blocks and/or their f16 expansion (batched) -- both counted, the choice is made at run time
        total += (act_bytes(kind, b->ne[0], ncols) + kBufferAlign - 1) & ~(kBufferAlign - 1);
        if (ncols > 8) {
            const size_t big = std::max(act_bytes(kind + 3, b->ne[0], ncols),
                                        kind == 1 ? act_bytes(8, b->ne[0], ncols) : kind == 0 ? act_bytes(9, b->ne[0], ncols) : 0);
            total += (big + kBufferAlign - 1) & ~(kBufferAlign - 1);
        }
    }
    return total;
}

// ---- decode-regime fusion: quantize-in-kernel GEMV, independent mul_mats in one launch ----

static bool overlaps(const ggml_tensor * a, const ggml_tensor * b) {
    const char * a0 = (const char *) a->data;
    const char * b0 = (const char *) b->data;
    return a0 < b0 + ggml_nbytes(b) && b0 < a0 + ggml_nbytes(a);
}

static bool fused_mv_eligible(const ggml_tensor * n) {
    if (n->op != GGML_OP_MUL_MAT || is_split_tensor(n->src[0])) return false;
    const ggml_tensor * a = n->src[0];
    const ggml_tensor * b = n->src[1];
    if (b->type != GGML_TYPE_F32 || !mi_mmv_fused_supported(a->type, a->ne[0], b->ne[1])) return false;
    if (a->ne[2] != 1 || a->ne[3] != 1 || b->ne[2] != 1 || b->ne[3] != 1) return false;
    if (a->nb[0] != ggml_type_size(a->type) || b->nb[0] != sizeof(float) || n->nb[0] != sizeof(float)) return false;
    if (((uintptr_t) a->data | a->nb[1]) % 16 != 0 || ((uintptr_t) b->data | b->nb[1]) % 16 != 0) return false;
    return true;
}

static bool same_group_shape(const ggml_tensor * x, const ggml_tensor * y) {
    const ggml_tensor * xa = x->src[0];
    const ggml_tensor * ya = y->src[0];
    return xa->type == ya->type && xa->ne[0] == ya->ne[0] && xa->ne[1] == ya->ne[1] && xa->nb[1] == ya->nb[1] &&
           x->src[1]->ne[1] == y->src[1]->ne[1] && x->src[1]->nb[1] == y->src[1]->nb[1] && x->nb[1] == y->nb[1];
}

// Launches nodes[i] and following independent same-shape mul_mats as one fused kernel.
// Returns the index of the last node consumed.
static int run_fused_group(mi_backend_ctx * ctx, ggml_cgraph * cgraph, int i) {
    static_assert(sizeof(mi_mmv_group) < 4096, "kernel argument block");
    ggml_tensor * first = cgraph->nodes[i];
    std::vector<ggml_tensor *> members = {first};
    int last = i;
    std::vector<int> at = {i};
    // scan up to 4 launches' worth, then split the run evenly (36 -> 18 + 18, not 32 + 4: a
    // launch of few members is all prologue)
    for (int j = i + 1; j < cgraph->n_nodes && (int) members.size() < 4 * kMiMaxMembers; j++) {
        ggml_tensor * n = cgraph->nodes[j];
        if (is_noop(n)) continue;
        if (!fused_mv_eligible(n) || !same_group_shape(first, n)) break;
        bool independent = true;
        for (ggml_tensor * m : members) {
            if (overlaps(n->src[1], m) || overlaps(n->src[0], m) || overlaps(n, m->src[0]) || overlaps(n, m->src[1]) || overlaps(n, m)) {
                independent = false;
                break;
            }
        }
        if (!independent) break;
        members.push_back(n);
        at.push_back(j);
    }
    {
        const int runs = ((int) members.size() + kMiMaxMembers - 1) / kMiMaxMembers;
        const int take = ((int) members.size() + runs - 1) / runs;
        members.resize(take);
        last = at[take - 1];
    }
    mi_mmv_group g;
    g.type = first->src[0]->type;
    g.n = (int) members.size();
    g.ncols = (int) first->src[1]->ne[1];
    g.K = first->src[0]->ne[0];
    g.N = first->src[0]->ne[1];
    g.nb01 = first->src[0]->nb[1];
    g.xcol = first->src[1]->nb[1];
    g.ycol = first->nb[1];
    const ggml_tensor * wts[kMiMaxMembers];
    for (int m = 0; m < g.n; m++) {
        g.m[m].W = members[m]->src[0]->data;
        g.m[m].X = (const char *) members[m]->src[1]->data;
        g.m[m].dst = (float *) members[m]->data;
        wts[m] = members[m]->src[0];
    }
    q40r_apply(ctx, g, wts);
    mi_mul_mat_q_fused(g, ctx->stream);
    ctx->last_launches++;
    for (ggml_tensor * m : members) invalidate_activations(ctx, m);
    return last;
}

// ---- node fusion (same results: each fused step is rounded exactly as its own node would be) ----
//
// Patterns of the GPT-2 / LLaMA graphs (examples/gpt-2/main-backend.cpp:442-717):
//   NORM|RMS_NORM -> MUL(., g[E]) -> ADD(., b[E])             one k_norm launch
//   MUL_MAT(F16, few cols) -> ADD(., bias[N]) [-> ADD(., resid) | -> GELU]   one GEMV launch
//   SCALE -> DIAG_MASK_INF -> SOFT_MAX                          one k_soft_max launch
// An intermediate may be skipped only if the next node is its sole consumer and it is not a graph
// output; views of a tensor count as consumers of it.

// A graph handed over by ggml_backend_sched is a view of one split (ggml_graph_view,
// ggml-backend.c:1549; size == 0, no hash table): a tensor may also be read by a later split that
// this backend never sees, so no use count taken over the view proves an intermediate private and
// every node output is stored (`partial`).
struct mi_uses {
    std::unordered_map<const ggml_tensor *, int> n;
    bool partial = false;
    int of(const ggml_tensor * t) const {
        if (partial) return 1 << 20;
        auto it = n.find(t);
        return it == n.end() ? 0 : it->second;
    }
};

// uses(X) = edges (consumer node, src == X) + views of X; a view V of X that is itself consumed
// counts once for X (as the view) and once per consumer for V
static void count_uses(const ggml_cgraph * g, mi_uses & u) {
    u.n.clear();
    u.partial = g->size == 0 && g->visited_hash_table.size == 0;
    for (int i = 0; i < g->n_nodes; i++) {
        const ggml_tensor * t = g->nodes[i];
        for (int s = 0; s < GGML_MAX_SRC; s++) {
            if (t->src[s]) u.n[t->src[s]]++;
        }
        if (t->view_src) u.n[t->view_src]++;
    }
}

// nodes already executed inside another node's fused kernel (set per graph by plan_attention)
static thread_local const std::vector<uint8_t> * tl_absorbed = nullptr;

static bool absorbed(int j) { return tl_absorbed && j < (int) tl_absorbed->size() && (*tl_absorbed)[j]; }

static int next_node(const ggml_cgraph * g, int i) {
    for (int j = i + 1; j < g->n_nodes; j++) {
        if (!is_noop(g->nodes[j]) && !absorbed(j)) return j;
    }
    return -1;
}

static bool private_intermediate(const ggml_tensor * t, const mi_uses & u) {
    return u.of(t) == 1 && !(t->flags & GGML_TENSOR_FLAG_OUTPUT);
}

// a fused kernel may write `out` over an input only when both are the same elements (each lane
// reads its element before writing it); any other overlap would race across workgroups
static bool safe_alias(const ggml_tensor * out, const ggml_tensor * in) {
    if (!in || !overlaps(out, in)) return true;
    return out->data == in->data && ggml_are_same_shape(out, in) && memcmp(out->nb, in->nb, sizeof(out->nb)) == 0;
}

static bool is_vec_f32(const ggml_tensor * t, int64_t n) {
    return t && t->type == GGML_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1 &&
           t->nb[0] == sizeof(float);
}

// ADD(x, other) or ADD(other, x): returns `other`, or null
static const ggml_tensor * add_operand(const ggml_tensor * add, const ggml_tensor * x) {
    if (add->op != GGML_OP_ADD) return nullptr;
    if (add->src[0] == x) return add->src[1];
    if (add->src[1] == x) return add->src[0];
    return nullptr;
}

static int try_fuse_softmax(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u) {
    ggml_tensor * sc = g->nodes[i];
    const int j = next_node(g, i);
    if (j < 0 || !private_intermediate(sc, u)) return -1;
    ggml_tensor * dm = g->nodes[j];
    if (dm->op != GGML_OP_DIAG_MASK_INF || dm->src[0] != sc) return -1;
    const int k = next_node(g, j);
    if (k < 0 || !private_intermediate(dm, u)) return -1;
    ggml_tensor * sm = g->nodes[k];
    if (sm->op != GGML_OP_SOFT_MAX || sm->src[0] != dm || sm->src[1] != nullptr || op_param_f(sm, 1) != 0.0f) return -1;
    const ggml_tensor * a = sc->src[0];
    if (a->type != GGML_TYPE_F32 || !ggml_is_contiguous(a) || !ggml_are_same_shape(a, sm)) return -1;
    if (!safe_alias(sm, a)) return -1;
    const int n_past = ((const int32_t *) dm->op_params)[0];
    mi_op_soft_max(desc(sm), desc(a), desc(nullptr), op_param_f(sm, 0), op_tables(ctx), op_param_f(sc, 0), n_past, ctx->stream);
    ctx->last_launches++;
    return k;
}

// The graph's nodes right after mul_mat g->nodes[i] that a GEMV epilogue absorbs: ADD(bias[N]),
// then ADD(resid) or GELU, then up to two CPY nodes of row views of the result (GPT-2's K/V cache
// writes, main-backend.cpp:556-561). Fills `e` (mi_f16_epilogue or mi_mmv_group::epilogue: same
// fields), *out_p = the node holding the final value; returns the last absorbed node, or -1.
template <class E>
static int collect_epilogue(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u, const ggml_tensor * w,
                            const ggml_tensor * x, E & e, ggml_tensor ** out_p, const ggml_tensor ** bias_p,
                            const ggml_tensor ** res_p) {
    ggml_tensor * mm = g->nodes[i];
    const int64_t N = w->ne[1];
    const ggml_tensor * bias_t = nullptr, * res_t = nullptr;
    ggml_tensor * out = mm;
    int last = i;
    int j = next_node(g, i);
    if (j >= 0 && private_intermediate(mm, u)) {
        ggml_tensor * add = g->nodes[j];
        const ggml_tensor * bias = add_operand(add, mm);
        if (bias && is_vec_f32(bias, N) && ggml_are_same_shape(add, mm) && add->nb[0] == sizeof(float)) {
            e.bias = (const float *) bias->data;
            bias_t = bias;
            out = add;
            last = j;
            const int k = next_node(g, j);
            if (k >= 0 && private_intermediate(add, u)) {
                ggml_tensor * n2 = g->nodes[k];
                const ggml_tensor * res = add_operand(n2, add);
                if (res && res != add && res->type == GGML_TYPE_F32 && ggml_are_same_shape(res, add) && res->nb[0] == sizeof(float) &&
                    n2->nb[0] == sizeof(float) && ggml_are_same_shape(n2, add)) {
                    e.resid = (const char *) res->data;
                    e.resid_nb1 = res->nb[1];
                    res_t = res;
                    out = n2;
                    last = k;
                } else if (n2->op == GGML_OP_UNARY && ggml_get_unary_op(n2) == GGML_UNARY_OP_GELU && n2->src[0] == add &&
                           n2->type == GGML_TYPE_F32 && n2->nb[0] == sizeof(float) && ggml_are_same_shape(n2, add)) {
                    e.gelu_table = op_tables(ctx) + 65536;
                    out = n2;
                    last = k;
                }
            }
        }
    }
    if (out->type != GGML_TYPE_F32 || out->nb[0] != sizeof(float)) return -1;
    // the graph's CPY nodes of row views of `out` that follow right away (GPT-2 writes the K and V
    // rows of c_attn's output into its caches, main-backend.cpp:556-561): stored by the epilogue
    int ncopy = 0;
    for (int j = next_node(g, last); j >= 0 && ncopy < 2; j = next_node(g, j)) {
        ggml_tensor * cp = g->nodes[j];
        if (cp->op != GGML_OP_CPY) break;
        const ggml_tensor * v = cp->src[0];
        // a row view of `out`, or `out` itself (e.g. the logits copied into a host staging tensor)
        if ((v->view_src != out && v != out) || v->type != GGML_TYPE_F32 || v->nb[0] != sizeof(float) || v->view_offs % sizeof(float)) break;
        if (v->ne[2] != 1 || v->ne[3] != 1 || v->ne[1] != out->ne[1] || (v->ne[1] > 1 && v->nb[1] != out->nb[1])) break;
        const int64_t r0 = v == out ? 0 : (int64_t) (v->view_offs / sizeof(float));
        if (r0 + v->ne[0] > N) break;
        if (cp->type != GGML_TYPE_F32 || !ggml_is_contiguous(cp) || ggml_nelements(cp) != ggml_nelements(v)) break;
        if (overlaps(cp, w) || overlaps(cp, x) || overlaps(cp, out) || (bias_t && overlaps(cp, bias_t)) || (res_t && overlaps(cp, res_t))) break;
        if (ncopy == 1 && overlaps(cp, g->nodes[last])) break;
        e.copy[ncopy].row0 = r0;
        e.copy[ncopy].row1 = r0 + v->ne[0];
        e.copy[ncopy].ptr = (char *) cp->data;
        e.copy[ncopy].col_stride = (size_t) v->ne[0] * sizeof(float);
        ncopy++;
        last = j;
    }
    *out_p = out;
    *bias_p = bias_t;
    *res_p = res_t;
    return last;
}

// stores a value left as partial sums (ctx->pend) before anything else reads it
static void flush_pending(mi_backend_ctx * ctx) {
    if (!ctx->pend.out) return;
    mi_sum_parts((float *) ctx->pend.out->data, ctx->pend.parts, ctx->pend.nparts, ctx->pend.n, ctx->stream);
    ctx->last_launches++;
    ctx->pend = {};
}

// pro / pro_x: the src1 of this mul_mat is the output of a norm chain (norm -> mul g -> add b)
// that the kernel computes itself from pro_x (pro->parts: pro_x is the pending partial-sum value)
static int try_fuse_f16_gemv(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u,
                             const mi_norm_prologue * pro = nullptr, const ggml_tensor * pro_x = nullptr) {
    ggml_tensor * mm = g->nodes[i];
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = pro_x ? pro_x : mm->src[1];
    if (is_split_tensor(w)) return -1;
    if (w->type != GGML_TYPE_F16 || x->type != GGML_TYPE_F32) return -1;
    if (w->ne[2] != 1 || w->ne[3] != 1 || x->ne[2] != 1 || x->ne[3] != 1 || x->ne[1] > 8) return -1;
    if (w->nb[0] != 2 || w->nb[1] % 16 != 0 || (uintptr_t) w->data % 16 != 0 || x->nb[0] != sizeof(float)) return -1;
    if (!mi_mul_mat_f16_fused_supported(w->ne[0], x->ne[1])) return -1;
    const int64_t N = w->ne[1];
    mi_f16_epilogue e;
    const ggml_tensor * bias_t = nullptr, * res_t = nullptr;
    ggml_tensor * out = mm;
    const int last = collect_epilogue(ctx, g, i, u, w, x, e, &out, &bias_t, &res_t);
    if (last < 0) return -1;
    // every workgroup reads all of X and W; resid/bias are read per element. When the graph
    // allocator has placed `out` over X (X's last reader is this mul_mat), X is first converted
    // into the backend's scratch so no workgroup can see it overwritten.
    if (overlaps(out, w)) return -1;
    if (bias_t && overlaps(out, bias_t)) return -1;
    if (res_t && !safe_alias(out, res_t)) return -1;
    const uint16_t * xh = nullptr;
    if (pro && (overlaps(out, x) || (x->nb[1] % sizeof(float)) != 0)) return -1;
    if (pro && pro->parts) {
        // only the tree-order kernel sums partials
        if (mi_mmv_order() != 0 || !mi_mul_mat_f16_fast_supported(w->ne[0], x->ne[1], src_cols(x), nullptr, *pro)) return -1;
        // x (stored by the first workgroup) must not be read by the others through the epilogue
        if ((bias_t && overlaps(x, bias_t)) || (res_t && overlaps(x, res_t))) return -1;
        mi_mul_mat_f16_fast(w->data, w->nb[1], w->ne[0], N, src_cols(x), nullptr, x->ne[1], (float *) out->data, out->nb[1], e, *pro,
                            ctx->stream);
        ctx->last_launches++;
        return last;
    }
    if (overlaps(out, x)) {
        uint16_t * tmp = (uint16_t *) scratch_take(ctx, act_bytes(2, w->ne[0], x->ne[1]));
        mi_convert_f16(src_cols(x), w->ne[0], tmp, ctx->stream);
        ctx->last_launches++;
        xh = tmp;
    }
    const mi_norm_prologue none;
    mi_mul_mat_f16_fused(w->data, w->nb[1], w->ne[0], N, src_cols(x), xh, x->ne[1], (float *) out->data, out->nb[1], e,
                         pro ? *pro : none, ctx->stream);
    ctx->last_launches++;
    return last;
}

// Q4_0/Q8_0/Q4_K/Q5_K decode GEMV with the graph's bias / residual / GELU and K/V row copies in
// the streaming kernel's store (a one-member k_mmv_stream group); -1 if nothing follows that it
// can absorb (then the node goes through the grouped path).
static int fuse_mask_q() {
    static const int m = getenv("GGML_MI355X_NO_FUSED_MMV") ? 0 : (getenv("GGML_MI355X_FUSE_MASK") ? atoi(getenv("GGML_MI355X_FUSE_MASK")) : 0xff);
    return m;
}

// pro / pro_x: as for try_fuse_f16_gemv (the norm chain producing src1, computed in the kernel)
static int try_fuse_q_gemv(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u,
                           const mi_norm_prologue * pro = nullptr, const ggml_tensor * pro_x = nullptr) {
    ggml_tensor * mm = g->nodes[i];
    if (!fused_mv_eligible(mm)) return -1;
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = pro_x ? pro_x : mm->src[1];
    if (pro && (w->ne[0] > kMiMmvProMaxK || x->nb[1] % sizeof(float) != 0 || x->ne[1] != mm->src[1]->ne[1])) return -1;
    mi_mmv_group grp;
    if (pro) {
        grp.pro.g = pro->g;
        grp.pro.b = pro->b;
        grp.pro.eps = pro->eps;
        grp.pro.mode = pro->mode;
    }
    const ggml_tensor * bias_t = nullptr, * res_t = nullptr;
    ggml_tensor * out = mm;
    const int last = collect_epilogue(ctx, g, i, u, w, x, grp.epi, &out, &bias_t, &res_t);
    if (last < 0 || (last == i && !pro)) return -1;
    // every workgroup quantizes all of X in its prologue and reads resid/bias per element: the
    // output may not overlap W, X or the bias, and may alias the residual only element for element
    if (overlaps(out, w) || overlaps(out, x) || (bias_t && overlaps(out, bias_t)) || !safe_alias(out, res_t)) return -1;
    if (out->nb[1] % sizeof(float) != 0) return -1;
    grp.type = w->type;
    grp.n = 1;
    grp.ncols = (int) x->ne[1];
    grp.K = w->ne[0];
    grp.N = w->ne[1];
    grp.nb01 = w->nb[1];
    grp.xcol = x->nb[1];
    grp.ycol = out->nb[1];
    grp.m[0].W = w->data;
    grp.m[0].X = (const char *) x->data;
    grp.m[0].dst = (float *) out->data;
    q40r_apply(ctx, grp, &w);
    mi_mul_mat_q_fused(grp, ctx->stream);
    ctx->last_launches++;
    return last;
}

static int try_fuse_norm(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u) {
    ggml_tensor * norm = g->nodes[i];
    const int64_t E = norm->ne[0];
    const int j = next_node(g, i);
    if (j < 0 || !private_intermediate(norm, u)) return -1;
    ggml_tensor * mul = g->nodes[j];
    if (mul->op != GGML_OP_MUL || mul->src[0] != norm || !is_vec_f32(mul->src[1], E) || !ggml_are_same_shape(mul, norm)) return -1;
    ggml_tensor * out = mul;
    const float * bias = nullptr;
    int last = j;
    const int k = next_node(g, j);
    if (k >= 0 && private_intermediate(mul, u)) {
        ggml_tensor * add = g->nodes[k];
        if (add->op == GGML_OP_ADD && add->src[0] == mul && is_vec_f32(add->src[1], E) && ggml_are_same_shape(add, mul)) {
            out = add;
            bias = (const float *) add->src[1]->data;
            last = k;
        }
    }
    if (out->type != GGML_TYPE_F32 || out->nb[0] != sizeof(float)) return -1;
    // norm chain feeding an F16 GEMV as its only consumer: one kernel for all of it
    const int m = next_node(g, last);
    if (m >= 0 && private_intermediate(out, u) && g->nodes[m]->op == GGML_OP_MUL_MAT && g->nodes[m]->src[1] == out &&
        norm->src[0]->type == GGML_TYPE_F32 && norm->src[0]->nb[0] == sizeof(float) && ggml_are_same_shape(norm->src[0], out)) {
        mi_norm_prologue pro;
        pro.g = (const float *) mul->src[1]->data;
        pro.b = bias;
        pro.eps = op_param_f(norm, 0);
        pro.mode = norm->op == GGML_OP_RMS_NORM ? 2 : 1;
        if (ctx->pend.out && ctx->pend.out == norm->src[0] && ctx->pend.n == E) {
            // the norm's input is still partial sums (try_fuse_attn_proj): added in the prologue,
            // stored by the GEMV's first workgroup
            mi_norm_prologue pp = pro;
            pp.parts = ctx->pend.parts;
            pp.nparts = ctx->pend.nparts;
            pp.store = (float *) ctx->pend.out->data;
            const int r = try_fuse_f16_gemv(ctx, g, m, u, &pp, norm->src[0]);
            if (r >= 0) {
                ctx->pend = {};
                return r;
            }
        }
        flush_pending(ctx);
        int r = try_fuse_f16_gemv(ctx, g, m, u, &pro, norm->src[0]);
        if (r < 0 && (fuse_mask_q() & 32)) r = try_fuse_q_gemv(ctx, g, m, u, &pro, norm->src[0]);
        if (r >= 0) return r;
    }
    flush_pending(ctx);
    if (!safe_alias(out, norm->src[0]) || overlaps(out, mul->src[1]) || (bias && overlaps(out, g->nodes[last]->src[1]))) return -1;
    mi_op_norm(desc(out), desc(norm->src[0]), op_param_f(norm, 0), norm->op == GGML_OP_RMS_NORM,
               (const float *) mul->src[1]->data, bias, ctx->stream);
    ctx->last_launches++;
    return last;
}

// ---- attention subgraph (examples/gpt-2/main-backend.cpp:552-608) -----------------------------
//   KQ = mul_mat(K, permute(cont(Q))); scale; diag_mask_inf; soft_max;
//   KQV = mul_mat(cont(permute(V)), soft_max); cont(permute(KQV))
// becomes one k_attn_ordered launch at the KQV node; the conts of Q and V and the KQ chain are
// absorbed (they only feed this block), reading Q, K, V through their source strides.

struct mi_attn_plan {
    int kqv;  // node index of KQV
    const ggml_tensor * merged;  // the absorbed cont node the kernel writes
    mi_attn_desc d;
    // Q is read through its source strides at the KQV node. The graph allocator considers that
    // source dead after the (absorbed) cont of Q, so `merged` may have been placed over it: then
    // Q is copied to the backend's scratch at the cont's position instead.
    int q_copy_at = -1;          // node index of the cont of Q, or -1
    mi_tensor_desc q_src;        // Q through its source strides, [D, N, H]
};

// byte range [lo, hi) touched by a strided [ne0, ne1, ne2] view
static void strided_range(const char * base, const int64_t * ne, const size_t * nb, int n, const char ** lo, const char ** hi) {
    size_t span = 4;
    for (int k = 0; k < n; k++) span += (size_t) (ne[k] - 1) * nb[k];
    *lo = base;
    *hi = base + span;
}

static int node_index(const ggml_cgraph * g, const ggml_tensor * t, const std::unordered_map<const ggml_tensor *, int> & idx) {
    auto it = idx.find(t);
    return it == idx.end() ? -1 : it->second;
}

// virtual strides of a PERMUTE view P of a CONT node C, read through C's source
static bool permute_of_cont_strides(const ggml_tensor * P, size_t nb[3], const char ** base) {
    if (P->op != GGML_OP_PERMUTE || P->ne[3] != 1) return false;
    const ggml_tensor * C = P->src[0];
    if (!C || C->op != GGML_OP_CONT || C->type != GGML_TYPE_F32) return false;
    const ggml_tensor * S = C->src[0];
    if (!S || S->type != GGML_TYPE_F32 || S->nb[0] != sizeof(float)) return false;
    size_t vc[4];
    if (ggml_are_same_shape(S, C)) {
        for (int k = 0; k < 4; k++) vc[k] = S->nb[k];
    } else if (S->ne[2] == 1 && S->ne[3] == 1 && C->ne[3] == 1 && C->ne[0] * C->ne[1] == S->ne[0] && C->ne[2] == S->ne[1]) {
        vc[0] = sizeof(float);
        vc[1] = (size_t) C->ne[0] * sizeof(float);
        vc[2] = S->nb[1];
        vc[3] = 0;
    } else {
        return false;
    }
    const int32_t * ax = (const int32_t *) P->op_params;
    size_t vp[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4; k++) {
        if (ax[k] < 0 || ax[k] > 3) return false;
        vp[ax[k]] = vc[k];
    }
    for (int k = 0; k < 3; k++) nb[k] = vp[k];
    *base = (const char *) S->data;
    return true;
}

static void plan_attention(const ggml_cgraph * g, const mi_uses & u, std::vector<uint8_t> & absorbed_nodes,
                           std::vector<mi_attn_plan> & plans) {
    plans.clear();
    absorbed_nodes.assign(g->n_nodes, 0);
    std::unordered_map<const ggml_tensor *, int> idx;
    for (int i = 0; i < g->n_nodes; i++) idx[g->nodes[i]] = i;
    static const bool dbg = getenv("GGML_MI355X_DEBUG_FUSION") != nullptr;
#define MI_ATTN_SKIP(why) { if (dbg && kqv->src[1] && kqv->src[1]->op == GGML_OP_SOFT_MAX) fprintf(stderr, "attn plan: node %d: %s\n", j, why); continue; }
    for (int j = 0; j < g->n_nodes; j++) {
        const ggml_tensor * kqv = g->nodes[j];
        if (kqv->op != GGML_OP_MUL_MAT || kqv->type != GGML_TYPE_F32) continue;
        const ggml_tensor * vt = kqv->src[0];
        const ggml_tensor * sm = kqv->src[1];
        if (!vt || vt->op != GGML_OP_CONT || vt->type != GGML_TYPE_F32 || u.of(vt) != 1) MI_ATTN_SKIP("check 1")
        const ggml_tensor * vsrc = vt->src[0];
        if (!vsrc || vsrc->type != GGML_TYPE_F32 || !ggml_are_same_shape(vsrc, vt)) MI_ATTN_SKIP("check 2")
        if (sm->op != GGML_OP_SOFT_MAX || sm->src[1] || op_param_f(sm, 1) != 0.0f || u.of(sm) != 1) MI_ATTN_SKIP("check 3")
        // the causal mask: diag_mask_inf(scale(KQ)) (single-sequence graphs), or scale(KQ) + mask with an
        // F32 [n_kv, N] mask tensor broadcast over heads (batched decode across sequences)
        const ggml_tensor * dm = sm->src[0];
        const ggml_tensor * mask = nullptr;
        if (dm->op == GGML_OP_ADD && dm->type == GGML_TYPE_F32 && dm->src[1] && dm->src[1]->type == GGML_TYPE_F32) mask = dm->src[1];
        else if (dm->op != GGML_OP_DIAG_MASK_INF) MI_ATTN_SKIP("check 4")
        if (u.of(dm) != 1) MI_ATTN_SKIP("check 4")
        const ggml_tensor * sc = dm->src[0];
        if (sc->op != GGML_OP_SCALE || u.of(sc) != 1) MI_ATTN_SKIP("check 5")
        const ggml_tensor * kq = sc->src[0];
        if (kq->op != GGML_OP_MUL_MAT || kq->type != GGML_TYPE_F32 || u.of(kq) != 1) MI_ATTN_SKIP("check 6")
        const ggml_tensor * K = kq->src[0];
        const ggml_tensor * Qp = kq->src[1];
        if (K->type != GGML_TYPE_F32 || K->ne[3] != 1 || Qp->type != GGML_TYPE_F32 || u.of(Qp) != 1) MI_ATTN_SKIP("check 7")
        const ggml_tensor * qc = Qp->src[0];
        if (!qc || u.of(qc) != 2) continue;  // the permute view only (src + view_src)
        // KQV consumer: permute -> cont (merged, contiguous)
        int jp = -1, jm = -1;
        for (int k = j + 1; k < g->n_nodes && jm < 0; k++) {
            const ggml_tensor * n = g->nodes[k];
            if (jp < 0 && n->op == GGML_OP_PERMUTE && n->src[0] == kqv) jp = k;
            else if (jp >= 0 && n->op == GGML_OP_CONT && n->src[0] == g->nodes[jp]) jm = k;
        }
        if (jp < 0 || jm < 0 || u.of(kqv) != 2 || u.of(g->nodes[jp]) != 1) MI_ATTN_SKIP("check 8")
        const ggml_tensor * P2 = g->nodes[jp];
        const ggml_tensor * M = g->nodes[jm];
        if (M->type != GGML_TYPE_F32 || !ggml_is_contiguous(M) || P2->ne[3] != 1) MI_ATTN_SKIP("check 9")

        mi_attn_desc d;
        const char * qbase = nullptr;
        if (!permute_of_cont_strides(Qp, d.q_nb, &qbase)) MI_ATTN_SKIP("check 10")
        d.q = qbase;
        d.D = (int) K->ne[0];
        d.n_kv = (int) K->ne[1];
        d.H = (int) Qp->ne[2];
        d.N = (int) Qp->ne[1];
        if (Qp->ne[0] != K->ne[0] || K->ne[2] == 0 || d.H % K->ne[2] != 0) MI_ATTN_SKIP("check 11")
        d.r2 = d.H / (int) K->ne[2];
        if (vt->ne[0] != d.n_kv || vt->ne[1] != d.D || vt->ne[2] != K->ne[2]) MI_ATTN_SKIP("check 12")
        if (!mi_attn_supported(d.D, d.n_kv)) MI_ATTN_SKIP("check 13")
        d.k = (const char *) K->data;
        d.v = (const char *) vsrc->data;
        for (int k = 0; k < 3; k++) {
            d.k_nb[k] = K->nb[k];
            d.v_nb[k] = vsrc->nb[k];
        }
        // KQV (d, t, h) -> merged: linear index in P2's (permuted) order, M contiguous
        const int32_t * ax = (const int32_t *) P2->op_params;
        const size_t c[4] = {1, (size_t) P2->ne[0], (size_t) (P2->ne[0] * P2->ne[1]), (size_t) (P2->ne[0] * P2->ne[1] * P2->ne[2])};
        bool ok = true;
        for (int k = 0; k < 3; k++) {
            if (ax[k] < 0 || ax[k] > 3) ok = false;
            else d.o_nb[k] = c[ax[k]] * sizeof(float);
        }
        if (!ok) MI_ATTN_SKIP("check 14")
        d.out = (char *) M->data;
        if (mask) {
            if (mask->ne[0] != d.n_kv || mask->ne[1] != d.N || mask->ne[2] != 1 || mask->ne[3] != 1 ||
                mask->nb[0] != sizeof(float) || !mask->data || mask == sc) MI_ATTN_SKIP("check 4m")
            d.mask = (const char *) mask->data;
            d.mask_nb1 = mask->nb[1];
            d.n_past = INT32_MAX / 2;  // never: the mask carries the causal structure
        } else {
            d.n_past = ((const int32_t *) dm->op_params)[0];
        }
        d.pre_scale = op_param_f(sc, 0);
        d.sm_scale = op_param_f(sm, 0);
        const int absorbed_ids[] = {node_index(g, vt, idx), node_index(g, qc, idx), node_index(g, kq, idx), node_index(g, sc, idx),
                                    node_index(g, dm, idx), node_index(g, sm, idx), jm};
        bool all = true;
        for (int a : absorbed_ids) all &= a >= 0;
        if (!all) MI_ATTN_SKIP("check 15")
        // the fused kernel writes M while other workgroups still read Q, K, V
        const char * mlo = (const char *) M->data;
        const char * mhi = mlo + ggml_nbytes(M);
        const char * lo, * hi;
        const int64_t kne[3] = {K->ne[0], K->ne[1], K->ne[2]};
        strided_range(d.k, kne, d.k_nb, 3, &lo, &hi);
        if (lo < mhi && mlo < hi) MI_ATTN_SKIP("check 16")
        const int64_t vne[3] = {vsrc->ne[0], vsrc->ne[1], vsrc->ne[2]};
        strided_range(d.v, vne, d.v_nb, 3, &lo, &hi);
        if (lo < mhi && mlo < hi) MI_ATTN_SKIP("check 17")
        mi_attn_plan pl;
        pl.kqv = j;
        pl.merged = M;
        pl.d = d;
        const int64_t qne[3] = {d.D, d.N, d.H};
        strided_range(d.q, qne, d.q_nb, 3, &lo, &hi);
        if (lo < mhi && mlo < hi) {
            pl.q_copy_at = node_index(g, qc, idx);
            pl.q_src.data = (char *) d.q;
            pl.q_src.type = GGML_TYPE_F32;
            for (int k = 0; k < 3; k++) {
                pl.q_src.ne[k] = qne[k];
                pl.q_src.nb[k] = d.q_nb[k];
            }
            pl.q_src.ne[3] = 1;
            pl.q_src.nb[3] = 0;
        }
        // Q, K and V are now read at the KQV node instead of at cont(Q) (or the copy that replaces
        // it), KQ and cont(V): no node that still runs in between may write over them
        std::vector<uint8_t> mine(g->n_nodes, 0);
        for (int a : absorbed_ids) mine[a] = 1;
        auto clobbered = [&](int from, const char * xlo, const char * xhi) {
            for (int k = from + 1; k < j; k++) {
                const ggml_tensor * n = g->nodes[k];
                if (mine[k] || absorbed_nodes[k] || is_noop(n) || !n->data) continue;
                const char * nlo = (const char *) n->data;
                if (nlo < xhi && xlo < nlo + ggml_nbytes(n)) return true;
            }
            return false;
        };
        strided_range(d.k, kne, d.k_nb, 3, &lo, &hi);
        if (clobbered(node_index(g, kq, idx), lo, hi)) MI_ATTN_SKIP("check 18")
        strided_range(d.v, vne, d.v_nb, 3, &lo, &hi);
        if (clobbered(node_index(g, vt, idx), lo, hi)) MI_ATTN_SKIP("check 19")
        if (pl.q_copy_at < 0) {
            strided_range(d.q, qne, d.q_nb, 3, &lo, &hi);
            if (clobbered(node_index(g, qc, idx), lo, hi)) MI_ATTN_SKIP("check 20")
        }
        if (mask) {  // read at KQV instead of at the ADD; also must not overlap the merged output
            const char * mlo2 = (const char *) mask->data;
            const char * mhi2 = mlo2 + ggml_nbytes(mask);
            if (clobbered(node_index(g, dm, idx), mlo2, mhi2) || (mlo2 < mhi && mlo < mhi2)) MI_ATTN_SKIP("check 21")
        }
        for (int a : absorbed_ids) absorbed_nodes[a] = 1;
        plans.push_back(pl);
    }
#undef MI_ATTN_SKIP
}

// At an attention block's KQV node: the block, the F16 output projection consuming its merged
// output (GPT-2's c_proj, main-backend.cpp:610-620) and that projection's bias and residual ADDs
// as one k_attn_proj launch, whose result stays as per-head partial sums (ctx->pend) until its
// consumer adds them (tree-order decode mode only). Returns the last node covered, or -1.
static int try_fuse_attn_proj(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_attn_plan & pl, const mi_uses & u) {
    if (mi_mmv_order() != 0 || g_mi_tuning.attn_variant != 0 || pl.d.N != 1) return -1;
    const int j = next_node(g, i);
    if (j < 0) return -1;
    ggml_tensor * mm = g->nodes[j];
    const ggml_tensor * M = pl.merged;
    if (mm->op != GGML_OP_MUL_MAT || mm->src[1] != M || u.of(M) != 1 || (M->flags & GGML_TENSOR_FLAG_OUTPUT)) return -1;
    const ggml_tensor * w = mm->src[0];
    if (is_split_tensor(w) || w->type != GGML_TYPE_F16 || w->ne[2] != 1 || w->ne[3] != 1 || w->nb[0] != 2) return -1;
    if (M->ne[0] != w->ne[0] || M->ne[1] != 1 || M->ne[2] != 1 || M->ne[3] != 1) return -1;
    if (!mi_attn_proj_supported(pl.d, w->ne[0], w->ne[1], w->nb[1], w->data)) return -1;
    const int64_t N = w->ne[1];
    const int k1 = next_node(g, j);
    if (k1 < 0 || !private_intermediate(mm, u)) return -1;
    ggml_tensor * a1 = g->nodes[k1];
    const ggml_tensor * bias = add_operand(a1, mm);
    if (!bias || !is_vec_f32(bias, N) || !ggml_are_same_shape(a1, mm) || a1->nb[0] != sizeof(float)) return -1;
    const int k2 = next_node(g, k1);
    if (k2 < 0 || !private_intermediate(a1, u)) return -1;
    ggml_tensor * a2 = g->nodes[k2];
    const ggml_tensor * res = add_operand(a2, a1);
    if (!res || res == a1 || !is_vec_f32(res, N) || !is_vec_f32(a2, N)) return -1;
    if ((size_t) pl.d.H * N * sizeof(float) > (size_t) (w->ne[0] / 64) * N * sizeof(float)) return -1;  // graph_scratch_bytes
    float * parts = (float *) scratch_take(ctx, (size_t) pl.d.H * N * sizeof(float));
    mi_attn_proj_desc p;
    p.W = (const uint8_t *) w->data;
    p.nb01 = w->nb[1];
    p.N = N;
    p.bias = (const float *) bias->data;
    p.resid = (const float *) res->data;
    p.parts = parts;
    mi_attn_proj(pl.d, p, ctx->stream);
    ctx->last_launches++;
    ctx->pend.out = a2;
    ctx->pend.parts = parts;
    ctx->pend.nparts = pl.d.H;
    ctx->pend.n = N;
    return k2;
}

// Quantized prompt mul_mats in a reference-order graph (mmv_order 1, or -1 resolved to 1: a quantized
// model's graph): the int8-MFMA prefill GEMMs compute the reference's exact integer block sums but
// fold them in their own canonical order, and since every layer re-quantizes its activations an ulp
// there becomes a quant step (~1e-2 of max|logit|). Such a mul_mat -- any column count since round 6
// -- runs instead as the reference-order streaming GEMV (k_mmv_stream ORD: the CPU's vec_dot lane
// chains, bit-identical; ggml.c:12056-12096 runs every column through the same vec_dot) over
// 8-column chunks, up to kMiMaxMembers chunks per launch: each chunk is a member of one grouped
// launch over the same weight rows, so a 512-column prompt is one launch whose chunks re-read the
// weights from the caches rather than 64 dependent launches. GGML_MI355X_ORD_PREFILL_COLS /
// set_tuning("ord_prefill_cols", n) caps the column count (longer prompts take the MFMA GEMMs);
// 0 turns it off.
static int g_ord_prefill_cols = getenv("GGML_MI355X_ORD_PREFILL_COLS") ? atoi(getenv("GGML_MI355X_ORD_PREFILL_COLS")) : INT_MAX;

// (tree order: prompts of up to g_tree_prefill_cols columns take the same 8-column GEMV chunks;
// set_tuning("tree_prefill_cols", n), 0 = off)
static int g_tree_prefill_cols = getenv("GGML_MI355X_TREE_PREFILL_COLS") ? atoi(getenv("GGML_MI355X_TREE_PREFILL_COLS")) : 0;

static bool ord_prefill_chunked(const ggml_tensor * n) {
    if (n->op != GGML_OP_MUL_MAT || is_split_tensor(n->src[0])) return false;
    const ggml_tensor * a = n->src[0];
    const ggml_tensor * b = n->src[1];
    if (b->type != GGML_TYPE_F32 || b->ne[1] <= 8 || b->ne[1] > (mi_mmv_order() == 1 ? g_ord_prefill_cols : g_tree_prefill_cols)) return false;
    if (a->type != GGML_TYPE_Q4_K && a->type != GGML_TYPE_Q5_K && a->type != GGML_TYPE_Q4_0 && a->type != GGML_TYPE_Q8_0) return false;
    if (!mi_mmv_fused_supported(a->type, a->ne[0], 8)) return false;
    if (a->ne[2] != 1 || a->ne[3] != 1 || b->ne[2] != 1 || b->ne[3] != 1) return false;
    if (a->nb[0] != ggml_type_size(a->type) || b->nb[0] != sizeof(float) || n->nb[0] != sizeof(float)) return false;
    if (((uintptr_t) a->data | a->nb[1]) % 16 != 0 || ((uintptr_t) b->data | b->nb[1]) % 16 != 0 || n->nb[1] % sizeof(float)) return false;
    return !overlaps(n, a) && !overlaps(n, b);
}

static void run_ord_prefill_chunks(mi_backend_ctx * ctx, ggml_tensor * n) {
    const ggml_tensor * a = n->src[0];
    const ggml_tensor * b = n->src[1];
    const int64_t ncols = b->ne[1];
    const int64_t full = ncols / 8;  // 8-column chunks; the ragged tail (< 8 columns) is one more launch
    auto launch = [&](int64_t c_first, int64_t nchunks, int cols) {
        mi_mmv_group g;
        g.type = a->type;
        g.n = (int) nchunks;
        g.ncols = cols;
        g.K = a->ne[0];
        g.N = a->ne[1];
        g.nb01 = a->nb[1];
        g.xcol = b->nb[1];
        g.ycol = n->nb[1];
        for (int64_t k = 0; k < nchunks; k++) {
            const int64_t c0 = c_first + 8 * k;
            g.m[k].W = a->data;
            g.m[k].X = (const char *) b->data + c0 * b->nb[1];
            g.m[k].dst = (float *) ((char *) n->data + c0 * n->nb[1]);
        }
        mi_mul_mat_q_fused(g, ctx->stream);
        ctx->last_launches++;
    };
    if (full > 0) {
        // split evenly over launches of at most kMiMaxMembers chunks (as run_fused_group)
        const int64_t runs = (full + kMiMaxMembers - 1) / kMiMaxMembers;
        const int64_t take = (full + runs - 1) / runs;
        for (int64_t k0 = 0; k0 < full; k0 += take) launch(8 * k0, std::min<int64_t>(take, full - k0), 8);
    }
    if (ncols % 8) launch(8 * full, 1, (int) (ncols % 8));
}

// the activation kind of a MUL_MAT node that runs on an exact int8 prefill GEMM (Q4_K / Q5_K: 8,
// Q4_0 / Q8_0: 9; > 8 plain columns), or -1
static int prefill_mmx_kind(const ggml_tensor * n) {
    if (n->op != GGML_OP_MUL_MAT || is_split_tensor(n->src[0]) || ord_prefill_chunked(n)) return -1;
    const ggml_tensor * a = n->src[0], * b = n->src[1];
    if (b->type != GGML_TYPE_F32 || a->nb[0] != ggml_type_size(a->type) || b->nb[0] != sizeof(float) || n->nb[0] != sizeof(float)) return -1;
    if (a->ne[0] != b->ne[0]) return -1;
    const int k = mm_act_kind(mm_desc_of(n), b);
    return k == 8 || k == 9 ? k : -1;
}

// Batched (prompt) mul_mats that follow each other in the graph and are independent of each other
// (Q/K/V or gate/up projections of one prompt, independent prompts), same weight type, K and
// column count: their activations are quantized by ONE launch (each distinct src1 once) and their
// GEMMs run as ONE grouped launch (mi_mul_mat_mmqx_group: every member's tiles in one grid), so
// a short prompt pays two kernel boundaries per group instead of per mul_mat. Each member's
// output is what op_mul_mat computes for it, bit for bit (same kernels, same fold). Returns the
// index of the last node consumed, or -1 (fewer than two members).
static int run_prefill_group(mi_backend_ctx * ctx, ggml_cgraph * g, int i) {
    static const bool no_group = getenv("GGML_MI355X_NO_PREFILL_GROUP") != nullptr;
    ggml_tensor * first = g->nodes[i];
    const int kind = prefill_mmx_kind(first);
    if (no_group || kind < 0) return -1;
    const ggml_type type = first->src[0]->type;
    const int64_t K = first->src[0]->ne[0];
    auto cols_of = [](const ggml_tensor * n) { return n->src[1]->ne[1] * n->src[1]->ne[2] * n->src[1]->ne[3]; };
    const int64_t ncols = cols_of(first);
    std::vector<ggml_tensor *> members = {first};
    int last = i;
    std::vector<int> at = {i};
    for (int j = next_node(g, i); j >= 0 && (int) members.size() < 4 * kMiMaxPrefillMembers; j = next_node(g, j)) {
        ggml_tensor * n = g->nodes[j];
        if (prefill_mmx_kind(n) != kind || n->src[0]->type != type || n->src[0]->ne[0] != K || cols_of(n) != ncols) break;
        bool independent = true;
        for (ggml_tensor * m : members) {
            if (overlaps(n->src[1], m) || overlaps(n->src[0], m) || overlaps(n, m->src[0]) || overlaps(n, m->src[1]) || overlaps(n, m)) {
                independent = false;
                break;
            }
        }
        if (!independent) break;
        members.push_back(n);
        at.push_back(j);
    }
    {
        // split a long run evenly over its launches (as run_fused_group)
        const int runs = ((int) members.size() + kMiMaxPrefillMembers - 1) / kMiMaxPrefillMembers;
        const int take = ((int) members.size() + runs - 1) / runs;
        members.resize(take);
        last = at[take - 1];
    }
    if (members.size() < 2) return -1;
    // activations: cached conversions are reused; the missing distinct src1s in one quantizer launch
    mi_mmx_qgroup q;
    q.K = K;
    std::vector<void *> xa(members.size(), nullptr);
    for (size_t k = 0; k < members.size(); k++) {
        const ggml_tensor * x = members[k]->src[1];
        xa[k] = find_activations(ctx, x, kind);
        if (xa[k]) continue;
        void * dev = scratch_take(ctx, act_bytes(kind, K, ncols));
        q.m[q.n].x = src_cols(x);
        q.m[q.n].act = kind == 8 ? mi_act_mmx_carve(dev, K, ncols) : mi_act_mmx0_carve(dev, K, ncols);
        q.n++;
        cache_activations(ctx, x, kind, dev);
        xa[k] = dev;
    }
    if (q.n > 0) {
        if (kind == 8) mi_quantize_q8_K_mmx_group(q, ctx->stream);
        else mi_quantize_q8_0_mmx_group(q, ctx->stream);
        ctx->last_launches++;
    }
    mi_mmx_group gg;
    gg.type = type;
    gg.K = K;
    gg.n = (int) members.size();
    for (size_t k = 0; k < members.size(); k++) {
        const ggml_tensor * n = members[k];
        const mi_act_mmx act = kind == 8 ? mi_act_mmx_carve(xa[k], K, ncols) : mi_act_mmx0_carve(xa[k], K, ncols);
        gg.m[k] = mi_mmx_member{n->src[0]->data, n->src[0]->nb[1], n->src[0]->ne[1], act, (float *) n->data, n->nb[1], 0, planes_of(ctx, n->src[0], n->src[1])};
    }
    mi_mul_mat_mmqx_group(gg, ctx->stream);
    ctx->last_launches++;
    for (ggml_tensor * m : members) invalidate_activations(ctx, m);
    return last;
}

static bool is_copy(const ggml_tensor * t) {
    return (t->op == GGML_OP_CPY || t->op == GGML_OP_DUP || t->op == GGML_OP_CONT) && is_f16_or_f32(t->src[0]) && is_f16_or_f32(t) &&
           ggml_nelements(t) == ggml_nelements(t->src[0]);
}

// GET_ROWS(a, ia), GET_ROWS(b, ib), ADD of the two (GPT-2's token + position embedding,
// main-backend.cpp:475-478) as one launch; the two row sets must be private intermediates
static int try_fuse_embedding(mi_backend_ctx * ctx, ggml_cgraph * g, int i, const mi_uses & u) {
    ggml_tensor * g1 = g->nodes[i];
    const int j = next_node(g, i);
    if (j < 0) return -1;
    ggml_tensor * g2 = g->nodes[j];
    const int k = next_node(g, j);
    if (k < 0 || g2->op != GGML_OP_GET_ROWS) return -1;
    ggml_tensor * add = g->nodes[k];
    if (add->op != GGML_OP_ADD || !((add->src[0] == g1 && add->src[1] == g2) || (add->src[0] == g2 && add->src[1] == g1))) return -1;
    if (!private_intermediate(g1, u) || !private_intermediate(g2, u)) return -1;
    for (const ggml_tensor * t : {(const ggml_tensor *) g1, (const ggml_tensor *) g2}) {
        if (t->type != GGML_TYPE_F32 || t->ne[2] != 1 || t->ne[3] != 1 || t->src[1]->ne[1] != 1 || t->src[1]->ne[2] != 1) return -1;
        if (t->src[0]->ne[2] != 1 || t->src[0]->ne[3] != 1) return -1;
    }
    if (!ggml_are_same_shape(g1, g2) || !ggml_are_same_shape(add, g1) || add->type != GGML_TYPE_F32 || add->nb[0] != sizeof(float)) return -1;
    // the output is written while the row tables and indices are read
    for (const ggml_tensor * t : {g1->src[0], g1->src[1], g2->src[0], g2->src[1]}) {
        if (overlaps(add, t)) return -1;
    }
    mi_op_get_rows_add(desc(add), desc(g1->src[0]), desc(g1->src[1]), desc(g2->src[0]), desc(g2->src[1]), ctx->stream);
    ctx->last_launches++;
    return k;
}

// consecutive independent copies (GPT-2: K -> cache, V -> cache, cont(Q)) as one launch
static int try_fuse_copies(mi_backend_ctx * ctx, ggml_cgraph * g, int i) {
    std::vector<ggml_tensor *> grp = {g->nodes[i]};
    if (!is_copy(grp[0])) return -1;
    int last = i;
    for (int j = next_node(g, i); j >= 0 && (int) grp.size() < kMiMaxCopies; j = next_node(g, j)) {
        ggml_tensor * n = g->nodes[j];
        if (!is_copy(n)) break;
        bool indep = true;
        for (ggml_tensor * m : grp) {
            if (overlaps(n->src[0], m) || overlaps(n, m->src[0]) || overlaps(n, m)) indep = false;
        }
        if (!indep) break;
        grp.push_back(n);
        last = j;
    }
    if (grp.size() < 2) return -1;
    mi_tensor_desc d[kMiMaxCopies], a[kMiMaxCopies];
    for (size_t k = 0; k < grp.size(); k++) {
        d[k] = desc(grp[k]);
        a[k] = desc(grp[k]->src[0]);
    }
    mi_op_cpy_multi(d, a, (int) grp.size(), ctx->stream);
    ctx->last_launches++;
    return last;
}

static enum ggml_status mi_graph_launch_nodes(mi_backend_ctx * ctx, ggml_cgraph * cgraph);

static bool graphs_enabled(const mi_backend_ctx * ctx) {
    static const bool env_no_graphs = getenv("GGML_MI355X_DISABLE_GRAPHS") != nullptr;
    return ctx->graphs && !env_no_graphs && !ctx->perf;  // the per-node timer needs direct launches
}

// ---- per-node timer ----------------------------------------------------------------------------
// A dispatch unit is one pass of mi_graph_launch_nodes' loop: a node, or a fused chain of nodes
// run by one kernel. perf_mark records an event before each unit (after the store of partial sums
// an earlier unit deferred, which stays in that unit's time; nodes absorbed into another node's
// kernel get no mark); perf_finish records the end,
// waits for the stream and adds each unit's device time to the perf fields of its last node (the
// other nodes of a fused chain get a run with no time, as the reference's fused-away work would),
// and the whole graph's to the cgraph's (ggml.c:19907-19922). ggml_graph_print shows them.
static bool perf_active(const mi_backend_ctx * ctx) {
    if (!ctx->perf) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    MI_CHECK(hipStreamIsCapturing(ctx->stream, &cs));
    return cs == hipStreamCaptureStatusNone;
}

static void perf_mark(mi_backend_ctx * ctx, int i) {
    const size_t k = ctx->perf_at.size();
    if (k == ctx->perf_ev.size()) {
        hipEvent_t e;
        MI_CHECK(hipEventCreate(&e));
        ctx->perf_ev.push_back(e);
    }
    MI_CHECK(hipEventRecord(ctx->perf_ev[k], ctx->stream));
    ctx->perf_at.push_back(i);
}

static void perf_finish(mi_backend_ctx * ctx, ggml_cgraph * g, int64_t t_host0) {
    const size_t n = ctx->perf_at.size();
    perf_mark(ctx, g->n_nodes);
    MI_CHECK(hipEventSynchronize(ctx->perf_ev[n]));
    for (size_t k = 0; k < n; k++) {
        float ms = 0.0f;
        MI_CHECK(hipEventElapsedTime(&ms, ctx->perf_ev[k], ctx->perf_ev[k + 1]));
        const int lo = ctx->perf_at[k], hi = ctx->perf_at[k + 1];
        // the time goes to the unit's last node that is not executed inside another node's kernel
        // (absorbed nodes between two units ran in an earlier unit's kernel: a run, no time)
        int last = -1, last_any = -1;
        for (int j = lo; j < hi; j++) {
            if (is_noop(g->nodes[j])) continue;
            g->nodes[j]->perf_runs++;
            last_any = j;
            if (!absorbed(j)) last = j;
        }
        if (last < 0) last = last_any;
        if (last >= 0) {
            const int64_t us = (int64_t) llround(ms * 1000.0);
            g->nodes[last]->perf_time_us += us;
            g->nodes[last]->perf_cycles += us;  // (device time: no CPU cycles; microseconds here)
        }
    }
    float total = 0.0f;
    if (n) MI_CHECK(hipEventElapsedTime(&total, ctx->perf_ev[0], ctx->perf_ev[n]));
    g->perf_runs++;
    g->perf_time_us += (int64_t) llround(total * 1000.0);
    g->perf_cycles += ggml_time_us() - t_host0;  // host wall time of the call, microseconds
    ctx->perf_at.clear();
}

// a graph that can be captured: no split-buffer mul_mat (several streams, events, peer copies)
static bool graph_capturable(const ggml_cgraph * cgraph) {
    for (int i = 0; i < cgraph->n_nodes; i++) {
        const ggml_tensor * n = cgraph->nodes[i];
        if (n->op == GGML_OP_MUL_MAT && is_split_tensor(n->src[0])) return false;
    }
    return true;
}

// Everything the node pass does synchronously -- table uploads, scratch growth -- done up front,
// so that a capture of the pass only enqueues kernels on ctx->stream. Scratch: the pass's own
// estimate plus room for the attention planner's Q copies (at most every CONT node's bytes).
static int graph_decode_order(const ggml_cgraph * g);

static void prepare_for_capture(mi_backend_ctx * ctx, const ggml_cgraph * cgraph) {
    tl_mi_graph_order = graph_decode_order(cgraph);  // (the graph's order decides which weight copies it needs)
    op_tables(ctx);
    rope_tables_prepare(ctx, cgraph);
    size_t cont_bytes = 0;
    for (int i = 0; i < cgraph->n_nodes; i++) {
        if (cgraph->nodes[i]->op == GGML_OP_CONT) cont_bytes += (ggml_nbytes(cgraph->nodes[i]) + kBufferAlign - 1) & ~(kBufferAlign - 1);
    }
    scratch_reserve(ctx, graph_scratch_bytes(cgraph) + cont_bytes);
}

// Captures the node pass of `cgraph` into a hipGraph (nullptr if something in it could not be
// captured; the backend then launches directly from now on). The stream may still be running
// earlier work: the capture records only what follows.
static hipGraph_t capture_pass(mi_backend_ctx * ctx, ggml_cgraph * cgraph) {
    MI_CHECK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    const ggml_status st = mi_graph_launch_nodes(ctx, cgraph);
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
    if (st != GGML_STATUS_SUCCESS || ec != hipSuccess || !graph) {
        (void) hipGetLastError();
        if (graph) (void) hipGraphDestroy(graph);
        ctx->graphs = false;
        return nullptr;
    }
    ctx->graph_stats[0]++;
    return graph;
}

// The exact launch-relevant content of a graph: per node its output address, op, type, flags,
// shape, strides, op_params, view source and every source's address, type, flags, shape and
// strides; plus the
// scratch buffer the captured kernels use and the tuning knobs that choose kernels. Two graphs
// with equal keys launch identical kernels with identical arguments.
static void graph_key(const mi_backend_ctx * ctx, const ggml_cgraph * g, std::vector<uint64_t> & k) {
    k.clear();
    k.reserve((size_t) g->n_nodes * 40 + 16);
    k.push_back((uint64_t) g->n_nodes);
    k.push_back((uint64_t) (g->size == 0 && g->visited_hash_table.size == 0));  // mi_uses::partial
    k.push_back((uint64_t) (uintptr_t) ctx->scratch);
    k.push_back(ctx->scratch_gen);
    // captured long-prompt GEMMs bake in the repacked planes' addresses (mi_mmx_member::planes): a
    // planes entry created or dropped since (a weight buffer freed and another allocated at the same
    // address) must not replay a graph that reads freed planes
    k.push_back(mi_planes_generation());
    k.push_back((uint64_t) (uint32_t) g_ord_prefill_cols | ((uint64_t) (uint32_t) g_tree_prefill_cols << 32));  // (chunked prompt GEMVs)
    {
        uint64_t tw[(sizeof(mi_tuning) + 7) / 8] = {};
        memcpy(tw, &g_mi_tuning, sizeof(mi_tuning));
        for (uint64_t w : tw) k.push_back(w);
    }
    auto tensor = [&](const ggml_tensor * t) {
        k.push_back((uint64_t) (uintptr_t) t->data);
        // flags too: whether a node's value is stored or fused away depends on GGML_TENSOR_FLAG_OUTPUT
        k.push_back((uint64_t) t->type | ((uint64_t) t->op << 16) | ((uint64_t) (uint32_t) t->flags << 32));
        for (int d = 0; d < 4; d++) k.push_back((uint64_t) t->ne[d]);
        for (int d = 0; d < 4; d++) k.push_back((uint64_t) t->nb[d]);
    };
    for (int i = 0; i < g->n_nodes; i++) {
        const ggml_tensor * t = g->nodes[i];
        tensor(t);
        k.push_back((uint64_t) (uintptr_t) t->view_src);
        uint64_t pw[GGML_MAX_OP_PARAMS / 8];
        memcpy(pw, t->op_params, sizeof(pw));
        for (uint64_t w : pw) k.push_back(w);
        int ns = 0;
        for (int j = 0; j < GGML_MAX_SRC; j++) if (t->src[j]) ns = j + 1;
        k.push_back((uint64_t) ns);
        for (int j = 0; j < ns; j++) {
            if (t->src[j]) tensor(t->src[j]);
            else k.push_back(0);
        }
    }
}

// topology of a graph (ops, types, source counts): graphs that differ only in addresses, shapes
// or parameters -- a decode step at the next position -- share it, so the executable graph of one
// can be updated in place for the other
static uint64_t graph_topology(const ggml_cgraph * g) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    mix((uint64_t) g->n_nodes);
    for (int i = 0; i < g->n_nodes; i++) {
        const ggml_tensor * t = g->nodes[i];
        int ns = 0;
        for (int j = 0; j < GGML_MAX_SRC; j++) if (t->src[j]) ns = j + 1;
        mix((uint64_t) t->op | ((uint64_t) t->type << 8) | ((uint64_t) ns << 16) | ((uint64_t) (t->view_src != nullptr) << 24));
    }
    return h;
}

// captures below this many kernel launches are not worth a replay (one small graph launches
// faster directly than through hipGraphLaunch); GGML_MI355X_GRAPH_MIN_LAUNCHES overrides
static int graph_min_launches() {
    static const int v = getenv("GGML_MI355X_GRAPH_MIN_LAUNCHES") ? atoi(getenv("GGML_MI355X_GRAPH_MIN_LAUNCHES")) : 4;
    return v;
}

static constexpr size_t kGraphCacheEntries = 8;
static constexpr int kGraphMissDirect = 3;
static constexpr int kGraphRetry = 32;

static void gcache_launch(mi_backend_ctx * ctx, mi_backend_ctx::gcache_entry & e) {
    MI_CHECK(hipGraphLaunch(e.exec, ctx->stream));
    MI_CHECK(hipEventRecord(e.done, ctx->stream));
    e.last_use = ++ctx->gclock;
    ctx->last_launches = e.launches;
}

// graph_compute (ggml-cuda.cu:2456-2713 analogue: capture at :2576, exec update at :2690, the
// GGML_CUDA_DISABLE_GRAPHS switch at :2462). A graph whose exact content (graph_key) was captured
// before is replayed with one hipGraphLaunch. Otherwise: the first graph of a topology runs
// directly (its launch count decides whether capturing it pays); a later one is captured, an
// executable graph of the same topology is updated in place when only kernel arguments changed,
// else a new one is instantiated (at most kGraphCacheEntries per backend, least recently used
// evicted). Anything that cannot be captured runs directly.
static enum ggml_status mi_graph_compute(ggml_backend_t backend, ggml_cgraph * cgraph) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    mi_device_guard g(ctx->device);
    if (!graphs_enabled(ctx) || !graph_capturable(cgraph)) {
        ctx->graph_stats[3]++;
        return mi_graph_launch_nodes(ctx, cgraph);
    }
    // A topology whose graphs kept arriving with new kernel arguments and never replayed (a decode
    // step through graph_compute: the KV length moves every call) launches directly: a capture costs
    // a synchronous recording of every launch plus an update per call for nothing, where a direct
    // launch overlaps host and device. Decided after kGraphMissDirect (3) such captures in a row; the
    // key and the preparation are then skipped too. Measured on main-batched.cpp's decode loop
    // (bench gpt2_batched): 4.9 k tokens/s capturing every step vs 6.2-6.5 k direct.
    // The decision decays: every kGraphRetry-th direct run of such a topology looks its key up
    // again, and a replay (a graph that does repeat) resets the count; set_graph_capture resets all.
    const uint64_t topo = graph_topology(cgraph);
    bool direct_only = false;
    {
        auto m = ctx->topo_misses.find(topo);
        if (m != ctx->topo_misses.end() && m->second >= kGraphMissDirect) {
            m->second++;
            if ((m->second - kGraphMissDirect) % kGraphRetry != 0) {
                ctx->graph_stats[3]++;
                return mi_graph_launch_nodes(ctx, cgraph);
            }
            direct_only = true;
        }
    }
    prepare_for_capture(ctx, cgraph);
    static thread_local std::vector<uint64_t> key;
    graph_key(ctx, cgraph, key);
    for (auto & e : ctx->gcache) {
        if (e.key == key) {
            ctx->graph_stats[4]++;
            ctx->topo_misses[e.topo] = 0;
            gcache_launch(ctx, e);
            return GGML_STATUS_SUCCESS;
        }
    }
    if (direct_only) {
        ctx->graph_stats[3]++;
        return mi_graph_launch_nodes(ctx, cgraph);
    }
    auto seen = ctx->topo_launches.find(topo);
    if (seen == ctx->topo_launches.end() || seen->second < graph_min_launches()) {
        ctx->graph_stats[3]++;
        const ggml_status st = mi_graph_launch_nodes(ctx, cgraph);
        ctx->topo_launches[topo] = ctx->last_launches;
        return st;
    }
    ctx->topo_misses[topo]++;  // (reset by a replay of this topology)
    hipGraph_t graph = capture_pass(ctx, cgraph);
    if (!graph) {
        ctx->graph_stats[3]++;
        return mi_graph_launch_nodes(ctx, cgraph);
    }
    ctx->graph_stats[5]++;
    const int launches = ctx->last_launches;
    // An executable graph of this topology that is not in flight is updated in place (never one
    // still running). In a decode loop every step has a new key (the KV length moves) and the
    // previous step's executable is usually still running: rather than wait for it, a second one
    // per topology is instantiated, and the two then alternate. An entry whose update was refused
    // (a changed kernel choice) is no longer tried for updates; it still replays its own key.
    mi_backend_ctx::gcache_entry * slot = nullptr;
    auto try_update = [&](mi_backend_ctx::gcache_entry & e) {
        hipGraphNode_t err_node = nullptr;
        hipGraphExecUpdateResult res;
        if (hipGraphExecUpdate(e.exec, graph, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess) {
            ctx->graph_stats[2]++;
            slot = &e;
        } else {
            (void) hipGetLastError();
            e.no_update = true;
        }
    };
    int same_topo = 0;
    mi_backend_ctx::gcache_entry * busy = nullptr;
    for (auto & e : ctx->gcache) {
        if (e.topo != topo || e.no_update) continue;
        same_topo++;
        const hipError_t q = hipEventQuery(e.done);
        if (q == hipErrorNotReady) {
            (void) hipGetLastError();
            if (!busy || e.last_use < busy->last_use) busy = &e;
            continue;
        }
        MI_CHECK(q);
        try_update(e);
        break;
    }
    if (!slot && busy && same_topo >= 2) {
        MI_CHECK(hipEventSynchronize(busy->done));
        try_update(*busy);
    }
    if (!slot) {
        if (ctx->gcache.size() >= kGraphCacheEntries) {
            auto lru = std::min_element(ctx->gcache.begin(), ctx->gcache.end(),
                                        [](const auto & a, const auto & b) { return a.last_use < b.last_use; });
            MI_CHECK(hipEventSynchronize(lru->done));
            MI_CHECK(hipGraphExecDestroy(lru->exec));
            MI_CHECK(hipEventDestroy(lru->done));
            ctx->gcache.erase(lru);
        }
        ctx->gcache.emplace_back();
        slot = &ctx->gcache.back();
        MI_CHECK(hipGraphInstantiate(&slot->exec, graph, nullptr, nullptr, 0));
        MI_CHECK(hipEventCreateWithFlags(&slot->done, hipEventDisableTiming));
        ctx->graph_stats[1]++;
    }
    MI_CHECK(hipGraphDestroy(graph));
    slot->key = key;
    slot->topo = topo;
    slot->launches = launches;
    gcache_launch(ctx, *slot);
    return GGML_STATUS_SUCCESS;
}

// Graph plans (ggml_backend_graph_plan_create / _compute, ggml-backend.h): a plan is the graph's
// launches captured into a hipGraph, so computing it is one hipGraphLaunch instead of one host
// launch per kernel (~3 us each). A caller that knows its next graph early -- a decode loop,
// whose next graph depends on positions only -- creates the plan while the device still runs the
// current one. Executable graphs are pooled per backend: a new plan updates a pooled one in place
// (hipGraphExecUpdate) when only kernel arguments changed (KV length, cache offsets), and
// instantiates otherwise.
struct mi_graph_plan {
    ggml_cgraph graph;              // the caller's graph (node arrays stay the caller's)
    hipGraphExec_t exec = nullptr;  // null: launched directly at compute time
    uint64_t scratch_gen = 0;       // the scratch buffer generation the capture refers to
    int launches = 0;
};

// consecutive refused updates after which a backend stops capturing (as ggml-cuda.cu's
// disable_due_to_too_many_updates)
static constexpr int kGraphMaxFailStreak = 4;

static ggml_backend_graph_plan_t mi_graph_plan_create(ggml_backend_t backend, const ggml_cgraph * cgraph) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    mi_device_guard g(ctx->device);
    auto * plan = new mi_graph_plan();
    plan->graph = *cgraph;
    if (!graphs_enabled(ctx) || !graph_capturable(cgraph)) return plan;
    prepare_for_capture(ctx, cgraph);
    hipGraph_t graph = capture_pass(ctx, &plan->graph);
    if (!graph) return plan;
    plan->scratch_gen = ctx->scratch_gen;
    plan->launches = ctx->last_launches;
    while (!ctx->exec_pool.empty() && !plan->exec) {
        hipGraphExec_t ex = ctx->exec_pool.back();
        ctx->exec_pool.pop_back();
        hipGraphNode_t err_node = nullptr;
        hipGraphExecUpdateResult res;
        if (hipGraphExecUpdate(ex, graph, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess) {
            plan->exec = ex;
        } else {
            (void) hipGetLastError();
            MI_CHECK(hipGraphExecDestroy(ex));
        }
    }
    if (plan->exec) {
        ctx->graph_stats[2]++;
        ctx->graph_fail_streak = 0;
    } else {
        MI_CHECK(hipGraphInstantiate(&plan->exec, graph, nullptr, nullptr, 0));
        ctx->graph_stats[1]++;
        if (ctx->graph_stats[1] > 2 && ++ctx->graph_fail_streak >= kGraphMaxFailStreak) ctx->graphs = false;
    }
    MI_CHECK(hipGraphDestroy(graph));
    return plan;
}

static void mi_graph_plan_free(ggml_backend_t backend, ggml_backend_graph_plan_t p) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    auto * plan = (mi_graph_plan *) p;
    if (plan->exec) {
        // kept for the next plan to update in place (at most a few per backend)
        if (ctx->exec_pool.size() < 4) ctx->exec_pool.push_back(plan->exec);
        else MI_CHECK(hipGraphExecDestroy(plan->exec));
    }
    delete plan;
}

static enum ggml_status mi_graph_plan_compute(ggml_backend_t backend, ggml_backend_graph_plan_t p) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    auto * plan = (mi_graph_plan *) p;
    mi_device_guard g(ctx->device);
    // a plan captured against a scratch buffer that has since been reallocated (a later, larger
    // graph) would launch on freed memory: such a plan runs its nodes directly
    if (!plan->exec || plan->scratch_gen != ctx->scratch_gen) {
        ctx->graph_stats[3]++;
        return mi_graph_launch_nodes(ctx, &plan->graph);
    }
    MI_CHECK(hipGraphLaunch(plan->exec, ctx->stream));
    // GGML_MI355X_PLAN_FLUSH (A/B): 1 = a marker event behind the launch, 2 = hipStreamQuery, 0 (the
    // default) = nothing; no variant was faster than the noise in the GPT-2 decode loop (r03y2)
    static const int flush = getenv("GGML_MI355X_PLAN_FLUSH") ? atoi(getenv("GGML_MI355X_PLAN_FLUSH")) : 0;
    if (flush == 1) {
        if (!ctx->plan_marker) MI_CHECK(hipEventCreateWithFlags(&ctx->plan_marker, hipEventDisableTiming));
        MI_CHECK(hipEventRecord(ctx->plan_marker, ctx->stream));
    } else if (flush == 2) {
        (void) hipStreamQuery(ctx->stream);
    }
    ctx->last_launches = plan->launches;
    return GGML_STATUS_SUCCESS;
}

// mmv_order -1: the decode summation order of a graph. A quantized MUL_MAT whose src1 is computed
// in the graph re-quantizes it (quantize_row_q8_*: round(x / d)), so a 1-ulp difference upstream can
// move a quant by a whole step and the logits of a quantized model by ~1e-2
// (tests/test_gpt2.py::test_reference_quantized_gpt2_is_ulp_sensitive): such graphs run every decode
// reduction in the reference CPU's order (bit-identical). Any other graph (F16 models, a mul_mat of
// input data) keeps the tree order, within 1e-5 of the reference per op.
// A split input of the reference scheduler is a NONE tensor holding a value another split computed
// (ggml_backend_sched_split_graph creates it with ggml_dup_tensor_layout, ggml-backend.c:1498-1523).
// It cannot be told from a true graph input by its own fields (flags are set only when n_copies > 1,
// names may be truncated), but the graph says where it came from: the scheduler hands a backend
// views of its splits (ggml_graph_view, ggml-backend.c:1549: size 0, no hash table), and a full
// graph never holds such copies. So in a split view every NONE source counts as computed -- the
// reference order, bit-identical either way -- and in a full graph as input.
static bool sched_split_view(const ggml_cgraph * g) { return g->size == 0 && g->visited_hash_table.size == 0; }

static int graph_decode_order(const ggml_cgraph * g) {
    const bool view = sched_split_view(g);
    for (int i = 0; i < g->n_nodes; i++) {
        const ggml_tensor * n = g->nodes[i];
        if (n->op != GGML_OP_MUL_MAT || !ggml_is_quantized(n->src[0]->type)) continue;
        const ggml_tensor * x = n->src[1];
        while (x->view_src || x->op == GGML_OP_RESHAPE || x->op == GGML_OP_VIEW || x->op == GGML_OP_PERMUTE ||
               x->op == GGML_OP_TRANSPOSE) {
            x = x->view_src ? x->view_src : x->src[0];
        }
        if (x->op != GGML_OP_NONE || view) return 1;
    }
    return 0;
}

static enum ggml_status mi_graph_launch_nodes(mi_backend_ctx * ctx, ggml_cgraph * cgraph) {
    tl_mi_graph_order = graph_decode_order(cgraph);
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        MI_CHECK(hipStreamIsCapturing(ctx->stream, &cs));
        if (cs == hipStreamCaptureStatusNone) rope_tables_prepare(ctx, cgraph);
    }
    scratch_reserve(ctx, graph_scratch_bytes(cgraph));
    ctx->scratch_used = 0;
    ctx->act_cache.clear();
    ctx->last_launches = 0;
    static const bool no_fuse = getenv("GGML_MI355X_NO_FUSED_MMV") != nullptr;
    static const bool no_node_fusion = getenv("GGML_MI355X_NO_NODE_FUSION") != nullptr;
    // bit mask of enabled node fusions (debug/A-B): 1 norm, 2 softmax, 4 f16 GEMV, 8 copies, 16 attention,
    // 64 embedding, 128 attention + output projection
    static const int fuse_mask = getenv("GGML_MI355X_FUSE_MASK") ? atoi(getenv("GGML_MI355X_FUSE_MASK")) : 0xff;
    ctx->pend = {};
    mi_uses uses;
    std::vector<uint8_t> absorbed_nodes;
    std::vector<mi_attn_plan> attn;
    if (!no_node_fusion) {
        count_uses(cgraph, uses);
        if (fuse_mask & 16) plan_attention(cgraph, uses, absorbed_nodes, attn);
    }
    size_t q_copy_bytes = 0;
    for (const auto & pl : attn) {
        if (pl.q_copy_at >= 0) q_copy_bytes += ((size_t) pl.d.D * pl.d.N * pl.d.H * sizeof(float) + kBufferAlign - 1) & ~(kBufferAlign - 1);
    }
    if (q_copy_bytes) {
        scratch_reserve(ctx, graph_scratch_bytes(cgraph) + q_copy_bytes);
        for (auto & pl : attn) {
            if (pl.q_copy_at < 0) continue;
            char * q = (char *) scratch_take(ctx, (size_t) pl.d.D * pl.d.N * pl.d.H * sizeof(float));
            pl.d.q = q;
            pl.d.q_nb[0] = sizeof(float);
            pl.d.q_nb[1] = (size_t) pl.d.D * sizeof(float);
            pl.d.q_nb[2] = (size_t) pl.d.D * pl.d.N * sizeof(float);
        }
    }
    tl_absorbed = &absorbed_nodes;
    size_t next_attn = 0;
    const bool perf = perf_active(ctx);
    const int64_t perf_t0 = perf ? ggml_time_us() : 0;
    ctx->perf_at.clear();
    for (int i = 0; i < cgraph->n_nodes; i++) {
        ggml_tensor * node = cgraph->nodes[i];
        if (absorbed(i) && q_copy_bytes) {
            for (const auto & pl : attn) {
                if (pl.q_copy_at != i) continue;
                if (perf) perf_mark(ctx, i);  // the Q copy: a unit of its own
                mi_tensor_desc dq = pl.q_src;
                dq.data = (char *) pl.d.q;
                for (int k = 0; k < 3; k++) dq.nb[k] = pl.d.q_nb[k];
                mi_op_cpy(dq, pl.q_src, ctx->stream);
                ctx->last_launches++;
            }
        }
        if (is_noop(node) || absorbed(i)) continue;
        if (ctx->pend.out) {
            // a value held as partial sums is stored before any node but its norm consumer runs
            const bool consumer = !no_node_fusion && (fuse_mask & 1) && (node->op == GGML_OP_NORM || node->op == GGML_OP_RMS_NORM) &&
                                  node->src[0] == ctx->pend.out;
            if (!consumer) flush_pending(ctx);  // (still timed with the unit that deferred it)
        }
        if (perf) perf_mark(ctx, i);
        if (next_attn < attn.size() && attn[next_attn].kqv == i) {
            const int lastp = (fuse_mask & 128) ? try_fuse_attn_proj(ctx, cgraph, i, attn[next_attn], uses) : -1;
            if (lastp < 0) {
                mi_attn_ordered(attn[next_attn].d, op_tables(ctx), ctx->stream);
                ctx->last_launches++;
            }
            invalidate_activations(ctx, attn[next_attn].merged);  // written here, at the KQV node
            for (int k = i + 1; k <= lastp; k++) invalidate_activations(ctx, cgraph->nodes[k]);
            if (lastp >= 0) i = lastp;
            next_attn++;
            continue;
        }
        if (node->op == GGML_OP_MUL_MAT && is_split_tensor(node->src[0])) {
            op_mul_mat_split(ctx, node);
            invalidate_activations(ctx, node);
            continue;
        }
        int last = -1;
        if (!no_node_fusion) {
            switch (node->op) {
                case GGML_OP_NORM:
                case GGML_OP_RMS_NORM: last = (fuse_mask & 1) ? try_fuse_norm(ctx, cgraph, i, uses) : -1; break;
                case GGML_OP_SCALE: last = (fuse_mask & 2) ? try_fuse_softmax(ctx, cgraph, i, uses) : -1; break;
                case GGML_OP_MUL_MAT:
                    last = (fuse_mask & 4) ? try_fuse_f16_gemv(ctx, cgraph, i, uses) : -1;
                    if (last < 0 && (fuse_mask & 32) && !no_fuse) last = try_fuse_q_gemv(ctx, cgraph, i, uses);
                    break;
                case GGML_OP_CPY:
                case GGML_OP_DUP:
                case GGML_OP_CONT: last = (fuse_mask & 8) ? try_fuse_copies(ctx, cgraph, i) : -1; break;
                case GGML_OP_GET_ROWS: last = (fuse_mask & 64) ? try_fuse_embedding(ctx, cgraph, i, uses) : -1; break;
                default: break;
            }
        }
        if (last >= 0) {
            for (int k = i; k <= last; k++) invalidate_activations(ctx, cgraph->nodes[k]);
            i = last;
            continue;
        }
        flush_pending(ctx);
        switch (node->op) {
            case GGML_OP_MUL_MAT: {
                if (!no_fuse && fused_mv_eligible(node)) {
                    i = run_fused_group(ctx, cgraph, i);
                    continue;
                }
                if (ord_prefill_chunked(node)) {
                    run_ord_prefill_chunks(ctx, node);
                    break;
                }
                const int lastg = run_prefill_group(ctx, cgraph, i);
                if (lastg >= 0) {
                    i = lastg;
                    continue;
                }
                op_mul_mat(ctx, node);
                break;
            }
            default:
                op_companion(ctx, node);
        }
        invalidate_activations(ctx, node);
    }
    flush_pending(ctx);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        tl_absorbed = nullptr;
        fprintf(stderr, "%s: kernel launch failed: %s\n", __func__, hipGetErrorString(err));
        return GGML_STATUS_FAILED;
    }
    if (perf) perf_finish(ctx, cgraph, perf_t0);
    tl_absorbed = nullptr;
    return GGML_STATUS_SUCCESS;
}

// ---------------------------------------------------------------------------------------------
// backend vtable
// ---------------------------------------------------------------------------------------------

static const char * mi_backend_name(ggml_backend_t backend) { return ((mi_backend_ctx *) backend->context)->name.c_str(); }

static void mi_backend_free(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    {
        mi_device_guard g(ctx->device);
        MI_CHECK(hipStreamSynchronize(ctx->stream));
        for (hipGraphExec_t ex : ctx->exec_pool) MI_CHECK(hipGraphExecDestroy(ex));
        for (auto & e : ctx->gcache) {
            MI_CHECK(hipGraphExecDestroy(e.exec));
            MI_CHECK(hipEventDestroy(e.done));
        }
        if (ctx->scratch) MI_CHECK(hipFree(ctx->scratch));
        if (ctx->tables) MI_CHECK(hipFree(ctx->tables));
        for (auto & t : ctx->rope_tables) MI_CHECK(hipFree(t.dev));
        if (ctx->plan_marker) MI_CHECK(hipEventDestroy(ctx->plan_marker));
        if (ctx->split_ready) MI_CHECK(hipEventDestroy(ctx->split_ready));
        for (hipEvent_t e : ctx->perf_ev) MI_CHECK(hipEventDestroy(e));
        MI_CHECK(hipStreamDestroy(ctx->stream));
    }
    delete ctx;
    delete backend;
}

static ggml_backend_buffer_type_t mi_backend_default_buft(ggml_backend_t backend) {
    return ggml_backend_mi355x_buffer_type(((mi_backend_ctx *) backend->context)->device);
}

static void mi_backend_set_tensor_async(ggml_backend_t backend, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    ggml_backend_buffer_t buf = tensor->view_src ? tensor->view_src->buffer : tensor->buffer;
    MI_ASSERT(buffer_is_mi355x(buf) && "unsupported buffer type");
    mi_device_guard g(ctx->device);
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, ctx->stream));
    mi_planes_refresh((char *) tensor->data + offset, size, ctx->stream);  // repacked planes over these bytes, after the copy
}

static void mi_backend_get_tensor_async(ggml_backend_t backend, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    ggml_backend_buffer_t buf = tensor->view_src ? tensor->view_src->buffer : tensor->buffer;
    MI_ASSERT(buffer_is_mi355x(buf) && "unsupported buffer type");
    mi_device_guard g(ctx->device);
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, ctx->stream));
}

static bool mi_backend_cpy_tensor_async(ggml_backend_t backend_src, ggml_backend_t backend_dst, const ggml_tensor * src, ggml_tensor * dst) {
    if (!ggml_backend_is_mi355x(backend_src) || !ggml_backend_is_mi355x(backend_dst)) return false;
    ggml_backend_buffer_t sbuf = src->view_src ? src->view_src->buffer : src->buffer;
    ggml_backend_buffer_t dbuf = dst->view_src ? dst->view_src->buffer : dst->buffer;
    if (!buffer_is_mi355x(sbuf) || !buffer_is_mi355x(dbuf)) return false;
    auto * cs = (mi_backend_ctx *) backend_src->context;
    auto * cd = (mi_backend_ctx *) backend_dst->context;
    if (cs->device == cd->device) {
        mi_device_guard g(cs->device);
        MI_CHECK(hipMemcpyAsync(dst->data, src->data, ggml_nbytes(dst), hipMemcpyDeviceToDevice, cd->stream));
        mi_planes_refresh(dst->data, ggml_nbytes(dst), cd->stream);
        return true;
    }
    // cross-device: copy on the source stream after its producers, destination waits on an event
    mi_device_guard g(cs->device);
    MI_CHECK(hipMemcpyPeerAsync(dst->data, cd->device, src->data, cs->device, ggml_nbytes(dst), cs->stream));
    hipEvent_t ev;
    MI_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    MI_CHECK(hipEventRecord(ev, cs->stream));
    {
        mi_device_guard g2(cd->device);
        MI_CHECK(hipStreamWaitEvent(cd->stream, ev, 0));
        mi_planes_refresh(dst->data, ggml_nbytes(dst), cd->stream);  // on the destination, behind the copy
    }
    MI_CHECK(hipEventDestroy(ev));
    return true;
}

static void mi_backend_synchronize(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    mi_device_guard g(ctx->device);
    MI_CHECK(hipStreamSynchronize(ctx->stream));
}

static ggml_backend_event_t mi_event_new(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    mi_device_guard g(ctx->device);
    hipEvent_t ev;
    MI_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    auto * e = new ggml_backend_event;
    e->backend = backend;
    e->context = ev;
    return e;
}

static void mi_event_free(ggml_backend_event_t event) {
    MI_CHECK(hipEventDestroy((hipEvent_t) event->context));
    delete event;
}

static void mi_event_record(ggml_backend_event_t event) {
    auto * ctx = (mi_backend_ctx *) event->backend->context;
    MI_CHECK(hipEventRecord((hipEvent_t) event->context, ctx->stream));
}

static void mi_event_wait(ggml_backend_t backend, ggml_backend_event_t event) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    if (ggml_backend_is_mi355x(event->backend)) {
        MI_CHECK(hipStreamWaitEvent(ctx->stream, (hipEvent_t) event->context, 0));
    } else {
        event->backend->iface.event_synchronize(event);
    }
}

static void mi_event_synchronize(ggml_backend_event_t event) { MI_CHECK(hipEventSynchronize((hipEvent_t) event->context)); }

static const ggml_backend_i k_mi_backend_i = {
    /* get_name                */ mi_backend_name,
    /* free                    */ mi_backend_free,
    /* get_default_buffer_type */ mi_backend_default_buft,
    /* set_tensor_async        */ mi_backend_set_tensor_async,
    /* get_tensor_async        */ mi_backend_get_tensor_async,
    /* cpy_tensor_async        */ mi_backend_cpy_tensor_async,
    /* synchronize             */ mi_backend_synchronize,
    /* graph_plan_create       */ mi_graph_plan_create,
    /* graph_plan_free         */ mi_graph_plan_free,
    /* graph_plan_compute      */ mi_graph_plan_compute,
    /* graph_compute           */ mi_graph_compute,
    /* supports_op             */ mi_supports_op,
    /* offload_op              */ mi_offload_op,
    /* event_new               */ mi_event_new,
    /* event_free              */ mi_event_free,
    /* event_record            */ mi_event_record,
    /* event_wait              */ mi_event_wait,
    /* event_synchronize       */ mi_event_synchronize,
};

static bool mi_buft_supports_backend(ggml_backend_buffer_type_t buft, ggml_backend_t backend) {
    if (!ggml_backend_is_mi355x(backend)) return false;
    return ((mi_buft_ctx *) buft->context)->device == ((mi_backend_ctx *) backend->context)->device;
}

// ---------------------------------------------------------------------------------------------
// public API
// ---------------------------------------------------------------------------------------------

extern "C" {

int ggml_backend_mi355x_get_device_count(void) { return device_count(); }

void ggml_backend_mi355x_get_device_description(int device, char * description, size_t description_size) {
    hipDeviceProp_t prop;
    MI_CHECK(hipGetDeviceProperties(&prop, device));
    snprintf(description, description_size, "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
}

void ggml_backend_mi355x_get_device_memory(int device, size_t * free, size_t * total) {
    mi_device_guard g(device);
    MI_CHECK(hipMemGetInfo(free, total));
}

bool ggml_backend_mi355x_register_host_buffer(void * buffer, size_t size) {
    if (getenv("GGML_MI355X_REGISTER_HOST") == nullptr) return false;
    const hipError_t err = hipHostRegister(buffer, size, hipHostRegisterPortable | hipHostRegisterReadOnly);
    if (err != hipSuccess) {
        (void) hipGetLastError();
        return false;
    }
    return true;
}

void ggml_backend_mi355x_unregister_host_buffer(void * buffer) {
    if (getenv("GGML_MI355X_REGISTER_HOST") == nullptr) return;
    (void) hipHostUnregister(buffer);
    (void) hipGetLastError();
}

ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device) {
    static std::mutex mutex;
    static ggml_backend_buffer_type types[GGML_MI355X_MAX_DEVICES];
    static mi_buft_ctx ctxs[GGML_MI355X_MAX_DEVICES];
    static bool initialized = false;
    std::lock_guard<std::mutex> lock(mutex);
    if (device < 0 || device >= device_count()) return nullptr;
    if (!initialized) {
        for (int i = 0; i < GGML_MI355X_MAX_DEVICES; i++) {
            ctxs[i] = mi_buft_ctx{i, "MI355X" + std::to_string(i)};
            types[i] = ggml_backend_buffer_type{k_mi_buft_i, &ctxs[i]};
        }
        initialized = true;
    }
    return &types[device];
}

ggml_backend_buffer_type_t ggml_backend_mi355x_host_buffer_type(void) {
    static ggml_backend_buffer_type buft = {
        {mi_host_buft_name, mi_host_buft_alloc, mi_host_buft_align, nullptr, nullptr, mi_host_buft_supports, mi_host_buft_is_host},
        nullptr,
    };
    return &buft;
}

ggml_backend_buffer_type_t ggml_backend_mi355x_split_buffer_type(const float * tensor_split) {
    // one buffer type per distinct split, kept for the process lifetime (ggml-cuda.cu:941-975);
    // tensor_split: GGML_MI355X_MAX_DEVICES proportions (all zero / null = equal rows per slot)
    static std::mutex mutex;
    static std::map<std::vector<float>, ggml_backend_buffer_type *> types;
    std::lock_guard<std::mutex> lock(mutex);
    const int n = split_slots();
    std::vector<float> cum(n, 0.0f);
    const bool all_zero = tensor_split == nullptr || std::all_of(tensor_split, tensor_split + n, [](float v) { return v == 0.0f; });
    float sum = 0.0f;
    for (int i = 0; i < n; i++) {
        cum[i] = sum;
        sum += all_zero ? 1.0f : std::max(tensor_split[i], 0.0f);
    }
    for (int i = 0; i < n; i++) cum[i] /= sum;
    auto it = types.find(cum);
    if (it != types.end()) return it->second;
    auto * buft = new ggml_backend_buffer_type{k_mi_split_buft_i, new mi_split_buft_ctx{cum}};
    types.emplace(cum, buft);
    return buft;
}

bool ggml_backend_is_mi355x(ggml_backend_t backend) {
    return backend != nullptr && ggml_guid_matches(backend->guid, mi_guid());
}

ggml_backend_t ggml_backend_mi355x_init(int device) {
    if (device < 0 || device >= device_count()) {
        fprintf(stderr, "%s: invalid device %d (have %d)\n", __func__, device, device_count());
        return nullptr;
    }
    auto * ctx = new mi_backend_ctx();
    ctx->device = device;
    ctx->name = "MI355X" + std::to_string(device);
    {
        mi_device_guard g(device);
        MI_CHECK(hipStreamCreate(&ctx->stream));
        op_tables(ctx);
    }
    auto * backend = new ggml_backend{mi_guid(), k_mi_backend_i, ctx};
    return backend;
}

void * ggml_backend_mi355x_get_stream(ggml_backend_t backend) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    return ((mi_backend_ctx *) backend->context)->stream;
}

int ggml_backend_mi355x_last_launch_count(ggml_backend_t backend) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    return ((mi_backend_ctx *) backend->context)->last_launches;
}

void ggml_backend_mi355x_set_graph_capture(ggml_backend_t backend, bool enable) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    auto * ctx = (mi_backend_ctx *) backend->context;
    ctx->graphs = enable;
    ctx->graph_fail_streak = 0;
    ctx->topo_misses.clear();  // topologies switched to direct launch get captured again
}

void ggml_backend_mi355x_set_perf(ggml_backend_t backend, bool enable) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    ((mi_backend_ctx *) backend->context)->perf = enable;
}

void ggml_backend_mi355x_graph_stats(ggml_backend_t backend, int64_t * stats4) {
    ggml_backend_mi355x_graph_stats_ex(backend, stats4, 4);
}

int ggml_backend_mi355x_graph_stats_ex(ggml_backend_t backend, int64_t * stats, int n) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    const auto * ctx = (const mi_backend_ctx *) backend->context;
    const int m = std::min(n, (int) (sizeof(ctx->graph_stats) / sizeof(ctx->graph_stats[0])));
    for (int i = 0; i < m; i++) stats[i] = ctx->graph_stats[i];
    return m;
}

bool ggml_backend_mi355x_set_tuning(const char * name, int value) {
    if (strcmp(name, "mmv_dma") == 0 && (value == 0 || (mi_diag_build() && ((value >= 1 && value <= 3) || (value >= 11 && value <= 13))))) {
        // (diagnostic builds only: measured slower than k_mmv_stream, profiles/r06h_gemv_lds_dma_ab.txt)
        g_mi_tuning.mmv_dma = value;
        return true;
    }
    if (strcmp(name, "f16_bp") == 0 && (value == 0 || (value == 1 && mi_diag_build()))) {  // (1: measured slower, diagnostic builds)
        g_mi_tuning.f16_bp = value;
        return true;
    }
    if (strcmp(name, "f16_bn") == 0 && value >= 0 && value % 10 <= 5 && value <= 15) {
        g_mi_tuning.f16_bn = value;
        return true;
    }
    if (strcmp(name, "mmv_blocks") == 0 && value >= 0) {
        g_mi_tuning.mmv_blocks = value;
        return true;
    }
    if (strcmp(name, "mmv_variant") == 0) {
        g_mi_tuning.mmv_variant = value;
        return true;
    }
    if (strcmp(name, "f16_variant") == 0) {
        g_mi_tuning.f16_variant = value;
        return true;
    }
    if (strcmp(name, "mmq_variant") == 0) {
        // the opt-in forms measured slower than the defaults (k_mmqp weight ring 4 2^19, k_mmqp
        // 64-column tiles 2^26; the k_mmf16p f32 fold behind 2^17) are compiled into diagnostic builds only
        if (!mi_diag_build() && (value & kMiMmqDiagBits)) return false;
        g_mi_tuning.mmq_variant = value;
        return true;
    }
    if (strcmp(name, "mmq_long") == 0 && (value == 0 || value == 2 || (mi_diag_build() && (value == 1 || value == 3 || value == 4 || value == 5 || (value >= 16 && value <= 24))))) {
        // 0 auto, 2 k_mmqt; diagnostic builds: 5 k_mmqt with the high half staggered, 3 k_mmqt with per-half stage synchronization, 4 k_mmqv: 1 k_mmqw for Q4_K, 16-23 k_mmqt stamps / ablations,
        // 24 k_mmqr per-step stamps
        g_mi_tuning.mmq_long = value;
        return true;
    }
    if (strcmp(name, "mmv_order") == 0 && value >= -1 && value <= 1) {
        g_mi_tuning.mmv_order = value;
        return true;
    }
    if (strcmp(name, "ord_prefill_cols") == 0 && value >= 0) {
        g_ord_prefill_cols = value;
        return true;
    }
    if (strcmp(name, "tree_prefill_cols") == 0 && value >= 0) {
        g_tree_prefill_cols = value;
        return true;
    }
    if (strcmp(name, "xfirst") == 0 && value >= -1 && value <= 1) {
        g_mi_tuning.xfirst = value;
        return true;
    }
    if (strcmp(name, "f16_nc") == 0 && value >= 0 && value <= 88 && value % 10 <= 8) {
        g_mi_tuning.f16_nc = value;
        return true;
    }
    if (strcmp(name, "planes") == 0 && value >= 0 && value <= 1) {
        g_mi_tuning.planes = value;
        return true;
    }
    if (strcmp(name, "q40r") == 0 && value >= 0 && value <= 1) {
        g_mi_tuning.q40r = value;
        return true;
    }
    if (strcmp(name, "q80r") == 0 && value >= 0 && value <= 1) {
        g_mi_tuning.q80r = value;
        return true;
    }
    if (strcmp(name, "f16_m8") == 0 && (value == 0 || (value == 1 && mi_diag_build()))) {  // (1: measured slower, diagnostic builds)
        g_mi_tuning.f16_m8 = value;
        return true;
    }
    if (strcmp(name, "f16_mt") == 0 && value >= 0 && value <= 1) {
        g_mi_tuning.f16_mt = value;
        return true;
    }
    if (strcmp(name, "mmv_pro4") == 0 && value >= 0 && value <= 1) {
        g_mi_tuning.mmv_pro4 = value;
        return true;
    }
    if (strcmp(name, "mmqt_short") == 0 && value >= 0) {
        g_mi_tuning.mmqt_short = value;
        return true;
    }
    if (strcmp(name, "f16_waves") == 0 && value >= 0) {
        g_mi_tuning.f16_waves = value;
        return true;
    }
    if (strcmp(name, "f16_norm_waves") == 0 && value >= 0 && value <= 8) {
        g_mi_tuning.f16_norm_waves = value;
        return true;
    }
    if (strcmp(name, "f16_ps_waves") == 0 && (value == 0 || value == 2 || value == 4 || value == 8)) {
        g_mi_tuning.f16_ps_waves = value;
        return true;
    }
    if (strcmp(name, "f16_rgs") == 0 && value >= 0 && value <= 8) {
        g_mi_tuning.f16_rgs = value;
        return true;
    }
    if (strcmp(name, "f16_threads") == 0 && (value == 0 || value == 64 || value == 128 || value == 256)) {
        g_mi_tuning.f16_threads = value;
        return true;
    }
    return false;
}

bool ggml_backend_mi355x_stamps_enable(size_t slots) { return mi_stamps_enable(slots); }
void ggml_backend_mi355x_stamps_reset(void) { mi_stamps_reset(); }
size_t ggml_backend_mi355x_stamps_read(uint64_t * words, size_t n, char * log, size_t log_size) {
    return mi_stamps_read(words, n, log, log_size);
}

size_t ggml_backend_mi355x_planes_stats(size_t * bytes) {
    if (bytes) *bytes = mi_planes_bytes();
    return mi_planes_count();
}

bool ggml_backend_mi355x_quantize_activations(ggml_backend_t backend, int vec_dot_type, const float * x, int64_t K,
                                              int64_t ncols, int8_t * qs, float * d, int16_t * s32) {
    MI_ASSERT(ggml_backend_is_mi355x(backend));
    const bool is_k = vec_dot_type == GGML_TYPE_Q8_K;
    if (!is_k && vec_dot_type != GGML_TYPE_Q8_0) return false;
    if (K % (is_k ? 256 : 32) != 0) return false;
    auto * ctx = (mi_backend_ctx *) backend->context;
    mi_device_guard g(ctx->device);
    const size_t xbytes = (size_t) K * ncols * sizeof(float);
    void * dx = nullptr;
    void * dq = nullptr;
    MI_CHECK(hipMalloc(&dx, xbytes));
    MI_CHECK(hipMalloc(&dq, mi_act_q8_bytes(K, ncols, is_k)));
    MI_CHECK(hipMemcpy(dx, x, xbytes, hipMemcpyHostToDevice));
    mi_src_cols src;
    src.base = (const char *) dx;
    src.ne1 = ncols;
    src.ne2 = src.ne3 = 1;
    src.nb1 = (size_t) K * sizeof(float);
    src.nb2 = src.nb3 = src.nb1 * ncols;
    const mi_act_q8 act = mi_act_q8_carve(dq, K, ncols, is_k);
    if (is_k) mi_quantize_q8_K(src, K, act, ctx->stream);
    else mi_quantize_q8_0(src, K, act, ctx->stream);
    MI_CHECK(hipStreamSynchronize(ctx->stream));
    MI_CHECK(hipMemcpy(qs, act.qs, (size_t) K * ncols, hipMemcpyDeviceToHost));
    MI_CHECK(hipMemcpy(d, act.d, (size_t) (K / (is_k ? 256 : 32)) * ncols * sizeof(float), hipMemcpyDeviceToHost));
    if (is_k && s32) MI_CHECK(hipMemcpy(s32, act.s32, (size_t) (K / 32) * ncols * sizeof(int16_t), hipMemcpyDeviceToHost));
    MI_CHECK(hipFree(dx));
    MI_CHECK(hipFree(dq));
    return true;
}

static ggml_backend_t mi_reg_init(const char * params, void * user_data) {
    (void) params;
    return ggml_backend_mi355x_init((int) (intptr_t) user_data);
}

int ggml_backend_mi355x_reg_devices(void) {
    static int registered = -1;
    if (registered >= 0) return registered;
    const int n = device_count();
    for (int i = 0; i < n; i++) {
        char name[128];
        snprintf(name, sizeof(name), "MI355X%d", i);
        ggml_backend_register(name, mi_reg_init, ggml_backend_mi355x_buffer_type(i), (void *) (intptr_t) i);
    }
    registered = n;
    return n;
}

} // extern "C"

// Plugging into the reference libggml (whose registry only knows the backends compiled into
// it, ggml-backend.c:417-450): with GGML_MI355X_AUTOREGISTER=1 the library registers its
// devices when loaded (e.g. LD_PRELOAD into the unmodified test-backend-ops). The reference
// registers its CPU entry on the first ggml_backend_reg_get_count() call, which keeps CPU at
// index 0 as there. The repo's own runtime instead looks this library up lazily on its first
// registry query (csrc/core/ggml_backend_rt.cpp), so loading it never touches the GPU.
__attribute__((constructor)) static void mi_autoregister(void) {
    const char * env = getenv("GGML_MI355X_AUTOREGISTER");
    if (!env || atoi(env) == 0) return;
    (void) ggml_backend_reg_get_count();
    ggml_backend_mi355x_reg_devices();
}
