// ggml_backend_rt.cpp -- the backend plumbing every device backend plugs into:
// buffer-type / buffer / backend dispatch wrappers, tensor copies, events, the backend
// registry and a host (pageable) buffer type. Mirrors src/ggml-backend.c:15-996 of the
// reference (NAIST-Archlab/ggml-imax @ v2); the vtable layouts are in include/ggml_abi.h.

#include "ggml_abi.h"

#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <vector>

extern "C" {

// ---- buffer type (ggml-backend.c:15-55) ------------------------------------------------------

const char * ggml_backend_buft_name(ggml_backend_buffer_type_t buft) { return buft->iface.get_name(buft); }

ggml_backend_buffer_t ggml_backend_buft_alloc_buffer(ggml_backend_buffer_type_t buft, size_t size) {
    return buft->iface.alloc_buffer(buft, size);
}

size_t ggml_backend_buft_get_alignment(ggml_backend_buffer_type_t buft) { return buft->iface.get_alignment(buft); }

size_t ggml_backend_buft_get_max_size(ggml_backend_buffer_type_t buft) {
    return buft->iface.get_max_size ? buft->iface.get_max_size(buft) : SIZE_MAX;
}

size_t ggml_backend_buft_get_alloc_size(ggml_backend_buffer_type_t buft, struct ggml_tensor * tensor) {
    if (buft->iface.get_alloc_size) {
        const size_t size = buft->iface.get_alloc_size(buft, tensor);
        GGML_ASSERT(size >= ggml_nbytes(tensor));
        return size;
    }
    return ggml_nbytes(tensor);
}

bool ggml_backend_buft_supports_backend(ggml_backend_buffer_type_t buft, ggml_backend_t backend) {
    return buft->iface.supports_backend(buft, backend);
}

bool ggml_backend_buft_is_host(ggml_backend_buffer_type_t buft) {
    return buft->iface.is_host ? buft->iface.is_host(buft) : false;
}

// ---- buffer (ggml-backend.c:57-160) ----------------------------------------------------------

ggml_backend_buffer_t ggml_backend_buffer_init(ggml_backend_buffer_type_t buft, struct ggml_backend_buffer_i iface,
                                               ggml_backend_buffer_context_t context, size_t size) {
    auto * b = (ggml_backend_buffer *) malloc(sizeof(ggml_backend_buffer));
    b->iface = iface;
    b->buft = buft;
    b->context = context;
    b->size = size;
    b->usage = GGML_BACKEND_BUFFER_USAGE_ANY;
    return b;
}

const char * ggml_backend_buffer_name(ggml_backend_buffer_t buffer) { return buffer->iface.get_name(buffer); }

void ggml_backend_buffer_free(ggml_backend_buffer_t buffer) {
    if (!buffer) return;
    if (buffer->iface.free_buffer) buffer->iface.free_buffer(buffer);
    free(buffer);
}

size_t ggml_backend_buffer_get_size(ggml_backend_buffer_t buffer) { return buffer->size; }

void * ggml_backend_buffer_get_base(ggml_backend_buffer_t buffer) {
    void * base = buffer->iface.get_base(buffer);
    GGML_ASSERT(base != NULL && "backend buffer base cannot be NULL");
    return base;
}

void ggml_backend_buffer_init_tensor(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor) {
    if (buffer->iface.init_tensor) buffer->iface.init_tensor(buffer, tensor);
}

ggml_backend_buffer_type_t ggml_backend_buffer_get_type(ggml_backend_buffer_t buffer) { return buffer->buft; }
size_t ggml_backend_buffer_get_alignment(ggml_backend_buffer_t buffer) { return ggml_backend_buft_get_alignment(buffer->buft); }
size_t ggml_backend_buffer_get_max_size(ggml_backend_buffer_t buffer) { return ggml_backend_buft_get_max_size(buffer->buft); }

size_t ggml_backend_buffer_get_alloc_size(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor) {
    return ggml_backend_buft_get_alloc_size(buffer->buft, tensor);
}

void ggml_backend_buffer_clear(ggml_backend_buffer_t buffer, uint8_t value) { buffer->iface.clear(buffer, value); }
bool ggml_backend_buffer_is_host(ggml_backend_buffer_t buffer) { return ggml_backend_buft_is_host(buffer->buft); }

void ggml_backend_buffer_set_usage(ggml_backend_buffer_t buffer, enum ggml_backend_buffer_usage usage) {
    buffer->usage = usage;
    if (ggml_backend_buffer_is_multi_buffer(buffer)) ggml_backend_multi_buffer_set_usage(buffer, usage);
}

void ggml_backend_buffer_reset(ggml_backend_buffer_t buffer) {
    if (buffer->iface.reset) buffer->iface.reset(buffer);
}

bool ggml_backend_buffer_copy_tensor(const struct ggml_tensor * src, struct ggml_tensor * dst) {
    ggml_backend_buffer_t dst_buf = dst->view_src ? dst->view_src->buffer : dst->buffer;
    if (dst_buf->iface.cpy_tensor) return dst_buf->iface.cpy_tensor(dst_buf, src, dst);
    return false;
}

// ---- backend (ggml-backend.c:162-300) --------------------------------------------------------

ggml_guid_t ggml_backend_guid(ggml_backend_t backend) { return backend ? backend->guid : nullptr; }
const char * ggml_backend_name(ggml_backend_t backend) { return backend ? backend->iface.get_name(backend) : "NULL"; }

void ggml_backend_free(ggml_backend_t backend) {
    if (backend) backend->iface.free(backend);
}

ggml_backend_buffer_type_t ggml_backend_get_default_buffer_type(ggml_backend_t backend) {
    return backend->iface.get_default_buffer_type(backend);
}

ggml_backend_buffer_t ggml_backend_alloc_buffer(ggml_backend_t backend, size_t size) {
    return ggml_backend_buft_alloc_buffer(ggml_backend_get_default_buffer_type(backend), size);
}

size_t ggml_backend_get_alignment(ggml_backend_t backend) { return ggml_backend_buft_get_alignment(ggml_backend_get_default_buffer_type(backend)); }
size_t ggml_backend_get_max_size(ggml_backend_t backend) { return ggml_backend_buft_get_max_size(ggml_backend_get_default_buffer_type(backend)); }

void ggml_backend_tensor_set_async(ggml_backend_t backend, struct ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    GGML_ASSERT(tensor->data != NULL && "tensor not allocated");
    GGML_ASSERT(offset + size <= ggml_nbytes(tensor) && "tensor write out of bounds");
    if (backend->iface.set_tensor_async == NULL) ggml_backend_tensor_set(tensor, data, offset, size);
    else backend->iface.set_tensor_async(backend, tensor, data, offset, size);
}

void ggml_backend_tensor_get_async(ggml_backend_t backend, const struct ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    GGML_ASSERT(tensor->data != NULL && "tensor not allocated");
    GGML_ASSERT(offset + size <= ggml_nbytes(tensor) && "tensor read out of bounds");
    if (backend->iface.get_tensor_async == NULL) ggml_backend_tensor_get(tensor, data, offset, size);
    else backend->iface.get_tensor_async(backend, tensor, data, offset, size);
}

void ggml_backend_tensor_set(struct ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    ggml_backend_buffer_t buf = tensor->view_src ? tensor->view_src->buffer : tensor->buffer;
    GGML_ASSERT(buf != NULL && "tensor buffer not set");
    GGML_ASSERT(tensor->data != NULL && "tensor not allocated");
    GGML_ASSERT(offset + size <= ggml_nbytes(tensor) && "tensor write out of bounds");
    if (!size) return;
    buf->iface.set_tensor(buf, tensor, data, offset, size);
}

void ggml_backend_tensor_get(const struct ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    ggml_backend_buffer_t buf = tensor->view_src ? tensor->view_src->buffer : tensor->buffer;
    GGML_ASSERT(buf != NULL && "tensor buffer not set");
    GGML_ASSERT(tensor->data != NULL && "tensor not allocated");
    GGML_ASSERT(offset + size <= ggml_nbytes(tensor) && "tensor read out of bounds");
    if (!size) return;
    buf->iface.get_tensor(buf, tensor, data, offset, size);
}

void ggml_backend_synchronize(ggml_backend_t backend) {
    if (backend->iface.synchronize) backend->iface.synchronize(backend);
}

ggml_backend_graph_plan_t ggml_backend_graph_plan_create(ggml_backend_t backend, struct ggml_cgraph * cgraph) {
    GGML_ASSERT(backend->iface.graph_plan_create != NULL);
    return backend->iface.graph_plan_create(backend, cgraph);
}

void ggml_backend_graph_plan_free(ggml_backend_t backend, ggml_backend_graph_plan_t plan) {
    GGML_ASSERT(backend->iface.graph_plan_free != NULL);
    backend->iface.graph_plan_free(backend, plan);
}

enum ggml_status ggml_backend_graph_plan_compute(ggml_backend_t backend, ggml_backend_graph_plan_t plan) {
    GGML_ASSERT(backend->iface.graph_plan_compute != NULL);
    return backend->iface.graph_plan_compute(backend, plan);
}

// ggml-backend.c:275-283: compute = async compute + synchronize
enum ggml_status ggml_backend_graph_compute(ggml_backend_t backend, struct ggml_cgraph * cgraph) {
    const enum ggml_status err = ggml_backend_graph_compute_async(backend, cgraph);
    ggml_backend_synchronize(backend);
    return err;
}

enum ggml_status ggml_backend_graph_compute_async(ggml_backend_t backend, struct ggml_cgraph * cgraph) {
    return backend->iface.graph_compute(backend, cgraph);
}

bool ggml_backend_supports_op(ggml_backend_t backend, const struct ggml_tensor * op) { return backend->iface.supports_op(backend, op); }

bool ggml_backend_offload_op(ggml_backend_t backend, const struct ggml_tensor * op) {
    return backend->iface.offload_op ? backend->iface.offload_op(backend, op) : false;
}

// ---- copies (ggml-backend.c:302-359) ---------------------------------------------------------

static bool layout_equal(const ggml_tensor * a, const ggml_tensor * b) {
    if (a->type != b->type) return false;
    for (int i = 0; i < GGML_MAX_DIMS; i++) {
        if (a->ne[i] != b->ne[i] || a->nb[i] != b->nb[i]) return false;
    }
    return true;
}

void ggml_backend_tensor_copy(struct ggml_tensor * src, struct ggml_tensor * dst) {
    GGML_ASSERT(layout_equal(src, dst) && "cannot copy tensors with different layouts");
    if (src == dst) return;
    if (ggml_backend_buffer_is_host(src->buffer)) {
        ggml_backend_tensor_set(dst, src->data, 0, ggml_nbytes(src));
    } else if (ggml_backend_buffer_is_host(dst->buffer)) {
        ggml_backend_tensor_get(src, dst->data, 0, ggml_nbytes(src));
    } else if (!ggml_backend_buffer_copy_tensor(src, dst)) {
        std::vector<uint8_t> staging(ggml_nbytes(src));
        ggml_backend_tensor_get(src, staging.data(), 0, staging.size());
        ggml_backend_tensor_set(dst, staging.data(), 0, staging.size());
    }
}

void ggml_backend_tensor_copy_async(ggml_backend_t backend_src, ggml_backend_t backend_dst, struct ggml_tensor * src, struct ggml_tensor * dst) {
    GGML_ASSERT(layout_equal(src, dst) && "cannot copy tensors with different layouts");
    if (src == dst) return;
    if (backend_dst->iface.cpy_tensor_async != NULL && backend_dst->iface.cpy_tensor_async(backend_src, backend_dst, src, dst)) return;
    // a host-side endpoint can be copied asynchronously by the device side, otherwise sync
    if (ggml_backend_buffer_is_host(src->buffer)) {
        ggml_backend_tensor_set_async(backend_dst, dst, src->data, 0, ggml_nbytes(src));
    } else {
        ggml_backend_synchronize(backend_src);
        ggml_backend_tensor_copy(src, dst);
        ggml_backend_synchronize(backend_dst);
    }
}

// ---- events (ggml-backend.c:363-393) ---------------------------------------------------------

ggml_backend_event_t ggml_backend_event_new(ggml_backend_t backend) {
    return backend->iface.event_new ? backend->iface.event_new(backend) : nullptr;
}

void ggml_backend_event_free(ggml_backend_event_t event) {
    if (event) event->backend->iface.event_free(event);
}

void ggml_backend_event_record(ggml_backend_event_t event) {
    GGML_ASSERT(event->backend->iface.event_record != NULL);
    event->backend->iface.event_record(event);
}

void ggml_backend_event_synchronize(ggml_backend_event_t event) {
    GGML_ASSERT(event->backend->iface.event_synchronize != NULL);
    event->backend->iface.event_synchronize(event);
}

void ggml_backend_event_wait(ggml_backend_t backend, ggml_backend_event_t event) {
    GGML_ASSERT(backend->iface.event_wait != NULL);
    backend->iface.event_wait(backend, event);
}

// ---- tensor placement (ggml-backend.c:1888-1913) ---------------------------------------------

void ggml_backend_tensor_alloc(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor, void * addr) {
    GGML_ASSERT(tensor->buffer == NULL);
    GGML_ASSERT(tensor->data == NULL);
    GGML_ASSERT(tensor->view_src == NULL);
    GGML_ASSERT(addr >= ggml_backend_buffer_get_base(buffer));
    GGML_ASSERT((char *) addr + ggml_backend_buffer_get_alloc_size(buffer, tensor) <=
                (char *) ggml_backend_buffer_get_base(buffer) + ggml_backend_buffer_get_size(buffer));
    tensor->buffer = buffer;
    tensor->data = addr;
    ggml_backend_buffer_init_tensor(buffer, tensor);
}

void ggml_backend_view_init(ggml_backend_buffer_t buffer, struct ggml_tensor * tensor) {
    GGML_ASSERT(tensor->buffer == NULL);
    GGML_ASSERT(tensor->view_src != NULL);
    GGML_ASSERT(tensor->view_src->buffer != NULL);
    GGML_ASSERT(tensor->view_src->data != NULL);
    tensor->buffer = buffer;
    tensor->data = (char *) tensor->view_src->data + tensor->view_offs;
    tensor->backend = tensor->view_src->backend;
    ggml_backend_buffer_init_tensor(buffer, tensor);
}

// ---- host buffer type (no compute: CPU-side staging / outputs) -------------------------------

static const char * host_buffer_name(ggml_backend_buffer_t) { return "Host"; }
static void * host_buffer_base(ggml_backend_buffer_t b) { return b->context; }
static void host_buffer_free(ggml_backend_buffer_t b) { free(b->context); }
static void host_buffer_set(ggml_backend_buffer_t, ggml_tensor * t, const void * data, size_t off, size_t size) {
    memcpy((char *) t->data + off, data, size);
}
static void host_buffer_get(ggml_backend_buffer_t, const ggml_tensor * t, void * data, size_t off, size_t size) {
    memcpy(data, (const char *) t->data + off, size);
}
static bool host_buffer_cpy(ggml_backend_buffer_t, const ggml_tensor * src, ggml_tensor * dst) {
    if (src->buffer && ggml_backend_buffer_is_host(src->buffer)) {
        memcpy(dst->data, src->data, ggml_nbytes(src));
        return true;
    }
    return false;
}
static void host_buffer_clear(ggml_backend_buffer_t b, uint8_t v) { memset(b->context, v, b->size); }

static const ggml_backend_buffer_i k_host_buffer_i = {
    host_buffer_name, host_buffer_free, host_buffer_base, nullptr, host_buffer_set, host_buffer_get,
    host_buffer_cpy, host_buffer_clear, nullptr,
};

static const ggml_backend_buffer_i k_host_buffer_from_ptr_i = {
    host_buffer_name, nullptr, host_buffer_base, nullptr, host_buffer_set, host_buffer_get,
    host_buffer_cpy, host_buffer_clear, nullptr,
};

static const char * host_buft_name(ggml_backend_buffer_type_t) { return "Host"; }

static ggml_backend_buffer_t host_buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    void * p = aligned_alloc(64, GGML_PAD(size ? size : 1, 64));
    if (!p) return nullptr;
    return ggml_backend_buffer_init(buft, k_host_buffer_i, p, size);
}

static size_t host_buft_align(ggml_backend_buffer_type_t) { return 32; }
static bool host_buft_supports(ggml_backend_buffer_type_t, ggml_backend_t) { return false; }
static bool host_buft_is_host(ggml_backend_buffer_type_t) { return true; }

ggml_backend_buffer_type_t ggml_backend_cpu_buffer_type(void) {
    static ggml_backend_buffer_type buft = {
        {host_buft_name, host_buft_alloc, host_buft_align, nullptr, nullptr, host_buft_supports, host_buft_is_host},
        nullptr,
    };
    return &buft;
}

ggml_backend_buffer_t ggml_backend_cpu_buffer_from_ptr(void * ptr, size_t size) {
    GGML_ASSERT(((uintptr_t) ptr % 32) == 0 && "buffer pointer must be aligned");
    return ggml_backend_buffer_init(ggml_backend_cpu_buffer_type(), k_host_buffer_from_ptr_i, ptr, size);
}

// ---- multi-buffer (ggml-backend.c:922-996) ---------------------------------------------------

struct multi_buffer_ctx {
    std::vector<ggml_backend_buffer_t> buffers;
};

static const char * multi_name(ggml_backend_buffer_t b) {
    return ((multi_buffer_ctx *) b->context)->buffers[0]->iface.get_name(((multi_buffer_ctx *) b->context)->buffers[0]);
}
static void multi_free(ggml_backend_buffer_t b) {
    auto * ctx = (multi_buffer_ctx *) b->context;
    for (auto * sub : ctx->buffers) ggml_backend_buffer_free(sub);
    delete ctx;
}
static void multi_clear(ggml_backend_buffer_t b, uint8_t v) {
    for (auto * sub : ((multi_buffer_ctx *) b->context)->buffers) ggml_backend_buffer_clear(sub, v);
}

static const ggml_backend_buffer_i k_multi_buffer_i = {
    multi_name, multi_free, nullptr, nullptr, nullptr, nullptr, nullptr, multi_clear, nullptr,
};

ggml_backend_buffer_t ggml_backend_multi_buffer_alloc_buffer(ggml_backend_buffer_t * buffers, size_t n_buffers) {
    auto * ctx = new multi_buffer_ctx();
    size_t total = 0;
    for (size_t i = 0; i < n_buffers; i++) {
        ctx->buffers.push_back(buffers[i]);
        total += ggml_backend_buffer_get_size(buffers[i]);
    }
    return ggml_backend_buffer_init(buffers[0]->buft, k_multi_buffer_i, ctx, total);
}

bool ggml_backend_buffer_is_multi_buffer(ggml_backend_buffer_t buffer) { return buffer->iface.get_name == multi_name; }

void ggml_backend_multi_buffer_set_usage(ggml_backend_buffer_t buffer, enum ggml_backend_buffer_usage usage) {
    GGML_ASSERT(ggml_backend_buffer_is_multi_buffer(buffer));
    for (auto * sub : ((multi_buffer_ctx *) buffer->context)->buffers) ggml_backend_buffer_set_usage(sub, usage);
}

// ---- registry (ggml-backend.c:395-541) -------------------------------------------------------

namespace {
struct reg_entry {
    char name[128];
    ggml_backend_init_fn init_fn;
    ggml_backend_buffer_type_t default_buffer_type;
    void * user_data;
};
reg_entry g_registry[16];
size_t g_registry_count = 0;
std::recursive_mutex g_registry_mutex;
}

// Analogue of ggml_backend_registry_init (ggml-backend.c:417-450), which calls the compiled-in
// backends' reg_devices(). Here backends are separate libraries: on the first registry query
// every loaded device backend that exports a reg_devices entry point registers itself. There
// is no CPU compute backend in this runtime.
static void registry_init(void) {
    static std::once_flag once;
    std::call_once(once, [] {
        typedef int (*reg_fn)(void);
        static const char * const k_backends[] = {"ggml_backend_mi355x_reg_devices"};
        for (const char * sym : k_backends) {
            if (auto fn = (reg_fn) dlsym(RTLD_DEFAULT, sym)) fn();
        }
    });
}

void ggml_backend_register(const char * name, ggml_backend_init_fn init_fn, ggml_backend_buffer_type_t default_buffer_type, void * user_data) {
    std::lock_guard<std::recursive_mutex> lock(g_registry_mutex);
    GGML_ASSERT(g_registry_count < 16);
    reg_entry & e = g_registry[g_registry_count++];
    snprintf(e.name, sizeof(e.name), "%s", name);
    e.init_fn = init_fn;
    e.default_buffer_type = default_buffer_type;
    e.user_data = user_data;
}

size_t ggml_backend_reg_get_count(void) {
    registry_init();
    return g_registry_count;
}

size_t ggml_backend_reg_find_by_name(const char * name) {
    registry_init();
    for (size_t i = 0; i < g_registry_count; i++) if (strcmp(g_registry[i].name, name) == 0) return i;
    return SIZE_MAX;
}

ggml_backend_t ggml_backend_reg_init_backend_from_str(const char * backend_str) {
    const char * params = strchr(backend_str, ':');
    char name[128];
    if (!params) {
        snprintf(name, sizeof(name), "%s", backend_str);
        params = "";
    } else {
        snprintf(name, sizeof(name), "%.*s", (int) (params - backend_str), backend_str);
        params++;
    }
    const size_t i = ggml_backend_reg_find_by_name(name);
    if (i == SIZE_MAX) {
        fprintf(stderr, "%s: backend %s not found\n", __func__, name);
        return nullptr;
    }
    return ggml_backend_reg_init_backend(i, params);
}

const char * ggml_backend_reg_get_name(size_t i) {
    registry_init();
    GGML_ASSERT(i < g_registry_count);
    return g_registry[i].name;
}

ggml_backend_t ggml_backend_reg_init_backend(size_t i, const char * params) {
    registry_init();
    GGML_ASSERT(i < g_registry_count);
    return g_registry[i].init_fn(params, g_registry[i].user_data);
}

ggml_backend_buffer_type_t ggml_backend_reg_get_default_buffer_type(size_t i) {
    registry_init();
    GGML_ASSERT(i < g_registry_count);
    return g_registry[i].default_buffer_type;
}

ggml_backend_buffer_t ggml_backend_reg_alloc_buffer(size_t i, size_t size) {
    registry_init();
    GGML_ASSERT(i < g_registry_count);
    return ggml_backend_buft_alloc_buffer(g_registry[i].default_buffer_type, size);
}

} // extern "C"
