// gguf.cpp -- GGUF v3 model files: the reference's gguf_* API (include/ggml/ggml.h:2247-2380,
// src/ggml.c:21671-22866) re-implemented over C++ containers.
//
// On disk (little endian): "GGUF", u32 version, u64 n_tensors, u64 n_kv; n_kv key/values
// (string key = u64 length + bytes, i32 type, value; arrays = i32 element type, u64 count,
// elements); n_tensors tensor infos (name, u32 n_dims, i64 ne[n_dims], i32 ggml_type, u64 offset
// into the data section); zero padding to `general.alignment` (u32, default 32); the data
// section, every tensor padded to the alignment. Files written here are byte-identical to the
// reference's for the same calls (tests/test_gguf.py). Loading maps the data section into one
// I8 tensor of a new ggml_context (or, with no_alloc, creates metadata-only tensors to be
// placed in a backend buffer -- the MI355X path, ggml_mi355x/gguf.py).
//
// Error behaviour: malformed files make gguf_init_from_file print a message and return NULL,
// as the reference does for I/O and header errors; where the reference asserts on a malformed
// file (unknown value type, bad tensor dims/type) this returns NULL too. API misuse (wrong
// getter type, bad key id, duplicate tensor name) aborts with GGML_ASSERT like the reference.

#include "ggml_abi.h"

#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

// the reference's in-memory string layout (struct gguf_str), exposed through gguf_get_arr_data
// for string arrays
struct str_view {
    uint64_t n;
    char * data;
};

size_t scalar_size(int t) {
    switch (t) {
        case GGUF_TYPE_UINT8: case GGUF_TYPE_INT8: case GGUF_TYPE_BOOL: return 1;
        case GGUF_TYPE_UINT16: case GGUF_TYPE_INT16: return 2;
        case GGUF_TYPE_UINT32: case GGUF_TYPE_INT32: case GGUF_TYPE_FLOAT32: return 4;
        case GGUF_TYPE_UINT64: case GGUF_TYPE_INT64: case GGUF_TYPE_FLOAT64: return 8;
        default: return 0;  // string, array: not fixed-size
    }
}

const char * const kTypeNames[GGUF_TYPE_COUNT] = {"u8", "i8", "u16", "i16", "u32", "i32", "f32",
                                                  "bool", "str", "arr", "u64", "i64", "f64"};

struct kv_entry {
    std::string key;
    int32_t type = GGUF_TYPE_UINT8;
    union {
        uint8_t u8;
        int8_t i8;
        uint16_t u16;
        int16_t i16;
        uint32_t u32;
        int32_t i32;
        float f32;
        uint64_t u64;
        int64_t i64;
        double f64;
        bool b;
        unsigned char bytes[8];
    } num{};
    std::string str;
    // arrays
    int32_t arr_type = GGUF_TYPE_UINT8;
    uint64_t arr_n = 0;
    std::vector<uint8_t> raw;        // fixed-size elements
    std::vector<std::string> strs;   // string elements
    std::vector<str_view> views;     // reference-layout view of strs

    void set_strings(std::vector<std::string> v) {
        strs = std::move(v);
        views.resize(strs.size());
        for (size_t i = 0; i < strs.size(); i++) views[i] = {strs[i].size(), &strs[i][0]};
    }
};

struct tensor_info {
    std::string name;
    uint32_t n_dims = 0;
    int64_t ne[GGML_MAX_DIMS] = {1, 1, 1, 1};
    int32_t type = GGML_TYPE_F32;
    uint64_t offset = 0;    // from the start of the data section
    const void * data = nullptr;  // writing API
    size_t size = 0;
};

// sequential little-endian reader with the file offset and the bytes left
struct reader {
    FILE * f;
    size_t offset = 0;
    size_t file_size = 0;

    bool bytes(void * dst, size_t n) {
        const size_t got = fread(dst, 1, n, f);
        offset += got;
        return got == n;
    }
    template <class T> bool el(T & v) { return bytes(&v, sizeof(T)); }
    size_t left() const { return file_size > offset ? file_size - offset : 0; }
    bool str(std::string & s) {
        uint64_t n = 0;
        if (!el(n) || n > left()) return false;
        s.resize(n);
        return n == 0 || bytes(&s[0], n);
    }
};

// byte sink: append to a vector, or only count (gguf_get_meta_size)
struct writer {
    std::vector<uint8_t> * out;
    size_t n = 0;
    void bytes(const void * p, size_t k) {
        if (out) out->insert(out->end(), (const uint8_t *) p, (const uint8_t *) p + k);
        n += k;
    }
    template <class T> void el(const T & v) { bytes(&v, sizeof(T)); }
    void str(const std::string & s) {
        el((uint64_t) s.size());
        bytes(s.data(), s.size());
    }
    void zeros(size_t k) {
        static const uint8_t z[64] = {};
        while (k) {
            const size_t c = k < sizeof(z) ? k : sizeof(z);
            bytes(z, c);
            k -= c;
        }
    }
};

} // namespace

struct gguf_context {
    uint32_t version = GGUF_VERSION;
    std::vector<std::unique_ptr<kv_entry>> kv;        // stable addresses for returned strings
    std::vector<std::unique_ptr<tensor_info>> infos;
    size_t alignment = GGUF_DEFAULT_ALIGNMENT;
    size_t offset = 0;   // file offset of the data section
    size_t size = 0;     // size of the data section
    void * data = nullptr;

    kv_entry & at(int key_id) const {
        GGML_ASSERT(key_id >= 0 && key_id < (int) kv.size());
        return *kv[key_id];
    }
    kv_entry & get_or_add(const char * key) {
        const int i = gguf_find_key(this, key);
        if (i >= 0) {
            // the reference overwrites in place; drop any previous payload
            kv_entry & e = *kv[i];
            e.str.clear();
            e.raw.clear();
            e.strs.clear();
            e.views.clear();
            e.arr_n = 0;
            return e;
        }
        kv.emplace_back(new kv_entry);
        kv.back()->key = key;
        return *kv.back();
    }
};

namespace {

bool read_value(reader & r, kv_entry & e) {
    if (e.type == GGUF_TYPE_STRING) return r.str(e.str);
    if (e.type == GGUF_TYPE_ARRAY) {
        if (!r.el(e.arr_type) || !r.el(e.arr_n)) return false;
        if (e.arr_type == GGUF_TYPE_STRING) {
            if (e.arr_n > r.left() / 8) return false;  // every element holds at least its length
            std::vector<std::string> v(e.arr_n);
            for (auto & s : v)
                if (!r.str(s)) return false;
            e.set_strings(std::move(v));
            return true;
        }
        const size_t es = scalar_size(e.arr_type);
        if (es == 0) {
            fprintf(stderr, "gguf_init_from_file: invalid array element type %d\n", e.arr_type);
            return false;
        }
        if (e.arr_n > r.left() / es) {
            fprintf(stderr, "gguf_init_from_file: array size is too large (%" PRIu64 ")\n", e.arr_n);
            return false;
        }
        e.raw.resize(e.arr_n * es);
        return e.raw.empty() || r.bytes(e.raw.data(), e.raw.size());
    }
    const size_t es = scalar_size(e.type);
    if (es == 0) {
        fprintf(stderr, "gguf_init_from_file: invalid value type %d\n", e.type);
        return false;
    }
    return r.bytes(e.num.bytes, es);
}

void write_meta(const gguf_context * ctx, writer & w) {
    w.bytes(GGUF_MAGIC, 4);
    w.el(ctx->version);
    w.el((uint64_t) ctx->infos.size());
    w.el((uint64_t) ctx->kv.size());
    for (const auto & p : ctx->kv) {
        const kv_entry & e = *p;
        w.str(e.key);
        w.el(e.type);
        if (e.type == GGUF_TYPE_STRING) {
            w.str(e.str);
        } else if (e.type == GGUF_TYPE_ARRAY) {
            w.el(e.arr_type);
            w.el(e.arr_n);
            if (e.arr_type == GGUF_TYPE_STRING) {
                for (const auto & s : e.strs) w.str(s);
            } else {
                GGML_ASSERT(scalar_size(e.arr_type) != 0 && "invalid type");
                w.bytes(e.raw.data(), e.raw.size());
            }
        } else {
            GGML_ASSERT(scalar_size(e.type) != 0 && "invalid type");
            w.bytes(e.num.bytes, scalar_size(e.type));
        }
    }
    for (const auto & p : ctx->infos) {
        const tensor_info & t = *p;
        w.str(t.name);
        w.el(t.n_dims);
        for (uint32_t j = 0; j < t.n_dims; j++) w.el(t.ne[j]);
        w.el(t.type);
        w.el(t.offset);
    }
    w.zeros(GGML_PAD(w.n, ctx->alignment) - w.n);
}

void update_offsets(gguf_context * ctx, size_t from) {
    for (size_t i = from; i < ctx->infos.size(); i++) {
        const tensor_info & prev = *ctx->infos[i - 1];
        ctx->infos[i]->offset = prev.offset + GGML_PAD(prev.size, ctx->alignment);
    }
}

} // namespace

extern "C" {

struct gguf_context * gguf_init_empty(void) { return new gguf_context; }

void gguf_free(struct gguf_context * ctx) { delete ctx; }

struct gguf_context * gguf_init_from_file(const char * fname, struct gguf_init_params params) {
    FILE * f = fopen(fname, "rb");
    if (!f) return nullptr;
    reader r{f};
    fseek(f, 0, SEEK_END);
    r.file_size = (size_t) ftell(f);
    fseek(f, 0, SEEK_SET);
    auto fail = [&](const char * what) -> gguf_context * {
        if (what) fprintf(stderr, "gguf_init_from_file: %s\n", what);
        fclose(f);
        return nullptr;
    };

    char magic[4] = {0, 0, 0, 0};
    r.bytes(magic, 4);
    if (memcmp(magic, GGUF_MAGIC, 4) != 0) {
        fprintf(stderr, "gguf_init_from_file: invalid magic characters '%c%c%c%c'\n", magic[0], magic[1], magic[2], magic[3]);
        return fail(nullptr);
    }
    std::unique_ptr<gguf_context> ctx(new gguf_context);
    uint64_t n_tensors = 0, n_kv = 0;
    if (!r.el(ctx->version) || !r.el(n_tensors) || !r.el(n_kv)) return fail("failed to read header");
    if (ctx->version == 1) return fail("GGUFv1 is no longer supported. please use a more up-to-date version");
    // every kv holds >= 12 bytes and every tensor info >= 24: bounds the allocations below
    if (n_kv > r.left() / 12 || n_tensors > r.left() / 24) return fail("failed to read header");

    for (uint64_t i = 0; i < n_kv; i++) {
        std::unique_ptr<kv_entry> e(new kv_entry);
        if (!r.str(e->key) || !r.el(e->type) || !read_value(r, *e)) return fail("failed to read key-value pairs");
        ctx->kv.push_back(std::move(e));
    }

    for (uint64_t i = 0; i < n_tensors; i++) {
        std::unique_ptr<tensor_info> t(new tensor_info);
        bool ok = r.str(t->name) && r.el(t->n_dims) && t->n_dims <= GGML_MAX_DIMS;
        for (uint32_t j = 0; ok && j < t->n_dims; j++) ok = r.el(t->ne[j]) && t->ne[j] > 0;
        ok = ok && r.el(t->type) && r.el(t->offset) && t->type >= 0 && t->type < GGML_TYPE_COUNT;
        // element count must not overflow int64
        ok = ok && INT64_MAX / t->ne[1] > t->ne[0] && INT64_MAX / t->ne[2] > t->ne[0] * t->ne[1] &&
             INT64_MAX / t->ne[3] > t->ne[0] * t->ne[1] * t->ne[2];
        if (ok && gguf_find_tensor(ctx.get(), t->name.c_str()) >= 0) {
            fprintf(stderr, "gguf_init_from_file: duplicated tensor name %s\n", t->name.c_str());
            ok = false;
        }
        if (!ok) return fail("failed to read tensor info");
        ctx->infos.push_back(std::move(t));
    }

    const int ai = gguf_find_key(ctx.get(), "general.alignment");
    if (ai >= 0) {
        if (ctx->kv[ai]->type != GGUF_TYPE_UINT32) return fail("general.alignment is not a u32");
        ctx->alignment = ctx->kv[ai]->num.u32;
        if (ctx->alignment == 0 || (ctx->alignment & (ctx->alignment - 1)) != 0) return fail("general.alignment is not a power of 2");
    }

    // the data section starts at the next multiple of the alignment
    const size_t pad = r.offset % ctx->alignment;
    if (pad != 0) {
        r.offset += ctx->alignment - pad;
        fseek(f, (long) r.offset, SEEK_SET);
    }
    ctx->offset = r.offset;

    ctx->size = 0;
    for (const auto & p : ctx->infos) {
        const tensor_info & t = *p;
        const int64_t ne = t.ne[0] * t.ne[1] * t.ne[2] * t.ne[3];
        if (ne % ggml_blck_size((enum ggml_type) t.type) != 0) {
            fprintf(stderr, "gguf_init_from_file: tensor '%s' of type %d (%s) number of elements (%" PRId64 ") is not a multiple of block size (%d)\n",
                    t.name.c_str(), t.type, ggml_type_name((enum ggml_type) t.type), ne, ggml_blck_size((enum ggml_type) t.type));
            return fail(nullptr);
        }
        ctx->size += GGML_PAD(ggml_row_size((enum ggml_type) t.type, ne), ctx->alignment);
    }

    if (params.ctx != nullptr) {
        const size_t n = ctx->infos.size();
        const size_t mem = params.no_alloc ? n * ggml_tensor_overhead() : (n + 1) * ggml_tensor_overhead() + ctx->size;
        ggml_init_params ip = {mem, nullptr, params.no_alloc};
        ggml_context * gctx = ggml_init(ip);
        if (!gctx) return fail("failed to create the ggml context");
        ggml_tensor * blob = nullptr;
        if (!params.no_alloc) {
            // the whole data section as one I8 tensor; the tensors below point into it
            blob = ggml_new_tensor_1d(gctx, GGML_TYPE_I8, (int64_t) ctx->size);
            if (!blob || !r.bytes(blob->data, ctx->size)) {
                ggml_free(gctx);
                return fail("failed to read tensor data");
            }
            ctx->data = blob->data;
        }
        ggml_set_no_alloc(gctx, true);
        for (const auto & p : ctx->infos) {
            ggml_tensor * cur = ggml_new_tensor(gctx, (enum ggml_type) p->type, (int) p->n_dims, p->ne);
            if (!cur) {
                ggml_free(gctx);
                return fail("failed to read the tensor data");
            }
            ggml_set_name(cur, p->name.c_str());
            if (blob) cur->data = (char *) blob->data + p->offset;
        }
        ggml_set_no_alloc(gctx, params.no_alloc);
        *params.ctx = gctx;
    }
    fclose(f);
    return ctx.release();
}

const char * gguf_type_name(enum gguf_type type) {
    return (int) type >= 0 && type < GGUF_TYPE_COUNT ? kTypeNames[type] : nullptr;
}

int gguf_get_version(const struct gguf_context * ctx) { return (int) ctx->version; }
size_t gguf_get_alignment(const struct gguf_context * ctx) { return ctx->alignment; }
size_t gguf_get_data_offset(const struct gguf_context * ctx) { return ctx->offset; }
void * gguf_get_data(const struct gguf_context * ctx) { return ctx->data; }
int gguf_get_n_kv(const struct gguf_context * ctx) { return (int) ctx->kv.size(); }

int gguf_find_key(const struct gguf_context * ctx, const char * key) {
    for (size_t i = 0; i < ctx->kv.size(); i++)
        if (ctx->kv[i]->key == key) return (int) i;
    return -1;
}

const char * gguf_get_key(const struct gguf_context * ctx, int key_id) { return ctx->at(key_id).key.c_str(); }
enum gguf_type gguf_get_kv_type(const struct gguf_context * ctx, int key_id) { return (enum gguf_type) ctx->at(key_id).type; }

enum gguf_type gguf_get_arr_type(const struct gguf_context * ctx, int key_id) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type == GGUF_TYPE_ARRAY);
    return (enum gguf_type) e.arr_type;
}

const void * gguf_get_arr_data(const struct gguf_context * ctx, int key_id) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type == GGUF_TYPE_ARRAY);
    return e.arr_type == GGUF_TYPE_STRING ? (const void *) e.views.data() : (const void *) e.raw.data();
}

const char * gguf_get_arr_str(const struct gguf_context * ctx, int key_id, int i) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type == GGUF_TYPE_ARRAY);
    GGML_ASSERT(e.arr_type == GGUF_TYPE_STRING && i >= 0 && (size_t) i < e.strs.size());
    return e.strs[i].c_str();
}

int gguf_get_arr_n(const struct gguf_context * ctx, int key_id) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type == GGUF_TYPE_ARRAY);
    return (int) e.arr_n;
}

#define MI_GGUF_GETTER(NAME, CT, TYPE, FIELD)                                  \
    CT gguf_get_val_##NAME(const struct gguf_context * ctx, int key_id) {      \
        const kv_entry & e = ctx->at(key_id);                                  \
        GGML_ASSERT(e.type == TYPE);                                           \
        return e.num.FIELD;                                                    \
    }
MI_GGUF_GETTER(u8, uint8_t, GGUF_TYPE_UINT8, u8)
MI_GGUF_GETTER(i8, int8_t, GGUF_TYPE_INT8, i8)
MI_GGUF_GETTER(u16, uint16_t, GGUF_TYPE_UINT16, u16)
MI_GGUF_GETTER(i16, int16_t, GGUF_TYPE_INT16, i16)
MI_GGUF_GETTER(u32, uint32_t, GGUF_TYPE_UINT32, u32)
MI_GGUF_GETTER(i32, int32_t, GGUF_TYPE_INT32, i32)
MI_GGUF_GETTER(f32, float, GGUF_TYPE_FLOAT32, f32)
MI_GGUF_GETTER(u64, uint64_t, GGUF_TYPE_UINT64, u64)
MI_GGUF_GETTER(i64, int64_t, GGUF_TYPE_INT64, i64)
MI_GGUF_GETTER(f64, double, GGUF_TYPE_FLOAT64, f64)
MI_GGUF_GETTER(bool, bool, GGUF_TYPE_BOOL, b)
#undef MI_GGUF_GETTER

const char * gguf_get_val_str(const struct gguf_context * ctx, int key_id) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type == GGUF_TYPE_STRING);
    return e.str.c_str();
}

const void * gguf_get_val_data(const struct gguf_context * ctx, int key_id) {
    const kv_entry & e = ctx->at(key_id);
    GGML_ASSERT(e.type != GGUF_TYPE_ARRAY);
    GGML_ASSERT(e.type != GGUF_TYPE_STRING);
    return e.num.bytes;
}

int gguf_get_n_tensors(const struct gguf_context * ctx) { return (int) ctx->infos.size(); }

int gguf_find_tensor(const struct gguf_context * ctx, const char * name) {
    for (size_t i = 0; i < ctx->infos.size(); i++)
        if (ctx->infos[i]->name == name) return (int) i;
    return -1;
}

size_t gguf_get_tensor_offset(const struct gguf_context * ctx, int i) { return ctx->infos[i]->offset; }
char * gguf_get_tensor_name(const struct gguf_context * ctx, int i) { return &ctx->infos[i]->name[0]; }
enum ggml_type gguf_get_tensor_type(const struct gguf_context * ctx, int i) { return (enum ggml_type) ctx->infos[i]->type; }

void gguf_remove_key(struct gguf_context * ctx, const char * key) {
    const int i = gguf_find_key(ctx, key);
    if (i >= 0) ctx->kv.erase(ctx->kv.begin() + i);
}

#define MI_GGUF_SETTER(NAME, CT, TYPE, FIELD)                                         \
    void gguf_set_val_##NAME(struct gguf_context * ctx, const char * key, CT val) {   \
        kv_entry & e = ctx->get_or_add(key);                                          \
        e.type = TYPE;                                                                \
        e.num = {};                                                                   \
        e.num.FIELD = val;                                                            \
    }
MI_GGUF_SETTER(u8, uint8_t, GGUF_TYPE_UINT8, u8)
MI_GGUF_SETTER(i8, int8_t, GGUF_TYPE_INT8, i8)
MI_GGUF_SETTER(u16, uint16_t, GGUF_TYPE_UINT16, u16)
MI_GGUF_SETTER(i16, int16_t, GGUF_TYPE_INT16, i16)
MI_GGUF_SETTER(u32, uint32_t, GGUF_TYPE_UINT32, u32)
MI_GGUF_SETTER(i32, int32_t, GGUF_TYPE_INT32, i32)
MI_GGUF_SETTER(f32, float, GGUF_TYPE_FLOAT32, f32)
MI_GGUF_SETTER(u64, uint64_t, GGUF_TYPE_UINT64, u64)
MI_GGUF_SETTER(i64, int64_t, GGUF_TYPE_INT64, i64)
MI_GGUF_SETTER(f64, double, GGUF_TYPE_FLOAT64, f64)
MI_GGUF_SETTER(bool, bool, GGUF_TYPE_BOOL, b)
#undef MI_GGUF_SETTER

void gguf_set_val_str(struct gguf_context * ctx, const char * key, const char * val) {
    kv_entry & e = ctx->get_or_add(key);
    e.type = GGUF_TYPE_STRING;
    e.str = val;
}

void gguf_set_arr_data(struct gguf_context * ctx, const char * key, enum gguf_type type, const void * data, int n) {
    const size_t es = scalar_size(type);
    GGML_ASSERT(es != 0 && n >= 0 && "gguf_set_arr_data: fixed-size element type");
    kv_entry & e = ctx->get_or_add(key);
    e.type = GGUF_TYPE_ARRAY;
    e.arr_type = type;
    e.arr_n = (uint64_t) n;
    e.raw.assign((const uint8_t *) data, (const uint8_t *) data + (size_t) n * es);
}

void gguf_set_arr_str(struct gguf_context * ctx, const char * key, const char ** data, int n) {
    kv_entry & e = ctx->get_or_add(key);
    e.type = GGUF_TYPE_ARRAY;
    e.arr_type = GGUF_TYPE_STRING;
    e.arr_n = (uint64_t) n;
    e.set_strings(std::vector<std::string>(data, data + n));
}

void gguf_set_kv(struct gguf_context * ctx, struct gguf_context * src) {
    for (const auto & p : src->kv) {
        const kv_entry & s = *p;
        GGML_ASSERT(!(s.type == GGUF_TYPE_ARRAY && s.arr_type == GGUF_TYPE_ARRAY) && "nested arrays not supported");
        if (s.type == GGUF_TYPE_STRING) {
            gguf_set_val_str(ctx, s.key.c_str(), s.str.c_str());
        } else if (s.type == GGUF_TYPE_ARRAY && s.arr_type == GGUF_TYPE_STRING) {
            std::vector<const char *> v;
            for (const auto & x : s.strs) v.push_back(x.c_str());
            gguf_set_arr_str(ctx, s.key.c_str(), v.data(), (int) v.size());
        } else if (s.type == GGUF_TYPE_ARRAY) {
            gguf_set_arr_data(ctx, s.key.c_str(), (enum gguf_type) s.arr_type, s.raw.data(), (int) s.arr_n);
        } else {
            GGML_ASSERT(scalar_size(s.type) != 0 && "invalid type");
            kv_entry & e = ctx->get_or_add(s.key.c_str());
            e.type = s.type;
            e.num = s.num;
        }
    }
}

void gguf_add_tensor(struct gguf_context * ctx, const struct ggml_tensor * tensor) {
    GGML_ASSERT(gguf_find_tensor(ctx, tensor->name) == -1 && "duplicated tensor name");
    std::unique_ptr<tensor_info> t(new tensor_info);
    t->name = tensor->name;
    t->n_dims = (uint32_t) ggml_n_dims(tensor);
    for (uint32_t i = 0; i < t->n_dims; i++) t->ne[i] = tensor->ne[i];
    t->type = tensor->type;
    t->data = tensor->data;
    t->size = ggml_nbytes(tensor);
    ctx->infos.push_back(std::move(t));
    if (ctx->infos.size() > 1) update_offsets(ctx, ctx->infos.size() - 1);
}

void gguf_set_tensor_type(struct gguf_context * ctx, const char * name, enum ggml_type type) {
    const int i = gguf_find_tensor(ctx, name);
    GGML_ASSERT(i >= 0 && "tensor not found");
    ctx->infos[i]->type = type;
}

void gguf_set_tensor_data(struct gguf_context * ctx, const char * name, const void * data, size_t size) {
    const int i = gguf_find_tensor(ctx, name);
    GGML_ASSERT(i >= 0 && "tensor not found");
    ctx->infos[i]->data = data;
    ctx->infos[i]->size = size;
    update_offsets(ctx, (size_t) i + 1);
}

void gguf_write_to_file(const struct gguf_context * ctx, const char * fname, bool only_meta) {
    FILE * f = fopen(fname, "wb");
    GGML_ASSERT(f && "failed to open file for writing");
    std::vector<uint8_t> buf;
    writer w{&buf};
    write_meta(ctx, w);
    fwrite(buf.data(), 1, buf.size(), f);
    if (!only_meta) {
        // tensor data, each padded to the alignment, streamed (no copy of the whole section)
        size_t off = 0;
        static const uint8_t zeros[256] = {};
        for (const auto & p : ctx->infos) {
            GGML_ASSERT(off == p->offset);
            if (p->size) fwrite(p->data, 1, p->size, f);
            size_t padn = GGML_PAD(p->size, ctx->alignment) - p->size;
            while (padn) {
                const size_t c = padn < sizeof(zeros) ? padn : sizeof(zeros);
                fwrite(zeros, 1, c, f);
                padn -= c;
            }
            off += GGML_PAD(p->size, ctx->alignment);
        }
    }
    fclose(f);
}

size_t gguf_get_meta_size(const struct gguf_context * ctx) {
    writer w{nullptr};
    write_meta(ctx, w);
    return w.n;
}

void gguf_get_meta_data(const struct gguf_context * ctx, void * data) {
    std::vector<uint8_t> buf;
    writer w{&buf};
    write_meta(ctx, w);
    memcpy(data, buf.data(), buf.size());
}

} // extern "C"
