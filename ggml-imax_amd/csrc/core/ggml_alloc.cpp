// ggml_alloc.cpp -- tensor and graph allocators (include/ggml/ggml-alloc.h API of the reference,
// src/ggml-alloc.c:60-981).
//
// ggml_tallocr / ggml_backend_alloc_ctx_tensors_from_buft follow the reference placement rules
// (linear, aligned, views initialised against their base). The graph allocator is our own
// planner, built for a device with 288 GB of HBM: leafs and inputs get private,
// non-overlapping slots for the whole graph (so host-side tensor_set of any leaf can never be
// clobbered by an earlier node), intermediates are packed by liveness (last consumer, views
// resolved to their base) with best-fit reuse of freed ranges, and outputs are never freed.

#include "ggml_abi.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <unordered_map>
#include <vector>

static size_t align_up(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

extern "C" {

struct ggml_tallocr ggml_tallocr_new(ggml_backend_buffer_t buffer) {
    void * base = ggml_backend_buffer_get_base(buffer);
    const size_t align = ggml_backend_buffer_get_alignment(buffer);
    GGML_ASSERT(align && !(align & (align - 1)));
    ggml_tallocr t;
    t.buffer = buffer;
    t.base = base;
    t.alignment = align;
    t.offset = (align - ((uintptr_t) base % align)) % align;
    return t;
}

void ggml_tallocr_alloc(struct ggml_tallocr * talloc, struct ggml_tensor * tensor) {
    const size_t size = GGML_PAD(ggml_backend_buffer_get_alloc_size(talloc->buffer, tensor), talloc->alignment);
    if (talloc->offset + size > ggml_backend_buffer_get_size(talloc->buffer)) {
        fprintf(stderr, "%s: not enough space in the buffer to allocate %s (needed %zu, available %zu)\n", __func__,
                tensor->name, size, ggml_backend_buffer_get_size(talloc->buffer) - talloc->offset);
        GGML_ASSERT(!"not enough space in the buffer");
    }
    void * addr = (char *) ggml_backend_buffer_get_base(talloc->buffer) + talloc->offset;
    talloc->offset += size;
    ggml_backend_tensor_alloc(talloc->buffer, tensor, addr);
}

// src/ggml-alloc.c:879-981
static bool alloc_tensor_range(ggml_context * ctx, ggml_tensor * first, ggml_tensor * last, ggml_backend_buffer_type_t buft,
                               size_t size, std::vector<ggml_backend_buffer_t> & buffers) {
    ggml_backend_buffer_t buffer = ggml_backend_buft_alloc_buffer(buft, size);
    if (!buffer) {
        for (auto * b : buffers) ggml_backend_buffer_free(b);
        buffers.clear();
        return false;
    }
    ggml_tallocr talloc = ggml_tallocr_new(buffer);
    for (ggml_tensor * t = first; t != last; t = ggml_get_next_tensor(ctx, t)) {
        if (t->data == NULL) {
            if (t->view_src == NULL) ggml_tallocr_alloc(&talloc, t);
            else if (t->buffer == NULL) ggml_backend_view_init(buffer, t);
        } else if (t->view_src != NULL && t->buffer == NULL) {
            ggml_backend_view_init(buffer, t);
        }
    }
    buffers.push_back(buffer);
    return true;
}

ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors_from_buft(struct ggml_context * ctx, ggml_backend_buffer_type_t buft) {
    GGML_ASSERT(ggml_get_no_alloc(ctx) == true);
    const size_t alignment = ggml_backend_buft_get_alignment(buft);
    const size_t max_size = ggml_backend_buft_get_max_size(buft);
    std::vector<ggml_backend_buffer_t> buffers;
    size_t cur = 0;
    ggml_tensor * first = ggml_get_first_tensor(ctx);
    for (ggml_tensor * t = first; t != NULL; t = ggml_get_next_tensor(ctx, t)) {
        size_t this_size = 0;
        if (t->data == NULL && t->view_src == NULL) this_size = GGML_PAD(ggml_backend_buft_get_alloc_size(buft, t), alignment);
        if (this_size > max_size) {
            fprintf(stderr, "%s: tensor %s is too large to fit in a %s buffer (tensor size: %zu, max buffer size: %zu)\n",
                    __func__, t->name, ggml_backend_buft_name(buft), this_size, max_size);
            for (auto * b : buffers) ggml_backend_buffer_free(b);
            return NULL;
        }
        if (cur + this_size > max_size) {
            if (!alloc_tensor_range(ctx, first, t, buft, cur, buffers)) return NULL;
            first = t;
            cur = this_size;
        } else {
            cur += this_size;
        }
    }
    if (cur > 0 && !alloc_tensor_range(ctx, first, NULL, buft, cur, buffers)) return NULL;
    if (buffers.empty()) return NULL;
    if (buffers.size() == 1) return buffers[0];
    return ggml_backend_multi_buffer_alloc_buffer(buffers.data(), buffers.size());
}

ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors(struct ggml_context * ctx, ggml_backend_t backend) {
    return ggml_backend_alloc_ctx_tensors_from_buft(ctx, ggml_backend_get_default_buffer_type(backend));
}

} // extern "C"

// ---------------------------------------------------------------------------------------------
// graph allocator
// ---------------------------------------------------------------------------------------------

namespace {

// best-fit free-range arena over [0, inf); tracks the high-water mark
struct arena {
    size_t align;
    size_t high = 0;
    std::map<size_t, size_t> free_ranges;  // offset -> size

    size_t alloc(size_t size) {
        size = align_up(size ? size : align, align);
        auto best = free_ranges.end();
        for (auto it = free_ranges.begin(); it != free_ranges.end(); ++it) {
            if (it->second >= size && (best == free_ranges.end() || it->second < best->second)) best = it;
        }
        if (best != free_ranges.end()) {
            const size_t off = best->first, rem = best->second - size;
            free_ranges.erase(best);
            if (rem) free_ranges[off + size] = rem;
            return off;
        }
        // grow: merge with a free tail if present
        if (!free_ranges.empty()) {
            auto last = std::prev(free_ranges.end());
            if (last->first + last->second == high) {
                const size_t off = last->first;
                free_ranges.erase(last);
                high = off + size;
                return off;
            }
        }
        const size_t off = high;
        high += size;
        return off;
    }

    void release(size_t off, size_t size) {
        size = align_up(size ? size : align, align);
        auto it = free_ranges.emplace(off, size).first;
        auto next = std::next(it);
        if (next != free_ranges.end() && it->first + it->second == next->first) {
            it->second += next->second;
            free_ranges.erase(next);
        }
        if (it != free_ranges.begin()) {
            auto prev = std::prev(it);
            if (prev->first + prev->second == it->first) {
                prev->second += it->second;
                free_ranges.erase(it);
            }
        }
    }
};

struct plan_entry {
    int buffer_id;
    size_t offset;
};

} // namespace

// per graph position (node i / leaf i) placement of the last full plan: reused as long as a new
// graph has the same shape of positions and every tensor fits its planned slot -- the reserve()
// of a worst-case graph followed by cheap per-step assignment, as ggml-alloc.c:668-737 does
struct slot {
    int buffer_id;   // -1: the position needs no memory
    size_t offset;
    size_t size;
};

struct ggml_gallocr {
    std::vector<ggml_backend_buffer_type_t> bufts;
    std::vector<ggml_backend_buffer_t> buffers;
    std::vector<size_t> planned;  // planned size per buffer
    std::vector<int> node_buffer_ids;
    std::vector<int> leaf_buffer_ids;
    std::vector<slot> node_slots, leaf_slots;
};

static ggml_tensor * base_of(ggml_tensor * t) { return t->view_src ? t->view_src : t; }

// Plans offsets for every graph tensor that needs memory. Returns per-buffer sizes.
static std::vector<size_t> plan_graph(ggml_gallocr * ga, ggml_cgraph * g, std::unordered_map<ggml_tensor *, plan_entry> & out) {
    const int nb = (int) ga->bufts.size();
    std::vector<arena> arenas(nb);
    for (int i = 0; i < nb; i++) arenas[i].align = ggml_backend_buft_get_alignment(ga->bufts[i]);

    auto needs_alloc = [](ggml_tensor * t) { return t->data == NULL && t->view_src == NULL; };
    auto leaf_buf = [&](int i) { return (int) ga->leaf_buffer_ids.size() > i ? ga->leaf_buffer_ids[i] : 0; };
    auto node_buf = [&](int i) { return (int) ga->node_buffer_ids.size() > i ? ga->node_buffer_ids[i] : 0; };

    std::unordered_map<ggml_tensor *, int> owner_buf;
    for (int i = 0; i < g->n_leafs; i++) owner_buf[g->leafs[i]] = leaf_buf(i);
    for (int i = 0; i < g->n_nodes; i++) owner_buf[g->nodes[i]] = node_buf(i);

    // last use of every base tensor (node index), outputs pinned to the end
    std::unordered_map<ggml_tensor *, int> last_use;
    for (int i = 0; i < g->n_nodes; i++) {
        ggml_tensor * n = g->nodes[i];
        last_use[base_of(n)] = std::max(last_use[base_of(n)], i);
        for (int s = 0; s < GGML_MAX_SRC; s++) {
            if (n->src[s]) last_use[base_of(n->src[s])] = std::max(last_use[base_of(n->src[s])], i);
        }
    }

    auto size_of = [&](ggml_tensor * t, int buf) { return ggml_backend_buft_get_alloc_size(ga->bufts[buf], t); };
    auto place = [&](ggml_tensor * t) {
        if (!needs_alloc(t) || out.count(t)) return;
        const int buf = owner_buf.count(t) ? owner_buf[t] : 0;
        out[t] = {buf, arenas[buf].alloc(size_of(t, buf))};
    };

    // 1) leafs and inputs: private slots for the whole graph
    for (int i = 0; i < g->n_leafs; i++) place(g->leafs[i]);
    for (int i = 0; i < g->n_nodes; i++) {
        ggml_tensor * n = g->nodes[i];
        if (n->flags & GGML_TENSOR_FLAG_INPUT) place(n);
        for (int s = 0; s < GGML_MAX_SRC; s++) if (n->src[s] && (n->src[s]->flags & GGML_TENSOR_FLAG_INPUT)) place(n->src[s]);
    }
    std::unordered_map<ggml_tensor *, bool> pinned;
    for (auto & kv : out) pinned[kv.first] = true;

    // 2) nodes in order; a base is released kFreeDelay nodes after its last consumer, so the
    //    outputs of the next few nodes never land on it. A backend that executes a short chain
    //    of nodes as one kernel (ggml-mi355x.cpp node fusion) then never finds the chain's output
    //    placed over the chain's inputs.
    constexpr int kFreeDelay = 4;
    std::vector<std::vector<ggml_tensor *>> release_at(g->n_nodes + kFreeDelay + 1);
    for (int i = 0; i < g->n_nodes; i++) {
        ggml_tensor * n = g->nodes[i];
        for (int s = 0; s < GGML_MAX_SRC; s++) if (n->src[s]) place(base_of(n->src[s]));
        place(n);
        for (ggml_tensor * p : release_at[i]) {
            const plan_entry e = out[p];
            arenas[e.buffer_id].release(e.offset, size_of(p, e.buffer_id));
        }
        for (int s = 0; s < GGML_MAX_SRC; s++) {
            ggml_tensor * p = n->src[s] ? base_of(n->src[s]) : nullptr;
            if (!p || !out.count(p) || pinned.count(p) || (p->flags & GGML_TENSOR_FLAG_OUTPUT)) continue;
            if (last_use[p] == i) {
                release_at[i + kFreeDelay].push_back(p);
                pinned[p] = true;  // never release twice
            }
        }
    }
    std::vector<size_t> sizes(nb);
    for (int i = 0; i < nb; i++) sizes[i] = arenas[i].high;
    auto slot_of = [&](ggml_tensor * t) -> slot {
        auto it = out.find(t);
        if (it == out.end()) return {-1, 0, 0};
        return {it->second.buffer_id, it->second.offset, size_of(t, it->second.buffer_id)};
    };
    ga->node_slots.resize(g->n_nodes);
    ga->leaf_slots.resize(g->n_leafs);
    for (int i = 0; i < g->n_nodes; i++) ga->node_slots[i] = slot_of(g->nodes[i]);
    for (int i = 0; i < g->n_leafs; i++) ga->leaf_slots[i] = slot_of(g->leafs[i]);
    return sizes;
}

// every tensor needing memory sits at a position whose planned slot holds it
static bool slots_fit(ggml_gallocr * ga, ggml_cgraph * g) {
    if ((int) ga->node_slots.size() != g->n_nodes || (int) ga->leaf_slots.size() != g->n_leafs || ga->buffers.empty()) return false;
    auto fits = [&](ggml_tensor * t, const slot & sl) {
        const bool needs = t->data == NULL && t->view_src == NULL;
        if (!needs) return sl.buffer_id < 0 || t->data != NULL || t->view_src != NULL;
        return sl.buffer_id >= 0 && ga->buffers[sl.buffer_id] != NULL &&
               ggml_backend_buft_get_alloc_size(ga->bufts[sl.buffer_id], t) <= sl.size;
    };
    for (int i = 0; i < g->n_leafs; i++) if (!fits(g->leafs[i], ga->leaf_slots[i])) return false;
    for (int i = 0; i < g->n_nodes; i++) if (!fits(g->nodes[i], ga->node_slots[i])) return false;
    return true;
}

extern "C" {

ggml_gallocr_t ggml_gallocr_new_n(ggml_backend_buffer_type_t * bufts, int n_bufs) {
    auto * ga = new ggml_gallocr();
    for (int i = 0; i < n_bufs; i++) ga->bufts.push_back(bufts[i]);
    ga->buffers.assign(n_bufs, nullptr);
    ga->planned.assign(n_bufs, 0);
    return ga;
}

ggml_gallocr_t ggml_gallocr_new(ggml_backend_buffer_type_t buft) { return ggml_gallocr_new_n(&buft, 1); }

void ggml_gallocr_free(ggml_gallocr_t galloc) {
    if (!galloc) return;
    for (size_t i = 0; i < galloc->buffers.size(); i++) {
        bool dup = false;
        for (size_t j = 0; j < i; j++) dup |= galloc->buffers[j] == galloc->buffers[i];
        if (!dup) ggml_backend_buffer_free(galloc->buffers[i]);
    }
    delete galloc;
}

static bool ensure_buffers(ggml_gallocr_t ga, const std::vector<size_t> & sizes) {
    for (size_t i = 0; i < sizes.size(); i++) {
        const size_t cur = ga->buffers[i] ? ggml_backend_buffer_get_size(ga->buffers[i]) : 0;
        if (sizes[i] > cur || (!ga->buffers[i] && sizes[i] > 0)) {
            ggml_backend_buffer_free(ga->buffers[i]);
            ga->buffers[i] = ggml_backend_buft_alloc_buffer(ga->bufts[i], sizes[i]);
            if (!ga->buffers[i]) {
                fprintf(stderr, "%s: failed to allocate %s buffer of size %zu\n", __func__, ggml_backend_buft_name(ga->bufts[i]), sizes[i]);
                return false;
            }
        }
        ga->planned[i] = std::max(ga->planned[i], sizes[i]);
    }
    return true;
}

bool ggml_gallocr_reserve_n(ggml_gallocr_t galloc, struct ggml_cgraph * graph, const int * node_buffer_ids, const int * leaf_buffer_ids) {
    galloc->node_buffer_ids.assign(node_buffer_ids ? node_buffer_ids : nullptr, node_buffer_ids ? node_buffer_ids + graph->n_nodes : nullptr);
    galloc->leaf_buffer_ids.assign(leaf_buffer_ids ? leaf_buffer_ids : nullptr, leaf_buffer_ids ? leaf_buffer_ids + graph->n_leafs : nullptr);
    std::unordered_map<ggml_tensor *, plan_entry> plan;
    return ensure_buffers(galloc, plan_graph(galloc, graph, plan));
}

bool ggml_gallocr_reserve(ggml_gallocr_t galloc, struct ggml_cgraph * graph) { return ggml_gallocr_reserve_n(galloc, graph, NULL, NULL); }

bool ggml_gallocr_alloc_graph(ggml_gallocr_t galloc, struct ggml_cgraph * graph) {
    auto init_view = [&](ggml_tensor * t) {
        if (t->view_src && t->buffer == NULL && t->view_src->buffer != NULL) ggml_backend_view_init(t->view_src->buffer, t);
    };
    if (slots_fit(galloc, graph)) {
        // fast path: same positions, every tensor fits its planned slot
        for (int i = 0; i < (int) galloc->buffers.size(); i++) {
            if (galloc->buffers[i]) ggml_backend_buffer_reset(galloc->buffers[i]);
        }
        auto put = [&](ggml_tensor * t, const slot & sl) {
            if (sl.buffer_id < 0 || t->data != NULL || t->view_src != NULL) return;
            ggml_backend_buffer_t buf = galloc->buffers[sl.buffer_id];
            ggml_backend_tensor_alloc(buf, t, (char *) ggml_backend_buffer_get_base(buf) + sl.offset);
        };
        for (int i = 0; i < graph->n_leafs; i++) put(graph->leafs[i], galloc->leaf_slots[i]);
        for (int i = 0; i < graph->n_nodes; i++) put(graph->nodes[i], galloc->node_slots[i]);
        for (int i = 0; i < graph->n_nodes; i++) {
            ggml_tensor * n = graph->nodes[i];
            for (int s = 0; s < GGML_MAX_SRC; s++) if (n->src[s]) init_view(n->src[s]);
            init_view(n);
        }
        for (int i = 0; i < graph->n_leafs; i++) init_view(graph->leafs[i]);
        return true;
    }
    std::unordered_map<ggml_tensor *, plan_entry> plan;
    const std::vector<size_t> sizes = plan_graph(galloc, graph, plan);
    for (size_t i = 0; i < sizes.size(); i++) {
        const size_t cur = galloc->buffers[i] ? ggml_backend_buffer_get_size(galloc->buffers[i]) : 0;
        if (sizes[i] > cur && galloc->bufts.size() > 1) return false;  // multi-buffer: caller must reserve_n
    }
    if (!ensure_buffers(galloc, sizes)) return false;
    for (int i = 0; i < galloc->buffers.size(); i++) {
        if (galloc->buffers[i]) ggml_backend_buffer_reset(galloc->buffers[i]);
    }
    // assign addresses in graph order, then initialise views against their bases
    auto assign = [&](ggml_tensor * t) {
        auto it = plan.find(t);
        if (it == plan.end() || t->data != NULL) return;
        ggml_backend_buffer_t buf = galloc->buffers[it->second.buffer_id];
        ggml_backend_tensor_alloc(buf, t, (char *) ggml_backend_buffer_get_base(buf) + it->second.offset);
    };
    for (int i = 0; i < graph->n_leafs; i++) assign(graph->leafs[i]);
    for (int i = 0; i < graph->n_nodes; i++) {
        ggml_tensor * n = graph->nodes[i];
        for (int s = 0; s < GGML_MAX_SRC; s++) {
            if (!n->src[s]) continue;
            assign(base_of(n->src[s]));
            init_view(n->src[s]);
        }
        assign(n);
        init_view(n);
    }
    for (int i = 0; i < graph->n_leafs; i++) init_view(graph->leafs[i]);
    return true;
}

size_t ggml_gallocr_get_buffer_size(ggml_gallocr_t galloc, int buffer_id) {
    GGML_ASSERT(buffer_id >= 0 && buffer_id < (int) galloc->buffers.size());
    return galloc->buffers[buffer_id] ? ggml_backend_buffer_get_size(galloc->buffers[buffer_id]) : 0;
}

} // extern "C"
