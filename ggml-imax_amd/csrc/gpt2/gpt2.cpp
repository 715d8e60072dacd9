// gpt2.cpp -- GPT-2 model driver over the ggml backend API (BASELINE config 4).
//
// Behaviour follows examples/gpt-2/main-backend.cpp of NAIST-Archlab/ggml-imax:
//   file format + loader  :101-439   (legacy ggml magic, hparams, vocab, tensors by name,
//                                     wte doubles as lm_head when the file has none :426-433)
//   graph                 :442-717   (node-for-node the same ops, so a backend that passes the
//                                     reference's test-backend-ops runs it unchanged)
//   eval                  :728-786
//   compute-buffer sizing :832-846   (worst case: n_batch tokens at the end of the context)
// and the tokenizer of examples/common.cpp:272-329. Only the ggml API is used: the same source is
// linked against this repo's runtime (product) and against the reference libggml (checker build in
// oracle/, which gives the CPU logits).

#include "gpt2-mi355x.h"
#ifdef GPT2_WITH_SCHED
#include "ggml_sched_abi.h"
#endif

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <regex>
#include <string>
#include <vector>

namespace {

constexpr int kMaxNodes = 4096;  // GPT2_MAX_NODES

struct layer_w {
    ggml_tensor * ln_1_g, * ln_1_b, * ln_2_g, * ln_2_b;
    ggml_tensor * c_attn_attn_w, * c_attn_attn_b, * c_attn_proj_w, * c_attn_proj_b;
    ggml_tensor * c_mlp_fc_w, * c_mlp_fc_b, * c_mlp_proj_w, * c_mlp_proj_b;
};

struct vocab_t {
    std::map<std::string, int32_t> token_to_id;
    std::vector<std::string> id_to_token;
};

int64_t now_us() { return ggml_time_us(); }

} // namespace

struct gpt2_model {
    gpt2_hparams_c hp = {50257, 1024, 768, 12, 12, 1, 1e-5f};
    ggml_tensor * ln_f_g = nullptr, * ln_f_b = nullptr;
    ggml_tensor * wte = nullptr, * wpe = nullptr, * lm_head = nullptr;
    std::vector<layer_w> layers;
    ggml_tensor * memory_k = nullptr, * memory_v = nullptr;
    ggml_context * ctx_w = nullptr, * ctx_kv = nullptr;
    ggml_backend_t backend = nullptr;
    ggml_backend_buffer_t buffer_w = nullptr, buffer_kv = nullptr;
    ggml_gallocr_t allocr = nullptr;
    std::map<std::string, ggml_tensor *> tensors;
    vocab_t vocab;
    size_t weight_bytes = 0;
    // two graph arenas: the next decode token's graph is built (and allocated) in one while the
    // device still runs the graph of the other
    std::vector<uint8_t> graph_buf[2];
    int graph_slot = 0;                   // arena of the graph last computed
    ggml_cgraph * next_gf = nullptr;      // prebuilt + allocated graph of (next_n_past, 1 token)
    int next_n_past = -1;
    ggml_backend_graph_plan_t next_plan = nullptr;  // next_gf as a backend graph plan (if supported)
    int last_nodes = 0;
    int64_t us_build = 0, us_alloc = 0, us_inputs = 0, us_compute = 0;
    // within us_compute: enqueue of the graph, next-graph build, wait for the device, logits copy
    int64_t us_launch = 0, us_prebuild = 0, us_wait = 0, us_readback = 0;
    std::vector<int32_t> tok, pos;  // input staging, alive until the next eval
    // gpt2_model_load_ex with a host buffer type: the token ids and positions live in host memory
    // the device reads in place (no upload), and the logits come back through a host staging
    // tensor copied into right behind the graph on the backend's queue
    bool host_io = false;
    ggml_tensor * logits_host = nullptr;
    // scheduler mode (examples/gpt-2/main-sched.cpp): layers split over backends
    std::vector<ggml_backend_t> backends;       // [gpu, ..., cpu]
    std::vector<ggml_backend_buffer_t> buffers_w;
    ggml_backend_buffer_t buffer_input = nullptr;
    ggml_context * ctx_in = nullptr;
    ggml_backend_buffer_t buffer_pos = nullptr;  // host_io: the constant positions, device-resident
    ggml_context * ctx_pos = nullptr;
    ggml_tensor * embd_in = nullptr, * pos_in = nullptr;  // persistent input tensors
    void * sched = nullptr;                     // ggml_backend_sched_t
    int n_gpu_layers = 0;
    int sched_flags = 0;                        // GPT2_SCHED_*
    // batched independent sequences (examples/gpt-2/main-batched.cpp:76-102): the KV cache as
    // cells, each holding a position and the set of sequences that see it, filled from `kv_head`
    struct kv_cell {
        int32_t pos = -1;
        std::vector<int32_t> seq;
        bool has(int32_t s) const { return std::find(seq.begin(), seq.end(), s) != seq.end(); }
    };
    std::vector<kv_cell> cells;
    uint32_t kv_head = 0, kv_n = 0;
    // batched decode inputs, host_io: one pinned staging block and one device block [tokens | pos |
    // KQ mask] (one async copy per step; the graph's inputs are views of the device block), and the
    // next step's graph built + allocated + planned while the device runs the current one
    ggml_backend_buffer_type_t host_buft = nullptr;
    ggml_context * ctx_bin = nullptr;
    ggml_backend_buffer_t buf_bin_host = nullptr, buf_bin_dev = nullptr;
    ggml_tensor * bin_host = nullptr, * bin_dev = nullptr;
    ggml_cgraph * bnext_gf = nullptr;                 // prebuilt batched graph of (bnext_tokens, bnext_head)
    int bnext_tokens = -1, bnext_head = -1;
    ggml_backend_graph_plan_t bnext_plan = nullptr;
    int64_t batch_plans = 0, batch_direct = 0;       // steps launched as a prebuilt plan / built on the spot
    int batch_reserved = 0;                           // batch size the compute buffer is reserved for
};

namespace {

template <typename T> bool rd(std::ifstream & f, T & v) { return (bool) f.read((char *) &v, sizeof(T)); }

// main-sched.cpp:306-366: wte/wpe on the GPU only when every layer is, ln_f/lm_head on the GPU
// when any layer is, layer il on the GPU when il >= n_layer - n_gpu_layers; one buffer per backend
bool place_weights_sched(gpt2_model & m) {
    ggml_backend_t gpu = m.backends.front(), cpu = m.backends.back();
    const int first_gpu_layer = m.hp.n_layer - m.n_gpu_layers;
    std::map<ggml_tensor *, ggml_backend_t> where;
    for (auto & kv : m.tensors) {
        const std::string & name = kv.first;
        ggml_backend_t b = cpu;
        if (name == "model/wte" || name == "model/wpe") b = m.n_gpu_layers > m.hp.n_layer ? gpu : cpu;
        else if (name == "model/ln_f/g" || name == "model/ln_f/b" || name == "model/lm_head") b = m.n_gpu_layers > 0 ? gpu : cpu;
        else if (name.compare(0, 7, "model/h") == 0) {
            const int il = std::stoi(name.substr(7, 2));
            b = il >= first_gpu_layer ? gpu : cpu;
            // GPT2_SCHED_SPLIT_MID: the previous layer's attention half on the GPU too
            if ((m.sched_flags & GPT2_SCHED_SPLIT_MID) && il == first_gpu_layer - 1 &&
                (name.find("/attn/") != std::string::npos || name.find("/ln_1/") != std::string::npos)) b = gpu;
        }
        where[kv.second] = b;
    }
    for (ggml_backend_t b : m.backends) {
        size_t size = 0;
        for (auto & kv : where) if (kv.second == b) size += ggml_nbytes(kv.first) + 512;
        if (size == 0) {
            m.buffers_w.push_back(nullptr);
            continue;
        }
        ggml_backend_buffer_t buf = ggml_backend_alloc_buffer(b, size);
        if (!buf) {
            fprintf(stderr, "gpt2_model_load: %s weight buffer allocation failed\n", ggml_backend_name(b));
            return false;
        }
        ggml_backend_buffer_set_usage(buf, GGML_BACKEND_BUFFER_USAGE_WEIGHTS);
        m.buffers_w.push_back(buf);
        ggml_tallocr alloc = ggml_tallocr_new(buf);
        for (auto & kv : where) if (kv.second == b) ggml_tallocr_alloc(&alloc, kv.first);
    }
    return true;
}

bool load_file(gpt2_model & m, const char * fname, int n_ctx_override) {
    std::ifstream fin(fname, std::ios::binary);
    if (!fin) {
        fprintf(stderr, "gpt2_model_load: failed to open '%s'\n", fname);
        return false;
    }
    uint32_t magic = 0;
    rd(fin, magic);
    if (magic != GGML_FILE_MAGIC) {
        fprintf(stderr, "gpt2_model_load: invalid model file '%s' (bad magic)\n", fname);
        return false;
    }
    auto & hp = m.hp;
    rd(fin, hp.n_vocab);
    rd(fin, hp.n_ctx);
    rd(fin, hp.n_embd);
    rd(fin, hp.n_head);
    rd(fin, hp.n_layer);
    rd(fin, hp.ftype);
    hp.ftype %= GGML_QNT_VERSION_FACTOR;

    int32_t n_vocab = 0;
    rd(fin, n_vocab);
    if (n_vocab != hp.n_vocab) {
        fprintf(stderr, "gpt2_model_load: invalid model file '%s' (bad vocab size %d != %d)\n", fname, n_vocab, hp.n_vocab);
        return false;
    }
    m.vocab.id_to_token.resize(n_vocab);
    for (int i = 0; i < n_vocab; i++) {
        uint32_t len = 0;
        rd(fin, len);
        std::string w(len, '\0');
        fin.read(&w[0], len);
        m.vocab.token_to_id[w] = i;
        m.vocab.id_to_token[i] = w;
    }

    const ggml_type wtype = ggml_ftype_to_ggml_type((ggml_ftype) hp.ftype);
    if (wtype == GGML_TYPE_COUNT) {
        fprintf(stderr, "gpt2_model_load: invalid model file '%s' (bad ftype value %d)\n", fname, hp.ftype);
        return false;
    }

    // weights context + tensors (main-backend.cpp:186-297)
    {
        ggml_init_params ip = {ggml_tensor_overhead() * (size_t) (2 + 6 + 12 * hp.n_layer), nullptr, true};
        m.ctx_w = ggml_init(ip);
        if (!m.ctx_w) return false;
        ggml_context * ctx = m.ctx_w;
        const int E = hp.n_embd;
        m.layers.resize(hp.n_layer);
        m.ln_f_g = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
        m.ln_f_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
        m.wte = ggml_new_tensor_2d(ctx, wtype, E, hp.n_vocab);
        m.wpe = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, E, hp.n_ctx);
        m.lm_head = ggml_new_tensor_2d(ctx, wtype, E, hp.n_vocab);
        m.tensors["model/ln_f/g"] = m.ln_f_g;
        m.tensors["model/ln_f/b"] = m.ln_f_b;
        m.tensors["model/wte"] = m.wte;
        m.tensors["model/wpe"] = m.wpe;
        m.tensors["model/lm_head"] = m.lm_head;
        for (int i = 0; i < hp.n_layer; i++) {
            layer_w & L = m.layers[i];
            L.ln_1_g = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            L.ln_1_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            L.ln_2_g = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            L.ln_2_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            L.c_attn_attn_w = ggml_new_tensor_2d(ctx, wtype, E, 3 * E);
            L.c_attn_attn_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, 3 * E);
            L.c_attn_proj_w = ggml_new_tensor_2d(ctx, wtype, E, E);
            L.c_attn_proj_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            L.c_mlp_fc_w = ggml_new_tensor_2d(ctx, wtype, E, 4 * E);
            L.c_mlp_fc_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, 4 * E);
            L.c_mlp_proj_w = ggml_new_tensor_2d(ctx, wtype, 4 * E, E);
            L.c_mlp_proj_b = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, E);
            const std::string p = "model/h" + std::to_string(i);
            m.tensors[p + "/ln_1/g"] = L.ln_1_g;
            m.tensors[p + "/ln_1/b"] = L.ln_1_b;
            m.tensors[p + "/ln_2/g"] = L.ln_2_g;
            m.tensors[p + "/ln_2/b"] = L.ln_2_b;
            m.tensors[p + "/attn/c_attn/w"] = L.c_attn_attn_w;
            m.tensors[p + "/attn/c_attn/b"] = L.c_attn_attn_b;
            m.tensors[p + "/attn/c_proj/w"] = L.c_attn_proj_w;
            m.tensors[p + "/attn/c_proj/b"] = L.c_attn_proj_b;
            m.tensors[p + "/mlp/c_fc/w"] = L.c_mlp_fc_w;
            m.tensors[p + "/mlp/c_fc/b"] = L.c_mlp_fc_b;
            m.tensors[p + "/mlp/c_proj/w"] = L.c_mlp_proj_w;
            m.tensors[p + "/mlp/c_proj/b"] = L.c_mlp_proj_b;
        }
    }
    if (m.backends.empty()) {
        m.buffer_w = ggml_backend_alloc_ctx_tensors(m.ctx_w, m.backend);
        if (!m.buffer_w) {
            fprintf(stderr, "gpt2_model_load: weight buffer allocation failed\n");
            return false;
        }
    } else if (!place_weights_sched(m)) {
        return false;
    }

    if (n_ctx_override > 0) hp.n_ctx = n_ctx_override;

    // KV memory, f32, n_layer*n_ctx*n_embd each (:306-343; main-sched.cpp:367-403 puts it on the
    // GPU when at least half the layers are there)
    {
        ggml_init_params ip = {ggml_tensor_overhead() * 2, nullptr, true};
        m.ctx_kv = ggml_init(ip);
        if (!m.ctx_kv) return false;
        const int64_t n_elements = (int64_t) hp.n_embd * hp.n_layer * hp.n_ctx;
        m.memory_k = ggml_new_tensor_1d(m.ctx_kv, GGML_TYPE_F32, n_elements);
        m.memory_v = ggml_new_tensor_1d(m.ctx_kv, GGML_TYPE_F32, n_elements);
        ggml_backend_t be_kv = m.backend;
        if (!m.backends.empty()) be_kv = m.n_gpu_layers >= hp.n_layer / 2 ? m.backends.front() : m.backends.back();
        m.buffer_kv = ggml_backend_alloc_ctx_tensors(m.ctx_kv, be_kv);
        if (!m.buffer_kv) {
            fprintf(stderr, "gpt2_model_load: KV buffer allocation failed\n");
            return false;
        }
    }

    // tensors by name (:346-435)
    bool has_lm_head = false;
    std::vector<char> buf;
    for (;;) {
        int32_t n_dims = 0, length = 0, ttype = 0;
        rd(fin, n_dims);
        rd(fin, length);
        rd(fin, ttype);
        if (fin.eof()) break;
        int32_t ne[2] = {1, 1};
        int64_t nelements = 1;
        for (int i = 0; i < n_dims; i++) {
            rd(fin, ne[i]);
            nelements *= ne[i];
        }
        std::string name(length, '\0');
        fin.read(&name[0], length);
        auto it = m.tensors.find(name);
        if (it == m.tensors.end()) {
            fprintf(stderr, "gpt2_model_load: unknown tensor '%s' in model file\n", name.c_str());
            return false;
        }
        ggml_tensor * t = it->second;
        ggml_set_name(t, name.c_str());
        if (ggml_nelements(t) != nelements || t->ne[0] != ne[0] || t->ne[1] != ne[1]) {
            fprintf(stderr, "gpt2_model_load: tensor '%s' has wrong shape in model file\n", name.c_str());
            return false;
        }
        const size_t bpe = ggml_type_size((ggml_type) ttype);
        if ((nelements * bpe) / ggml_blck_size(t->type) != ggml_nbytes(t)) {
            fprintf(stderr, "gpt2_model_load: tensor '%s' has wrong size in model file\n", name.c_str());
            return false;
        }
        const size_t nb = ggml_nbytes(t);
        if (t->buffer && ggml_backend_buffer_is_host(t->buffer)) {
            fin.read((char *) t->data, nb);
        } else {
            buf.resize(nb);
            fin.read(buf.data(), nb);
            ggml_backend_tensor_set(t, buf.data(), 0, nb);
        }
        if (!fin) {
            fprintf(stderr, "gpt2_model_load: truncated model file at '%s'\n", name.c_str());
            return false;
        }
        if (name == "model/wte" && !has_lm_head) m.lm_head = t;  // tied embedding
        if (name == "model/lm_head") has_lm_head = true;
        m.weight_bytes += nb;
    }
    return true;
}

// gpt2_graph, main-backend.cpp:442-717
ggml_cgraph * build_graph(gpt2_model & m, int n_past, int N, int slot = 0) {
    const auto & hp = m.hp;
    const int n_embd = hp.n_embd, n_layer = hp.n_layer, n_ctx = hp.n_ctx, n_head = hp.n_head;

    const size_t buf_size = ggml_tensor_overhead() * kMaxNodes + ggml_graph_overhead_custom(kMaxNodes, false);
    std::vector<uint8_t> & arena = m.graph_buf[slot];
    if (arena.size() != buf_size) arena.resize(buf_size);
    ggml_init_params ip = {buf_size, arena.data(), true};
    ggml_context * ctx = ggml_init(ip);
    ggml_cgraph * gf = ggml_new_graph_custom(ctx, kMaxNodes, false);

    ggml_tensor * embd, * position;
    if (m.host_io) {
        // pinned host token ids read in place; pos_in (device) holds 0 .. n_ctx - 1 for good, so a graph's positions are a
        // view at n_past and only the token ids change per eval
        embd = ggml_view_1d(ctx, m.embd_in, N, 0);
        position = ggml_view_1d(ctx, m.pos_in, N, (size_t) n_past * sizeof(int32_t));
    } else if (m.embd_in) {
        // scheduler mode: views of persistent input tensors (main-sched.cpp:562-570)
        embd = ggml_view_1d(ctx, m.embd_in, N, 0);
        position = ggml_view_1d(ctx, m.pos_in, N, 0);
    } else {
        embd = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, N);
        ggml_set_name(embd, "embd");
        ggml_set_input(embd);
        position = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, N);
        ggml_set_name(position, "position");
        ggml_set_input(position);
    }

    ggml_tensor * inpL = ggml_add(ctx, ggml_get_rows(ctx, m.wte, embd), ggml_get_rows(ctx, m.wpe, position));

    const size_t esk = ggml_element_size(m.memory_k), esv = ggml_element_size(m.memory_v);
    for (int il = 0; il < n_layer; ++il) {
        const layer_w & L = m.layers[il];
        ggml_tensor * cur = ggml_norm(ctx, inpL, hp.eps);
        cur = ggml_add(ctx, ggml_mul(ctx, cur, L.ln_1_g), L.ln_1_b);

        cur = ggml_mul_mat(ctx, L.c_attn_attn_w, cur);
        cur = ggml_add(ctx, cur, L.c_attn_attn_b);

        {
            ggml_tensor * Qcur = ggml_view_2d(ctx, cur, n_embd, N, cur->nb[1], 0 * sizeof(float) * n_embd);
            ggml_tensor * Kcur = ggml_view_2d(ctx, cur, n_embd, N, cur->nb[1], 1 * sizeof(float) * n_embd);
            ggml_tensor * Vcur = ggml_view_2d(ctx, cur, n_embd, N, cur->nb[1], 2 * sizeof(float) * n_embd);

            ggml_tensor * k = ggml_view_1d(ctx, m.memory_k, (int64_t) N * n_embd, (esk * n_embd) * (il * n_ctx + n_past));
            ggml_tensor * v = ggml_view_1d(ctx, m.memory_v, (int64_t) N * n_embd, (esv * n_embd) * (il * n_ctx + n_past));
            ggml_build_forward_expand(gf, ggml_cpy(ctx, Kcur, k));
            ggml_build_forward_expand(gf, ggml_cpy(ctx, Vcur, v));

            ggml_tensor * Q = ggml_permute(ctx, ggml_cont_3d(ctx, Qcur, n_embd / n_head, n_head, N), 0, 2, 1, 3);
            ggml_tensor * K = ggml_permute(
                ctx,
                ggml_reshape_3d(ctx, ggml_view_1d(ctx, m.memory_k, (int64_t) (n_past + N) * n_embd, il * n_ctx * esk * n_embd),
                                n_embd / n_head, n_head, n_past + N),
                0, 2, 1, 3);
            ggml_tensor * KQ = ggml_mul_mat(ctx, K, Q);
            ggml_tensor * KQ_scaled = ggml_scale(ctx, KQ, 1.0f / sqrtf(float(n_embd) / n_head));
            ggml_tensor * KQ_masked = ggml_diag_mask_inf(ctx, KQ_scaled, n_past);
            ggml_tensor * KQ_soft_max = ggml_soft_max(ctx, KQ_masked);
            ggml_tensor * V_trans = ggml_cont_3d(
                ctx,
                ggml_permute(ctx,
                             ggml_reshape_3d(ctx,
                                             ggml_view_1d(ctx, m.memory_v, (int64_t) (n_past + N) * n_embd, il * n_ctx * esv * n_embd),
                                             n_embd / n_head, n_head, n_past + N),
                             1, 2, 0, 3),
                n_past + N, n_embd / n_head, n_head);
            ggml_tensor * KQV = ggml_mul_mat(ctx, V_trans, KQ_soft_max);
            ggml_tensor * KQV_merged = ggml_permute(ctx, KQV, 0, 2, 1, 3);
            cur = ggml_cont_2d(ctx, KQV_merged, n_embd, N);
        }

        cur = ggml_mul_mat(ctx, L.c_attn_proj_w, cur);
        cur = ggml_add(ctx, cur, L.c_attn_proj_b);
        cur = ggml_add(ctx, cur, inpL);
        ggml_tensor * inpFF = cur;

        cur = ggml_norm(ctx, inpFF, hp.eps);
        cur = ggml_add(ctx, ggml_mul(ctx, cur, L.ln_2_g), L.ln_2_b);
        cur = ggml_mul_mat(ctx, L.c_mlp_fc_w, cur);
        cur = ggml_add(ctx, cur, L.c_mlp_fc_b);
        cur = ggml_gelu(ctx, cur);
        cur = ggml_mul_mat(ctx, L.c_mlp_proj_w, cur);
        cur = ggml_add(ctx, cur, L.c_mlp_proj_b);

        inpL = ggml_add(ctx, cur, inpFF);
    }

    inpL = ggml_norm(ctx, inpL, hp.eps);
    inpL = ggml_add(ctx, ggml_mul(ctx, inpL, m.ln_f_g), m.ln_f_b);
    inpL = ggml_mul_mat(ctx, m.lm_head, inpL);
    ggml_set_name(inpL, "logits");
    ggml_set_output(inpL);
    ggml_build_forward_expand(gf, inpL);
    ggml_free(ctx);  // the context memory is graph_buf; the graph stays valid until the next build
    return gf;
}

// gpt2_graph of examples/gpt-2/main-batched.cpp:552-717: n_tokens tokens of any sequences at
// their own positions, written to the KV cells kv_head.., attending to the first n_kv cells
// through KQ_mask ([n_kv, n_tokens], 0 or -inf, broadcast over the heads)
ggml_cgraph * build_graph_batched(gpt2_model & m, int n_tokens, int n_kv, int kv_head, int slot = 0) {
    const auto & hp = m.hp;
    const int n_embd = hp.n_embd, n_layer = hp.n_layer, n_ctx = hp.n_ctx, n_head = hp.n_head;
    const size_t buf_size = ggml_tensor_overhead() * kMaxNodes + ggml_graph_overhead_custom(kMaxNodes, false);
    std::vector<uint8_t> & arena = m.graph_buf[slot];
    if (arena.size() != buf_size) arena.resize(buf_size);
    ggml_init_params ip = {buf_size, arena.data(), true};
    ggml_context * ctx = ggml_init(ip);
    ggml_cgraph * gf = ggml_new_graph_custom(ctx, kMaxNodes, false);

    ggml_tensor * inp_tokens = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, n_tokens);
    ggml_tensor * position = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, n_tokens);
    ggml_tensor * KQ_mask = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, n_kv, n_tokens, 1);
    if (m.bin_dev) {
        // placed in the persistent device input block [tokens | pos | mask] (one async copy per
        // step; the graph allocator leaves tensors that already have memory alone)
        char * base = (char *) m.bin_dev->data;
        inp_tokens->data = base;
        position->data = base + (size_t) n_tokens * 4;
        KQ_mask->data = base + (size_t) 2 * n_tokens * 4;
        inp_tokens->buffer = position->buffer = KQ_mask->buffer = m.buf_bin_dev;
    }
    ggml_set_name(inp_tokens, "inp_tokens");
    ggml_set_input(inp_tokens);
    ggml_set_name(position, "position");
    ggml_set_input(position);
    ggml_tensor * inpL = ggml_add(ctx, ggml_get_rows(ctx, m.wte, inp_tokens), ggml_get_rows(ctx, m.wpe, position));
    ggml_set_name(KQ_mask, "KQ_mask");
    ggml_set_input(KQ_mask);

    const size_t esk = ggml_element_size(m.memory_k), esv = ggml_element_size(m.memory_v);
    for (int il = 0; il < n_layer; ++il) {
        const layer_w & L = m.layers[il];
        ggml_tensor * cur = ggml_norm(ctx, inpL, hp.eps);
        cur = ggml_add(ctx, ggml_mul(ctx, cur, L.ln_1_g), L.ln_1_b);
        cur = ggml_mul_mat(ctx, L.c_attn_attn_w, cur);
        cur = ggml_add(ctx, cur, L.c_attn_attn_b);
        {
            ggml_tensor * Qcur = ggml_view_2d(ctx, cur, n_embd, n_tokens, cur->nb[1], 0 * sizeof(float) * n_embd);
            ggml_tensor * Kcur = ggml_view_2d(ctx, cur, n_embd, n_tokens, cur->nb[1], 1 * sizeof(float) * n_embd);
            ggml_tensor * Vcur = ggml_view_2d(ctx, cur, n_embd, n_tokens, cur->nb[1], 2 * sizeof(float) * n_embd);
            ggml_tensor * k = ggml_view_1d(ctx, m.memory_k, (int64_t) n_tokens * n_embd, (esk * n_embd) * (il * n_ctx + kv_head));
            ggml_tensor * v = ggml_view_1d(ctx, m.memory_v, (int64_t) n_tokens * n_embd, (esv * n_embd) * (il * n_ctx + kv_head));
            ggml_build_forward_expand(gf, ggml_cpy(ctx, Kcur, k));
            ggml_build_forward_expand(gf, ggml_cpy(ctx, Vcur, v));

            ggml_tensor * Q = ggml_permute(ctx, ggml_cont_3d(ctx, Qcur, n_embd / n_head, n_head, n_tokens), 0, 2, 1, 3);
            ggml_tensor * K = ggml_permute(
                ctx,
                ggml_reshape_3d(ctx, ggml_view_1d(ctx, m.memory_k, (int64_t) n_kv * n_embd, il * n_ctx * esk * n_embd),
                                n_embd / n_head, n_head, n_kv),
                0, 2, 1, 3);
            ggml_tensor * KQ = ggml_mul_mat(ctx, K, Q);
            ggml_tensor * KQ_scaled = ggml_scale(ctx, KQ, 1.0f / sqrtf(float(n_embd) / n_head));
            ggml_tensor * KQ_masked = ggml_add(ctx, KQ_scaled, KQ_mask);
            ggml_tensor * KQ_soft_max = ggml_soft_max(ctx, KQ_masked);
            ggml_tensor * V_trans = ggml_cont_3d(
                ctx,
                ggml_permute(ctx,
                             ggml_reshape_3d(ctx, ggml_view_1d(ctx, m.memory_v, (int64_t) n_kv * n_embd, il * n_ctx * esv * n_embd),
                                             n_embd / n_head, n_head, n_kv),
                             1, 2, 0, 3),
                n_kv, n_embd / n_head, n_head);
            ggml_tensor * KQV = ggml_mul_mat(ctx, V_trans, KQ_soft_max);
            ggml_tensor * KQV_merged = ggml_permute(ctx, KQV, 0, 2, 1, 3);
            cur = ggml_cont_2d(ctx, KQV_merged, n_embd, n_tokens);
        }
        cur = ggml_mul_mat(ctx, L.c_attn_proj_w, cur);
        cur = ggml_add(ctx, cur, L.c_attn_proj_b);
        cur = ggml_add(ctx, cur, inpL);
        ggml_tensor * inpFF = cur;
        cur = ggml_norm(ctx, inpFF, hp.eps);
        cur = ggml_add(ctx, ggml_mul(ctx, cur, L.ln_2_g), L.ln_2_b);
        cur = ggml_mul_mat(ctx, L.c_mlp_fc_w, cur);
        cur = ggml_add(ctx, cur, L.c_mlp_fc_b);
        cur = ggml_gelu(ctx, cur);
        cur = ggml_mul_mat(ctx, L.c_mlp_proj_w, cur);
        cur = ggml_add(ctx, cur, L.c_mlp_proj_b);
        inpL = ggml_add(ctx, cur, inpFF);
    }
    inpL = ggml_norm(ctx, inpL, hp.eps);
    inpL = ggml_add(ctx, ggml_mul(ctx, inpL, m.ln_f_g), m.ln_f_b);
    inpL = ggml_mul_mat(ctx, m.lm_head, inpL);
    ggml_set_name(inpL, "logits");
    ggml_set_output(inpL);
    ggml_build_forward_expand(gf, inpL);
    ggml_free(ctx);
    return gf;
}

void split_words(std::string str, std::vector<std::string> & words) {
    // examples/common.cpp:272-283
    static const std::regex re(R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
    std::smatch sm;
    while (std::regex_search(str, sm, re)) {
        for (auto x : sm) words.push_back(x);
        str = sm.suffix();
    }
}

} // namespace

extern "C" {

gpt2_model * gpt2_model_load(const char * fname, ggml_backend_t backend, int n_ctx, int n_batch) {
    return gpt2_model_load_ex(fname, backend, n_ctx, n_batch, nullptr);
}

gpt2_model * gpt2_model_load_ex(const char * fname, ggml_backend_t backend, int n_ctx, int n_batch,
                                ggml_backend_buffer_type_t host_buft) {
    if (!backend) {
        fprintf(stderr, "gpt2_model_load: no backend\n");
        return nullptr;
    }
    auto * m = new gpt2_model();
    m->backend = backend;
    if (!load_file(*m, fname, n_ctx)) {
        gpt2_model_free(m);
        return nullptr;
    }
    const int n_tokens = std::min(m->hp.n_ctx, n_batch > 0 ? n_batch : 8);
    if (host_buft) {
        ggml_init_params ip = {ggml_tensor_overhead() * 3, nullptr, true};
        m->ctx_in = ggml_init(ip);
        m->embd_in = ggml_new_tensor_1d(m->ctx_in, GGML_TYPE_I32, m->hp.n_ctx);
        m->logits_host = ggml_new_tensor_2d(m->ctx_in, GGML_TYPE_F32, m->hp.n_vocab, n_tokens);
        // positions never change (0 .. n_ctx - 1, a graph views its slice): they live on the
        // device, so a decode step's only host read is its token id
        m->ctx_pos = ggml_init(ip);
        m->pos_in = ggml_new_tensor_1d(m->ctx_pos, GGML_TYPE_I32, m->hp.n_ctx);
        m->buffer_pos = ggml_backend_alloc_ctx_tensors(m->ctx_pos, backend);
        ggml_set_name(m->embd_in, "in/embd");
        ggml_set_name(m->pos_in, "in/position");
        ggml_set_name(m->logits_host, "out/logits");
        m->host_buft = host_buft;
        m->buffer_input = ggml_backend_alloc_ctx_tensors_from_buft(m->ctx_in, host_buft);
        // the device reads these in place: a buffer the type fell back to (e.g. pageable memory,
        // another buffer type) will not do
        if (!m->buffer_input || m->buffer_input->buft != host_buft || !ggml_backend_buffer_is_host(m->buffer_input) ||
            !m->buffer_pos) {
            fprintf(stderr, "gpt2_model_load: host input buffer allocation failed (or not a host buffer type)\n");
            gpt2_model_free(m);
            return nullptr;
        }
        std::vector<int32_t> pos(m->hp.n_ctx);
        for (int i = 0; i < m->hp.n_ctx; i++) pos[i] = i;
        ggml_backend_tensor_set(m->pos_in, pos.data(), 0, pos.size() * sizeof(int32_t));
        m->host_io = true;
    }
    m->allocr = ggml_gallocr_new(ggml_backend_get_default_buffer_type(backend));
    ggml_cgraph * gf = build_graph(*m, m->hp.n_ctx - n_tokens, n_tokens);
    if (!ggml_gallocr_reserve(m->allocr, gf)) {
        fprintf(stderr, "gpt2_model_load: compute buffer reservation failed\n");
        gpt2_model_free(m);
        return nullptr;
    }
    return m;
}

gpt2_model * gpt2_model_load_sched(const char * fname, ggml_backend_t * backends, int n_backends, int n_gpu_layers, int n_ctx,
                                   int n_batch) {
    return gpt2_model_load_sched_ex(fname, backends, n_backends, n_gpu_layers, n_ctx, n_batch, 0, nullptr);
}

gpt2_model * gpt2_model_load_sched_ex(const char * fname, ggml_backend_t * backends, int n_backends, int n_gpu_layers,
                                      int n_ctx, int n_batch, int flags, ggml_backend_buffer_type_t input_buft) {
#ifdef GPT2_WITH_SCHED
    if (!backends || n_backends < 1) {
        fprintf(stderr, "gpt2_model_load_sched: no backends\n");
        return nullptr;
    }
    auto * m = new gpt2_model();
    m->backends.assign(backends, backends + n_backends);
    m->backend = backends[n_backends - 1];
    m->n_gpu_layers = n_backends > 1 ? n_gpu_layers : 0;
    m->sched_flags = flags;
    if (!load_file(*m, fname, n_ctx)) {
        gpt2_model_free(m);
        return nullptr;
    }
    // persistent inputs (main-sched.cpp:512-534): on the GPU only when every layer is
    {
        ggml_init_params ip = {ggml_tensor_overhead() * 2, nullptr, true};
        m->ctx_in = ggml_init(ip);
        m->embd_in = ggml_new_tensor_1d(m->ctx_in, GGML_TYPE_I32, m->hp.n_ctx);
        m->pos_in = ggml_new_tensor_1d(m->ctx_in, GGML_TYPE_I32, m->hp.n_ctx);
        ggml_set_name(m->embd_in, "in/embd");
        ggml_set_name(m->pos_in, "in/position");
        ggml_backend_t be_in = m->n_gpu_layers >= m->hp.n_layer ? m->backends.front() : m->backends.back();
        m->buffer_input = input_buft ? ggml_backend_alloc_ctx_tensors_from_buft(m->ctx_in, input_buft)
                                     : ggml_backend_alloc_ctx_tensors(m->ctx_in, be_in);
        if (!m->buffer_input) {
            gpt2_model_free(m);
            return nullptr;
        }
    }
    auto * sched = ggml_backend_sched_new(m->backends.data(), nullptr, n_backends, kMaxNodes, (flags & GPT2_SCHED_PARALLEL) != 0);
    m->sched = sched;
    const int n_tokens = std::min(m->hp.n_ctx, n_batch > 0 ? n_batch : 8);
    ggml_cgraph * gf = build_graph(*m, m->hp.n_ctx - n_tokens, n_tokens);
    if (!ggml_backend_sched_reserve(sched, gf)) {
        fprintf(stderr, "gpt2_model_load_sched: compute buffer reservation failed\n");
        gpt2_model_free(m);
        return nullptr;
    }
    return m;
#else
    (void) fname; (void) backends; (void) n_backends; (void) n_gpu_layers; (void) n_ctx; (void) n_batch; (void) flags;
    (void) input_buft;
    fprintf(stderr, "gpt2_model_load_sched: this build has no ggml_backend_sched (link the driver against a libggml "
                    "that provides it, e.g. oracle/_ref/libgpt2_ref.so)\n");
    return nullptr;
#endif
}

int gpt2_sched_n_splits(const gpt2_model * m) {
#ifdef GPT2_WITH_SCHED
    return m->sched ? ggml_backend_sched_get_n_splits((ggml_backend_sched_t) m->sched) : 0;
#else
    (void) m;
    return 0;
#endif
}

void gpt2_model_free(gpt2_model * m) {
    if (!m) return;
    if (m->next_plan) {
        ggml_backend_synchronize(m->backend);
        ggml_backend_graph_plan_free(m->backend, m->next_plan);
    }
#ifdef GPT2_WITH_SCHED
    if (m->sched) ggml_backend_sched_free((ggml_backend_sched_t) m->sched);
#endif
    if (m->bnext_plan) {
        ggml_backend_synchronize(m->backend);
        ggml_backend_graph_plan_free(m->backend, m->bnext_plan);
    }
    if (m->buf_bin_host) ggml_backend_buffer_free(m->buf_bin_host);
    if (m->buf_bin_dev) ggml_backend_buffer_free(m->buf_bin_dev);
    if (m->ctx_bin) ggml_free(m->ctx_bin);
    if (m->buffer_input) ggml_backend_buffer_free(m->buffer_input);
    if (m->ctx_in) ggml_free(m->ctx_in);
    if (m->buffer_pos) ggml_backend_buffer_free(m->buffer_pos);
    if (m->ctx_pos) ggml_free(m->ctx_pos);
    for (ggml_backend_buffer_t b : m->buffers_w) if (b) ggml_backend_buffer_free(b);
    if (m->allocr) ggml_gallocr_free(m->allocr);
    if (m->buffer_w) ggml_backend_buffer_free(m->buffer_w);
    if (m->buffer_kv) ggml_backend_buffer_free(m->buffer_kv);
    if (m->ctx_w) ggml_free(m->ctx_w);
    if (m->ctx_kv) ggml_free(m->ctx_kv);
    delete m;
}

void gpt2_model_hparams(const gpt2_model * m, gpt2_hparams_c * out) { *out = m->hp; }

// ---- batched independent sequences (examples/gpt-2/main-batched.cpp) ------------------------------

void gpt2_kv_cache_clear(gpt2_model * m) {
    m->cells.assign((size_t) m->hp.n_ctx, gpt2_model::kv_cell());
    m->kv_head = m->kv_n = 0;
}

// gpt2_kv_cache_seq_cp (main-batched.cpp:814-827): cells of seq_src at positions [p0, p1) are seen by
// seq_dst too (p0 < 0: from 0, p1 < 0: to the end)
void gpt2_kv_cache_seq_cp(gpt2_model * m, int32_t seq_src, int32_t seq_dst, int32_t p0, int32_t p1) {
    if (m->cells.size() != (size_t) m->hp.n_ctx) gpt2_kv_cache_clear(m);
    if (p0 < 0) p0 = 0;
    if (p1 < 0) p1 = INT32_MAX;
    for (auto & c : m->cells) {
        if (c.has(seq_src) && c.pos >= p0 && c.pos < p1 && !c.has(seq_dst)) c.seq.push_back(seq_dst);
    }
}

// gpt2_decode (main-batched.cpp:854-968): the batch's tokens go into KV cells kv_head.., the graph
// attends to cells [0, kv_head + n_tokens) through the host-built KQ mask (a cell is visible to a
// token when it belongs to the token's sequence at a position <= the token's)
// the batched path's prebuilt graph / plan (arenas and allocator are shared with gpt2_eval's)
static void drop_batch_prebuilt(gpt2_model * m) {
    if (m->bnext_plan) {
        ggml_backend_synchronize(m->backend);
        ggml_backend_graph_plan_free(m->backend, m->bnext_plan);
        m->bnext_plan = nullptr;
    }
    m->bnext_gf = nullptr;
    m->bnext_tokens = m->bnext_head = -1;
}

// host_io: the pinned staging block and the device input block, grown to hold n_tokens tokens and
// positions and an n_ctx x n_tokens mask
static bool batch_inputs_reserve(gpt2_model * m, int n_tokens) {
    const size_t need = (size_t) 2 * n_tokens * 4 + (size_t) m->hp.n_ctx * n_tokens * 4;
    if (!m->bin_dev || ggml_nbytes(m->bin_dev) < need) {
        drop_batch_prebuilt(m);
        ggml_backend_synchronize(m->backend);
        if (m->buf_bin_host) ggml_backend_buffer_free(m->buf_bin_host);
        if (m->buf_bin_dev) ggml_backend_buffer_free(m->buf_bin_dev);
        if (m->ctx_bin) ggml_free(m->ctx_bin);
        m->bin_host = m->bin_dev = nullptr;
        m->buf_bin_host = m->buf_bin_dev = nullptr;
        ggml_init_params ip = {ggml_tensor_overhead() * 2, nullptr, true};
        m->ctx_bin = ggml_init(ip);
        ggml_tensor * h = ggml_new_tensor_1d(m->ctx_bin, GGML_TYPE_F32, (int64_t) (need / 4));
        ggml_tensor * d = ggml_new_tensor_1d(m->ctx_bin, GGML_TYPE_F32, (int64_t) (need / 4));
        ggml_set_name(h, "in/batch_host");
        ggml_set_name(d, "in/batch");
        m->buf_bin_host = ggml_backend_buft_alloc_buffer(m->host_buft, ggml_backend_buft_get_alloc_size(m->host_buft, h));
        m->buf_bin_dev = ggml_backend_alloc_buffer(m->backend, ggml_nbytes(d) + 256);
        if (!m->buf_bin_host || !m->buf_bin_dev) return false;
        ggml_tallocr ah = ggml_tallocr_new(m->buf_bin_host);
        ggml_tallocr_alloc(&ah, h);
        ggml_tallocr ad = ggml_tallocr_new(m->buf_bin_dev);
        ggml_tallocr_alloc(&ad, d);
        m->bin_host = h;
        m->bin_dev = d;
    }
    if (m->batch_reserved < n_tokens) {
        // the compute buffer sized for this batch at a full KV cache, once, while nothing runs: a
        // graph allocated during the previous step's execution must never grow (reallocate) it
        drop_batch_prebuilt(m);
        ggml_backend_synchronize(m->backend);
        ggml_cgraph * worst = build_graph_batched(*m, n_tokens, m->hp.n_ctx, m->hp.n_ctx - n_tokens, m->graph_slot ^ 1);
        if (!ggml_gallocr_reserve(m->allocr, worst)) return false;
        m->batch_reserved = n_tokens;
    }
    return true;
}

int gpt2_decode_batch(gpt2_model * m, int n_tokens, const int32_t * tokens, const int32_t * pos, const int32_t * seq_id,
                      float * logits, int all_logits) {
    if (n_tokens <= 0 || !tokens || !pos || !seq_id) {
        fprintf(stderr, "gpt2_decode_batch: empty batch\n");
        return -1;
    }
    if (m->sched) {
        fprintf(stderr, "gpt2_decode_batch: not available in scheduler mode\n");
        return -1;
    }
    if (m->cells.size() != (size_t) m->hp.n_ctx) gpt2_kv_cache_clear(m);
    if (m->kv_head + (uint32_t) n_tokens > (uint32_t) m->hp.n_ctx) {
        fprintf(stderr, "gpt2_decode_batch: KV cache full (%u + %d > %d)\n", m->kv_head, n_tokens, m->hp.n_ctx);
        return -2;
    }
    // the decode loop's prebuilt graph (gpt2_eval) would reuse the arena and allocator: dropped
    if (m->next_plan) {
        ggml_backend_synchronize(m->backend);
        ggml_backend_graph_plan_free(m->backend, m->next_plan);
        m->next_plan = nullptr;
    }
    m->next_gf = nullptr;
    const int64_t t0 = now_us();
    for (int i = 0; i < n_tokens; i++) {
        auto & c = m->cells[m->kv_head + i];
        c.pos = pos[i];
        c.seq.clear();
        c.seq.push_back(seq_id[i]);
    }
    m->kv_n = m->kv_head + (uint32_t) n_tokens;
    const int n_kv = (int) m->kv_n;
    const size_t nv = (size_t) m->hp.n_vocab;
    const size_t lg_off = all_logits ? 0 : sizeof(float) * nv * (n_tokens - 1), lg_size = sizeof(float) * nv * (all_logits ? n_tokens : 1);
    // host_io (pinned staging): inputs in one async copy, the step launched as a plan prebuilt during
    // the previous step, the logits staged behind it, the next step prebuilt while this one runs
    const bool fast = m->host_io && m->backend->iface.graph_plan_create && lg_size <= ggml_nbytes(m->logits_host) &&
                      batch_inputs_reserve(m, n_tokens);
    ggml_cgraph * gf = nullptr;
    ggml_backend_graph_plan_t plan = nullptr;
    int64_t t1, t2;
    if (fast && m->bnext_gf && m->bnext_tokens == n_tokens && m->bnext_head == (int) m->kv_head) {
        gf = m->bnext_gf;
        plan = m->bnext_plan;
        m->bnext_plan = nullptr;
        m->bnext_gf = nullptr;
        m->graph_slot ^= 1;
        m->batch_plans++;
        t1 = t2 = now_us();
    } else {
        drop_batch_prebuilt(m);
        m->graph_slot ^= 1;
        gf = build_graph_batched(*m, n_tokens, n_kv, (int) m->kv_head, m->graph_slot);
        t1 = now_us();
        if (!ggml_gallocr_alloc_graph(m->allocr, gf)) {
            fprintf(stderr, "gpt2_decode_batch: graph allocation failed\n");
            return 1;
        }
        m->batch_direct++;
        t2 = now_us();
    }
    if (fast) {
        // [tokens | pos | mask] into the pinned block, one async copy into the device block
        char * hb = (char *) m->bin_host->data;
        memcpy(hb, tokens, (size_t) n_tokens * 4);
        memcpy(hb + (size_t) n_tokens * 4, pos, (size_t) n_tokens * 4);
        float * mask = (float *) (hb + (size_t) 2 * n_tokens * 4);
        for (int j = 0; j < n_tokens; j++) {
            for (int i = 0; i < n_kv; i++) {
                const auto & c = m->cells[i];
                mask[(size_t) j * n_kv + i] = (!c.has(seq_id[j]) || c.pos > pos[j]) ? -INFINITY : 0.0f;
            }
        }
        ggml_backend_tensor_set_async(m->backend, m->bin_dev, hb, 0, (size_t) 2 * n_tokens * 4 + (size_t) n_kv * n_tokens * 4);
    } else {
        ggml_backend_tensor_set(ggml_graph_get_tensor(gf, "inp_tokens"), tokens, 0, (size_t) n_tokens * sizeof(int32_t));
        ggml_backend_tensor_set(ggml_graph_get_tensor(gf, "position"), pos, 0, (size_t) n_tokens * sizeof(int32_t));
        std::vector<float> mask((size_t) n_kv * n_tokens, 0.0f);
        for (int j = 0; j < n_tokens; j++) {
            for (int i = 0; i < n_kv; i++) {
                const auto & c = m->cells[i];
                if (!c.has(seq_id[j]) || c.pos > pos[j]) mask[(size_t) j * n_kv + i] = -INFINITY;
            }
        }
        ggml_backend_tensor_set(ggml_graph_get_tensor(gf, "KQ_mask"), mask.data(), 0, mask.size() * sizeof(float));
    }
    const int64_t t3 = now_us();
    ggml_tensor * out = ggml_graph_get_tensor(gf, "logits");
    m->kv_head += (uint32_t) n_tokens;
    m->last_nodes = gf->n_nodes;
    if (!fast) {
        if (ggml_backend_graph_compute(m->backend, gf) != GGML_STATUS_SUCCESS) {
            fprintf(stderr, "gpt2_decode_batch: graph compute failed\n");
            return 1;
        }
        // logits == nullptr: into the pinned staging, read in place by the caller (gpt2_logits_host)
        float * dl = logits ? logits : (m->host_io && lg_size <= ggml_nbytes(m->logits_host) ? (float *) m->logits_host->data : nullptr);
        if (!dl) {
            fprintf(stderr, "gpt2_decode_batch: no logits destination (staging too small)\n");
            return -3;
        }
        ggml_backend_tensor_get(out, dl, lg_off, lg_size);
    } else {
        const ggml_status st = plan ? ggml_backend_graph_plan_compute(m->backend, plan) : ggml_backend_graph_compute_async(m->backend, gf);
        if (st != GGML_STATUS_SUCCESS) {
            fprintf(stderr, "gpt2_decode_batch: graph compute failed\n");
            if (plan) ggml_backend_graph_plan_free(m->backend, plan);
            return 1;
        }
        ggml_backend_tensor_get_async(m->backend, out, m->logits_host->data, lg_off, lg_size);
        // the next step of the same batch size (one token per sequence: main-batched.cpp's loop),
        // built, allocated and captured while the device runs this one; its inputs are data
        const int nh = (int) m->kv_head;
        if (nh + n_tokens <= m->hp.n_ctx) {
            ggml_cgraph * nx = build_graph_batched(*m, n_tokens, nh + n_tokens, nh, m->graph_slot ^ 1);
            if (ggml_gallocr_alloc_graph(m->allocr, nx)) {
                m->bnext_gf = nx;
                m->bnext_tokens = n_tokens;
                m->bnext_head = nh;
                m->bnext_plan = ggml_backend_graph_plan_create(m->backend, nx);
            }
        }
        ggml_backend_synchronize(m->backend);
        if (plan) ggml_backend_graph_plan_free(m->backend, plan);  // its graph has run
        if (logits) memcpy(logits, m->logits_host->data, lg_size);  // else: the caller reads gpt2_logits_host()
    }
    m->us_build = t1 - t0;
    m->us_alloc = t2 - t1;
    m->us_inputs = t3 - t2;
    m->us_compute = now_us() - t3;
    return 0;
}

void gpt2_batch_stats(const gpt2_model * m, int64_t * out2) {
    out2[0] = m->batch_plans;
    out2[1] = m->batch_direct;
}

size_t gpt2_model_size(const gpt2_model * m) { return m->weight_bytes; }
size_t gpt2_compute_buffer_size(const gpt2_model * m) { return ggml_gallocr_get_buffer_size(m->allocr, 0); }

int gpt2_eval(gpt2_model * m, int n_past, const int32_t * tokens, int N, float * logits, int all_logits) {
    // positions index wpe, which has the file's context length even when the KV cache is larger
    if (N <= 0 || n_past < 0 || n_past + N > m->hp.n_ctx || n_past + N > m->wpe->ne[1]) {
        fprintf(stderr, "gpt2_eval: bad token range (n_past %d, n_tokens %d, n_ctx %d, wpe rows %d)\n", n_past, N,
                m->hp.n_ctx, (int) m->wpe->ne[1]);
        return 1;
    }
    for (int i = 0; i < N; i++) {
        if (tokens[i] < 0 || tokens[i] >= m->hp.n_vocab) {
            fprintf(stderr, "gpt2_eval: token %d out of range\n", tokens[i]);
            return 1;
        }
    }
#ifdef GPT2_WITH_SCHED
    if (m->sched) {
        // main-sched.cpp:854-884: inputs into the persistent tensors, sched reset + compute
        const int64_t t0 = now_us();
        ggml_backend_tensor_set(m->embd_in, tokens, 0, (size_t) N * sizeof(int32_t));
        m->pos.resize(N);
        for (int i = 0; i < N; i++) m->pos[i] = n_past + i;
        ggml_backend_tensor_set(m->pos_in, m->pos.data(), 0, (size_t) N * sizeof(int32_t));
        ggml_cgraph * gf = build_graph(*m, n_past, N);
        const int64_t t1 = now_us();
        auto * sched = (ggml_backend_sched_t) m->sched;
        ggml_backend_sched_reset(sched);
        if (ggml_backend_sched_graph_compute(sched, gf) != GGML_STATUS_SUCCESS) {
            fprintf(stderr, "gpt2_eval: scheduler compute failed\n");
            return 1;
        }
        ggml_tensor * out = gf->nodes[gf->n_nodes - 1];
        const size_t nv = (size_t) m->hp.n_vocab;
        if (all_logits) ggml_backend_tensor_get(out, logits, 0, sizeof(float) * nv * N);
        else ggml_backend_tensor_get(out, logits, sizeof(float) * nv * (N - 1), sizeof(float) * nv);
        m->last_nodes = gf->n_nodes;
        m->us_build = t1 - t0;
        m->us_alloc = m->us_inputs = 0;
        m->us_compute = now_us() - t1;
        return 0;
    }
#endif
    drop_batch_prebuilt(m);
    const int64_t t0 = now_us();
    ggml_cgraph * gf;
    int64_t t1, t1b;
    ggml_backend_graph_plan_t plan = nullptr;
    if (m->next_gf && m->next_n_past == n_past && N == 1) {
        // built and allocated while the device ran the previous token (graph_slot ^ 1)
        gf = m->next_gf;
        plan = m->next_plan;  // owned here from now on: freed once its graph has run
        m->next_plan = nullptr;
        m->graph_slot ^= 1;
        t1 = t1b = t0;
    } else {
        if (m->next_plan) ggml_backend_graph_plan_free(m->backend, m->next_plan);
        m->next_plan = nullptr;
        m->graph_slot ^= 1;
        gf = build_graph(*m, n_past, N, m->graph_slot);
        t1 = now_us();
        if (!ggml_gallocr_alloc_graph(m->allocr, gf)) {
            m->next_gf = nullptr;
            fprintf(stderr, "gpt2_eval: graph allocation failed\n");
            return 1;
        }
        t1b = now_us();
    }
    m->next_gf = nullptr;
    if (m->host_io) {
        // the device reads the ids in place: the previous eval synchronized, so nothing reads them now
        memcpy(m->embd_in->data, tokens, (size_t) N * sizeof(int32_t));
    } else {
        // inputs go in on the backend's queue, ordered before the graph (ggml_backend_tensor_set_async,
        // ggml-backend.h): no host round trip per input
        ggml_tensor * embd = ggml_graph_get_tensor(gf, "embd");
        ggml_tensor * position = ggml_graph_get_tensor(gf, "position");
        m->pos.resize(N);
        m->tok.assign(tokens, tokens + N);
        for (int i = 0; i < N; i++) m->pos[i] = n_past + i;
        ggml_backend_tensor_set_async(m->backend, embd, m->tok.data(), 0, (size_t) N * ggml_element_size(embd));
        ggml_backend_tensor_set_async(m->backend, position, m->pos.data(), 0, (size_t) N * sizeof(int32_t));
    }
    const int64_t t2 = now_us();
    const ggml_status st = plan ? ggml_backend_graph_plan_compute(m->backend, plan) : ggml_backend_graph_compute_async(m->backend, gf);
    if (st != GGML_STATUS_SUCCESS) {
        fprintf(stderr, "gpt2_eval: graph compute failed\n");
        if (plan) ggml_backend_graph_plan_free(m->backend, plan);
        return 1;
    }
    ggml_tensor * out = ggml_graph_get_tensor(gf, "logits");
    const size_t nv = (size_t) m->hp.n_vocab;
    const size_t lg_off = all_logits ? 0 : sizeof(float) * nv * (N - 1), lg_size = sizeof(float) * nv * (all_logits ? N : 1);
    // logits staged through host memory by a copy queued right behind the graph
    const bool staged = m->host_io && lg_size <= ggml_nbytes(m->logits_host);
    // (measured against an in-graph CPY into the staging that the lm_head GEMV's epilogue stores
    // over PCIe: slower, the host's next-graph preparation ran ~150 us longer per token, r03y2)
    if (staged) ggml_backend_tensor_get_async(m->backend, out, m->logits_host->data, lg_off, lg_size);
    const int64_t t2b = now_us();
    // While the device runs this graph, build and allocate the next decode step's (one token at
    // n_past + N) in the other arena: the graph depends on positions only, not on the token the
    // caller will pick from these logits. The allocator only assigns addresses in the compute
    // buffer; the next graph's kernels are queued after this one's on the same stream.
    const int np1 = n_past + N;
    if (np1 + 1 <= m->hp.n_ctx && np1 + 1 <= m->wpe->ne[1]) {
        ggml_cgraph * nx = build_graph(*m, np1, 1, m->graph_slot ^ 1);
        if (ggml_gallocr_alloc_graph(m->allocr, nx)) {
            m->next_gf = nx;
            m->next_n_past = np1;
            // and, where the backend has graph plans (MI355X: a captured hipGraph), prepared
            // for a single launch
            if (m->backend->iface.graph_plan_create) m->next_plan = ggml_backend_graph_plan_create(m->backend, nx);
        }
    }
    const int64_t t2c = now_us();
    ggml_backend_synchronize(m->backend);
    const int64_t t2d = now_us();
    if (staged) {
        if (logits) memcpy(logits, m->logits_host->data, lg_size);  // else: the caller reads gpt2_logits_host()
    } else {
        if (!logits) {
            fprintf(stderr, "gpt2_eval: logits == NULL needs the host staging of gpt2_model_load_ex\n");
            if (plan) ggml_backend_graph_plan_free(m->backend, plan);
            return 1;
        }
        ggml_backend_tensor_get(out, logits, lg_off, lg_size);
    }
    const int64_t t3 = now_us();
    if (plan) ggml_backend_graph_plan_free(m->backend, plan);  // its graph has run
    m->us_launch = t2b - t2;
    m->us_prebuild = t2c - t2b;
    m->us_wait = t2d - t2c;
    m->us_readback = t3 - t2d;
    m->last_nodes = gf->n_nodes;
    m->us_build = t1 - t0;
    m->us_alloc = t1b - t1;
    m->us_inputs = t2 - t1b;
    m->us_compute = t3 - t2;
    return 0;
}

const char * gpt2_token_text(const gpt2_model * m, int32_t id) {
    if (id < 0 || id >= (int32_t) m->vocab.id_to_token.size()) return nullptr;
    return m->vocab.id_to_token[id].c_str();
}

int gpt2_tokenize(const gpt2_model * m, const char * text, int32_t * out, int max_tokens) {
    std::vector<std::string> words;
    split_words(text, words);
    // longest vocabulary prefix at each position (examples/common.cpp:322-340)
    int n = 0;
    for (const auto & w : words) {
        for (int i = 0; i < (int) w.size();) {
            for (int j = (int) w.size() - 1; j >= i; j--) {
                auto it = m->vocab.token_to_id.find(w.substr(i, j - i + 1));
                if (it != m->vocab.token_to_id.end()) {
                    if (n < max_tokens) out[n] = it->second;
                    n++;
                    i = j + 1;
                    break;
                } else if (j == i) {
                    fprintf(stderr, "gpt2_tokenize: unknown token '%s'\n", w.substr(i, 1).c_str());
                    i++;
                }
            }
        }
    }
    return n;
}

const float * gpt2_logits_host(const gpt2_model * m) { return m->host_io ? (const float *) m->logits_host->data : nullptr; }

void gpt2_last_eval_timing(const gpt2_model * m, int64_t * us4) {
    us4[0] = m->us_launch;
    us4[1] = m->us_prebuild;
    us4[2] = m->us_wait;
    us4[3] = m->us_readback;
}

void gpt2_last_eval_stats(const gpt2_model * m, int * n_nodes, int64_t * us_build, int64_t * us_alloc, int64_t * us_inputs,
                          int64_t * us_compute) {
    if (n_nodes) *n_nodes = m->last_nodes;
    if (us_build) *us_build = m->us_build;
    if (us_alloc) *us_alloc = m->us_alloc;
    if (us_inputs) *us_inputs = m->us_inputs;
    if (us_compute) *us_compute = m->us_compute;
}

} // extern "C"
