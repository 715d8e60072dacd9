// gpt2-mi355x.h -- GPT-2 decode driver over the ggml backend API (BASELINE config 4).
//
// The model code of examples/gpt-2/main-backend.cpp (NAIST-Archlab/ggml-imax) as a C library:
// the same legacy-ggml file format (:102-439), the same graph (gpt2_graph :442-717) and the same
// evaluation contract (gpt2_eval :728-786), but with the backend passed in by the caller, so one
// build runs on ggml_backend_mi355x_init(dev) and on the reference CPU backend alike.
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

struct gpt2_model;

struct gpt2_hparams_c {
    int32_t n_vocab;
    int32_t n_ctx;    // KV-cache context (the -c override, main-backend.cpp:304)
    int32_t n_embd;
    int32_t n_head;
    int32_t n_layer;
    int32_t ftype;
    float eps;
};

// gpt2_model_load (main-backend.cpp:101): weights and KV cache in `backend`'s default buffer type,
// and a graph allocator reserved for the worst-case graph of n_batch tokens (:832-846).
// n_ctx <= 0 keeps the file's context. Returns NULL (with a message on stderr) on failure.
GGML_API struct gpt2_model * gpt2_model_load(const char * fname, ggml_backend_t backend, int n_ctx, int n_batch);
// The same, with host_buft (a host buffer type the backend's kernels can read, e.g.
// ggml_backend_mi355x_host_buffer_type(); NULL = gpt2_model_load) holding the token ids and
// positions, which the device then reads in place instead of receiving an upload per eval, and a
// staging copy of the logits, copied into right behind the graph on the backend's queue.
GGML_API struct gpt2_model * gpt2_model_load_ex(const char * fname, ggml_backend_t backend, int n_ctx, int n_batch,
                                                ggml_backend_buffer_type_t host_buft);
// examples/gpt-2/main-sched.cpp: layers split over `backends` (the last one is the CPU fallback,
// as ggml_backend_sched requires) by n_gpu_layers, executed through ggml_backend_sched. Needs a
// ggml runtime that provides the scheduler (the reference libggml: oracle/_ref/libgpt2_ref.so);
// other builds return NULL with a message.
GGML_API struct gpt2_model * gpt2_model_load_sched(const char * fname, ggml_backend_t * backends, int n_backends, int n_gpu_layers,
                                                   int n_ctx, int n_batch);
// The same with scheduler options (all off = gpt2_model_load_sched):
//   GPT2_SCHED_PARALLEL   ggml_backend_sched_new(..., parallel = true): input copies + backend
//                         events (ggml-backend.c:1647-1710, :1751-1755)
//   GPT2_SCHED_SPLIT_MID  the attention weights of the last CPU layer go to the GPU as well, so a
//                         split boundary falls inside a layer (between attention and MLP)
// input_buft: buffer type of the persistent input tensors (NULL = main-sched.cpp's choice), e.g.
// ggml_backend_mi355x_host_buffer_type() for pinned host inputs read by both backends.
#define GPT2_SCHED_PARALLEL  1
#define GPT2_SCHED_SPLIT_MID 2
GGML_API struct gpt2_model * gpt2_model_load_sched_ex(const char * fname, ggml_backend_t * backends, int n_backends,
                                                      int n_gpu_layers, int n_ctx, int n_batch, int flags,
                                                      ggml_backend_buffer_type_t input_buft);
GGML_API int gpt2_sched_n_splits(const struct gpt2_model * model);
GGML_API void gpt2_model_free(struct gpt2_model * model);
GGML_API void gpt2_model_hparams(const struct gpt2_model * model, struct gpt2_hparams_c * out);
GGML_API size_t gpt2_model_size(const struct gpt2_model * model);   // bytes of weight data read
GGML_API size_t gpt2_compute_buffer_size(const struct gpt2_model * model);

// gpt2_eval (main-backend.cpp:728): runs n_tokens tokens at positions n_past.. and writes the
// logits of the last token (n_vocab floats), or of all tokens (n_tokens*n_vocab) if all_logits.
// logits may be NULL for a model loaded with a host buffer type (gpt2_model_load_ex): the logits
// are then only in gpt2_logits_host(), valid until the next eval. Returns 0 on success.
GGML_API int gpt2_eval(struct gpt2_model * model, int n_past, const int32_t * tokens, int n_tokens, float * logits,
                       int all_logits);
// Batched independent sequences (examples/gpt-2/main-batched.cpp): the KV cache as cells with
// positions and sequence ids. gpt2_decode_batch (gpt2_decode, :854-968) runs n_tokens tokens, token i
// of sequence seq_id[i] at position pos[i], writing them into the next free cells and attending
// through main-batched's KQ mask; logits of the last token (n_vocab floats) or of all tokens.
// Returns 0 on success, -2 when the cache is full. gpt2_kv_cache_seq_cp (:814-827) lets seq_dst see
// seq_src's cells at positions [p0, p1) (-1: open end), e.g. a shared prompt; gpt2_kv_cache_clear
// empties the cache. (Not in scheduler mode; do not interleave with gpt2_eval on one model.)
GGML_API int gpt2_decode_batch(struct gpt2_model * model, int n_tokens, const int32_t * tokens, const int32_t * pos,
                               const int32_t * seq_id, float * logits, int all_logits);
GGML_API void gpt2_kv_cache_seq_cp(struct gpt2_model * model, int32_t seq_src, int32_t seq_dst, int32_t p0, int32_t p1);
GGML_API void gpt2_kv_cache_clear(struct gpt2_model * model);
// batched steps launched as a graph plan prebuilt during the previous step ([0]) and built on the
// spot ([1]); with a host buffer type (gpt2_model_load_ex) a step's inputs go in as one async copy
GGML_API void gpt2_batch_stats(const struct gpt2_model * model, int64_t * out2);
// the host staging of the logits (gpt2_model_load_ex with a host buffer type), or NULL
GGML_API const float * gpt2_logits_host(const struct gpt2_model * model);

// the vocabulary from the model file and the word-split + longest-match tokenizer of
// examples/common.cpp:272-329. gpt2_tokenize returns the token count (may exceed max_tokens;
// only max_tokens are written).
GGML_API const char * gpt2_token_text(const struct gpt2_model * model, int32_t id);
GGML_API int gpt2_tokenize(const struct gpt2_model * model, const char * text, int32_t * out, int max_tokens);

// last-evaluated graph statistics: nodes, and wall-clock microseconds of graph build / graph
// allocation / input upload / compute (incl. reading the logits back)
GGML_API void gpt2_last_eval_stats(const struct gpt2_model * model, int * n_nodes, int64_t * us_build, int64_t * us_alloc,
                                   int64_t * us_inputs, int64_t * us_compute);

// the parts of us_compute of the last direct-backend eval, microseconds: us4[0] host time to
// enqueue the graph (ggml_backend_graph_compute_async), [1] to build + allocate the next decode
// step's graph while the device runs this one, [2] waiting for the device, [3] the logits copy
GGML_API void gpt2_last_eval_timing(const struct gpt2_model * model, int64_t * us4);

#ifdef __cplusplus
}
#endif
