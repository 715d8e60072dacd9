// ggml_sched_abi.h -- the reference's backend scheduler API (include/ggml/ggml-backend.h:167-204 of
// NAIST-Archlab/ggml-imax). Declared separately from ggml_abi.h because this repo's runtime
// (libggml_core) does not implement the scheduler: these symbols come from the reference libggml,
// under which the MI355X backend is exercised as a drop-in (oracle/Makefile `gpt2`: the GPT-2
// driver is built with -DGPT2_WITH_SCHED only there;
// tests/test_gpt2.py::test_gpt2_partial_offload_under_reference_scheduler).
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

struct ggml_backend_sched;
typedef struct ggml_backend_sched * ggml_backend_sched_t;
typedef bool (*ggml_backend_sched_eval_callback)(struct ggml_tensor * t, bool ask, void * user_data);

GGML_API ggml_backend_sched_t ggml_backend_sched_new(ggml_backend_t * backends, ggml_backend_buffer_type_t * bufts, int n_backends,
                                                     size_t graph_size, bool parallel);
GGML_API void ggml_backend_sched_free(ggml_backend_sched_t sched);
GGML_API bool ggml_backend_sched_reserve(ggml_backend_sched_t sched, struct ggml_cgraph * measure_graph);
GGML_API int ggml_backend_sched_get_n_splits(ggml_backend_sched_t sched);
GGML_API int ggml_backend_sched_get_n_copies(ggml_backend_sched_t sched);
GGML_API size_t ggml_backend_sched_get_buffer_size(ggml_backend_sched_t sched, ggml_backend_t backend);
GGML_API void ggml_backend_sched_set_tensor_backend(ggml_backend_sched_t sched, struct ggml_tensor * node, ggml_backend_t backend);
GGML_API ggml_backend_t ggml_backend_sched_get_tensor_backend(ggml_backend_sched_t sched, struct ggml_tensor * node);
GGML_API bool ggml_backend_sched_alloc_graph(ggml_backend_sched_t sched, struct ggml_cgraph * graph);
GGML_API enum ggml_status ggml_backend_sched_graph_compute(ggml_backend_sched_t sched, struct ggml_cgraph * graph);
GGML_API void ggml_backend_sched_synchronize(ggml_backend_sched_t sched);
GGML_API void ggml_backend_sched_reset(ggml_backend_sched_t sched);

#ifdef __cplusplus
}
#endif
