// ggml-mi355x.h -- C-ABI entry points of the MI355X (gfx950) ggml backend.
//
// Drop-in counterpart of the reference's device-backend header src/ggml-cuda.h:19-40
// (NAIST-Archlab/ggml-imax @ v2); each function cites the declaration it replaces. Everything
// else a caller needs goes through the generic ggml_backend_* API (include/ggml_abi.h), exactly
// as with the CUDA and Metal backends. The library also registers one registry entry per
// device ("MI355X0", "MI355X1", ...) from an ELF constructor, so registry-driven tools
// (tests/test-backend-ops.cpp, ggml_backend_reg_init_backend_from_str) find it unmodified.
#pragma once

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_MI355X_MAX_DEVICES 16

// ggml-cuda.h:21  ggml_backend_cuda_init(int device)
GGML_API ggml_backend_t ggml_backend_mi355x_init(int device);

// ggml-cuda.h:23  ggml_backend_is_cuda(ggml_backend_t)
GGML_API bool ggml_backend_is_mi355x(ggml_backend_t backend);

// ggml-cuda.h:26  ggml_backend_cuda_buffer_type(int device): device-resident (HBM) buffers
GGML_API ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device);

// ggml-cuda.h:29  ggml_backend_cuda_split_buffer_type(const float * tensor_split): rows of a
// matrix split across devices (tensor-split row path); tensor_split = GGML_MI355X_MAX_DEVICES
// proportions (NULL / all zero = equal), slices rounded to 64-row GEMM tiles
GGML_API ggml_backend_buffer_type_t ggml_backend_mi355x_split_buffer_type(const float * tensor_split);

// ggml-cuda.h:32  ggml_backend_cuda_host_buffer_type(): pinned host memory for fast H2D/D2H
GGML_API ggml_backend_buffer_type_t ggml_backend_mi355x_host_buffer_type(void);

// ggml-cuda.h:34-36
GGML_API int  ggml_backend_mi355x_get_device_count(void);
GGML_API void ggml_backend_mi355x_get_device_description(int device, char * description, size_t description_size);
GGML_API void ggml_backend_mi355x_get_device_memory(int device, size_t * free, size_t * total);

// ggml-cuda.h:38-39
GGML_API bool ggml_backend_mi355x_register_host_buffer(void * buffer, size_t size);
GGML_API void ggml_backend_mi355x_unregister_host_buffer(void * buffer);

// ggml-cuda.cu:3024-3042 ggml_backend_cuda_reg_devices (called by the reference registry init;
// here also run from the library constructor). Returns the number of devices registered.
GGML_API int ggml_backend_mi355x_reg_devices(void);

// --- MI355X extensions (no reference counterpart) ---

// hipStream_t the backend launches on (for external timing with HIP events / stream interop)
GGML_API void * ggml_backend_mi355x_get_stream(ggml_backend_t backend);

// Number of kernels launched by the last graph_compute (for tests / profiling).
GGML_API int ggml_backend_mi355x_last_launch_count(ggml_backend_t backend);

// hipGraphs. graph_compute captures a graph's launches and replays the capture whenever the same
// graph (same nodes, addresses, shapes, parameters) is computed again, updating an executable
// graph of the same topology in place when only kernel arguments changed (the reference's CUDA
// graphs, ggml-cuda.cu:2456-2713); the first graph of a topology, and graphs of fewer than 4
// kernel launches (GGML_MI355X_GRAPH_MIN_LAUNCHES), launch directly. Graph plans
// (ggml_backend_graph_plan_create / _compute) are captured at creation and computed with one
// hipGraphLaunch. GGML_MI355X_DISABLE_GRAPHS=1 (process-wide, as GGML_CUDA_DISABLE_GRAPHS,
// ggml-cuda.cu:2462) or set_graph_capture(false) makes both launch directly.
GGML_API void ggml_backend_mi355x_set_graph_capture(ggml_backend_t backend, bool enable);
// Per-node timer, the reference's GGML_PERF (ggml.c:19195-19205, :19907-19922) for this backend:
// with it on (or GGML_MI355X_PERF set), graphs launch directly and every node's device time is
// measured with HIP events around the kernel that computes it; node->perf_runs / perf_time_us (and
// perf_cycles, in microseconds) and the cgraph's totals accumulate as the reference's CPU executor
// fills them, and ggml_graph_print() prints them. A fused chain's time goes to its last node, the
// others get runs without time. Timing synchronizes the stream once per graph.
GGML_API void ggml_backend_mi355x_set_perf(ggml_backend_t backend, bool enable);
// counters since init: [0] captures (plans and graph_compute), [1] graph instantiations,
// [2] in-place updates, [3] direct (uncaptured) computes
GGML_API void ggml_backend_mi355x_graph_stats(ggml_backend_t backend, int64_t * stats4);
// the same counters and more: [4] graph_compute replays of a cached capture, [5] graph_compute
// captures; fills min(n, available) entries and returns that count
GGML_API int ggml_backend_mi355x_graph_stats_ex(ggml_backend_t backend, int64_t * stats, int n);

// Launch-shape knobs of the streaming kernels, for A/B tuning inside one process:
// "mmv_blocks" (resident workgroups of the fused GEMV), "mmv_variant" (see mi355x_kernels.h).
// Returns false for an unknown name.
GGML_API bool ggml_backend_mi355x_set_tuning(const char * name, int value);

// Runs the device activation quantizer that GGML_OP_MUL_MAT uses for `vec_dot_type`
// (GGML_TYPE_Q8_0 or GGML_TYPE_Q8_K) on ncols host columns of K floats and returns its
// structure-of-arrays result: qs [ncols*K], d [ncols*K/QK], s32 [ncols*K/32] (Q8_K only,
// sums of 32 quants). Lets tests compare the device rounding with the reference bit for bit.
GGML_API bool ggml_backend_mi355x_quantize_activations(ggml_backend_t backend, int vec_dot_type, const float * x,
                                                       int64_t K, int64_t ncols, int8_t * qs, float * d, int16_t * s32);

// Device phase stamps (diagnostic builds, `make -C ggml-imax_amd diaglib`): with slots > 0 the
// decode kernels (k_mmv_stream, the F16 GEMVs, k_attn_proj, k_get_rows_add) write s_memrealtime
// stamps (100 MHz chip clock) of every workgroup's first wave into a device buffer of `slots` words,
// 8 per workgroup and launch, in launch order; slots = 0 turns them off. Returns false in release
// builds (whose kernels carry no stamps). _read copies up to n words into `words` and the launch
// log ("kernel workgroups offset" lines) into `log`, and returns the number of words written since
// the last _reset.
GGML_API bool ggml_backend_mi355x_stamps_enable(size_t slots);
GGML_API void ggml_backend_mi355x_stamps_reset(void);
GGML_API size_t ggml_backend_mi355x_stamps_read(uint64_t * words, size_t n, char * log, size_t log_size);
// Repacked MFMA planes of Q4_K / Q5_K weights kept for long prompts (no reference counterpart: the
// reference's CPU mul_mat dequantizes per call): how many weight tensors carry them, and their bytes
GGML_API size_t ggml_backend_mi355x_planes_stats(size_t * bytes);

#ifdef __cplusplus
}
#endif
