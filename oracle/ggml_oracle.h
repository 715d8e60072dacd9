// ggml_oracle.h -- TEST INFRASTRUCTURE ONLY (see ggml_oracle.c header).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

// numeric values equal enum ggml_type (include/ggml/ggml.h:348-381)
enum {
    ORC_F32 = 0, ORC_F16 = 1, ORC_Q4_0 = 2, ORC_Q8_0 = 8,
    ORC_Q4_K = 12, ORC_Q5_K = 13, ORC_Q8_K = 15,
};

uint16_t orc_fp32_to_fp16(float f);
float    orc_fp16_to_fp32(uint16_t h);
int      orc_block_size(int type);
int      orc_type_size(int type);
size_t   orc_row_size(int type, int64_t n);
int      orc_vec_dot_type(int type);
size_t   orc_quantize_chunk(int type, const float * src, void * dst, int64_t nrows, int64_t n_per_row);
void     orc_quantize_act(int vec_dot_type, const float * x, void * dst, int64_t n);
void     orc_dequantize_row(int type, const void * src, float * y, int64_t k);
float    orc_vec_dot(int type, int n, const void * x, const void * y);
void     orc_mul_mat(int type, const void * W, int64_t K, int64_t N, const float * X, int64_t B, float * Y, int nthreads);

#ifdef __cplusplus
}
#endif
