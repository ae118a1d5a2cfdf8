// Replaces /root/reference/include/thaDNN/thaDNN_mha.hpp:5-47 — the reference's three-kernel
// attention split.  pos[] is a HOST array, pos_d[]/size_batch[] are DEVICE copies of it.
#pragma once
#include "../thaBLAS.hpp"
#ifdef __cplusplus
extern "C" {
#endif

// ---- v1: KV cache laid out [b][layer][seq_len][kv_dim] (the live path, src/thaDNN.cpp:52-54)
// scores: s_att[b][h][t] = q_b[h*hs:(h+1)*hs] . K_b[loff + t*kv_dim + (h/kv_mul)*hs] / sqrtf(hs), t <= pos[b]
// (reference src/thaDNN/thaDNN_mha.cpp:246-304)
thablasStatus_t thaDNN_s_multiheads_1_v1_batch(thablasHandle_t* handle, int n_batches, int pos[],
                                               int pos_d[], int n_heads, int n_layers,
                                               float* s_q_batch, float* s_att_batch,
                                               float* s_key_cache_batch, int head_size,
                                               int seq_len, int loff, int kv_dim, int dim,
                                               int kv_mul);
// in-place softmax of s_att[b][h][0..size_batch[b]] (reference mha.cpp:306-374)
thablasStatus_t thaDNN_s_multiheads_2_v1_batch(thablasHandle_t* handle, int n_batches,
                                               float* s_att_batch, int size_batch[], int seq_len,
                                               int n_heads);
// s_xb[b][h*hs + i] = sum_{t<=pos_d[b]} s_att[b][h][t] * V_b[loff + t*kv_dim + (h/kv_mul)*hs + i]
// (reference mha.cpp:376-426)
thablasStatus_t thaDNN_s_multiheads_3_v1_batch(thablasHandle_t* handle, int n_batches, int pos_d[],
                                               int n_heads, float* s_xb_batch, float* s_att_batch,
                                               float* s_value_cache_batch, int head_size,
                                               int seq_len, int loff, int kv_dim, int kv_mul,
                                               int dim, int n_layers);

// ---- v2: KV laid out [t][batch_size][kv_dim] for one layer (pipeline path, mha.cpp:60-244;
// not on the live path, kept for API completeness).
thablasStatus_t thaDNN_s_multiheads_1_v2_batch(thablasHandle_t* handle, int batch_size,
                                               int pipe_size, int pos[], int pos_d[], int n_heads,
                                               float* s_q_batch, float* s_att_batch,
                                               float* s_key_cache_batch, int head_size,
                                               int n_words, int kv_dim, int dim, int kv_mul);
thablasStatus_t thaDNN_s_multiheads_2_batch(thablasHandle_t* handle, int n_batches,
                                            float* s_att_batch, int size_batch[], int seq_len,
                                            int n_heads);
thablasStatus_t thaDNN_s_multiheads_3_v2_batch(thablasHandle_t* handle, int batch_size, int pos_d[],
                                               int n_heads, float* s_xb_batch, float* s_att_batch,
                                               float* s_value_cache_batch, int head_size,
                                               int n_words, int kv_dim, int kv_mul, int dim,
                                               int pipe_size);
#ifdef __cplusplus
}
#endif
