// models.hpp — the ABI the kernels index.  Replaces /root/reference/include/models.hpp:10-70
// (Config / TransformerWeights / RunState / Transformer, field order and types identical, so a
// caller written against the reference compiles and links unchanged) and the loader / device
// upload entry points of /root/reference/include/utils.hpp:41-71.
//
// Layout contract (same as the reference, src/models.cpp:86-179, src/thaDNN.cpp:13-81):
//  * weights row-major [out][in]; layer l of wq at wq + l*dim*dim, etc.;
//  * batched RunState: x, xb, xb2, q [B][dim]; hb, hb2 [B][hidden]; att [B][H][seq_len];
//    logits [B][vocab]; key_cache / value_cache [B][L][seq_len][kv_dim].
#pragma once
#include <stddef.h>
#include <sys/types.h>
#include "thaBLAS.hpp"

#ifdef __cplusplus
extern "C" {
#endif

// reference include/models.hpp:10-18 (28-byte model.bin v0 header)
typedef struct {
  int dim;         // transformer dimension
  int hidden_dim;  // for ffn layers
  int n_layers;    // number of layers
  int n_heads;     // number of query heads
  int n_kv_heads;  // number of key/value heads
  int vocab_size;  // vocabulary size (negative in the file = unshared classifier)
  int seq_len;     // max sequence length
} Config;

// reference include/models.hpp:20-39
typedef struct {
  float* token_embedding_table;  // (vocab_size, dim)
  float* rms_att_weight;         // (layer, dim)
  float* rms_ffn_weight;         // (layer, dim)
  float* wq;                     // (layer, dim, n_heads * head_size)
  float* wk;                     // (layer, dim, n_kv_heads * head_size)
  float* wv;                     // (layer, dim, n_kv_heads * head_size)
  float* wo;                     // (layer, n_heads * head_size, dim)
  float* w1;                     // (layer, hidden_dim, dim)
  float* w2;                     // (layer, dim, hidden_dim)
  float* w3;                     // (layer, hidden_dim, dim)
  float* rms_final_weight;       // (dim,)
  float* wcls;                   // (vocab_size, dim)
} TransformerWeights;

// reference include/models.hpp:41-60 (all fields kept, including the pipeline-only ones)
typedef struct {
  float* x;
  float* xb;
  float* xb2;
  float* hb;
  float* hb2;
  float* q;
  float* k;
  float* v;
  float* att;
  float* logits;
  float* key_cache;
  float* value_cache;
  float* key_matmul;
  float* value_matmul;
  float* key_layer_cache;
  float* value_layer_cache;
} RunState;

// reference include/models.hpp:62-70
typedef struct {
  Config config;
  TransformerWeights weights;
  RunState state;
  int fd;
  float* data;
  ssize_t file_size;
} Transformer;

// ---- host loader (reference src/utils.cpp:85-177): mmap a llama2.c v0 fp32 model.bin.
void malloc_run_state(RunState* s, Config* p);
void memory_map_weights(TransformerWeights* w, Config* p, float* ptr, int shared_weights);
void read_checkpoint(char* checkpoint, Config* config, TransformerWeights* weights, int* fd,
                     float** data, ssize_t* file_size);
void build_transformer(Transformer* t, char* checkpoint_path);
void free_run_state(RunState* s);
void free_transformer(Transformer* t);
void print_transformer(Transformer* t);

// ---- device residency (reference include/models.hpp:120-134, src/models.cpp:86-179).  Unlike
// the reference, the weights live in ONE device arena laid out exactly like the file payload,
// so a single H2D copy (or one RCCL broadcast) moves the whole model.  The out-parameters are
// the reference's C++ references (`TransformerWeights* &w_d`) for C++ callers, so its
// src/llama.cpp compiles unchanged; the C ABI (C callers, FFIs) sees the same symbol taking a
// pointer to the pointer.
#ifdef __cplusplus
#define THALLAMA_OUT(T) T*&
#else
#define THALLAMA_OUT(T) T**
#endif
// reference include/models.hpp:121
void copy_transformer_to_device(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(Transformer) t_d);
// reference include/models.hpp:122
void copy_weight_to_device(Transformer* t_h, THALLAMA_OUT(TransformerWeights) w_d);
// reference include/models.hpp:123 (one sequence)
void alloc_state_to_device(Transformer* t_h, THALLAMA_OUT(RunState) s_d);
// reference include/models.hpp:124
void alloc_state_to_device_batch(Transformer* t_h, THALLAMA_OUT(RunState) s_d_batch, int batch_size);
void free_weight_device(TransformerWeights* w_d);
void free_state_device(RunState* s_d);

// ---- pipeline, layer-swap and 70B staging (reference include/models.hpp:120,
// 125-134, src/models.cpp:181-758) for the drivers in thaDNN.hpp.  A stage's weights are one device
// arena (free with free_weight_device), its state the decoder's layout [batch][layers][seq][kv_dim]
// (free_state_device).  The swap variants keep EVERY position on the device (an MI355X holds the
// cache; the host state is an empty struct), and the 70B device state holds every layer's K/V
// rows; the 70B device weights hold the embedding, final norm, classifier and two layer staging
// slots (the per-layer fields point at slot 0).
void set_transformer(void);
void copy_transformer_pipeline_to_device(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(Transformer) t_d, int pipe_size, int pipe_id);
void copy_transformer_pipeline_to_device_batch(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(Transformer) t_d, int pipe_size, int pipe_id, int batch_size);
void copy_transformer_weight_pipeline_to_device_batch(Transformer* t_h, THALLAMA_OUT(TransformerWeights) w_d, int pipe_size, int pipe_id, int batch_size);
void alloc_run_state_to_device_batch(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(RunState) s_d, int pipe_size, int pipe_id, int batch_size);
void alloc_swap_run_state_on_host_batch(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(RunState) s_h, int pipe_size, int pipe_id, int batch_size, int n_buffer_words);
void alloc_swap_run_state_to_device_batch(thablasHandle_t handle, Transformer* t_h, THALLAMA_OUT(RunState) s_d, int pipe_size, int pipe_id, int batch_size, int n_buffer_words);
void copy_transformer_to_host_70B(Transformer* storage_t, TransformerWeights* h_w[], RunState* h_s[], int n_devices);
void alloc_state_to_device_70B(Transformer* t_h, THALLAMA_OUT(RunState) d_s);
void alloc_weight_to_device_70B(Transformer* h_t, THALLAMA_OUT(TransformerWeights) d_w);
void free_transformer_device(void);

// Number of floats in the v0 payload after the 28-byte header (including the unused
// freq_cis block and, when unshared, wcls) — the size of the device arena.
size_t thallama_v0_payload_floats(const Config* p, int shared_weights);
// Point w at the arena (device or host) exactly like memory_map_weights.
void thallama_map_weights(TransformerWeights* w, const Config* p, float* arena, int shared_weights);

#ifdef __cplusplus
}  // extern "C"

// reference include/models.hpp:72-117: the fp16 mirrors and the paged-KV block (declared by the
// reference, used by none of its live paths; kept so code naming them still compiles)
#include <hip/hip_fp16.h>
typedef struct {
  float* addr;
  int occupied;
} KVBlock;
typedef struct {
  __half *token_embedding_table, *rms_att_weight, *rms_ffn_weight, *wq, *wk, *wv, *wo, *w1, *w2, *w3,
      *rms_final_weight, *wcls;
} TransformerWeightsHalf;
typedef struct {
  __half *x, *xb, *xb2, *hb, *hb2, *q, *k, *v, *att, *logits, *key_cache, *value_cache;
} RunStateHalf;
#endif
