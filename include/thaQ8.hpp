// thaQ8.hpp — the int8 (Q8_0) twin of the decode path.  The reference has no GPU int8
// path: its int8 forward exists only as the CPU program runq.c (matmul :317-342,
// quantize :145-171, forward :344-481, v2 "ak42" file :189-251).  These entry points are
// ADDITIONS to the thaBLAS/thaDNN surface, named and laid out after runq.c so a caller
// moving from runq finds the same structures.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include "thaBLAS.hpp"
#include "models.hpp"

#ifdef __cplusplus
extern "C" {
#endif

// runq.c:34-37
typedef struct {
  int8_t* q;  // quantized values
  float* s;   // scaling factors, one per group of GS
} QuantizedTensor;

// runq.c:39-59 field order.  Host struct; q/s/float pointers are DEVICE pointers; the
// per-layer arrays (wq ... w3) are HOST arrays of n_layers entries.
typedef struct {
  QuantizedTensor* q_tokens;      // (vocab_size, dim)
  float* token_embedding_table;   // same, dequantized fp32 (runq.c:199-201)
  float* rms_att_weight;          // (layer, dim)
  float* rms_ffn_weight;          // (layer, dim)
  QuantizedTensor* wq;
  QuantizedTensor* wk;
  QuantizedTensor* wv;
  QuantizedTensor* wo;
  QuantizedTensor* w1;
  QuantizedTensor* w2;
  QuantizedTensor* w3;
  float* rms_final_weight;        // (dim,)
  QuantizedTensor* wcls;          // one entry (== q_tokens when shared)
  int group_size;                 // GS (runq.c:19)
} Q8TransformerWeights;

// Bytes of the v2 payload after its 256-byte header (export.py version2_export order).
size_t thallama_q8_payload_bytes(const Config* p, int shared_classifier, int group_size);

// Map a device copy of the v2 payload exactly like runq.c memory_map_weights (:189-217):
// allocates the host per-layer arrays; token_embedding_table is set to emb_f32 (a device
// buffer of vocab*dim floats the caller owns, filled by thallama_q8_dequant_embedding).
int thallama_q8_map(Q8TransformerWeights* w, const Config* p, void* payload_dev, int shared_classifier,
                    int group_size, float* emb_f32);
void thallama_q8_unmap(Q8TransformerWeights* w);

// A v2 ("ak42") checkpoint opened like runq.c read_checkpoint (:219-251): the 256-byte header
// parsed, the file mmapped read-only, `payload` pointing just past the header (host memory).
typedef struct {
  Config config;           // vocab_size as stored (positive)
  int shared_classifier;   // header flag byte
  int group_size;          // GS
  int fd;
  void* data;              // the whole mapping
  size_t file_size;
  const void* payload;     // data + 256
  size_t payload_bytes;    // file_size - 256 (>= thallama_q8_payload_bytes)
} Q8Checkpoint;
// 0 on success; -1 unreadable, -2 bad magic, -3 bad version, -4 truncated payload.
int thallama_q8_read_checkpoint(const char* path, Q8Checkpoint* ck);
void thallama_q8_close_checkpoint(Q8Checkpoint* ck);

// token_embedding_table[i] = q_tokens.q[i] * q_tokens.s[i / GS]  (runq.c:139-143)
int thallama_q8_dequant_embedding(const Q8TransformerWeights* w, const Config* p, hipStream_t stream);

// Quantise fp32 device weights (layout of thallama_map_weights) into a device v2 payload with
// train/export.py:46-70 semantics (scale = max|w|/127, q = round-half-even(w/scale)).
int thallama_q8_quantize_model(void* payload_dev, const TransformerWeights* w_fp32, const Config* p,
                               int shared_classifier, int group_size, hipStream_t stream);

// Activation quantisation, runq.c:145-171 semantics (round half away from zero), for
// n_batches rows of n floats at x + b*x_stride -> q + b*n, s + b*(n/gs).
thablasStatus_t thaBLAS_q8_quantize_batch(thablasHandle_t* handle, int n_batches, int8_t* q, float* s,
                                          float* x, int n, int group_size, int x_stride);

// C[b*C_batch_size + i] = sum_g (sum_{k in g} xq_b[k] * wq[i*K+k]) * ws[i*K/GS + g] * xs_b[g]
// where (xq_b, xs_b) = quantize(x + b*x_batch_size) — runq.c quantize + matmul fused.
thablasStatus_t thaBLAS_q8_matmul_batch(thablasHandle_t* handle, int n_batches, float* C, float* x,
                                        int8_t* wq, float* ws, int K, int M, int group_size,
                                        int C_batch_size, int x_batch_size);

// The int8 decode step (runq.c forward :344-481 for n_batches sequences), same contract as
// thaDNN_s_forward_batch.
thablasStatus_t thaDNN_q8_forward_batch(thablasHandle_t handle, int n_batches, Config* p,
                                        Q8TransformerWeights* w, RunState* s_batch, int token[], int pos[],
                                        float* logits_host);

#ifdef __cplusplus
}
#endif
