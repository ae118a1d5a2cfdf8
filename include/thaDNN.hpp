// thaDNN.hpp — drop-in replacement for /root/reference/include/thaDNN.hpp.
#pragma once
#include "thaBLAS.hpp"
#include "models.hpp"
#include "thaDNN/thaDNN_rmsnorm.hpp"
#include "thaDNN/thaDNN_rope.hpp"
#include "thaDNN/thaDNN_mha.hpp"
#include "thaDNN/thaDNN_softmax.hpp"
#include "thaDNN/thaDNN_swiglu.hpp"

#include "utils.hpp"
// the reference's thaDNN.hpp includes <omp.h> (its pipeline driver takes omp_lock_t*)
#if defined(__has_include)
#if __has_include(<omp.h>)
#include <omp.h>
#define THALLAMA_OMP_LOCK omp_lock_t
#endif
#endif
#ifndef THALLAMA_OMP_LOCK
#define THALLAMA_OMP_LOCK void
#endif

#ifdef __cplusplus
extern "C" {
#endif

// reference include/thaDNN.hpp:12-25
typedef enum {
  thaDNNStatusSuccess = 0,
  thaDNNStatusNotInitialized = 1,
  thaDNNStatusInvalidValue = 2,
  thaDNNStatusBadParm = 3,
  thaDNNStatusAllocFailed = 4,
  thaDNNStatusInternalError = 5,
  thaDNNStatusNotImplemented = 6,
  thaDNNStatusUnknownError = 7,
  thaDNNStatusUnsupportedOp = 8,
  thaDNNStatusGpuOperationsSkipped = 9,
  thaDNNStatusVersionMismatch = 10,
} thaDNNStatus_t;

// One decode step for n_batches independent sequences (reference include/thaDNN.hpp:69,
// src/thaDNN.cpp:13-81).  token[]/pos[] are HOST arrays (sequence b processes token[b] at
// position pos[b]); w and s_batch hold DEVICE pointers; logits_host is a HOST buffer of
// n_batches*vocab floats (pinned or pageable).  On return the logits are in logits_host
// (the reference ends with hipDeviceSynchronize, src/thaDNN.cpp:78).  All work runs on
// handle1.calc_stream; handle2/handle3 are accepted for signature compatibility.
thablasStatus_t thaDNN_s_forward_batch(thablasHandle_t handle1, thablasHandle_t handle2,
                                       thablasHandle_t handle3, int n_batches, Config* p,
                                       TransformerWeights* w, RunState* s_batch, int token[],
                                       int pos[], float* logits_host);

// ---- the 70B layer-streaming and the pipeline / layer-swap drivers (reference
// include/thaDNN.hpp:72-80, src/thaDNN.cpp:83-427), on the decoder's kernels:
//  * thaDNN_s_forward_70B: batch 1; layer l + 1's weights (h_w, pinned host memory from
//    copy_transformer_to_host_70B) copied into a device staging slot while layer l computes;
//    every layer's K/V rows stay in d_s (h_s unused);
//  * the pipelines: stage g = layers [g*pipe, (g+1)*pipe) on the device of handle[g]'s stream with
//    w[g] / s_batch[g] (models.hpp staging), the residual stream handed to the next stage by an
//    asynchronous peer copy + event, logits from the last stage into logits_host (synchronised).
//    The reference's host-thread bookkeeping and device locks are accepted and not needed (each
//    caller runs on its own streams and states); the layer-swap variant swaps nothing (the device
//    holds every position).  n_layers must be a multiple of n_devices.
thablasStatus_t thaDNN_s_forward_70B(thablasHandle_t handle, int batch_size, Config* p, TransformerWeights* h_w[], RunState* h_s, TransformerWeights* d_w, RunState* d_s, int token[], int pos[], float* logits_host);
thablasStatus_t thaDNN_s_forward_batch_pipe_line(thablasHandle_t handle[], int n_devices, int n_batches, Transformer* transformer_d[], int token[], int pos[], float* logits_host);
thablasStatus_t thaDNN_s_forward_batch_multiple_pipe_line(thablasHandle_t handle[], int host_thread_id, int n_host_threads, int n_devices, int batch_size, Config* p, TransformerWeights* w[], RunState* s_batch[], int token[], int pos[], float* logits_host, int* host_thread_status, int* device_host_thread, THALLAMA_OMP_LOCK* device_mtx);
thablasStatus_t thaDNN_s_forward_batch_multiple_pipe_line_layer_swap(thablasHandle_t handle[], int thread_id, int n_host_threads, int n_devices, int batch_size, int n_buffer_words, Config* p, TransformerWeights* w[], RunState* s_batch[], RunState* s_host_batch[], int token[], int pos[], float* logits_host, THALLAMA_OMP_LOCK* device_locks);

#ifdef __cplusplus
}
#endif
