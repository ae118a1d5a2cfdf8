// thaDNN.hpp — drop-in replacement for /root/reference/include/thaDNN.hpp.
#pragma once
#include "thaBLAS.hpp"
#include "models.hpp"
#include "thaDNN/thaDNN_rmsnorm.hpp"
#include "thaDNN/thaDNN_rope.hpp"
#include "thaDNN/thaDNN_mha.hpp"
#include "thaDNN/thaDNN_softmax.hpp"
#include "thaDNN/thaDNN_swiglu.hpp"

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

#ifdef __cplusplus
}
#endif
