// Replaces /root/reference/include/thaDNN/thaDNN_rmsnorm.hpp:4-10.
#pragma once
#include "../thaBLAS.hpp"
#ifdef __cplusplus
extern "C" {
#endif
// o_batch[b*dim + i] = weight[i] * (ss_b * x_batch[b*dim + i]),  i < size,
// ss_b = 1/sqrtf(sum_i x^2 / size + 1e-5f)  (reference src/thaDNN/thaDNN_rmsnorm.cpp:35-65,
// CPU twin src/seq.cpp:3-16).  o may alias x.
thablasStatus_t thaDNN_s_rmsnorm_v2_batch(thablasHandle_t* handle, int n_batches, float* o_batch,
                                          float* x_batch, float* weight, int size, int dim);
#ifdef __cplusplus
}
#endif
