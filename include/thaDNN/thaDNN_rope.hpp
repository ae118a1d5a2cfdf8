// Replaces /root/reference/include/thaDNN/thaDNN_rope.hpp:5-11.
#pragma once
#include "../thaBLAS.hpp"
#ifdef __cplusplus
extern "C" {
#endif
// Rotate pairs (i, i+1) of q (i < dim) and k (i < kv_dim) by pos * 10000^(-(i%head_size)/head_size)
// (reference src/thaDNN/thaDNN_rope.cpp:25-43, CPU src/seq.cpp:87-101).  In place.
thablasStatus_t thaDNN_s_rope(thablasHandle_t* handle, int dim, int head_size, int kv_dim, int pos,
                              float* q, float* k);
#ifdef __cplusplus
}
#endif
