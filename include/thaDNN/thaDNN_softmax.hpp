// Replaces /root/reference/include/thaDNN/thaDNN_softmax.hpp:5-7.  The reference header
// takes the handle by pointer while its definition takes it by value
// (src/thaDNN/thaDNN_softmax.cpp:102): the header wins.
#pragma once
#include "../thaBLAS.hpp"
#ifdef __cplusplus
extern "C" {
#endif
// In-place numerically stable softmax of x[0..size) (reference src/thaDNN/thaDNN_softmax.cpp:62-97,
// CPU src/seq.cpp:18-36).  Enqueued on handle->calc_stream.
thablasStatus_t thaDNN_s_softmax_v2(thablasHandle_t* handle, float* x, int size);
#ifdef __cplusplus
}
#endif
