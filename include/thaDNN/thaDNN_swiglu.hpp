// Replaces /root/reference/include/thaDNN/thaDNN_swiglu.hpp:4-7.
#pragma once
#include "../thaBLAS.hpp"
#ifdef __cplusplus
extern "C" {
#endif
// hb[i] = hb[i] * (1/(1+expf(-hb[i]))) * hb2[i]  (reference src/thaDNN/thaDNN_swiglu.cpp:5-14,
// CPU src/seq.cpp:159-166).
thablasStatus_t thaDNN_s_swiglu(thablasHandle_t* handle, float* hb, float* hb2, int hidden_dim);
#ifdef __cplusplus
}
#endif
