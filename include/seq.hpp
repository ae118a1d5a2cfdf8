// seq.hpp — drop-in for /root/reference/include/seq.hpp: the CPU forward of the caller's own
// src/seq.cpp (the reference's oracle, src/seq.cpp:3-183).  Caller-side: libthallama.so does not
// define these; a build that uses them compiles the reference's seq.cpp beside its driver.
#pragma once
#include "utils.hpp"

#ifdef __cplusplus
// reference include/seq.hpp:3-11
void rmsnorm(float* o, float* x, float* weight, int size);
void softmax(float* x, int size);
void matmul(float* xout, float* x, float* w, int n, int d);
float* forward(Transformer* transformer, int token, int pos);
#endif
