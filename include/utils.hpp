// utils.hpp — drop-in for /root/reference/include/utils.hpp.
//
// Two halves, as in the reference:
//  * the host loader (malloc_run_state, memory_map_weights, read_checkpoint, build_transformer,
//    free_run_state, free_transformer, print_transformer; reference utils.hpp:42-54) and the
//    device-residency entry points (utils.hpp:57-71) are declared in models.hpp and exported by
//    libthallama.so with C linkage;
//  * the small caller-side helpers below (reference utils.hpp:20-34) are defined by the caller's
//    own src/utils.cpp, which may also be compiled in: its loader definitions then take the
//    place of the library's (same names, same semantics, src/utils.cpp:85-204).
#pragma once
#include <ctype.h>
#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include "hip_helper.hpp"
#include "thaBLAS.hpp"
#include "models.hpp"

#ifdef __cplusplus
#include <fstream>
#include <iostream>
#include <string>

// reference include/utils.hpp:20-34 (caller-side, src/utils.cpp:20-83)
void alloc_mat(float** m, int R, int C);
void util_free(void* m);
void alloc_vec(float** m, int N);
void rand_mat(float* m, int R, int C);
void rand_vec(float* m, int N);
void zero_mat(float* m, int R, int C);
void zero_vec(float* m, int N);
bool compareFiles(const std::string& filePath1, const std::string& filePath2);
#endif
