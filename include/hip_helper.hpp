// hip_helper.hpp — error convention of the drop-in boundary.
//
// Replaces /root/reference/include/hip_helper.hpp:4-11 (CHECK_HIP: print and
// exit(EXIT_FAILURE) on any HIP error) and :49-51 (WARP_SIZE / MAX_BLOCK_SIZE).
// The reference's dead CHECK_thaBLAS_ERROR macro (:23-47, names an enum that
// does not exist) is not reproduced.
#pragma once
#include <stdio.h>
#include <stdlib.h>
#include <hip/hip_runtime.h>

#define CHECK_HIP(cmd)                                                          \
  do {                                                                          \
    hipError_t error_ = (cmd);                                                  \
    if (error_ != hipSuccess) {                                                 \
      fprintf(stderr, "HIP Error: %s (%d): %s:%d\n", hipGetErrorString(error_), \
              (int)error_, __FILE__, __LINE__);                                 \
      fflush(stdout);                                                           \
      exit(EXIT_FAILURE);                                                       \
    }                                                                           \
  } while (0)

#define MAX_NUM_SUPPORTED_GPUS 32
#define WARP_SIZE 64        // CDNA wavefront (reference hip_helper.hpp:50)
#define MAX_BLOCK_SIZE 1024
