// thaBLAS.hpp — drop-in replacement for /root/reference/include/thaBLAS.hpp.
//
// Same type names, enum values, struct layout and entry-point signatures as
// the reference (every declaration cites the line it replaces), exported with
// C linkage so the library can be bound from C, C++ (the reference's own
// src/llama.cpp includes this header unchanged) or any FFI (ctypes).
//
// Conventions kept from the reference:
//  * all float* are DEVICE pointers unless noted; the caller allocates
//    (reference src/models.cpp:86-179);
//  * kernels are enqueued asynchronously on handle->calc_stream
//    (reference src/thaBLAS.cpp:223) and the wrappers return
//    THABLAS_STATUS_SUCCESS; HIP runtime failures abort via CHECK_HIP.
//  * New: arguments that would make a kernel fault (null pointers, negative
//    sizes) return THABLAS_STATUS_INVALID_VALUE instead of launching — the
//    reference has that validation commented out (src/thaBLAS.cpp:212-216).
#pragma once

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

// reference include/thaBLAS.hpp:5-19
typedef enum {
  THABLAS_STATUS_SUCCESS = 0,
  THABLAS_STATUS_NOT_INITIALIZED = 1,
  THABLAS_STATUS_ALLOC_FAILED = 2,
  THABLAS_STATUS_INVALID_VALUE = 3,
  THABLAS_STATUS_MAPPING_ERROR = 4,
  THABLAS_STATUS_EXECUTION_FAILED = 5,
  THABLAS_STATUS_INTERNAL_ERROR = 6,
  THABLAS_STATUS_NOT_SUPPORTED = 7,
  THABLAS_STATUS_ARCH_MISMATCH = 8,
  THABLAS_STATUS_HANDLE_IS_NULLPTR = 9,
  THABLAS_STATUS_INVALID_ENUM = 10,
  THABLAS_STATUS_UNKNOWN = 11,
} thablasStatus_t;

// reference include/thaBLAS.hpp:21-25
typedef struct {
  int current_gpu_id;
  hipStream_t calc_stream;
  hipStream_t copy_stream;
} thablasHandle_t;

// reference include/thaBLAS.hpp:27 / src/thaBLAS.cpp:49-58
thablasStatus_t thablasCreate(thablasHandle_t* handle);
// reference include/thaBLAS.hpp:29 / src/thaBLAS.cpp:60-64 (the reference leaks
// both streams; this one destroys them)
thablasStatus_t thablasDestroy(thablasHandle_t handle);

// ---------------------------------------------------------------- level 1
// B = A / val.  reference include/thaBLAS.hpp:57 / src/thaBLAS.cpp:79-95
thablasStatus_t thablas_Svds(thablasHandle_t handle, int n, float* A, float* B, float val);
// a += b (residual add).  reference include/thaBLAS.hpp:61 / src/thaBLAS.cpp:110-126
thablasStatus_t thaBLAS_s_vecaddvec(thablasHandle_t* handle, float* a, float* b, int size);

// ---------------------------------------------------------------- level 2
// C[M] = A[M][K] . B[K].  reference include/thaBLAS.hpp:70 / src/thaBLAS.cpp:239-241
thablasStatus_t thaBLAS_s_matmulvec(thablasHandle_t handle, float* C, float* B, float* A, int K, int M);
// same math; the header takes the handle by value (include/thaBLAS.hpp:72) while
// the reference definition takes a pointer (src/thaBLAS.cpp:260) — the header wins.
thablasStatus_t thaDNN_s_matmulvec_v2(thablasHandle_t handle, float* C, float* B, float* A, int K, int M);

// ---------------------------------------------------------------- level 3
// C[m][n] = A[m][k] . B[k][n], all row-major.
// reference include/thaBLAS.hpp:103 / src/thaBLAS.cpp:154-170
thablasStatus_t thaBLAS_s_matmul(thablasHandle_t handle, int m, int n, int k, float* A, float* B, float* C);

// The live decode GEMV (reference include/thaBLAS.hpp:106-117, src/thaBLAS.cpp:191-228):
//   for b < n_batches, i < M:
//     C_batch[Coff + has_pos*pos_d[b] + b*C_batch_size + i] = sum_k A[i*K+k] * B_batch[b*B_batch_size + k]
// A is row-major [M][K]; pos_d is a DEVICE int array.  Offsets are computed in
// 64-bit here (the reference overflows int at b*C_batch_size >= 2^31).
thablasStatus_t thaBLAS_s_matmul_batch(thablasHandle_t* handle, int n_batches, float* C_batch,
                                       float* B_batch, float* A, int K, int M, int Coff,
                                       int has_pos, int pos_d[], int C_batch_size,
                                       int B_batch_size);

// C[j][i] = sum_k A[i][k] * B[j][k]  (B, C "column-major" = [N][K], [N][M]).
// reference include/thaBLAS.hpp:119-125 / src/thaBLAS.cpp:281-319
thablasStatus_t thaBLAS_s_matmul_reduction(thablasHandle_t* handle, float* A, float* B, float* C,
                                           int M, int N, int K);

// D[n][m] = sum_k A[m][k] * B[n][k] for N = 16 on the f32 matrix cores.
// reference include/thaBLAS.hpp:127-133 / src/thaBLAS.cpp:321-351 (MFMA 16x16x4 f32).
thablasStatus_t thaBLAS_s_sgemm_Mx16xK(thablasHandle_t* handle, float* d_A, float* d_B, float* d_D,
                                       int M, int N, int K);

// reference include/thaBLAS.hpp:135-141 / src/thaBLAS.cpp:353-359 (compile-time switch
// between the two above; here a runtime choice: MFMA when N % 16 == 0 and M % 16 == 0).
thablasStatus_t thaBLAS_s_matmul_ifdef(thablasHandle_t* handle, float* d_A, float* d_B, float* d_D,
                                       int M, int N, int K);

#ifdef __cplusplus
}  // extern "C"
#endif
