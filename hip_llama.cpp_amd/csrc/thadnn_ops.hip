// thadnn_ops.hip — the stand-alone thaDNN operators (include/thaDNN/*.hpp) on gfx950.
//
// These keep the reference's operator-level API (one call = one op, reference
// src/thaDNN/*.cpp).  The fused decode step (forward.hip) does not call them:
// it folds RMSNorm, RoPE, SwiGLU and the residual adds into the GEMV
// prologue/epilogues and runs attention as one kernel.  They exist so a caller
// of the reference's op API gets the same results, and they are the unit
// under test for each op's numerics.
#include <math.h>
#include "../../include/thaDNN.hpp"
#include "../../include/hip_helper.hpp"
#include "common.hpp"
#include "libm_exact.hpp"

using tl::f4;

static inline thablasStatus_t launch_status(hipError_t e) {
  return e == hipSuccess ? THABLAS_STATUS_SUCCESS : THABLAS_STATUS_EXECUTION_FAILED;
}

// ------------------------------------------------------------------ RMSNorm
// reference src/thaDNN/thaDNN_rmsnorm.cpp:35-65 ; CPU src/seq.cpp:3-16
__global__ void __launch_bounds__(256) k_rmsnorm(float* o_batch, const float* x_batch, const float* w,
                                                 int size, long long dim, bool vec) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const float* x = x_batch + b * dim;
  float* o = o_batch + b * dim;
  float ss = 0.f;
  if (vec) {
    const f4* x4 = reinterpret_cast<const f4*>(x);
    for (int i = threadIdx.x; i < size / 4; i += 256) {
      f4 v = x4[i];
      ss = fmaf(v.x, v.x, ss); ss = fmaf(v.y, v.y, ss); ss = fmaf(v.z, v.z, ss); ss = fmaf(v.w, v.w, ss);
    }
  } else {
    for (int i = threadIdx.x; i < size; i += 256) ss = fmaf(x[i], x[i], ss);
  }
  ss = tl::block_sum(ss, red);
  ss = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(ss, (float)size), 1e-5f)));
  if (vec) {
    const f4* x4 = reinterpret_cast<const f4*>(x);
    const f4* w4 = reinterpret_cast<const f4*>(w);
    f4* o4 = reinterpret_cast<f4*>(o);
    for (int i = threadIdx.x; i < size / 4; i += 256) {
      f4 v = x4[i], g = w4[i];
      o4[i] = f4{__fmul_rn(g.x, __fmul_rn(ss, v.x)), __fmul_rn(g.y, __fmul_rn(ss, v.y)),
                 __fmul_rn(g.z, __fmul_rn(ss, v.z)), __fmul_rn(g.w, __fmul_rn(ss, v.w))};
    }
  } else {
    for (int i = threadIdx.x; i < size; i += 256) o[i] = __fmul_rn(w[i], __fmul_rn(ss, x[i]));
  }
}

extern "C" thablasStatus_t thaDNN_s_rmsnorm_v2_batch(thablasHandle_t* handle, int n_batches, float* o_batch,
                                                     float* x_batch, float* weight, int size, int dim) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches < 0 || size < 0 || (n_batches > 1 && dim < size)) return THABLAS_STATUS_INVALID_VALUE;
  if (n_batches == 0 || size == 0) return THABLAS_STATUS_SUCCESS;
  if (!o_batch || !x_batch || !weight) return THABLAS_STATUS_INVALID_VALUE;
  const bool vec = (size % 4 == 0) && (dim % 4 == 0) &&
                   ((((uintptr_t)o_batch) | ((uintptr_t)x_batch) | ((uintptr_t)weight)) & 15) == 0;
  hipLaunchKernelGGL(k_rmsnorm, dim3(n_batches), dim3(256), 0, handle->calc_stream, o_batch, x_batch,
                     weight, size, (long long)dim, vec);
  return launch_status(hipGetLastError());
}

// ------------------------------------------------------------------ RoPE
// reference src/thaDNN/thaDNN_rope.cpp:25-43 ; CPU src/seq.cpp:87-101
__global__ void __launch_bounds__(256) k_rope(int dim, int head_size, int kv_dim, int pos, float* q, float* k) {
  tl::keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  const int i = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (i >= dim) return;  // like the reference, dim is taken as even
  const int head_dim = i % head_size;
  const float freq = __fdiv_rn(1.0f, powf(10000.0f, __fdiv_rn((float)head_dim, (float)head_size)));
  const float val = __fmul_rn((float)pos, freq);
  const float fcr = cosf(val), fci = sinf(val);
  const int rotn = i < kv_dim ? 2 : 1;
  for (int v = 0; v < rotn; ++v) {
    float* vec = v == 0 ? q : k;
    const float v0 = vec[i], v1 = vec[i + 1];
    vec[i] = __fsub_rn(__fmul_rn(v0, fcr), __fmul_rn(v1, fci));
    vec[i + 1] = __fadd_rn(__fmul_rn(v0, fci), __fmul_rn(v1, fcr));
  }
}

extern "C" thablasStatus_t thaDNN_s_rope(thablasHandle_t* handle, int dim, int head_size, int kv_dim, int pos,
                                         float* q, float* k) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (dim < 0 || head_size <= 0 || kv_dim < 0 || pos < 0 || !q || (kv_dim > 0 && !k))
    return THABLAS_STATUS_INVALID_VALUE;
  if (dim == 0) return THABLAS_STATUS_SUCCESS;
  const int pairs = (dim + 1) / 2;
  hipLaunchKernelGGL(k_rope, dim3((pairs + 255) / 256), dim3(256), 0, handle->calc_stream, dim, head_size,
                     kv_dim, pos, q, k);
  return launch_status(hipGetLastError());
}

// ------------------------------------------------------------------ SwiGLU
// reference src/thaDNN/thaDNN_swiglu.cpp:5-14 ; CPU src/seq.cpp:159-166
__device__ __forceinline__ float swiglu1(float a, float b) {
  float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, tl::expf_libm(-a)));
  return __fmul_rn(__fmul_rn(a, s), b);
}

__global__ void __launch_bounds__(256) k_swiglu(float* hb, const float* hb2, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) hb[i] = swiglu1(hb[i], hb2[i]);
}

extern "C" thablasStatus_t thaDNN_s_swiglu(thablasHandle_t* handle, float* hb, float* hb2, int hidden_dim) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (hidden_dim < 0 || ((!hb || !hb2) && hidden_dim)) return THABLAS_STATUS_INVALID_VALUE;
  if (hidden_dim == 0) return THABLAS_STATUS_SUCCESS;
  int blocks = (hidden_dim + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_swiglu, dim3(blocks), dim3(256), 0, handle->calc_stream, hb, hb2, hidden_dim);
  return launch_status(hipGetLastError());
}

// ------------------------------------------------------------------ softmax
// One block per row (row stride `stride`); reference src/thaDNN/thaDNN_softmax.cpp:62-97 and
// src/thaDNN/thaDNN_mha.cpp:306-352 ; CPU src/seq.cpp:18-36.  size_d (device) overrides n when set:
// row r has size_d[r / rows_per_size] + 1 elements.
__global__ void __launch_bounds__(256) k_softmax_rows(float* x, long long stride, int n, const int* size_d,
                                                      int rows_per_size) {
  __shared__ float red[16];
  const int r = blockIdx.x;
  float* row = x + r * stride;
  const int size = size_d ? size_d[r / rows_per_size] + 1 : n;
  float m = -3.402823466e+38f;
  for (int i = threadIdx.x; i < size; i += 256) m = fmaxf(m, row[i]);
  m = tl::block_max(m, red);
  float s = 0.f;
  for (int i = threadIdx.x; i < size; i += 256) {
    float e = tl::expf_libm(__fsub_rn(row[i], m));
    row[i] = e;
    s += e;
  }
  s = tl::block_sum(s, red);
  for (int i = threadIdx.x; i < size; i += 256) row[i] = __fdiv_rn(row[i], s);
}

extern "C" thablasStatus_t thaDNN_s_softmax_v2(thablasHandle_t* handle, float* x, int size) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  // reference src/thaDNN/thaDNN_softmax.cpp:103-106 rejects size == 0 / null x
  if (size <= 0 || !x || handle->current_gpu_id < 0) return THABLAS_STATUS_INVALID_VALUE;
  hipLaunchKernelGGL(k_softmax_rows, dim3(1), dim3(256), 0, handle->calc_stream, x, 0LL, size, nullptr, 1);
  return launch_status(hipGetLastError());
}

// ------------------------------------------------------------------ attention, 3-kernel API
// Scores.  Grid (key tiles of 32, head, batch); one wave per key, lanes stride the head dim.
// k_row(b, t) = K + b*kb_stride + t*kt_stride (+ head offset)
__global__ void __launch_bounds__(256) k_mha_scores(const int* pos_d, int n_heads, const float* q,
                                                    long long q_stride, float* att, long long att_b_stride,
                                                    long long att_h_stride, const float* kcache,
                                                    long long kb_stride, long long kt_stride, int head_size,
                                                    int kv_mul) {
  tl::keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int T = pos_d[b] + 1;
  const float* qh = q + b * q_stride + (long long)h * head_size;
  const float* kb = kcache + b * kb_stride + (long long)(h / kv_mul) * head_size;
  float* a = att + b * att_b_stride + h * att_h_stride;
  const float rs = sqrtf((float)head_size);
  for (int t = blockIdx.x * 32 + wave; t < min(T, (int)(blockIdx.x + 1) * 32); t += 4) {
    const float* k = kb + t * kt_stride;
    float d = 0.f;
    for (int i = lane; i < head_size; i += 64) d = fmaf(qh[i], k[i], d);
    d = tl::wave_sum(d);
    if (lane == 0) a[t] = __fdiv_rn(d, rs);
  }
}

// Weighted V sum.  Grid (head-dim tiles of 64, head, batch); wave w sums t = w mod 4.
__global__ void __launch_bounds__(256) k_mha_av(const int* pos_d, int n_heads, float* xb, long long xb_stride,
                                                const float* att, long long att_b_stride,
                                                long long att_h_stride, const float* vcache,
                                                long long vb_stride, long long vt_stride, int head_size,
                                                int kv_mul) {
  tl::keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  __shared__ float part[4][64];
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int T = pos_d[b] + 1;
  const float* a = att + b * att_b_stride + h * att_h_stride;
  const float* vb = vcache + b * vb_stride + (long long)(h / kv_mul) * head_size;
  float s = 0.f;
  if (i < head_size)
    for (int t = wave; t < T; t += 4) s = fmaf(a[t], vb[t * vt_stride + i], s);
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < head_size)
    xb[b * xb_stride + (long long)h * head_size + i] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

static int max_pos_host(const int* pos, int n) {
  int m = 0;
  for (int b = 0; b < n; ++b) m = pos[b] > m ? pos[b] : m;
  return m;
}

extern "C" thablasStatus_t thaDNN_s_multiheads_1_v1_batch(thablasHandle_t* handle, int n_batches, int pos[],
                                                          int pos_d[], int n_heads, int n_layers,
                                                          float* s_q_batch, float* s_att_batch,
                                                          float* s_key_cache_batch, int head_size,
                                                          int seq_len, int loff, int kv_dim, int dim,
                                                          int kv_mul) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches <= 0 || n_heads <= 0) return THABLAS_STATUS_SUCCESS;
  if (!pos || !pos_d || !s_q_batch || !s_att_batch || !s_key_cache_batch || head_size <= 0 || kv_mul <= 0)
    return THABLAS_STATUS_INVALID_VALUE;
  const int tiles = (max_pos_host(pos, n_batches) + 1 + 31) / 32;
  hipLaunchKernelGGL(k_mha_scores, dim3(tiles, n_heads, n_batches), dim3(256), 0, handle->calc_stream, pos_d,
                     n_heads, s_q_batch, (long long)dim, s_att_batch, (long long)n_heads * seq_len,
                     (long long)seq_len, s_key_cache_batch + (long long)loff,
                     (long long)n_layers * seq_len * kv_dim, (long long)kv_dim, head_size, kv_mul);
  return launch_status(hipGetLastError());
}

extern "C" thablasStatus_t thaDNN_s_multiheads_2_v1_batch(thablasHandle_t* handle, int n_batches,
                                                          float* s_att_batch, int size_batch[], int seq_len,
                                                          int n_heads) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches <= 0 || n_heads <= 0) return THABLAS_STATUS_SUCCESS;
  if (!s_att_batch || !size_batch) return THABLAS_STATUS_INVALID_VALUE;
  hipLaunchKernelGGL(k_softmax_rows, dim3(n_batches * n_heads), dim3(256), 0, handle->calc_stream, s_att_batch,
                     (long long)seq_len, 0, size_batch, n_heads);
  return launch_status(hipGetLastError());
}

extern "C" thablasStatus_t thaDNN_s_multiheads_2_batch(thablasHandle_t* handle, int n_batches, float* s_att_batch,
                                                       int size_batch[], int seq_len, int n_heads) {
  return thaDNN_s_multiheads_2_v1_batch(handle, n_batches, s_att_batch, size_batch, seq_len, n_heads);
}

extern "C" thablasStatus_t thaDNN_s_multiheads_3_v1_batch(thablasHandle_t* handle, int n_batches, int pos_d[],
                                                          int n_heads, float* s_xb_batch, float* s_att_batch,
                                                          float* s_value_cache_batch, int head_size,
                                                          int seq_len, int loff, int kv_dim, int kv_mul,
                                                          int dim, int n_layers) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches <= 0 || n_heads <= 0) return THABLAS_STATUS_SUCCESS;
  if (!pos_d || !s_xb_batch || !s_att_batch || !s_value_cache_batch || head_size <= 0 || kv_mul <= 0)
    return THABLAS_STATUS_INVALID_VALUE;
  hipLaunchKernelGGL(k_mha_av, dim3((head_size + 63) / 64, n_heads, n_batches), dim3(256), 0,
                     handle->calc_stream, pos_d, n_heads, s_xb_batch, (long long)dim, s_att_batch,
                     (long long)n_heads * seq_len, (long long)seq_len, s_value_cache_batch + (long long)loff,
                     (long long)n_layers * seq_len * kv_dim, (long long)kv_dim, head_size, kv_mul);
  return launch_status(hipGetLastError());
}

// v2 layout: K/V rows for step t of sequence b at cache + t*batch_size*kv_dim + b*kv_dim
// (reference src/thaDNN/thaDNN_mha.cpp:60-92, 182-205).
extern "C" thablasStatus_t thaDNN_s_multiheads_1_v2_batch(thablasHandle_t* handle, int batch_size, int pipe_size,
                                                          int pos[], int pos_d[], int n_heads, float* s_q_batch,
                                                          float* s_att_batch, float* s_key_cache_batch,
                                                          int head_size, int n_words, int kv_dim, int dim,
                                                          int kv_mul) {
  (void)pipe_size;
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (batch_size <= 0 || n_heads <= 0) return THABLAS_STATUS_SUCCESS;
  if (!pos || !pos_d || !s_q_batch || !s_att_batch || !s_key_cache_batch || head_size <= 0 || kv_mul <= 0)
    return THABLAS_STATUS_INVALID_VALUE;
  const int tiles = (max_pos_host(pos, batch_size) + 1 + 31) / 32;
  hipLaunchKernelGGL(k_mha_scores, dim3(tiles, n_heads, batch_size), dim3(256), 0, handle->calc_stream, pos_d,
                     n_heads, s_q_batch, (long long)dim, s_att_batch, (long long)n_heads * n_words,
                     (long long)n_words, s_key_cache_batch, (long long)kv_dim,
                     (long long)batch_size * kv_dim, head_size, kv_mul);
  return launch_status(hipGetLastError());
}

extern "C" thablasStatus_t thaDNN_s_multiheads_3_v2_batch(thablasHandle_t* handle, int batch_size, int pos_d[],
                                                          int n_heads, float* s_xb_batch, float* s_att_batch,
                                                          float* s_value_cache_batch, int head_size, int n_words,
                                                          int kv_dim, int kv_mul, int dim, int pipe_size) {
  (void)pipe_size;
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (batch_size <= 0 || n_heads <= 0) return THABLAS_STATUS_SUCCESS;
  if (!pos_d || !s_xb_batch || !s_att_batch || !s_value_cache_batch || head_size <= 0 || kv_mul <= 0)
    return THABLAS_STATUS_INVALID_VALUE;
  hipLaunchKernelGGL(k_mha_av, dim3((head_size + 63) / 64, n_heads, batch_size), dim3(256), 0,
                     handle->calc_stream, pos_d, n_heads, s_xb_batch, (long long)dim, s_att_batch,
                     (long long)n_heads * n_words, (long long)n_words, s_value_cache_batch, (long long)kv_dim,
                     (long long)batch_size * kv_dim, head_size, kv_mul);
  return launch_status(hipGetLastError());
}
