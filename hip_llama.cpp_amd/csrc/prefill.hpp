// prefill.hpp — batched prompt processing kernels (prefill.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tl {

// Y[t][m] (op)= sum_k X[t][k] W[m][k] for t < n, m < M, on the fp32 matrix cores; epilogue by
// mode (gemv.hpp GemvMode): GM_STORE, GM_RESID (+=), GM_SWIGLU (W1/W3 rows interleaved,
// Y = hb), GM_QKV (RoPE; q -> Y, k/v -> cache rows at pos0 + t).  K % 32 == 0.
struct PGemmArgs {
  const float* X;
  int ldx;
  int n, K, M;
  const float *W0, *W1, *W2;
  float* Y;
  int ldy;
  float *kc, *vc;  // this sequence's cache, layer offset applied
  int pos0, dim, kv_dim, head_size;
  const float2* rope;
};

hipError_t prefill_gemm(int mode, const PGemmArgs& a, hipStream_t s);
hipError_t prefill_embed(float* x, const float* emb, const int* tok, int n, int dim, hipStream_t s);
hipError_t prefill_rmsnorm(float* o, const float* x, const float* w, int n, int dim, hipStream_t s);
hipError_t prefill_positions(int* pos, int pos0, int n, hipStream_t s);

}  // namespace tl
