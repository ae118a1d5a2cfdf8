// prefill.hip — batched prompt processing.
//
// The reference feeds a prompt one token per decode step (src/llama.cpp:1029-1031: while
// pos < n_prompt-1 the next token is forced), i.e. n_prompt full passes over the weights.
// Here the prompt's n tokens go through each layer together: every projection is ONE
// [n x K] x [K x M] GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32,
// each output a k-ordered fmaf chain), the weights are read once per 64 prompt tokens
// instead of once per token, and the attention of all n queries is one launch of the decode
// attention kernel with the n positions as its "sequences" over one shared KV cache.
// Only the K/V cache rows (and the residual stream) are the product: no logits are formed
// for the forced tokens; the next decode step starts from the last prompt token.
//
// Semantics per token are the decode step's (src/seq.cpp:53-168): RMSNorm, QKV, RoPE, K/V
// written at pos0+p, causal attention over positions <= pos0+p, Wo + residual, RMSNorm,
// SwiGLU, W2 + residual.
#include <hip/hip_runtime.h>
#include "attention.hpp"
#include "common.hpp"
#include "gemv.hpp"
#include "prefill.hpp"

namespace tl {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GM_BM = 64;   // prompt tokens per block tile
constexpr int GM_BN = 128;  // weight rows per block tile
constexpr int GM_BK = 32;   // K per LDS stage
constexpr int GM_LD = GM_BK + 2;  // LDS row stride: 17*r mod 32 permutes the banks -> conflict free

struct PGemmParams {
  const float* X;      // [n][ldx] input rows
  int ldx;
  int n, K, M;         // tokens, reduction length, output rows (weight rows)
  const float* W0;     // QKV: Wq | SwiGLU: W1 | W
  const float* W1;     // QKV: Wk | SwiGLU: W3
  const float* W2;     // QKV: Wv
  float* Y;            // output rows [n][ldy] (QKV: q, RESID: x (+=), SwiGLU: hb)
  int ldy;
  // QKV: K/V cache rows at pos0 + p, RoPE from the host table
  float* kc;
  float* vc;           // cache base of this sequence + layer offset
  int pos0, dim, kv_dim, head_size;
  const float2* rope;
};

// Global weight row R of the phase (QKV: [Wq; Wk; Wv]; SwiGLU: W1/W3 rows interleaved,
// 2i = W1 row i, 2i+1 = W3 row i, so each SwiGLU pair sits in two adjacent output columns).
template <int MODE>
TL_DEVICE const float* wrow(const PGemmParams& p, int R) {
  const long long K = p.K;
  if constexpr (MODE == GM_SWIGLU) return ((R & 1) ? p.W1 : p.W0) + (long long)(R >> 1) * K;
  if constexpr (MODE == GM_QKV) {
    if (R < p.dim) return p.W0 + (long long)R * K;
    R -= p.dim;
    if (R < p.kv_dim) return p.W1 + (long long)R * K;
    return p.W2 + (long long)(R - p.kv_dim) * K;
  }
  return p.W0 + (long long)R * K;
}

// Block: 4 waves in 2 (tokens) x 2 (rows); wave tile 32 tokens x 64 rows = two 32x32 MFMA
// accumulators.  Operands stage through LDS 32 K at a time; the next stage's global loads
// are issued before the current stage's MFMAs.
template <int MODE>
__global__ void __launch_bounds__(256) prefill_gemm_kernel(PGemmParams p) {
  keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  __shared__ __attribute__((aligned(16))) float Xs[GM_BM * GM_LD];
  __shared__ __attribute__((aligned(16))) float Ws[GM_BN * GM_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = blockIdx.x * GM_BN, t0 = blockIdx.y * GM_BM;

  // global -> register staging: W 128x32 (4 float4 per thread), X 64x32 (2 per thread)
  const int sr = tid >> 3, sc = (tid & 7) * 4;  // row within a 32-row pass, k offset
  const float* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int R = m0 + sr + 32 * i;
    wsrc[i] = R < p.M ? wrow<MODE>(p, R) : nullptr;
  }
  const float* xsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int t = t0 + sr + 32 * i;
    xsrc[i] = t < p.n ? p.X + (long long)t * p.ldx : nullptr;
  }
  f4 wreg[4], xreg[2];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      wreg[i] = wsrc[i] ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(wsrc[i] + k0 + sc))
                        : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
      xreg[i] = xsrc[i] ? *reinterpret_cast<const f4*>(xsrc[i] + k0 + sc) : f4{0.f, 0.f, 0.f, 0.f};
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* d = Ws + (sr + 32 * i) * GM_LD + sc;
      *reinterpret_cast<float2*>(d) = make_float2(wreg[i].x, wreg[i].y);
      *reinterpret_cast<float2*>(d + 2) = make_float2(wreg[i].z, wreg[i].w);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float* d = Xs + (sr + 32 * i) * GM_LD + sc;
      *reinterpret_cast<float2*>(d) = make_float2(xreg[i].x, xreg[i].y);
      *reinterpret_cast<float2*>(d + 2) = make_float2(xreg[i].z, xreg[i].w);
    }
  };

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  const float* xa = Xs + (wr * 32 + (lane & 31)) * GM_LD + (lane >> 5);
  const float* wb0 = Ws + (wc * 64 + (lane & 31)) * GM_LD + (lane >> 5);
  const float* wb1 = wb0 + 32 * GM_LD;

  fetch(0);
  for (int k0 = 0; k0 < p.K; k0 += GM_BK) {
    __syncthreads();  // previous stage consumed
    stash();
    __syncthreads();
    if (k0 + GM_BK < p.K) fetch(k0 + GM_BK);
#pragma unroll
    for (int kk = 0; kk < GM_BK; kk += 2) {
      const float a = xa[kk];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, wb0[kk], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, wb1[kk], acc1, 0, 0, 0);
    }
  }

  // epilogue: lane owns output column m (a weight row) for 16 token rows
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const f32x16& acc = half ? acc1 : acc0;
    const int m = m0 + wc * 64 + half * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = t0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const float v = acc[r];
      // partner column m ^ 1 lives in lane ^ 1 (same token rows)
      const float pv = __shfl_xor(v, 1, 64);
      if (t >= p.n || m >= p.M) continue;
      if constexpr (MODE == GM_RESID) {
        float* y = p.Y + (long long)t * p.ldy + m;
        *y = __fadd_rn(*y, v);
      } else if constexpr (MODE == GM_SWIGLU) {
        if ((m & 1) == 0) p.Y[(long long)t * p.ldy + (m >> 1)] = silu_mul(v, pv);
      } else if constexpr (MODE == GM_QKV) {
        const int pos = p.pos0 + t;
        const bool odd = m & 1;
        const float a0 = odd ? pv : v, a1 = odd ? v : pv;
        float out = v;
        if (m < p.dim + p.kv_dim) {
          // RoPE on the (2i, 2i+1) pair (reference src/seq.cpp:86-101)
          const int i = m < p.dim ? m : m - p.dim;
          const float2 cs = p.rope[(long long)pos * (p.head_size >> 1) + ((i % p.head_size) >> 1)];
          out = odd ? __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x))
                    : __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        }
        if (m < p.dim) {
          p.Y[(long long)t * p.ldy + m] = out;
        } else if (m < p.dim + p.kv_dim) {
          p.kc[(long long)pos * p.kv_dim + (m - p.dim)] = out;
        } else {
          p.vc[(long long)pos * p.kv_dim + (m - p.dim - p.kv_dim)] = out;
        }
      } else {
        p.Y[(long long)t * p.ldy + m] = v;
      }
    }
  }
}

// x[t] = emb[tok[t]]
__global__ void __launch_bounds__(256) k_embed_rows(float* x, const float* emb, const int* tok, int dim) {
  const int t = blockIdx.x;
  const f4* s = reinterpret_cast<const f4*>(emb + (long long)tok[t] * dim);
  f4* d = reinterpret_cast<f4*>(x + (long long)t * dim);
  for (int j = threadIdx.x; j < (dim >> 2); j += blockDim.x) d[j] = s[j];
}

// o[t] = w * (ss * x[t]), ss = 1/sqrt(sum x^2 / dim + 1e-5) (reference src/seq.cpp:3-16)
__global__ void __launch_bounds__(256) k_rmsnorm_rows(float* o, const float* x, const float* w, int dim) {
  __shared__ float red[16];
  const int t = blockIdx.x;
  const float* xr = x + (long long)t * dim;
  float s = 0.f;
  for (int j = threadIdx.x; j < dim; j += blockDim.x) s = fmaf(xr[j], xr[j], s);
  s = block_sum(s, red);
  const float ss = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(s, (float)dim), 1e-5f)));
  for (int j = threadIdx.x; j < dim; j += blockDim.x) o[(long long)t * dim + j] = __fmul_rn(w[j], __fmul_rn(ss, xr[j]));
}

__global__ void k_iota_pos(int* pos, int pos0, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) pos[t] = pos0 + t;
}

template <int MODE>
static hipError_t gemm(const PGemmParams& p, hipStream_t s) {
  dim3 grid((p.M + GM_BN - 1) / GM_BN, (p.n + GM_BM - 1) / GM_BM);
  hipLaunchKernelGGL(prefill_gemm_kernel<MODE>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t prefill_gemm(int mode, const PGemmArgs& a, hipStream_t s) {
  PGemmParams p = {};
  p.X = a.X; p.ldx = a.ldx; p.n = a.n; p.K = a.K; p.M = a.M;
  p.W0 = a.W0; p.W1 = a.W1; p.W2 = a.W2; p.Y = a.Y; p.ldy = a.ldy;
  p.kc = a.kc; p.vc = a.vc; p.pos0 = a.pos0; p.dim = a.dim; p.kv_dim = a.kv_dim; p.head_size = a.head_size;
  p.rope = a.rope;
  switch (mode) {
    case GM_QKV: return gemm<GM_QKV>(p, s);
    case GM_RESID: return gemm<GM_RESID>(p, s);
    case GM_SWIGLU: return gemm<GM_SWIGLU>(p, s);
    default: return gemm<GM_STORE>(p, s);
  }
}

hipError_t prefill_embed(float* x, const float* emb, const int* tok, int n, int dim, hipStream_t s) {
  hipLaunchKernelGGL(k_embed_rows, dim3(n), dim3(256), 0, s, x, emb, tok, dim);
  return hipGetLastError();
}

hipError_t prefill_rmsnorm(float* o, const float* x, const float* w, int n, int dim, hipStream_t s) {
  hipLaunchKernelGGL(k_rmsnorm_rows, dim3(n), dim3(256), 0, s, o, x, w, dim);
  return hipGetLastError();
}

hipError_t prefill_positions(int* pos, int pos0, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_iota_pos, dim3((n + 255) / 256), dim3(256), 0, s, pos, pos0, n);
  return hipGetLastError();
}

}  // namespace tl
