// gemv_mfma.hpp — the batched (2..16 sequences) decode GEMV on the fp32 matrix cores.
//
// With B sequences the VALU streaming kernel (gemv.hpp) multiplies every weight float4 by B
// activation float4s read back from LDS: at B = 8 that is 8x the weight bytes in LDS
// traffic, and the step runs at ~30% of the HBM roofline.  Here one wave computes a 16-row
// x 16-sequence tile with v_mfma_f32_16x16x4_f32: per 16-k step a lane loads ONE float4 of
// weights (row l&15, k = 4(l>>4)..+3) and ONE float4 of its sequence's activations
// (sequence l&15, same k), and four MFMAs consume them (component c of every lane is k-slot
// l>>4 of MFMA c, so A and B agree on k).  Activations come from L2 (every block reads the
// same B x K floats); the weights stream once, non-temporal.
//
// A block is 8 waves on the SAME 16 rows, splitting K (wave w takes 16-k steps w, w+8, ...),
// so even a 4096-row matrix gives 256 blocks x 8 waves; the 8 partial tiles are summed in
// LDS in a fixed order (deterministic), then the same fused epilogues as gemv.hpp (store
// at pos offsets, residual, SwiGLU over a W1/W3 pair of tiles, QKV + RoPE + KV write).
// Numerics: each wave's partial is a k-ordered fp32 fma chain.  An RMSNorm / embedding
// prologue runs ONCE per launch (gemv_prenorm_kernel, x' = w * (ss * x) as in
// src/seq.cpp:3-16) into scratch rows, not once per block.
#pragma once
#include "gemv.hpp"

namespace tl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMfmaWaves = 8;
constexpr int kMfmaUnr = 8;

// One output of the decode epilogues (gemv.hpp epilogue) for row/item `item`, sequence b.
template <int MODE>
TL_DEVICE void epi_one(const GemvParams& p, int item, int b, float v0, float v1) {
  if constexpr (MODE == GM_STORE) {
    float* y = p.y + p.y_off + (long long)b * p.y_stride + (p.has_pos ? (long long)p.has_pos * p.pos[b] : 0);
    y[item] = v0;
  } else if constexpr (MODE == GM_RESID) {
    float* y = p.y + (long long)b * p.y_stride + item;
    *y = __fadd_rn(*y, v0);
  } else if constexpr (MODE == GM_SWIGLU) {
    p.y[(long long)b * p.y_stride + item] = silu_mul(v0, v1);
  } else {  // GM_QKV: item = row pair (2 item, 2 item + 1) -> (v0, v1)
    int row = 2 * item;
    const int pb = p.pos[b];
    float a0 = v0, a1 = v1;
    if (row < p.dim + p.kv_dim) {
      const int i = row < p.dim ? row : row - p.dim;
      const float2 cs = p.rope[(long long)pb * (p.head_size >> 1) + ((i % p.head_size) >> 1)];
      const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
      const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
      a0 = r0; a1 = r1;
    }
    if (row < p.dim) {
      float* qd = p.y + (long long)b * p.y_stride + row;
      qd[0] = a0; qd[1] = a1;
    } else {
      row -= p.dim;
      float* base = p.kc;
      if (row >= p.kv_dim) { row -= p.kv_dim; base = p.vc; }
      float* dd = base + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)pb * p.kv_dim + row;
      dd[0] = a0; dd[1] = a1;
    }
  }
}

// xn[b] = rms_w * (ss_b * x_b) (or x_b itself without a norm); x_b is the embedding row
// tok[b] when tok is set, and then also copied to x_out (the residual stream).
static __global__ void __launch_bounds__(256) gemv_prenorm_kernel(GemvParams p) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int n4 = p.K >> 2;
  const f4* src = reinterpret_cast<const f4*>(p.tok ? p.emb + (long long)p.tok[b] * p.K : p.x + b * p.x_stride);
  f4* dst = reinterpret_cast<f4*>(p.xn + (long long)b * p.K);
  float sq = 0.f;
  for (int j = threadIdx.x; j < n4; j += blockDim.x) {
    const f4 v = src[j];
    if (p.tok) reinterpret_cast<f4*>(p.x_out + b * p.x_stride)[j] = v;
    sq = fmaf(v.x, v.x, sq); sq = fmaf(v.y, v.y, sq); sq = fmaf(v.z, v.z, sq); sq = fmaf(v.w, v.w, sq);
  }
  float s = 1.f;
  if (p.rms_w) {
    const float t = block_sum(sq, red);
    s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)p.K), 1e-5f)));
  }
  for (int j = threadIdx.x; j < n4; j += blockDim.x) {
    const f4 v = src[j];
    if (p.rms_w) {
      const f4 w = reinterpret_cast<const f4*>(p.rms_w)[j];
      dst[j] = f4{__fmul_rn(w.x, __fmul_rn(s, v.x)), __fmul_rn(w.y, __fmul_rn(s, v.y)),
                  __fmul_rn(w.z, __fmul_rn(s, v.z)), __fmul_rn(w.w, __fmul_rn(s, v.w))};
    } else {
      dst[j] = v;
    }
  }
}

template <int MODE, bool NT>
__global__ void __launch_bounds__(kMfmaWaves * 64) gemv_mfma_kernel(GemvParams p) {
  constexpr int W = kMfmaWaves, U = kMfmaUnr;
  constexpr bool TWO = MODE == GM_SWIGLU;  // two weight tiles (W1, W3) share the activations
  __shared__ float red[W][TWO ? 2 : 1][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int K = p.K, nb = p.nb;
  const long long Kl = K;

  // this lane's weight row(s): tile of 16 rows (QKV: 8 row pairs; SwiGLU: 16 items)
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
  const int r = blockIdx.x * 16 + i;
  const bool rv = r < n_rows;
  const int rr = rv ? r : 0;
  const float* w0;
  const float* w1 = nullptr;
  if constexpr (MODE == GM_SWIGLU) {
    w0 = p.W0 + rr * Kl;
    w1 = p.W1 + rr * Kl;
  } else if constexpr (MODE == GM_QKV) {
    w0 = item_row<GM_QKV>(p, rr >> 1, rr & 1);
  } else {
    w0 = p.W0 + rr * Kl;
  }
  // this lane's sequence (column i); the launcher has already applied any RMSNorm /
  // embedding prologue (gemv_prenorm_kernel), so x holds the GEMV input rows
  const bool jv = i < nb;
  const float* xr = jv ? p.x + (long long)i * p.x_stride : nullptr;

  const int nsteps = K >> 4;
  auto wl = [&](const float* w, int s) {
    const f4* a = reinterpret_cast<const f4*>(w + 16 * s + 4 * q);
    if constexpr (NT) return __builtin_nontemporal_load(a);
    else return *a;
  };

  f4 wa[U], wb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int s = wave + W * u;
    if (s < nsteps) {
      wa[u] = wl(w0, s);
      if constexpr (TWO) wb[u] = wl(w1, s);
    }
  }

  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int g = 0; g * W * U < nsteps; ++g) {
    f4 xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = wave + W * (g * U + u);
      xv[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (s < nsteps && jv) xv[u] = *reinterpret_cast<const f4*>(xr + 16 * s + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = wave + W * (g * U + u);
      if (s < nsteps) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[u].x, xv[u].x, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[u].y, xv[u].y, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[u].z, xv[u].z, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[u].w, xv[u].w, acc0, 0, 0, 0);
        if constexpr (TWO) {
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[u].x, xv[u].x, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[u].y, xv[u].y, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[u].z, xv[u].z, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[u].w, xv[u].w, acc1, 0, 0, 0);
        }
      }
    }
    // next group's weights
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = wave + W * ((g + 1) * U + u);
      if (s < nsteps) {
        wa[u] = wl(w0, s);
        if constexpr (TWO) wb[u] = wl(w1, s);
      }
    }
  }

  // C layout (16x16): lane holds rows 4q..4q+3 of column i
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[wave][0][(4 * q + e) * 16 + i] = acc0[e];
    if constexpr (TWO) red[wave][TWO ? 1 : 0][(4 * q + e) * 16 + i] = acc1[e];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 256) {
    const int row = t >> 4, j = t & 15;
    const int R = blockIdx.x * 16 + row;
    if (j < nb && R < n_rows) {
      float v0 = red[0][0][t];
      for (int w = 1; w < W; ++w) v0 += red[w][0][t];
      if constexpr (MODE == GM_SWIGLU) {
        float v1 = red[0][TWO ? 1 : 0][t];
        for (int w = 1; w < W; ++w) v1 += red[w][TWO ? 1 : 0][t];
        epi_one<MODE>(p, R, j, v0, v1);
      } else if constexpr (MODE == GM_QKV) {
        if ((row & 1) == 0) {
          float v1 = red[0][0][t + 16];
          for (int w = 1; w < W; ++w) v1 += red[w][0][t + 16];
          epi_one<MODE>(p, R >> 1, j, v0, v1);
        }
      } else {
        epi_one<MODE>(p, R, j, v0, 0.f);
      }
    }
  }
}

}  // namespace tl
