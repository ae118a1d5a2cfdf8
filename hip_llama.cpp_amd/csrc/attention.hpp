// attention.hpp — fused single-token decode attention for one layer.
//
// Semantics: reference src/seq.cpp:103-136 (scores q.k/sqrtf(hs) for t <= pos,
// softmax, weighted sum of V), which the reference GPU path splits into three
// launches (src/thaDNN/thaDNN_mha.cpp:246-426).  Here it is ONE launch over a
// (head, sequence, key-split) grid plus, when the keys are split, a tiny
// combine launch (flash-decoding).  K/V stay in the reference layout
// [b][layer][seq_len][kv_dim]; each key row of a head is 4*hs contiguous bytes,
// read by hs/4 lanes with one float4 each.
#pragma once
#include "common.hpp"

namespace tl {

struct AttnParams {
  const float* q;       // [B][dim]  (RoPE already applied)
  const float* kc;      // key_cache base   [B][L][S][kv_dim]
  const float* vc;      // value_cache base
  long long kv_b_stride, kv_l_off;
  const int* pos;       // [B]
  float* out;           // [B][dim]
  float* part;          // [B][H][nsplit][hs + 4]  (o, m, l, pad) when nsplit > 1
  int dim, kv_dim, head_size, n_heads, kv_mul, seq_len, nsplit, min_chunk;
};

TL_DEVICE void split_range(int T, int nsplit, int min_chunk, int s, int& t0, int& t1) {
  int chunk = (T + nsplit - 1) / nsplit;
  chunk = max(chunk, min_chunk);
  t0 = s * chunk;
  t1 = min(T, t0 + chunk);
}

// LPK = lanes per key row = hs/4.
template <int LPK>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);  // 16
  float* sc = red + 16;                         // scores for this split (<= seq_len)
  constexpr int HS = LPK * 4;
  const int h = blockIdx.x, b = blockIdx.y, s = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = p.pos[b] + 1;
  int t0, t1;
  split_range(T, p.nsplit, p.min_chunk, s, t0, t1);
  if (t0 >= t1) return;  // nothing for this split (combine ignores it)
  const int n = t1 - t0;

  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const f4 qv = reinterpret_cast<const f4*>(p.q + (long long)b * p.dim + h * HS)[lane % LPK];
  const float rs = sqrtf((float)HS);

  // ---- scores: each wave handles KPW = 64/LPK keys per step
  constexpr int KPW = 64 / LPK;
  const int sub = lane / LPK;
  for (int t = t0 + wave * KPW + sub; t - sub < t1; t += 4 * KPW) {
    float d = 0.f;
    if (t < t1) {
      const f4 kv = reinterpret_cast<const f4*>(kbase + (long long)t * p.kv_dim)[lane % LPK];
      d = dot4(qv, kv, 0.f);
    }
    d = group_sum<LPK>(d);
    if (t < t1 && (lane % LPK) == 0) sc[t - t0] = __fdiv_rn(d, rs);
  }
  __syncthreads();

  // ---- softmax over this split (reference src/seq.cpp:18-36)
  float m = -3.402823466e+38f;
  for (int i = tid; i < n; i += 256) m = fmaxf(m, sc[i]);
  m = block_max(m, red);
  float l = 0.f;
  for (int i = tid; i < n; i += 256) {
    float e = expf(__fsub_rn(sc[i], m));
    sc[i] = e;
    l += e;
  }
  l = block_sum(l, red);
  const bool whole = p.nsplit == 1 || (t0 == 0 && t1 == T);
  if (whole) {
    for (int i = tid; i < n; i += 256) sc[i] = __fdiv_rn(sc[i], l);
    __syncthreads();
  }

  // ---- weighted V sum: LPK float4 columns x G groups over t
  constexpr int G = 256 / LPK;
  const int col = tid % LPK, g = tid / LPK;
  f4 o = {0.f, 0.f, 0.f, 0.f};
  for (int t = t0 + g; t < t1; t += G) {
    const float a = sc[t - t0];
    const f4 vv = reinterpret_cast<const f4*>(vbase + (long long)t * p.kv_dim)[col];
    o.x = fmaf(a, vv.x, o.x); o.y = fmaf(a, vv.y, o.y);
    o.z = fmaf(a, vv.z, o.z); o.w = fmaf(a, vv.w, o.w);
  }
  // reduce the G groups through LDS (reuse the score area after a barrier)
  __syncthreads();
  f4* ob = reinterpret_cast<f4*>(sc);
  ob[g * LPK + col] = o;
  __syncthreads();
  if (tid < LPK) {
    f4 r = ob[tid];
    for (int gg = 1; gg < G; ++gg) {
      f4 x = ob[gg * LPK + tid];
      r.x += x.x; r.y += x.y; r.z += x.z; r.w += x.w;
    }
    if (whole) {
      reinterpret_cast<f4*>(p.out + (long long)b * p.dim + h * HS)[tid] = r;
    } else {
      float* pp = p.part + (((long long)b * p.n_heads + h) * p.nsplit + s) * (HS + 4);
      reinterpret_cast<f4*>(pp)[tid] = r;  // records are HS+4 floats: 16-B aligned
      if (tid == 0) { pp[HS] = m; pp[HS + 1] = l; }
    }
  }
}

// out[b][h*hs + i] = sum_s o_s[i] e^{m_s-M} / sum_s l_s e^{m_s-M}
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnParams p) {
  const int h = blockIdx.x, b = blockIdx.y;
  const int hs = p.head_size;
  const int T = p.pos[b] + 1;
  int t0, t1;
  split_range(T, p.nsplit, p.min_chunk, 0, t0, t1);
  if (t1 == T) return;  // single split covered everything and wrote `out` directly
  const float* base = p.part + ((long long)b * p.n_heads + h) * p.nsplit * (hs + 4);
  float M = -3.402823466e+38f;
  int ns = 0;
  for (int s = 0; s < p.nsplit; ++s) {
    int a0, a1;
    split_range(T, p.nsplit, p.min_chunk, s, a0, a1);
    if (a0 >= a1) break;
    M = fmaxf(M, base[s * (hs + 4) + hs]);
    ns = s + 1;
  }
  float L = 0.f;
  for (int s = 0; s < ns; ++s) L += base[s * (hs + 4) + hs + 1] * expf(base[s * (hs + 4) + hs] - M);
  for (int i = threadIdx.x; i < hs; i += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < ns; ++s) acc = fmaf(base[s * (hs + 4) + i], expf(base[s * (hs + 4) + hs] - M), acc);
    p.out[(long long)b * p.dim + h * hs + i] = acc / L;
  }
}

}  // namespace tl
