// gemv_q8.hpp — the int8 (Q8_0) twin of the decode GEMV, written for gfx950.
//
// Semantics: runq.c (reference) — activations are quantised per group of GS with
// scale = max|x|/127 and q = round-half-away(x/scale) (runq.c:145-171); each row is
//   y[i] = sum_g ( sum_{k in g} xq[k]*wq[i][k] ) * ws[i][g] * xs[g]
// with the inner sum exact in int32 and the outer one in fp32 (runq.c:317-342).
//
// Layout: the runq v2 file layout, unchanged — per tensor an int8 block [M][K]
// followed by an fp32 scale block [M][K/GS] (runq.c:173-187).
//
// Design:
//  * one wave per row; lane l reads 16 int8 (one dwordx4) of a 1-KiB wave-load,
//    i.e. a GS=64 group spans 4 lanes; the int8 products use v_dot4_i32_i8
//    (__builtin_amdgcn_sdot4), the group's int32 sum is completed with two xor
//    shuffles and scaled once, exactly like runq's per-group float step;
//  * the activation quantisation (and the RMSNorm feeding it) is a block prologue:
//    every block normalises + quantises the activations into LDS (int8 + scales),
//    so no extra launch and no int8 activation round-trip through HBM.
#pragma once
#include "gemv.hpp"

namespace tl {

TL_DEVICE int q8_round(float v) {
  // C round(): half away from zero; NaN (all-zero group, scale 0) -> 0 like the x86 reference
  const float r = roundf(v);
  return r != r ? 0 : (int)r;
}

// Stage quantised activations for rows [kc, kc+kcn): xq [NB][kcn] int8, xsc [NB][kcn/gs].
template <int NB>
TL_DEVICE void stage_x_q8(const GemvParams& p, int8_t* xq, float* xsc, int kc, int kcn, const float* ss) {
  const int gs = p.gs, ng = kcn / gs;
  for (int e = threadIdx.x; e < NB * ng; e += blockDim.x) {
    const int b = e / ng, g = e % ng;
    int8_t* dq = xq + b * kcn + g * gs;
    if (b >= p.nb) {
      for (int i = 0; i < gs; i += 4) *reinterpret_cast<int*>(dq + i) = 0;
      xsc[b * ng + g] = 0.f;
      continue;
    }
    const float* src = p.tok ? p.emb + (long long)p.tok[b] * p.K : p.x + b * p.x_stride;
    const int k0 = kc + g * gs;
    // pass 1: max |x'| over the group (x' = RMSNorm output when fused)
    float wmax = 0.f;
    for (int i = 0; i < gs; i += 4) {
      f4 v = *reinterpret_cast<const f4*>(src + k0 + i);
      if (p.rms_w) {
        const f4 w = *reinterpret_cast<const f4*>(p.rms_w + k0 + i);
        v = f4{__fmul_rn(w.x, __fmul_rn(ss[b], v.x)), __fmul_rn(w.y, __fmul_rn(ss[b], v.y)),
               __fmul_rn(w.z, __fmul_rn(ss[b], v.z)), __fmul_rn(w.w, __fmul_rn(ss[b], v.w))};
      }
      wmax = fmaxf(wmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    const float scale = __fdiv_rn(wmax, 127.0f);
    xsc[b * ng + g] = scale;
    // pass 2: quantise (x/scale, round half away from zero)
    for (int i = 0; i < gs; i += 4) {
      f4 v = *reinterpret_cast<const f4*>(src + k0 + i);
      if (p.rms_w) {
        const f4 w = *reinterpret_cast<const f4*>(p.rms_w + k0 + i);
        v = f4{__fmul_rn(w.x, __fmul_rn(ss[b], v.x)), __fmul_rn(w.y, __fmul_rn(ss[b], v.y)),
               __fmul_rn(w.z, __fmul_rn(ss[b], v.z)), __fmul_rn(w.w, __fmul_rn(ss[b], v.w))};
      }
      const int q0 = q8_round(__fdiv_rn(v.x, scale)), q1 = q8_round(__fdiv_rn(v.y, scale));
      const int q2 = q8_round(__fdiv_rn(v.z, scale)), q3 = q8_round(__fdiv_rn(v.w, scale));
      *reinterpret_cast<int*>(dq + i) = (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
    }
  }
}

template <int MODE>
TL_DEVICE void q8_item_row(const GemvParams& p, int item, int r, const int8_t*& q, const float*& s) {
  const long long K = p.K, ng = p.K / p.gs;
  long long row;
  int which;
  if constexpr (MODE == GM_SWIGLU) {
    which = r;
    row = item;
  } else if constexpr (MODE == GM_QKV) {
    int rr = 2 * item;
    if (rr < p.dim) { which = 0; row = rr + r; }
    else if (rr - p.dim < p.kv_dim) { which = 1; row = rr - p.dim + r; }
    else { which = 2; row = rr - p.dim - p.kv_dim + r; }
  } else {
    which = 0;
    row = item;
  }
  const int8_t* Q = which == 0 ? p.Q0 : (which == 1 ? p.Q1 : p.Q2);
  const float* S = which == 0 ? p.S0 : (which == 1 ? p.S1 : p.S2);
  q = Q + row * K;
  s = S + row * ng;
}

// acc[b] += this lane's share of row . xq over [kc, kc + kcn); LPG = lanes per group.
template <int NB, int LPG, bool NT>
TL_DEVICE void q8_row_chunk(const int8_t* __restrict__ wq, const float* __restrict__ ws, const int8_t* xq,
                            const float* xsc, int kc, int kcn, int gs, int lane, float (&acc)[NB]) {
  typedef int i4 __attribute__((ext_vector_type(4)));
  const int nfull = kcn >> 10;  // whole 1-KiB wave-loads in the chunk
  const int gpl = 1024 / gs;    // groups per wave-load
  const int ng_chunk = kcn / gs;
  auto step = [&](int j, bool live) {
    const int kb = j * 1024 + lane * 16;  // byte offset inside the chunk
    i4 wv = live ? (NT ? __builtin_nontemporal_load(reinterpret_cast<const i4*>(wq + kc + kb))
                       : *reinterpret_cast<const i4*>(wq + kc + kb))
                 : i4{0, 0, 0, 0};
    const int g = j * gpl + lane / LPG;  // group index inside the chunk
    const float wsc = live ? ws[(kc / gs) + g] : 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const i4 xv = live ? *reinterpret_cast<const i4*>(xq + b * kcn + kb) : i4{0, 0, 0, 0};
      int d = __builtin_amdgcn_sdot4(wv.x, xv.x, 0, false);
      d = __builtin_amdgcn_sdot4(wv.y, xv.y, d, false);
      d = __builtin_amdgcn_sdot4(wv.z, xv.z, d, false);
      d = __builtin_amdgcn_sdot4(wv.w, xv.w, d, false);
#pragma unroll
      for (int o = LPG / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if ((lane % LPG) == 0 && live)
        acc[b] += __fmul_rn(__fmul_rn((float)d, wsc), xsc[b * ng_chunk + (g < ng_chunk ? g : 0)]);
    }
  };
  int j = 0;
  for (; j + 4 <= nfull; j += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) step(j + u, true);
  }
  for (; j < nfull; ++j) step(j, true);
  if (nfull * 1024 < kcn) step(nfull, nfull * 1024 + lane * 16 < kcn);
}

template <int MODE, int NB, int LPG, bool NT>
__global__ void __launch_bounds__(256) gemv_q8_kernel(GemvParams p, int kc_max) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);  // 16
  float* ss = red + 16;                         // NB (<= 64)
  float* xsc = ss + 64;                         // [NB][kc/gs]
  int8_t* xq = reinterpret_cast<int8_t*>(xsc + NB * (kc_max / p.gs));  // [NB][kc]
  constexpr int RPI = RowsPerItem<MODE>::v;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wave;
  float acc[RPI][NB];
#pragma unroll
  for (int r = 0; r < RPI; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[r][b] = 0.f;
  if (p.rms_w) {
    rms_scales<NB>(p, ss, red);
    __syncthreads();
  }
  if (p.tok && blockIdx.x == 0) {  // embedding row -> residual stream (fused lookup)
    for (int e = threadIdx.x; e < p.nb * (p.K / 4); e += blockDim.x) {
      const int b = e / (p.K / 4), j = e % (p.K / 4);
      reinterpret_cast<f4*>(p.x_out + b * p.x_stride)[j] =
          reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.K)[j];
    }
  }
  for (int kc = 0; kc < p.K; kc += kc_max) {
    const int kcn = min(kc_max, p.K - kc);
    if (kc) __syncthreads();
    stage_x_q8<NB>(p, xq, xsc, kc, kcn, ss);
    __syncthreads();
    if (item < p.n_items) {
#pragma unroll
      for (int r = 0; r < RPI; ++r) {
        const int8_t* q;
        const float* s;
        q8_item_row<MODE>(p, item, r, q, s);
        q8_row_chunk<NB, LPG, NT>(q, s, xq, xsc, kc, kcn, p.gs, lane, acc[r]);
      }
    }
  }
  if (item >= p.n_items) return;
  float v[2][NB];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) v[r][b] = r < RPI ? wave_sum(acc[r < RPI ? r : 0][b]) : 0.f;
  epilogue<MODE, NB>(p, item, v, lane);
}

}  // namespace tl
