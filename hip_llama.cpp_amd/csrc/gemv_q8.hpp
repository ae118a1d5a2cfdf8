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
//  * one wave per row group; lane l reads 16 int8 (one dwordx4) of each 1-KiB
//    wave-load, so a GS=64 group spans 4 lanes; products use v_dot4_i32_i8
//    (__builtin_amdgcn_sdot4) and a group's int32 sum is completed with two xor
//    shuffles and scaled once, exactly like runq's per-group float step;
//  * a wave keeps IPW items (x2 rows for SwiGLU / QKV pairs) in flight at once:
//    4 wave-loads per row per step, so 16-32 KiB per wave are outstanding;
//  * the activation quantisation (and the RMSNorm feeding it) is a cooperative
//    block prologue: GS/16 threads per group, each normalising and quantising 16
//    values, a shuffle max per group, one dwordx4 LDS store per thread — no extra
//    launch and no int8 activation round-trip through HBM.
#pragma once
#include "gemv.hpp"

namespace tl {

typedef int q8i4 __attribute__((ext_vector_type(4)));

// 16 (or 8) activations (one thread's slice of a group) -> int8 codes packed in dwords:
// q = round(x / scale), runq.c:167, bit-identical to the IEEE division and C round() (the
// division-free quotient and rounding of common.hpp q8_code_fast: the division costs ~10
// VALU instructions and every block of the persistent step quantises the whole vector).
template <int NF4>  // NF4 float4s -> NF4 dwords of int8 codes
TL_DEVICE void q8_pack(const f4 (&v)[NF4], float scale, int (&packed)[NF4]) {
  float q[4 * NF4];
#pragma unroll
  for (int u = 0; u < NF4; ++u) { q[4 * u] = v[u].x; q[4 * u + 1] = v[u].y; q[4 * u + 2] = v[u].z; q[4 * u + 3] = v[u].w; }
  int qi[4 * NF4];
  if (q8_fast_scale(scale)) {
    const float r = __fdiv_rn(1.0f, scale);
#pragma unroll
    for (int i = 0; i < 4 * NF4; ++i) qi[i] = q8_code_fast(q[i], scale, r);
  } else {
#pragma unroll
    for (int i = 0; i < 4 * NF4; ++i) qi[i] = q8_round(__fdiv_rn(q[i], scale));
  }
#pragma unroll
  for (int u = 0; u < NF4; ++u)
    packed[u] = (qi[4 * u] & 0xFF) | ((qi[4 * u + 1] & 0xFF) << 8) | ((qi[4 * u + 2] & 0xFF) << 16) |
                ((qi[4 * u + 3] & 0xFF) << 24);
}
typedef int q8i2 __attribute__((ext_vector_type(2)));
TL_DEVICE q8i4 q8_pack16(const f4 (&v)[4], float scale) {
  int p[4];
  q8_pack<4>(v, scale, p);
  return q8i4{p[0], p[1], p[2], p[3]};
}
TL_DEVICE q8i2 q8_pack8(const f4 (&v)[2], float scale) {
  int p[2];
  q8_pack<2>(v, scale, p);
  return q8i2{p[0], p[1]};
}

TL_DEVICE f4 rms_apply(f4 v, f4 w, float s) {
  return f4{__fmul_rn(w.x, __fmul_rn(s, v.x)), __fmul_rn(w.y, __fmul_rn(s, v.y)), __fmul_rn(w.z, __fmul_rn(s, v.z)),
            __fmul_rn(w.w, __fmul_rn(s, v.w))};
}

// Quantise activations [kc, kc+kcn) of every live sequence into xq [NB][kcn] int8 and
// xsc [NB][kcn/gs]; TPG = gs/16 threads per group, 16 values per thread.
template <int NB, int TPG>
TL_DEVICE void stage_x_q8(const GemvParams& p, int8_t* xq, float* xsc, int kc, int kcn, const float* ss) {
  const int n16 = kcn >> 4;  // 16-value slices per sequence
  for (int e = threadIdx.x; e < NB * n16; e += blockDim.x) {
    const int b = e / n16, sl = e % n16;  // TPG consecutive threads own one group
    const int k0 = kc + sl * 16;
    f4 v[4];
    if (b < p.nb) {
      const float* src = p.tok ? p.emb + (long long)p.tok[b] * p.K : p.x + b * p.x_stride;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = *reinterpret_cast<const f4*>(src + k0 + 4 * u);
        if (p.rms_w) v[u] = rms_apply(v[u], *reinterpret_cast<const f4*>(p.rms_w + k0 + 4 * u), ss[b]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = f4{0.f, 0.f, 0.f, 0.f};
    }
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
#pragma unroll
    for (int o = TPG / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const float scale = __fdiv_rn(m, 127.0f);
    *reinterpret_cast<q8i4*>(xq + b * kcn + sl * 16) = q8_pack16(v, scale);
    if ((sl % TPG) == 0) xsc[b * (kcn / (TPG * 16)) + sl / TPG] = scale;
  }
}

// Batched launches: quantise every live sequence's activations ONCE (RMSNorm / embedding
// fused as in stage_x_q8) into p.xq / p.xqs, instead of once per block (at 8 sequences the
// per-block prologue read 8 x K activations for every 16-32 weight rows).  One block per
// sequence; same arithmetic as stage_x_q8 (runq.c:145-171).
template <int LPG>
__global__ void __launch_bounds__(256) gemv_q8_prequant_kernel(GemvParams p) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int K = p.K, n16 = K >> 4, ng = K / (LPG * 16);
  const float* src = p.tok ? p.emb + (long long)p.tok[b] * K : p.x + b * p.x_stride;
  float s = 1.f;
  if (p.rms_w) {
    float sq = 0.f;
    for (int j = threadIdx.x; j < (K >> 2); j += blockDim.x) {
      const f4 v = reinterpret_cast<const f4*>(src)[j];
      sq = fmaf(v.x, v.x, sq); sq = fmaf(v.y, v.y, sq); sq = fmaf(v.z, v.z, sq); sq = fmaf(v.w, v.w, sq);
    }
    const float t = block_sum(sq, red);
    s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)K), 1e-5f)));
  }
  if (p.tok)
    for (int j = threadIdx.x; j < (K >> 2); j += blockDim.x)
      reinterpret_cast<f4*>(p.x_out + b * p.x_stride)[j] = reinterpret_cast<const f4*>(src)[j];
  // 256 threads = 64 quads... of LPG threads per group; every thread one 16-value slice
  for (int sl0 = 0; sl0 < n16; sl0 += blockDim.x) {
    const int sl = sl0 + threadIdx.x;
    const bool live = sl < n16;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = live ? reinterpret_cast<const f4*>(src + sl * 16)[u] : f4{0.f, 0.f, 0.f, 0.f};
      if (live && p.rms_w) v[u] = rms_apply(v[u], reinterpret_cast<const f4*>(p.rms_w + sl * 16)[u], s);
    }
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
#pragma unroll
    for (int o = LPG / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const float scale = __fdiv_rn(m, 127.0f);
    if (live) {
      *reinterpret_cast<q8i4*>(p.xq + (long long)b * K + sl * 16) = q8_pack16(v, scale);
      if ((sl % LPG) == 0) p.xqs[(long long)b * ng + sl / LPG] = scale;
    }
  }
}

// The same with every value loaded once, up front, and kept in registers through the norm's
// block sum (K <= 3 * 256 * 16 = 12288): one memory round trip instead of two dependent ones
// (the batched int8 step runs four of these per layer; 5 us each on one CU per sequence).
template <int LPG>
__global__ void __launch_bounds__(256) gemv_q8_prequant_reg_kernel(GemvParams p) {
  constexpr int MR = 3;
  __shared__ float red[16];
  const int b = blockIdx.x, t = threadIdx.x;
  const int K = p.K, n16 = K >> 4, ng = K / (LPG * 16);
  const float* src = p.tok ? p.emb + (long long)p.tok[b] * K : p.x + b * p.x_stride;
  f4 v[MR][4];
  float sq = 0.f;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int sl = r * 256 + t;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[r][u] = sl < n16 ? reinterpret_cast<const f4*>(src + sl * 16)[u] : f4{0.f, 0.f, 0.f, 0.f};
      sq = fmaf(v[r][u].x, v[r][u].x, sq); sq = fmaf(v[r][u].y, v[r][u].y, sq);
      sq = fmaf(v[r][u].z, v[r][u].z, sq); sq = fmaf(v[r][u].w, v[r][u].w, sq);
    }
    if (p.tok && sl < n16)
#pragma unroll
      for (int u = 0; u < 4; ++u) reinterpret_cast<f4*>(p.x_out + b * p.x_stride + sl * 16)[u] = v[r][u];
  }
  float s = 1.f;
  if (p.rms_w) s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(block_sum(sq, red), (float)K), 1e-5f)));
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    if (r * 256 >= n16) break;  // block-uniform
    const int sl = r * 256 + t;
    const bool live = sl < n16;
    f4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      w[u] = live && p.rms_w ? rms_apply(v[r][u], reinterpret_cast<const f4*>(p.rms_w + sl * 16)[u], s) : v[r][u];
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(w[u].x), fabsf(w[u].y)), fmaxf(fabsf(w[u].z), fabsf(w[u].w))));
    m = fmaxf(m, dpp_f<0xB1>(m));
    if (LPG >= 4) m = fmaxf(m, dpp_f<0x4E>(m));
    if (LPG >= 8) m = fmaxf(m, dpp_f<0x141>(m));
    const float scale = __fdiv_rn(m, 127.0f);
    if (live) {
      *reinterpret_cast<q8i4*>(p.xq + (long long)b * K + sl * 16) = q8_pack16(w, scale);
      if ((sl % LPG) == 0) p.xqs[(long long)b * ng + sl / LPG] = scale;
    }
  }
}

// Copy pre-quantised activations [kc, kc+kcn) of every live sequence into the LDS layout
// stage_x_q8 produces.
template <int NB, int LPG>
TL_DEVICE void stage_x_q8_pre(const GemvParams& p, int8_t* xq, float* xsc, int kc, int kcn) {
  typedef int i4 __attribute__((ext_vector_type(4)));
  const int n16 = kcn >> 4, gsz = LPG * 16, ngc = kcn / gsz, ng = p.K / gsz;
  for (int e = threadIdx.x; e < NB * n16; e += blockDim.x) {
    const int b = e / n16, sl = e % n16;
    i4 v = i4{0, 0, 0, 0};
    if (b < p.nb) v = *reinterpret_cast<const i4*>(p.xq + (long long)b * p.K + kc + sl * 16);
    *reinterpret_cast<i4*>(xq + b * kcn + sl * 16) = v;
  }
  for (int e = threadIdx.x; e < NB * ngc; e += blockDim.x) {
    const int b = e / ngc, gi = e % ngc;
    xsc[b * ngc + gi] = b < p.nb ? p.xqs[(long long)b * ng + kc / gsz + gi] : 0.f;
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


// One wave-load (16 int8 per lane) of one row against every sequence's activations.
template <int NB, int LPG>
TL_DEVICE void q8_dot(q8i4 wv, float wsc, const int8_t* xq, const float* xsc, int kcn, int gidx, int kb, int lane,
                      float (&acc)[NB]) {
  const int ng = kcn / (LPG * 16);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const q8i4 xv = *reinterpret_cast<const q8i4*>(xq + b * kcn + kb);
    int d = __builtin_amdgcn_sdot4(wv.x, xv.x, 0, false);
    d = __builtin_amdgcn_sdot4(wv.y, xv.y, d, false);
    d = __builtin_amdgcn_sdot4(wv.z, xv.z, d, false);
    d = __builtin_amdgcn_sdot4(wv.w, xv.w, d, false);
    d = lane_group_sum_i<LPG>(d);
    // runq.c:334: val += ((float)ival) * w.s * x.s, once per group (its first lane)
    if ((lane % LPG) == 0) acc[b] += __fmul_rn(__fmul_rn((float)d, wsc), xsc[b * ng + gidx]);
  }
}

// WAVES waves, IPW items per wave (RPI rows each) streamed together.
template <int MODE, int NB, int LPG, bool NT, int WAVES, int IPW>
__global__ void __launch_bounds__(WAVES * 64) gemv_q8_kernel(GemvParams p, int kc_max) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);  // 16
  float* ss = red + 16;                         // NB (<= 64)
  float* xsc = ss + 64;                         // [NB][kc/gs]
  int8_t* xq = reinterpret_cast<int8_t*>(xsc + NB * (kc_max / (LPG * 16)));  // [NB][kc]
  constexpr int RPI = RowsPerItem<MODE>::v;
  constexpr int R = IPW * RPI;  // rows in flight per wave
  constexpr int GS = LPG * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int item0 = blockIdx.x * (WAVES * IPW) + wave;

  float acc[R][NB];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[r][b] = 0.f;
  if (p.rms_w) rms_scales<NB>(p, ss, red);
  if (p.tok && blockIdx.x == 0) {  // embedding row -> residual stream (fused lookup)
    for (int e = threadIdx.x; e < p.nb * (p.K / 4); e += blockDim.x) {
      const int b = e / (p.K / 4), j = e % (p.K / 4);
      reinterpret_cast<f4*>(p.x_out + b * p.x_stride)[j] =
          reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.K)[j];
    }
  }
  // row pointers of this wave's items (rows of dead items point at row 0: loaded, never stored)
  const int8_t* wq[R];
  const float* ws[R];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int item = item0 + i * WAVES;
#pragma unroll
    for (int r = 0; r < RPI; ++r) q8_item_row<MODE>(p, item < p.n_items ? item : 0, r, wq[i * RPI + r], ws[i * RPI + r]);
  }

  for (int kc = 0; kc < p.K; kc += kc_max) {
    const int kcn = min(kc_max, p.K - kc);
    if (kc) __syncthreads();
    if (p.xq) stage_x_q8_pre<NB, LPG>(p, xq, xsc, kc, kcn);
    else stage_x_q8<NB, LPG>(p, xq, xsc, kc, kcn, ss);
    __syncthreads();
    const int nfull = kcn >> 10;
    int j = 0;
    for (; j + 2 <= nfull; j += 2) {  // 2 wave-loads x R rows in flight
      q8i4 wv[2][R];
      float sc[2][R];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int kb = (j + u) * 1024 + lane * 16;
          const q8i4* src = reinterpret_cast<const q8i4*>(wq[r] + kc + kb);
          wv[u][r] = NT ? __builtin_nontemporal_load(src) : *src;
          sc[u][r] = ws[r][(kc + kb) / GS];
        }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
          q8_dot<NB, LPG>(wv[u][r], sc[u][r], xq, xsc, kcn, ((j + u) * 1024 + lane * 16) / GS, (j + u) * 1024 + lane * 16,
                          lane, acc[r]);
    }
    for (; j * 1024 < kcn; ++j) {  // last full wave-load and/or the partial tail
      const int kb = j * 1024 + lane * 16;
      const bool live = kb < kcn;
      const int kbl = live ? kb : 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const q8i4* src = reinterpret_cast<const q8i4*>(wq[r] + kc + kbl);
        q8i4 wv = NT ? __builtin_nontemporal_load(src) : *src;
        float sc = ws[r][(kc + kbl) / GS];
        if (!live) { wv = q8i4{0, 0, 0, 0}; sc = 0.f; }
        q8_dot<NB, LPG>(wv, sc, xq, xsc, kcn, kbl / GS, kbl, lane, acc[r]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int item = item0 + i * WAVES;
    if (item >= p.n_items) continue;
    float v[2][NB];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int b = 0; b < NB; ++b) v[r][b] = r < RPI ? wave_sum_u(acc[i * RPI + (r < RPI ? r : 0)][b]) : 0.f;
    epilogue<MODE, NB>(p, item, v, lane);
  }
}

}  // namespace tl
