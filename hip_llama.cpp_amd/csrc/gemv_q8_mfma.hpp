// gemv_q8_mfma.hpp — the batched (4..8 sequences) int8 decode GEMV on the int8 matrix cores.
//
// runq.c:317-342 per output row: per group of GS = 64 the int32 dot of the weight and
// activation codes, then val += ((float)ival * w.s) * x.s.  The VALU kernel (gemv_q8.hpp)
// spends one v_dot4_i32_i8 per 4 weight bytes and sequence, so at 8 sequences it is
// VALU-bound; here one wave computes a 16-row x 16-sequence tile and ONE
// v_mfma_i32_16x16x64_i8 per quantisation group gives all 256 exact int32 group dots (lane
// (i, q) feeds row / sequence i with bytes 16q..16q+15 of the group).  The weight bytes take
// the fp32 matrix-core kernel's path (gemv_mfma.hpp): 256-B row runs (= 4 groups, 16 lanes x
// 16 B, four rows per load instruction) through a wave-private LDS tile padded by 16 B per
// row, read back in the MFMA layout; the activation codes (quantised once per launch,
// gemv_q8_prequant_kernel) come the same way, rows >= 8 stay zero.  The group scales of the
// run go through LDS too, and each lane scales its 4 int32 results per group in fp32.
// Splits, partial sums and epilogues are the fp32 kernel's (fixed orders: deterministic).
#pragma once
#include "gemv_mfma.hpp"

namespace tl {

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(kMfmaWaves * 64) gemv_q8_mfma_kernel(GemvParams p) {
  keep_implicit_args();  // common.hpp
  constexpr int W = kMfmaWaves;
  constexpr bool TWO = MODE == GM_SWIGLU;
  constexpr int NR = TWO ? 2 : 1;  // weight tiles per run; tile NR is the activation codes
  constexpr int U = 4;             // quantisation groups (64 B) per 256-B run
  constexpr int LPR = 16;          // lanes per row in a load (16 B each)
  constexpr int RPI = 64 / LPR;    // rows per load instruction
  constexpr int NI = 16 / RPI;     // load instructions per 16-row tile
  constexpr int XI = 2;            // activation rows 0..7 (nb <= 8): two load instructions
  constexpr int STR = 64 + 4;      // LDS row stride in dwords (256 B + 16 B pad)
  constexpr int TILE = 16 * STR;   // dwords per tile
  __shared__ __attribute__((aligned(16))) unsigned lds[W * (NR + 1) * TILE];
  __shared__ float scl[W][NR + 1][16][U];  // the run's group scales: [tile][row or sequence][group]
  __shared__ unsigned s_last;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int lr = lane / LPR, lc = lane % LPR;  // load map: row RPI v + lr, 16-B chunk lc
  const int K = p.K, nb = p.nb, ng = K >> 6;
  const int tile = blockIdx.x / p.msplit, split = blockIdx.x - tile * p.msplit;
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;

  // weight rows of this tile (clamped: rows past the matrix reuse the last, results dropped)
  const int8_t* wrow[NR][NI];
  const float* srow[NR][NI];
#pragma unroll
  for (int v = 0; v < NI; ++v) {
    const int r = RPI * v + lr;
    int R = tile * 16 + r;
    R = R < n_rows ? R : n_rows - 1;
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      if constexpr (MODE == GM_QKV) q8_item_row<GM_QKV>(p, R >> 1, R & 1, wrow[m][v], srow[m][v]);
      else q8_item_row<MODE>(p, R, m, wrow[m][v], srow[m][v]);
    }
  }
  // scale loads: lane l -> row (or sequence) l / 4, group l % 4 of the run
  const int sr = lane >> 2, sg = lane & 3;
  const float* wsrow[NR];
  {
    int R = tile * 16 + sr;
    R = R < n_rows ? R : n_rows - 1;
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      const int8_t* dummy;
      if constexpr (MODE == GM_QKV) q8_item_row<GM_QKV>(p, R >> 1, R & 1, dummy, wsrow[m]);
      else q8_item_row<MODE>(p, R, m, dummy, wsrow[m]);
    }
  }
  const bool sx = sr < nb;
  const float* xsrow = p.xqs + (long long)(sx ? sr : 0) * ng;

  const int nruns = K >> 8;
  const int r0 = split * p.msteps;
  const int r1 = r0 + p.msteps < nruns ? r0 + p.msteps : nruns;
  const int per = (r1 - r0 + W - 1) / W;
  const int ws_ = r0 + wave * per;
  const int we = ws_ + per < r1 ? ws_ + per : r1;
  const int nrun = we > ws_ ? we - ws_ : 0;

  auto wl = [&](const int8_t* w) {
    const f4* a = reinterpret_cast<const f4*>(w);
    if constexpr (NT) return __builtin_nontemporal_load(a);
    else return *a;
  };
  struct Run {
    f4 t[NR + 1][NI];
    float s[NR + 1];
  };
  auto load = [&](Run& t, int g) {
    const int kb = 256 * (ws_ + g);  // byte offset of the run
#pragma unroll
    for (int v = 0; v < NI; ++v) {
#pragma unroll
      for (int m = 0; m < NR; ++m) t.t[m][v] = wl(wrow[m][v] + kb + 16 * lc);
      if (v < XI) {
        const int rr = RPI * v + lr;
        const f4 x = *reinterpret_cast<const f4*>(p.xq + (long long)(rr < nb ? rr : 0) * K + kb + 16 * lc);
        t.t[NR][v] = rr < nb ? x : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int m = 0; m < NR; ++m) t.s[m] = wsrow[m][4 * (ws_ + g) + sg];
    t.s[NR] = sx ? xsrow[4 * (ws_ + g) + sg] : 0.f;
  };
  unsigned* my = lds + wave * (NR + 1) * TILE;
  // activation tile rows 8..15 stay zero
#pragma unroll
  for (int v = XI; v < NI; ++v)
    *reinterpret_cast<f4*>(my + NR * TILE + (RPI * v + lr) * STR + 4 * lc) = f4{0.f, 0.f, 0.f, 0.f};
  float acc[NR][4];
#pragma unroll
  for (int m = 0; m < NR; ++m)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[m][e] = 0.f;
  auto mma = [&](const Run& t) {
#pragma unroll
    for (int m = 0; m <= NR; ++m) {
#pragma unroll
      for (int v = 0; v < NI; ++v)
        if (m < NR || v < XI) *reinterpret_cast<f4*>(my + m * TILE + (RPI * v + lr) * STR + 4 * lc) = t.t[m][v];
      scl[wave][m][sr][sg] = t.s[m];
    }
    asm volatile("" ::: "memory");  // same-wave LDS ops execute in order
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i32x4 x = *reinterpret_cast<const i32x4*>(my + NR * TILE + i * STR + 16 * u + 4 * q);
      const float xs = scl[wave][NR][i][u];
#pragma unroll
      for (int m = 0; m < NR; ++m) {
        const i32x4 a = *reinterpret_cast<const i32x4*>(my + m * TILE + i * STR + 16 * u + 4 * q);
        const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, x, i32x4{0, 0, 0, 0}, 0, 0, 0);
        // output (row 4q + e, sequence i): runq.c:334 val += ((float)ival * w.s) * x.s
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[m][e] = __fadd_rn(acc[m][e], __fmul_rn(__fmul_rn((float)d[e], scl[wave][m][4 * q + e][u]), xs));
      }
    }
    asm volatile("" ::: "memory");
  };

  Run ta, tb;
  if (nrun > 0) load(ta, 0);
  for (int g = 0; g < nrun; g += 2) {
    if (g + 1 < nrun) load(tb, g + 1);
    mma(ta);
    if (g + 1 >= nrun) break;
    if (g + 2 < nrun) load(ta, g + 2);
    mma(tb);
  }

  __syncthreads();  // the staging tiles become the wave-partial buffer
  float* red = reinterpret_cast<float*>(lds);  // [W][NR][256]
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int m = 0; m < NR; ++m) red[(wave * NR + m) * 256 + (4 * q + e) * 16 + i] = acc[m][e];
  __syncthreads();
  auto wsum = [&](int m, int t) {
    float v = red[m * 256 + t];
    for (int w = 1; w < W; ++w) v += red[(w * NR + m) * 256 + t];
    return v;
  };
  const int msplit = p.msplit;
  float* tpart = p.mpart + (long long)tile * msplit * (NR * 256);
  if (msplit > 1) {
    for (int t = threadIdx.x; t < 256; t += W * 64) {
      st1_sc1(tpart + split * (NR * 256) + t, wsum(0, t));
      if constexpr (TWO) st1_sc1(tpart + split * (NR * 256) + 256 + t, wsum(1, t));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(p.mcnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)(msplit - 1);
    __syncthreads();
    if (!s_last) return;
  }
  auto tot = [&](int m, int t) {
    if (msplit == 1) return wsum(m, t);
    const float* b = tpart + m * 256 + t;
    float v = ld1_sc1(b);
    for (int sp = 1; sp < msplit; ++sp) v += ld1_sc1(b + sp * (NR * 256));
    return v;
  };
  for (int t = threadIdx.x; t < 256; t += W * 64) {
    const int row = t >> 4, j = t & 15;
    const int R = tile * 16 + row;
    if (j < nb && R < n_rows) {
      if constexpr (MODE == GM_SWIGLU) {
        epi_one<MODE>(p, R, j, tot(0, t), tot(NR - 1, t));
      } else if constexpr (MODE == GM_QKV) {
        if ((row & 1) == 0) epi_one<MODE>(p, R >> 1, j, tot(0, t), tot(0, t + 16));
      } else {
        epi_one<MODE>(p, R, j, tot(0, t), 0.f);
      }
    }
  }
  if (msplit > 1 && threadIdx.x == 0) __hip_atomic_store(p.mcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace tl
