// gemv_mfma.hpp — the batched (2..16 sequences) decode GEMV on the fp32 matrix cores.
//
// With B sequences the VALU streaming kernel (gemv.hpp) multiplies every weight float4 by B
// activation float4s read back from LDS: at B = 8 that is 8x the weight bytes in LDS
// traffic, and the step runs at ~30% of the HBM roofline.  Here one wave computes a 16-row
// x 16-sequence tile with v_mfma_f32_16x16x4_f32 (lane (i, q) holds row i / sequence i at
// k = 4q..4q+3 of each 16-k step; component c feeds MFMA c, so A and B agree on k).
// Activations come from L2 (every block reads the same B x K floats); the weights stream
// once, non-temporal.
//
// The launcher splits K across blocks until the grid fills every CU four blocks deep (a
// 4096-row matrix -> 256 tiles x 4 splits).  Wave partials are summed in LDS and split
// partials by the last block of the tile, both in a fixed order (deterministic), then the
// same fused epilogues as gemv.hpp (store at pos offsets, residual, SwiGLU over a W1/W3
// pair of tiles, QKV + RoPE + KV write).  An RMSNorm / embedding prologue runs ONCE per
// launch (gemv_prenorm_kernel, x' = w * (ss * x) as in src/seq.cpp:3-16) into scratch
// rows, not once per block.  The fp32 MFMA accumulates exactly-rounded products in fp32,
// within the reference's 1e-4 logits tolerance of its sequential loop.
// RMSNorm across launches: the residual launches (Wo, W2) also leave, per 16-row tile, the sum of
// squares of the rows they updated (a fixed order: rows 0..15 of the tile); the next normed
// launch (QKV, W1/W3, classifier) reduces those partials in a fixed order at its start (every
// block gets the same ss) and applies x' = w * (ss * x) as it loads the activations, so the
// prologue launch runs only where the input is the embedding row (layer 0).
#pragma once
#include "gemv.hpp"

namespace tl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 4 waves per block (the norm and epilogue maps assume 256 threads) and 4 16-k steps per group
// (256-B row runs, four rows per load instruction, which the launcher's XI counts assume; 8 steps =
// 512-B runs needed 226-254 VGPRs, one wave per SIMD, and lost 12% at batch 8:
// profiles/r04/mfma_u8_ab.txt)
constexpr int kMfmaWaves = 4;
constexpr int kMfmaU = 4;

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
template <int kUnused = 0>
__global__ void __launch_bounds__(256) gemv_prenorm_kernel(GemvParams p) {
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

// Block = kMfmaWaves waves on one 16-row tile and one K split (blockIdx = tile * msplit +
// split); wave w takes a contiguous run of the split's 16-k steps.  Per group of U 16-k steps a wave reads its
// 16-row weight tile (and the 16 activation rows) as 256-B contiguous runs per row (16
// lanes x 16 B, four rows per instruction), writes them to a wave-private LDS tile (rows
// padded by 16 B: conflict-free both ways) and reads them back in the MFMA lane layout
// (lane (i, q): row i, k = 16 u + 4 q).  Loading the MFMA layout straight from HBM (64 B
// per row per instruction) ran at 2.5-3.5 TB/s, these runs at 3.5-5.4 TB/s (profiles/
// r01_mfma_sweep.jsonl); LDS traffic is ~1 B per weight byte.  The weights of group g + 1
// are in flight while group g multiplies; steps past the run load a clamped (valid)
// address and multiply zero activations, so no load is predicated.
template <int MODE, bool NT, int XI>
__global__ void __launch_bounds__(kMfmaWaves * 64) gemv_mfma_kernel(GemvParams p) {
  keep_implicit_args();
  constexpr int W = kMfmaWaves;
  constexpr bool TWO = MODE == GM_SWIGLU;
  constexpr int NR = TWO ? 2 : 1;      // weight tiles per group; tile NR is the activations
  constexpr int U = kMfmaU;            // 16-k steps per group
  constexpr int LPR = U * 4;           // lanes per row in a load (16 B each): 256-B runs
  constexpr int RPI = 64 / LPR;        // rows per load instruction
  constexpr int NI = 16 / RPI;         // load instructions per 16-row tile
  static_assert(XI >= 1 && XI <= NI, "live activation load instructions");
  constexpr int STR = U * 16 + 4;      // LDS row stride in floats (padded)
  constexpr int TILE = 16 * STR;       // floats per tile
  static_assert(W * 64 == 256, "the norm and epilogue maps assume 256 threads");
  __shared__ __attribute__((aligned(16))) float lds[W * (NR + 1) * TILE];
  __shared__ unsigned s_last;
  __shared__ float s_red[256];
  __shared__ float s_ss[16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int lr = lane / LPR, lc = lane % LPR;  // load map: row RPI v + lr, 16-B chunk lc
  const int K = p.K, nb = p.nb;
  const long long Kl = K;
  const int tile = blockIdx.x / p.msplit, split = blockIdx.x - tile * p.msplit;
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;

  const float* wrow[NR][NI];
  const float* xrow[NI];
  bool xok[NI];
#pragma unroll
  for (int v = 0; v < NI; ++v) {
    const int r = RPI * v + lr;
    int R = tile * 16 + r;
    R = R < n_rows ? R : n_rows - 1;
    if constexpr (MODE == GM_SWIGLU) {
      wrow[0][v] = p.W0 + R * Kl;
      wrow[NR - 1][v] = p.W1 + R * Kl;
    } else if constexpr (MODE == GM_QKV) {
      wrow[0][v] = item_row<GM_QKV>(p, R >> 1, R & 1);
    } else {
      wrow[0][v] = p.W0 + R * Kl;
    }
    xok[v] = r < nb;
    xrow[v] = p.x + (long long)(r < nb ? r : 0) * p.x_stride;
  }

  // fused RMSNorm (p.rms_w set here only with p.ssq_in, see the launcher): ss_b from the producer's
  // per-tile sums of squares (<= 256 tiles) — thread (b, j) sums tiles j, j + 16, ..., then b sums
  // its 16 in order; run after the first weight loads are in flight (their latency covers it)
  const bool fnorm = p.rms_w != nullptr;
  float xs[NI];
  auto norm_scales = [&] {
    const int t = threadIdx.x, b = t >> 4, j = t & 15;
    float part[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) part[k] = b < nb && j + 16 * k < p.ssq_nt ? p.ssq_in[(long long)b * p.ssq_nt + j + 16 * k] : 0.f;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) a = __fadd_rn(a, part[k]);
    s_red[t] = a;
    __syncthreads();
    if (t < nb) {
      float v = 0.f;
      for (int k = 0; k < 16; ++k) v = __fadd_rn(v, s_red[t * 16 + k]);
      s_ss[t] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(v, (float)K), 1e-5f)));  // src/seq.cpp:3-16
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NI; ++v) {
      const int r = RPI * v + lr;
      xs[v] = r < nb ? s_ss[r] : 0.f;
    }
  };
  const int nsteps = K >> 4;
  const int s0 = split * p.msteps;
  const int s1 = s0 + p.msteps < nsteps ? s0 + p.msteps : nsteps;
  const int per = (s1 - s0 + W * U - 1) / (W * U) * U;
  const int ws = s0 + wave * per;
  const int we = ws + per < s1 ? ws + per : s1;
  const int ng = we > ws ? (we - ws + U - 1) / U : 0;
  // this lane's float offset in group g (clamped to a valid address past the run)
  auto kof = [&](int g, bool& ok) {
    const int st = ws + g * U + (lc >> 2);
    ok = st < we;
    return ok ? 16 * (ws + g * U) + 4 * lc : 16 * (nsteps - 1) + 4 * (lc & 3);
  };
  auto wl = [&](const float* w) {
    const f4* a = reinterpret_cast<const f4*>(w);
    if constexpr (NT) return __builtin_nontemporal_load(a);
    else return *a;
  };
  // activation rows >= nb are zero: only the first XI of the NI activation load instructions
  // are issued (XI * RPI >= nb, a compile-time count: a run-time skip made the compiler's
  // vmcnt waits conservative), the other tile rows stay zero from the start
  auto xlive = [&](int v) { return v < XI; };
  auto load = [&](f4 (&t)[NR + 1][NI], f4& rw, int g) {
    bool ok;
    const int k = kof(g, ok);
    if (fnorm) rw = *reinterpret_cast<const f4*>(p.rms_w + k);
#pragma unroll
    for (int v = 0; v < NI; ++v) {
#pragma unroll
      for (int m = 0; m < NR; ++m) t[m][v] = wl(wrow[m][v] + k);
      if (xlive(v)) {
        const f4 x = *reinterpret_cast<const f4*>(xrow[v] + k);
        t[NR][v] = (ok && xok[v]) ? x : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  float* my = lds + wave * (NR + 1) * TILE;
#pragma unroll
  for (int v = 0; v < NI; ++v)
    if (!xlive(v)) *reinterpret_cast<f4*>(my + NR * TILE + (RPI * v + lr) * STR + 4 * lc) = f4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc[NR];
#pragma unroll
  for (int m = 0; m < NR; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const f4 (&t)[NR + 1][NI], const f4& rw) {
#pragma unroll
    for (int m = 0; m <= NR; ++m)
#pragma unroll
      for (int v = 0; v < NI; ++v)
        if (m < NR || xlive(v)) {
          f4 e = t[m][v];
          if (m == NR && fnorm) {  // x' = w * (ss * x), as gemv_prenorm_kernel (zeros stay zero)
            const float sv = xs[v];
            e = f4{__fmul_rn(rw.x, __fmul_rn(sv, e.x)), __fmul_rn(rw.y, __fmul_rn(sv, e.y)),
                   __fmul_rn(rw.z, __fmul_rn(sv, e.z)), __fmul_rn(rw.w, __fmul_rn(sv, e.w))};
          }
          *reinterpret_cast<f4*>(my + m * TILE + (RPI * v + lr) * STR + 4 * lc) = e;
        }
    asm volatile("" ::: "memory");  // same-wave LDS ops execute in order
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 x = *reinterpret_cast<const f4*>(my + NR * TILE + i * STR + 16 * u + 4 * q);
#pragma unroll
      for (int m = 0; m < NR; ++m) {
        const f4 a = *reinterpret_cast<const f4*>(my + m * TILE + i * STR + 16 * u + 4 * q);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, x.x, acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, x.y, acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, x.z, acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, x.w, acc[m], 0, 0, 0);
      }
    }
    asm volatile("" ::: "memory");
  };

  f4 ta[NR + 1][NI], tb[NR + 1][NI];
  f4 rwa = f4{0.f, 0.f, 0.f, 0.f}, rwb = rwa;
  if (ng > 0) load(ta, rwa, 0);
  if (fnorm) norm_scales();  // (block barriers: every wave, live or not)
  for (int g = 0; g < ng; g += 2) {
    if (g + 1 < ng) load(tb, rwb, g + 1);
    mma(ta, rwa);
    if (g + 1 >= ng) break;
    if (g + 2 < ng) load(ta, rwa, g + 2);
    mma(tb, rwb);
  }

  __syncthreads();  // the staging tiles become the wave-partial buffer
  float* red = lds;  // [W][NR][256]
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
      } else if constexpr (MODE == GM_RESID) {
        float* y = p.y + (long long)j * p.y_stride + R;
        const float nv = __fadd_rn(*y, tot(0, t));
        *y = nv;
        if (p.ssq_out) s_red[t] = __fmul_rn(nv, nv);
      } else {
        epi_one<MODE>(p, R, j, tot(0, t), 0.f);
      }
    }
  }
  if constexpr (MODE == GM_RESID) {
    if (p.ssq_out) {  // this tile's sum of squares per sequence, rows in order (rows past the end: 0)
      const int row = threadIdx.x >> 4, j = threadIdx.x & 15;
      if (!(j < nb && tile * 16 + row < n_rows)) s_red[threadIdx.x] = 0.f;
      __syncthreads();
      if (threadIdx.x < nb) {
        float v = 0.f;
        for (int r = 0; r < 16; ++r) v = __fadd_rn(v, s_red[r * 16 + threadIdx.x]);
        p.ssq_out[(long long)threadIdx.x * p.ssq_nt + tile] = v;
      }
    }
  }
  if (msplit > 1 && threadIdx.x == 0) __hip_atomic_store(p.mcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace tl
