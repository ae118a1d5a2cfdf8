// q8_exact.hip — the multi-launch int8 (Q8_0, group size 64) decode step for 1..8 sequences in
// runq's own arithmetic order, so every sequence's logits are bit-identical to runq.c's forward
// (runq.c:344-481; the oracle's oracle_q8_forward).  The batch-1 persistent step (persist.hip)
// reaches the same bits with its own machinery; these are the launches the batched decoders use.
//
// runq re-quantises the activations before every matmul, so a last-bit fp32 difference anywhere
// upstream moves an int8 code and the decode leaves runq's within a few steps
// (tools/probes/q8drift.c).  Every fp32 operation whose result reaches a quantiser is done in
// runq's order with runq's roundings (the library is built with -ffp-contract=off):
//  * RMSNorm: the sum of squares is runq's sequential chain (runq.c:284-287), taken by one wave
//    with seqsum.hpp; then w * (ss * x) (runq.c:289-294) and the quantisation (runq.c:145-171),
//    once per launch and sequence (q8x_prequant_kernel);
//  * GEMV (runq.c:317-342): per group of 64 the int32 dot — one v_mfma_i32_16x16x64_i8 gives a
//    16-row x 16-sequence tile of them, exactly — then ((float)ival * w.s) * x.s kept per group
//    in LDS, and per (row, sequence) runq's left-to-right chain over the groups.  No K split
//    across blocks (a tile's chains need all its products): one 16-row tile per block, its K
//    runs dealt over the block's waves;
//  * attention (runq.c:396-434): one lane per key for the sequential q.k dot, / sqrtf(hs); the
//    softmax with glibc's expf restated (libm_exact.hpp) and the sequential sum (seqsum.hpp);
//    one lane per output column for the chain over the keys (attn_q8x_scores_kernel,
//    attn_q8x_out_kernel);
//  * SwiGLU (runq.c:458-467) in the W1/W3 epilogue with the exact expf (gemv.hpp silu_mul);
//    RoPE from the host-libm table; residual adds are single roundings.
#include <hip/hip_runtime.h>
#include <mutex>
#include <utility>
#include <vector>
#include "attention.hpp"
#include "gemv_q8.hpp"
#include "gemv_q8_mfma.hpp"
#include "q8_dispatch.hpp"

namespace tl {

// ---------------------------------------------------------------- activation quantisation
// One block per sequence: x (or the token's embedding row, also copied to x_out) -> RMSNorm
// with runq's sum of squares -> runq's quantisation into p.xq / p.xqs.  Dynamic LDS: the
// seqsum layout of K squares (when p.rms_w).
__global__ void __launch_bounds__(256) q8x_prequant_kernel(GemvParams p) {
  keep_implicit_args();
  constexpr int MR = 3;  // 16-value slices per thread (K <= 3 * 256 * 16 = 12288)
  extern __shared__ __attribute__((aligned(16))) float q8x_sq[];
  __shared__ float s_sum;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int K = p.K, n16 = K >> 4, ng = K >> 6;
  const float* src = p.tok ? p.emb + (long long)p.tok[b] * K : p.x + b * p.x_stride;
  // every value loaded once, up front, and kept in registers through the norm
  f4 v[MR][4];
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    const int sl = r * 256 + t;
#pragma unroll
    for (int u = 0; u < 4; ++u) v[r][u] = sl < n16 ? reinterpret_cast<const f4*>(src + sl * 16)[u] : f4{0.f, 0.f, 0.f, 0.f};
  }
  if (p.tok)
#pragma unroll
    for (int r = 0; r < MR; ++r)
      if (r * 256 + t < n16)
#pragma unroll
        for (int u = 0; u < 4; ++u) reinterpret_cast<f4*>(p.x_out + b * p.x_stride + (r * 256 + t) * 16)[u] = v[r][u];
  float s = 1.f;
  if (p.rms_w) {
    const int ch = seqsum_ch(K);
    for (int i = t; i < seqsum_floats(K); i += 256) q8x_sq[i] = 0.f;  // the padding adds +0
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      const int sl = r * 256 + t;
      if (sl < n16)
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // runq.c:286: x[j] * x[j], one rounding each
          float* d = q8x_sq + seqsum_index(sl * 16 + 4 * u, ch);  // ch % 4 == 0: one chunk
          d[0] = __fmul_rn(v[r][u].x, v[r][u].x); d[1] = __fmul_rn(v[r][u].y, v[r][u].y);
          d[2] = __fmul_rn(v[r][u].z, v[r][u].z); d[3] = __fmul_rn(v[r][u].w, v[r][u].w);
        }
    }
    __syncthreads();
    if (t < 64) {
      const float sum = K <= 4096 ? wave_seqsum_reg(q8x_sq, K, lane) : wave_seqsum(q8x_sq, K, lane);
      if (lane == 0) s_sum = sum;
    }
    __syncthreads();
    s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(s_sum, (float)K), 1e-5f)));  // runq.c:287-289
  }
  // 4 threads per group of 64, 16 values each (gemv_q8_prequant_reg_kernel's arithmetic)
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
    m = fmaxf(m, dpp_f<0x4E>(m));
    const float scale = __fdiv_rn(m, 127.0f);
    if (live) {
      *reinterpret_cast<q8i4*>(p.xq + (long long)b * K + sl * 16) = q8_pack16(w, scale);
      if ((sl & 3) == 0) p.xqs[(long long)b * ng + (sl >> 2)] = scale;
    }
  }
}

// ---------------------------------------------------------------- GEMV
// Dynamic LDS of one block: staging tiles (W waves x (NR + 1) tiles of 16 rows x 272 B), the
// runs' group scales, and the per-group products [NR][16 rows][8 sequences][ng + 4].
constexpr int kQxStr = 64 + 4, kQxTile = 16 * kQxStr;
inline size_t q8x_gemv_lds(int nr, int K, int W) {
  const int ngp = (K >> 6) + 4;
  return (size_t)W * (nr + 1) * kQxTile * 4 + (size_t)W * (nr + 1) * 16 * 4 * 4 + (size_t)nr * 128 * ngp * 4;
}

template <int MODE, bool NT, int W>
__global__ void __launch_bounds__(W * 64) gemv_q8_exact_kernel(GemvParams p) {
  keep_implicit_args();
  constexpr bool TWO = MODE == GM_SWIGLU;
  constexpr int NR = TWO ? 2 : 1;  // weight tiles per run; tile NR is the activation codes
  constexpr int U = 4;             // groups (64 B) per 256-B run
  constexpr int LPR = 16, RPI = 64 / LPR, NI = 16 / RPI, XI = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned q8x_lds[];
  unsigned* lds = q8x_lds;
  float* scl = reinterpret_cast<float*>(lds + W * (NR + 1) * kQxTile);  // [W][NR + 1][16][U]
  float* prod = scl + W * (NR + 1) * 16 * U;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int lr = lane / LPR, lc = lane % LPR;
  const int K = p.K, nb = p.nb, ng = K >> 6, ngp = ng + 4;
  const int tile = blockIdx.x;
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;

  const int8_t* wrow[NR][NI];
  const float* srow[NR][NI];
#pragma unroll
  for (int v = 0; v < NI; ++v) {
    int R = tile * 16 + RPI * v + lr;
    R = R < n_rows ? R : n_rows - 1;
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      if constexpr (MODE == GM_QKV) q8_item_row<GM_QKV>(p, R >> 1, R & 1, wrow[m][v], srow[m][v]);
      else q8_item_row<MODE>(p, R, m, wrow[m][v], srow[m][v]);
    }
  }
  const int sr = lane >> 2, sg = lane & 3;  // scale loads: row (or sequence) sr, group sg of the run
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
  const int per = (nruns + W - 1) / W;
  const int ws_ = wave * per < nruns ? wave * per : nruns;
  const int we = ws_ + per < nruns ? ws_ + per : nruns;
  const int nrun = we - ws_;

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
    const int kb = 256 * (ws_ + g);
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
  unsigned* my = lds + wave * (NR + 1) * kQxTile;
  float* mys = scl + wave * (NR + 1) * 16 * U;
#pragma unroll
  for (int v = XI; v < NI; ++v)
    *reinterpret_cast<f4*>(my + NR * kQxTile + (RPI * v + lr) * kQxStr + 4 * lc) = f4{0.f, 0.f, 0.f, 0.f};
  // products of run g: lane (i, q) holds (row 4q + e, sequence i) of each group u of the run
  auto mma = [&](const Run& t, int g) {
#pragma unroll
    for (int m = 0; m <= NR; ++m) {
#pragma unroll
      for (int v = 0; v < NI; ++v)
        if (m < NR || v < XI) *reinterpret_cast<f4*>(my + m * kQxTile + (RPI * v + lr) * kQxStr + 4 * lc) = t.t[m][v];
      mys[(m * 16 + sr) * U + sg] = t.s[m];
    }
    asm volatile("" ::: "memory");  // same-wave LDS ops execute in order
    const int g0 = 4 * (ws_ + g);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const i32x4 x = *reinterpret_cast<const i32x4*>(my + NR * kQxTile + i * kQxStr + 16 * u + 4 * q);
      const float xs = mys[(NR * 16 + i) * U + u];
#pragma unroll
      for (int m = 0; m < NR; ++m) {
        const i32x4 a = *reinterpret_cast<const i32x4*>(my + m * kQxTile + i * kQxStr + 16 * u + 4 * q);
        const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, x, i32x4{0, 0, 0, 0}, 0, 0, 0);
        if (i < nb) {
#pragma unroll
          for (int e = 0; e < 4; ++e)  // runq.c:336: ((float)ival * w.s) * x.s
            prod[((m * 16 + 4 * q + e) * 8 + i) * ngp + g0 + u] =
                __fmul_rn(__fmul_rn((float)d[e], mys[(m * 16 + 4 * q + e) * U + u]), xs);
        }
      }
    }
    asm volatile("" ::: "memory");
  };

  // three runs in flight per wave (one block per CU: the LDS holds every product of the tile)
  Run ta, tb, tc;
  if (nrun > 0) load(ta, 0);
  if (nrun > 1) load(tb, 1);
  for (int g = 0; g < nrun; g += 3) {
    if (g + 2 < nrun) load(tc, g + 2);
    mma(ta, g);
    if (g + 1 >= nrun) break;
    if (g + 3 < nrun) load(ta, g + 3);
    mma(tb, g + 1);
    if (g + 2 >= nrun) break;
    if (g + 4 < nrun) load(tb, g + 4);
    mma(tc, g + 2);
  }
  __syncthreads();  // every product is in LDS; the staging tiles become the row-value buffer
  // runq.c:330-338: each (row, sequence) value is the left-to-right chain over its groups
  float* red = reinterpret_cast<float*>(lds);  // [NR][16 rows][16]
  for (int t = threadIdx.x; t < NR * 128; t += W * 64) {
    const int m = t >> 7, row = (t >> 3) & 15, j = t & 7;
    float v = 0.f;
    if (j < nb) v = chain_f4<8>(reinterpret_cast<const f4*>(prod + ((m * 16 + row) * 8 + j) * ngp), ng >> 2, 0.f);
    red[m * 256 + row * 16 + j] = v;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += W * 64) {
    const int row = t >> 4, j = t & 15;
    const int R = tile * 16 + row;
    if (j < nb && R < n_rows) {
      if constexpr (MODE == GM_SWIGLU) {
        epi_one<MODE>(p, R, j, red[t], red[256 + t]);
      } else if constexpr (MODE == GM_QKV) {
        if ((row & 1) == 0) epi_one<MODE>(p, R >> 1, j, red[t], red[t + 16]);
      } else {
        epi_one<MODE>(p, R, j, red[t], 0.f);
      }
    }
  }
}

template <int MODE, bool NT, int W>
static hipError_t launch_q8x_w(const GemvParams& p, hipStream_t s, size_t lds) {
  const int rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
  hipLaunchKernelGGL((gemv_q8_exact_kernel<MODE, NT, W>), dim3((rows + 15) / 16), dim3(W * 64), lds, s, p);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_q8x_mode(const GemvParams& p0, hipStream_t s, bool nt) {
  if (p0.n_items <= 0 || p0.nb <= 0) return hipSuccess;
  if (p0.nb > 8 || !p0.xq || !p0.xqs) return hipErrorInvalidValue;
  GemvParams p = p0;
  if (!p.xq_ready) {
    const size_t lds = p.rms_w ? (size_t)64 * (4 * ((p.K + 255) >> 8) + 4) * 4 : 0;  // seqsum_floats(K)
    hipLaunchKernelGGL(q8x_prequant_kernel, dim3(p.nb), dim3(256), lds, s, p);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  p.rms_w = nullptr;
  p.tok = nullptr;
  p.x_out = nullptr;
  constexpr int NR = MODE == GM_SWIGLU ? 2 : 1;
  const size_t cap = 160 * 1024 - 256;
  for (int W : {8, 6, 4}) {
    const size_t lds = q8x_gemv_lds(NR, p.K, W);
    if (lds > cap) continue;
    if (W == 8) return nt ? launch_q8x_w<MODE, true, 8>(p, s, lds) : launch_q8x_w<MODE, false, 8>(p, s, lds);
    if (W == 6) return nt ? launch_q8x_w<MODE, true, 6>(p, s, lds) : launch_q8x_w<MODE, false, 6>(p, s, lds);
    return nt ? launch_q8x_w<MODE, true, 4>(p, s, lds) : launch_q8x_w<MODE, false, 4>(p, s, lds);
  }
  return hipErrorInvalidValue;  // (K too large for one block's products)
}

bool q8_exact_ok(int gs, int dim, int hidden, int hs, int seq_len) {
  return gs == 64 && dim % 256 == 0 && hidden % 256 == 0 && (hs == 64 || hs == 128) && hidden <= 12288 &&
         q8x_gemv_lds(1, hidden, 4) <= 160 * 1024 - 256 && seq_len <= 8192;
}

hipError_t launch_gemv_q8_exact(int mode, const GemvParams& p, hipStream_t s, bool nt) {
  if (p.gs != 64 || (p.K & 255)) return hipErrorInvalidValue;
  switch (mode) {
    case GM_STORE: return launch_q8x_mode<GM_STORE>(p, s, nt);
    case GM_RESID: return launch_q8x_mode<GM_RESID>(p, s, nt);
    case GM_SWIGLU: return launch_q8x_mode<GM_SWIGLU>(p, s, nt);
    case GM_QKV: return launch_q8x_mode<GM_QKV>(p, s, nt);
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------- attention
// Scores: block (b * H + h, y) scores keys t0 + lane, t0 = 64 (y + k gridDim.y), one lane per
// key: the key rows reach LDS by LDS-DMA transposed (piece i of key l at win[i * 256 + 4 l],
// conflict-free reads), then runq's sequential dot with q and / sqrtf(hs).  att: [B][H][S].
template <int HS>
__global__ void __launch_bounds__(64) attn_q8x_scores_kernel(AttnParams p, float* att) {
  keep_implicit_args();
  constexpr int PC = HS / 4;
  __shared__ __attribute__((aligned(16))) float qs[HS];
  __shared__ __attribute__((aligned(16))) float win[PC * 256];
  const int lane = threadIdx.x;
  const int b = blockIdx.x / p.n_heads, h = blockIdx.x % p.n_heads;
  const int T = p.pos[b] + 1;
  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  for (int c = lane; c < HS; c += 64) qs[c] = p.q[(long long)b * p.dim + h * HS + c];
  float* out = att + ((long long)b * p.n_heads + h) * p.seq_len;
  const float rs = sqrtf((float)HS);
  const f4* q4 = reinterpret_cast<const f4*>(qs);
  for (int t0 = 64 * blockIdx.y; t0 < T; t0 += 64 * gridDim.y) {
    wave_lds_fence();  // the previous window's reads are done
    if (t0 + lane < T) {
      const float* row = kbase + (long long)(t0 + lane) * p.kv_dim;
#pragma unroll
      for (int c = 0; c < PC; ++c) dma16(row + 4 * c, win + c * 256);
    }
    dma_wait_all();
    float sc = 0.f;
    constexpr int RA = 8;
    for (int c0 = 0; c0 < PC; c0 += RA) {
      f4 k4[RA], qv[RA];
#pragma unroll
      for (int c = 0; c < RA; ++c) {
        k4[c] = reinterpret_cast<const f4*>(win + 4 * lane)[(c0 + c) * 64];
        qv[c] = q4[c0 + c];
      }
#pragma unroll
      for (int c = 0; c < RA; ++c) {  // runq.c:410-413: score += q[i] * k[i]
        sc = __fadd_rn(sc, __fmul_rn(qv[c].x, k4[c].x));
        sc = __fadd_rn(sc, __fmul_rn(qv[c].y, k4[c].y));
        sc = __fadd_rn(sc, __fmul_rn(qv[c].z, k4[c].z));
        sc = __fadd_rn(sc, __fmul_rn(qv[c].w, k4[c].w));
      }
    }
    if (t0 + lane < T) out[t0 + lane] = __fdiv_rn(sc, rs);
  }
}

// Softmax + output columns: block (b * H + h, c) repeats the head's softmax (max, glibc expf,
// runq's sequential sum — identical in every block of the head) and chains its CW = HS / NG
// columns over the T keys (lane < CW owns one); V rows reach LDS by LDS-DMA in rounds.
// Dynamic LDS: the expf table, at [S], the seqsum layout of S values, the V window.
template <int HS, int NG>
__global__ void __launch_bounds__(64) attn_q8x_out_kernel(AttnParams p, const float* att, int rv) {
  keep_implicit_args();
  constexpr int CW = HS / NG, PPR = CW / 4, RPI = 64 / PPR;
  extern __shared__ __attribute__((aligned(16))) float q8xo[];
  uint64_t* etab = reinterpret_cast<uint64_t*>(q8xo);
  float* at = q8xo + 64;
  float* sa = at + ((p.seq_len + 3) & ~3);
  float* vw = sa + seqsum_floats(p.seq_len);
  const int lane = threadIdx.x;
  const int b = blockIdx.x / p.n_heads, h = blockIdx.x % p.n_heads, c = blockIdx.y;
  const int T = p.pos[b] + 1;
  {
    constexpr uint64_t tab[32] = TL_EXPF_TABLE;
    if (lane < 32) etab[lane] = tab[lane];
  }
  const int ch = seqsum_ch(T);
  for (int k = lane; k < seqsum_floats(T); k += 64) sa[k] = 0.f;
  const float* sc = att + ((long long)b * p.n_heads + h) * p.seq_len;
  float mx = -__builtin_inff();
  for (int t = lane; t < T; t += 64) {
    const float v = sc[t];
    at[t] = v;
    mx = fmaxf(mx, v);
  }
  mx = wave_max_u(mx);  // runq.c:300-304 (a maximum: exact in any order)
  wave_lds_fence();
  const unsigned chm = seqsum_magic(ch);
  for (int t = lane; t < T; t += 64) sa[seqsum_index_m(t, ch, chm)] = expf_libm_tab(__fsub_rn(at[t], mx), etab);
  wave_lds_fence();
  const float sum = T <= 512 ? wave_seqsum_short(sa, T) : T <= 4096 ? wave_seqsum_reg(sa, T, lane) : wave_seqsum(sa, T, lane);
  for (int t = lane; t < T; t += 64) at[t] = __fdiv_rn(sa[seqsum_index_m(t, ch, chm)], sum);  // runq.c:310
  wave_lds_fence();
  const int kvh = h / p.kv_mul;
  const int col0 = c * CW;
  const float* vbase = p.vc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS + col0;
  float o = 0.f;
  const int cl = lane < CW ? lane : 0;
  for (int r0 = 0; r0 < T; r0 += rv) {
    const int n = min(rv, T - r0);
    wave_lds_fence();  // the previous round's reads are done
    for (int k = 0; k * RPI < n; ++k) {
      const int rr = k * RPI + lane / PPR;
      if (rr < n) dma16(vbase + (long long)(r0 + rr) * p.kv_dim + (lane % PPR) * 4, vw + k * 256);
    }
    dma_wait_all();
    const int n16 = n & ~15;
    for (int u = 0; u < n16; u += 16) {  // runq.c:424-431: xb[i] += a * v[i], key by key
      f4 a4[4];
      float v16[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) a4[k] = *reinterpret_cast<const f4*>(at + r0 + u + 4 * k);
#pragma unroll
      for (int k = 0; k < 16; ++k) v16[k] = vw[(u + k) * CW + cl];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o = __fadd_rn(o, __fmul_rn(a4[k].x, v16[4 * k]));
        o = __fadd_rn(o, __fmul_rn(a4[k].y, v16[4 * k + 1]));
        o = __fadd_rn(o, __fmul_rn(a4[k].z, v16[4 * k + 2]));
        o = __fadd_rn(o, __fmul_rn(a4[k].w, v16[4 * k + 3]));
      }
    }
    for (int u = n16; u < n; ++u) o = __fadd_rn(o, __fmul_rn(at[r0 + u], vw[u * CW + cl]));
  }
  if (lane < CW) p.out[(long long)b * p.dim + h * HS + col0 + lane] = o;
}

template <int HS>
static hipError_t launch_attn_q8x_hs(const AttnParams& a, int B, float* att, hipStream_t s) {
  constexpr int NG = 8, CW = HS / NG;
  const int ky = (a.seq_len + 63) / 64 < 16 ? (a.seq_len + 63) / 64 : 16;
  hipLaunchKernelGGL((attn_q8x_scores_kernel<HS>), dim3(B * a.n_heads, ky), dim3(64), 0, s, a, att);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int rv = 256;  // V rows per round (a multiple of 16 and of the rows per DMA instruction)
  const size_t lds = (size_t)(64 + ((a.seq_len + 3) & ~3) + 64 * (4 * ((a.seq_len + 255) >> 8) + 4) + rv * CW) * 4;
  hipLaunchKernelGGL((attn_q8x_out_kernel<HS, NG>), dim3(B * a.n_heads, NG), dim3(64), lds, s, a, att, rv);
  return hipGetLastError();
}

// Raise every kernel's dynamic-LDS limit to 160 KiB on the current device, once per device (the
// attribute is per device): called when an exact int8 decoder is created, so no launch — and no
// graph capture — ever sets an attribute.
template <int MODE>
static hipError_t q8x_attr_mode() {
  const void* fns[] = {(const void*)gemv_q8_exact_kernel<MODE, true, 8>, (const void*)gemv_q8_exact_kernel<MODE, true, 6>,
                       (const void*)gemv_q8_exact_kernel<MODE, true, 4>, (const void*)gemv_q8_exact_kernel<MODE, false, 8>,
                       (const void*)gemv_q8_exact_kernel<MODE, false, 6>, (const void*)gemv_q8_exact_kernel<MODE, false, 4>};
  for (const void* f : fns) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t q8_exact_prepare() {
  static std::mutex mu;
  static std::vector<int> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  for (int d : done)
    if (d == dev) return hipSuccess;
  if ((e = q8x_attr_mode<GM_STORE>()) != hipSuccess || (e = q8x_attr_mode<GM_RESID>()) != hipSuccess ||
      (e = q8x_attr_mode<GM_SWIGLU>()) != hipSuccess || (e = q8x_attr_mode<GM_QKV>()) != hipSuccess)
    return e;
  for (const void* f : {(const void*)attn_q8x_out_kernel<128, 8>, (const void*)attn_q8x_out_kernel<64, 8>})
    if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)) != hipSuccess) return e;
  done.push_back(dev);
  return hipSuccess;
}

hipError_t launch_attn_q8_exact(const AttnParams& a, int B, float* att, hipStream_t s) {
  if (a.head_size == 128) return launch_attn_q8x_hs<128>(a, B, att, s);
  if (a.head_size == 64) return launch_attn_q8x_hs<64>(a, B, att, s);
  return hipErrorInvalidValue;
}

}  // namespace tl
