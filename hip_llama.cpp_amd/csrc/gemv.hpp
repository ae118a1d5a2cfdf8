// gemv.hpp — the decode weight x activation stream, written for gfx950.
//
// Computes, for NB sequences at once, y[b][r] = sum_k W[r][k] * x'[b][k] where
// W is the reference's row-major [M][K] fp32 weight (reference
// src/thaBLAS.cpp:191-208, CPU twin src/seq.cpp:40-51) and x' is either the
// raw activation or its RMSNorm (reference src/seq.cpp:3-16) fused as a
// prologue.  The epilogue is fused per use site (plain/offset store, residual
// add, SwiGLU, QKV + RoPE + KV-cache write).
//
// Design (why it looks like this on MI355X):
//  * HBM-bound: every weight byte is read exactly once per step for ALL NB
//    sequences (the reference re-reads each row once per sequence).
//  * One wavefront owns a row at a time; lane l reads float4 j*64+l of the
//    row, so one wave-instruction moves 1 KiB of contiguous weights
//    (global_load_dwordx4, fully coalesced); 16 loads per lane are issued
//    before the first FMA so 16 KiB per wave is in flight.
//  * The activation chunk is staged ONCE per block in LDS (normalised there
//    when RMSNorm is fused) and read back with ds_read_b128 — conflict-free
//    because consecutive lanes read consecutive 16-B slots.
//  * The K reduction is a 64-lane xor butterfly (no LDS, no barrier).
//  * Rows are dealt to blocks contiguously and to the 4 waves of a block
//    interleaved; there is no inter-block communication at all.
#pragma once
#include <stdlib.h>
#include "common.hpp"
#include "libm_exact.hpp"

namespace tl {

enum GemvMode : int {
  GM_STORE = 0,   // y[y_off + has_pos*pos[b] + b*y_stride + r] = v        (thaBLAS_s_matmul_batch)
  GM_RESID = 1,   // y[b*y_stride + r] += v                                  (Wo / W2 + residual)
  GM_SWIGLU = 2,  // y[b*y_stride + r] = silu(W1 x) * (W3 x)                (FFN up + SwiGLU)
  GM_QKV = 3,     // q / key_cache / value_cache with RoPE on q,k           (QKV + RoPE + KV write)
};

struct GemvParams {
  const float* W0;  // STORE/RESID: W; SWIGLU: W1; QKV: Wq
  const float* W1;  // SWIGLU: W3;     QKV: Wk
  const float* W2;  //                 QKV: Wv
  int K;            // reduction length (row length), multiple of 256
  int n_items;      // rows (STORE/RESID), hidden rows (SWIGLU), row PAIRS (QKV)
  int nb;           // live sequences (<= NB template)
  // input
  const float* x;        // [nb][x_stride]
  long long x_stride;
  const float* rms_w;    // non-null: input is rms_w[k] * (ss_b * x[b][k])
  const int* tok;        // non-null: input row b is emb[tok[b]] (embedding lookup fused)
  const float* emb;      //   embedding table [V][K]
  float* x_out;          //   and that row is also written to x_out[b*x_stride] (residual stream)
  // output
  float* y;
  long long y_stride;
  long long y_off;
  int has_pos;
  const int* pos;        // device [nb]
  // QKV only
  float* kc;             // key_cache base   [B][L][S][kv_dim]
  float* vc;             // value_cache base
  long long kv_b_stride; // L*S*kv_dim
  long long kv_l_off;    // l*S*kv_dim
  int dim, kv_dim, head_size;
  const float2* rope;    // [S][head_size/2] (cos, sin), computed on the host with libm
  // Q8_0 weights (gemv_q8.hpp): int8 rows + one fp32 scale per group of gs (runq.c:34-37)
  const int8_t* Q0; const int8_t* Q1; const int8_t* Q2;
  const float* S0; const float* S1; const float* S2;
  int gs;
  // optional scratch [nb][K] for the matrix-core path (gemv_mfma.hpp): when set, the
  // RMSNorm / embedding prologue runs once per launch into it instead of once per block
  float* xn;
  // optional int8 scratch (gemv_q8.hpp, batched): [<=8][K] codes + [<=8][K/gs] scales; when
  // set, the activations are quantised once per launch (gemv_q8_prequant_kernel) instead of
  // once per block
  signed char* xq;
  float* xqs;
  int xq_ready;  // xq/xqs already hold this launch's quantised activations (attention wrote them)
  // optional split-K scratch for the matrix-core path: per-block partial tiles
  // [tiles][splits][2][256] and one ticket per tile (zero between launches)
  float* mpart;
  unsigned* mcnt;
  int msplit, msteps;    // set by the launcher: K splits per tile, 16-k steps per split
  // matrix-core path, RMSNorm carried across launches (gemv_mfma.hpp): a RESID launch (Wo / W2)
  // leaves per-tile partial sums of squares of the rows it updated in ssq_out[b * ssq_nt + tile];
  // the next normed launch (ssq_in) reduces them in a fixed order and applies the norm as it
  // loads its activations, instead of a gemv_prenorm_kernel launch
  float* ssq_out;
  const float* ssq_in;
  int ssq_nt;            // tiles of the producing launch (its rows / 16)
};

// Blocks the matrix-core GEMV aims for: 4 per CU (6 and 8 lost 12-15% everywhere, 2 wins only for
// the residual launch with K <= 4096, mfma_splits' depth2).
inline int mfma_target_blocks() {
  static const int v = [] {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return ncu * 4;
  }();
  return v;
}

TL_DEVICE float silu_mul_tab(float a, float b, const uint64_t* etab) {
  // reference src/seq.cpp:159-166 / runq.c:455-462: val *= 1/(1+expf(-val)); val *= hb2, with
  // the host libm's expf bit for bit (libm_exact.hpp; etab: its table, e.g. an LDS copy)
  float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf_libm_tab(-a, etab)));
  return __fmul_rn(__fmul_rn(a, s), b);
}
TL_DEVICE float silu_mul(float a, float b) {
  constexpr uint64_t T[32] = TL_EXPF_TABLE;
  return silu_mul_tab(a, b, T);
}

// Stage x'[b][kc .. kc+kcn) into LDS as NB rows of kcn floats.  When the whole
// row fits (single chunk) and RMSNorm is fused, ss is computed from the staged
// copy (no second global read).  `ss` must already hold the per-b scales when
// several chunks are used.
template <int NB>
TL_DEVICE void stage_x(const GemvParams& p, f4* xs, int kc, int kcn, bool single, float* ss,
                       float* red) {
  const int n4 = kcn >> 2;
  const int tid = threadIdx.x, nt = blockDim.x;
  float sq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) sq[b] = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const bool live = b < p.nb;
    const f4* src = nullptr;
    if (live) {
      if (p.tok) src = reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.K + kc);
      else src = reinterpret_cast<const f4*>(p.x + b * p.x_stride + kc);
    }
    for (int j = tid; j < n4; j += nt) {
      f4 v = live ? src[j] : f4{0.f, 0.f, 0.f, 0.f};
      if (p.tok && live && blockIdx.x == 0)
        reinterpret_cast<f4*>(p.x_out + b * p.x_stride + kc)[j] = v;
      if (p.rms_w) {
        if (single) {
          sq[b] = fmaf(v.x, v.x, sq[b]); sq[b] = fmaf(v.y, v.y, sq[b]);
          sq[b] = fmaf(v.z, v.z, sq[b]); sq[b] = fmaf(v.w, v.w, sq[b]);
        } else {
          const f4 w = reinterpret_cast<const f4*>(p.rms_w + kc)[j];
          const float s = ss[b];
          v = f4{__fmul_rn(w.x, __fmul_rn(s, v.x)), __fmul_rn(w.y, __fmul_rn(s, v.y)),
                 __fmul_rn(w.z, __fmul_rn(s, v.z)), __fmul_rn(w.w, __fmul_rn(s, v.w))};
        }
      }
      xs[b * n4 + j] = v;
    }
  }
  if (p.rms_w && single) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      // reference rmsnorm: ss = 1/sqrtf(sum/size + 1e-5f)
      float t = block_sum(sq[b], red);
      ss[b] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)p.K), 1e-5f)));
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float s = ss[b];
      for (int j = tid; j < n4; j += nt) {
        const f4 w = reinterpret_cast<const f4*>(p.rms_w + kc)[j];
        f4 v = xs[b * n4 + j];
        xs[b * n4 + j] = f4{__fmul_rn(w.x, __fmul_rn(s, v.x)), __fmul_rn(w.y, __fmul_rn(s, v.y)),
                            __fmul_rn(w.z, __fmul_rn(s, v.z)), __fmul_rn(w.w, __fmul_rn(s, v.w))};
      }
    }
  }
}

// Sum of squares over the full row for every live b (multi-chunk RMSNorm).
template <int NB>
TL_DEVICE void rms_scales(const GemvParams& p, float* ss, float* red) {
  const int n4 = p.K >> 2;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float s = 0.f;
    if (b < p.nb) {
      const f4* src = p.tok ? reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.K)
                            : reinterpret_cast<const f4*>(p.x + b * p.x_stride);
      for (int j = threadIdx.x; j < n4; j += blockDim.x) {
        f4 v = src[j];
        s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
      }
    }
    float t = block_sum(s, red);
    ss[b] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)p.K), 1e-5f)));
  }
}

// Accumulate one row chunk: acc[b] += sum_j W[j*64+lane] . xs[b][j*64+lane], j < cnt.
// HASPRE: the first 16 wave-loads were issued earlier (before the activation staging
// barrier) and arrive in `pre`.
template <int NB, bool NT, bool HASPRE>
TL_DEVICE void row_chunk(const f4* __restrict__ w, const f4* xs, int n4, int cnt, int lane, float (&acc)[NB],
                         const f4 (&pre)[16]) {
  int j = 0;
  if constexpr (HASPRE) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = dot4(pre[u], xs[b * n4 + u * 64 + lane], acc[b]);
    }
    j = 16;
  }
  // 16 wave-loads in flight at one sequence; with several sequences every weight float4
  // meets NB activation reads, so fewer loads per step keep the registers (and the
  // occupancy) for the accumulators
  constexpr int UNR = NB == 1 ? 16 : (NB == 2 ? 8 : 4);
  for (; j + UNR <= cnt; j += UNR) {
    f4 wv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) wv[u] = load_w4<NT>(w + (j + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = dot4(wv[u], xs[b * n4 + (j + u) * 64 + lane], acc[b]);
    }
  }
  for (; j + 4 <= cnt; j += 4) {
    f4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = load_w4<NT>(w + (j + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = dot4(wv[u], xs[b * n4 + (j + u) * 64 + lane], acc[b]);
    }
  }
  for (; j < cnt; ++j) {
    f4 wv = load_w4<NT>(w + j * 64 + lane);
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = dot4(wv, xs[b * n4 + j * 64 + lane], acc[b]);
  }
}

template <int MODE>
struct RowsPerItem { static constexpr int v = (MODE == GM_SWIGLU || MODE == GM_QKV) ? 2 : 1; };

template <int MODE>
TL_DEVICE const float* item_row(const GemvParams& p, int item, int r) {
  const long long K = p.K;
  if constexpr (MODE == GM_SWIGLU) {
    return (r == 0 ? p.W0 : p.W1) + (long long)item * K;
  } else if constexpr (MODE == GM_QKV) {
    int row = 2 * item;
    if (row < p.dim) return p.W0 + (long long)(row + r) * K;
    row -= p.dim;
    if (row < p.kv_dim) return p.W1 + (long long)(row + r) * K;
    row -= p.kv_dim;
    return p.W2 + (long long)(row + r) * K;
  } else {
    return p.W0 + (long long)item * K;
  }
}

template <int MODE, int NB>
TL_DEVICE void epilogue(const GemvParams& p, int item, const float (&v)[2][NB], int lane) {
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (lane != b || b >= p.nb) continue;
    if constexpr (MODE == GM_STORE) {
      float* y = p.y + p.y_off + (long long)b * p.y_stride + (p.has_pos ? (long long)p.has_pos * p.pos[b] : 0);
      y[item] = v[0][b];
    } else if constexpr (MODE == GM_RESID) {
      float* y = p.y + (long long)b * p.y_stride + item;
      *y = __fadd_rn(*y, v[0][b]);
    } else if constexpr (MODE == GM_SWIGLU) {
      p.y[(long long)b * p.y_stride + item] = silu_mul(v[0][b], v[1][b]);
    } else {  // GM_QKV
      int row = 2 * item;
      const int pb = p.pos[b];
      float a0 = v[0][b], a1 = v[1][b];
      if (row < p.dim + p.kv_dim) {
        const int i = row < p.dim ? row : row - p.dim;
        const float2 cs = p.rope[(long long)pb * (p.head_size >> 1) + ((i % p.head_size) >> 1)];
        // reference src/seq.cpp:97-98 (no contraction, like the x86 reference build)
        const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
        a0 = r0; a1 = r1;
      }
      if (row < p.dim) {
        float* q = p.y + (long long)b * p.y_stride + row;
        q[0] = a0; q[1] = a1;
      } else {
        row -= p.dim;
        float* base = p.kc;
        if (row >= p.kv_dim) { row -= p.kv_dim; base = p.vc; }
        float* d = base + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)pb * p.kv_dim + row;
        d[0] = a0; d[1] = a1;
      }
    }
  }
}

// WAVES waves per block, IPW items per wave, up to kc_max floats of x staged per chunk.
// PF: when the activations fit one chunk, each wave issues its first row's first 16
// wave-loads BEFORE staging, so the staging (L2 reads + RMSNorm + barrier) hides under
// the weight stream's HBM latency.
template <int MODE, int NB, int IPW, bool NT, int WAVES, bool PF>
__global__ void __launch_bounds__(WAVES * 64) gemv_kernel(GemvParams p, int kc_max) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);          // 16 floats (block reductions)
  float* ss = red + 16;                                  // NB floats
  f4* xs = reinterpret_cast<f4*>(smem + 16 * 4 + 64 * 4); // [NB][kc/4]

  constexpr int RPI = RowsPerItem<MODE>::v;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int item0 = blockIdx.x * (WAVES * IPW) + wave;

  float acc[IPW][RPI][NB];
#pragma unroll
  for (int i = 0; i < IPW; ++i)
#pragma unroll
    for (int r = 0; r < RPI; ++r)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[i][r][b] = 0.f;

  const int K = p.K;
  const bool single = K <= kc_max;
  f4 pre[16];
  const bool use_pre = PF && single && (K >> 8) >= 16 && item0 < p.n_items;
  if (PF && use_pre) {
    const f4* w = reinterpret_cast<const f4*>(item_row<MODE>(p, item0, 0));
#pragma unroll
    for (int u = 0; u < 16; ++u) pre[u] = load_w4<NT>(w + u * 64 + lane);
  }
  if (p.rms_w && !single) rms_scales<NB>(p, ss, red);

  for (int kc = 0; kc < K; kc += kc_max) {
    const int kcn = min(kc_max, K - kc);
    if (kc) __syncthreads();
    stage_x<NB>(p, xs, kc, kcn, single, ss, red);
    __syncthreads();
    const int n4 = kcn >> 2;
    const int cnt = n4 >> 6;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int item = item0 + i * WAVES;
      if (item < p.n_items) {
#pragma unroll
        for (int r = 0; r < RPI; ++r) {
          const f4* w = reinterpret_cast<const f4*>(item_row<MODE>(p, item, r) + kc);
          if (PF && i == 0 && r == 0 && use_pre)
            row_chunk<NB, NT, true>(w, xs, n4, cnt, lane, acc[i][r], pre);
          else
            row_chunk<NB, NT, false>(w, xs, n4, cnt, lane, acc[i][r], pre);
        }
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
      for (int b = 0; b < NB; ++b) v[r][b] = r < RPI ? wave_sum_u(acc[i][r < RPI ? r : 0][b]) : 0.f;
    epilogue<MODE, NB>(p, item, v, lane);
  }
}

// Fallback for shapes the streaming kernel does not take (K % 256 != 0, unaligned
// pointers): one wave per (row, sequence), scalar loads.  Same epilogues.
template <int MODE>
__global__ void __launch_bounds__(256) gemv_generic_kernel(GemvParams p) {
  keep_implicit_args();
  __shared__ float red[16];
  (void)red;
  constexpr int RPI = RowsPerItem<MODE>::v;
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (item >= p.n_items) return;
  // input scale (RMSNorm) computed redundantly per wave
  const float* xin = p.tok ? p.emb + (long long)p.tok[b] * p.K : p.x + b * p.x_stride;
  float s = 1.f;
  if (p.rms_w) {
    float t = 0.f;
    for (int k = lane; k < p.K; k += 64) t = fmaf(xin[k], xin[k], t);
    t = wave_sum_u(t);
    s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)p.K), 1e-5f)));
  }
  if (p.tok && item == 0 && (threadIdx.x >> 6) == 0)
    for (int k = lane; k < p.K; k += 64) p.x_out[b * p.x_stride + k] = xin[k];
  float v[2][1] = {{0.f}, {0.f}};
  for (int r = 0; r < RPI; ++r) {
    const float* w = item_row<MODE>(p, item, r);
    float a = 0.f;
    for (int k = lane; k < p.K; k += 64) {
      float xv = xin[k];
      if (p.rms_w) xv = __fmul_rn(p.rms_w[k], __fmul_rn(s, xv));
      a = fmaf(w[k], xv, a);
    }
    v[r][0] = wave_sum_u(a);
  }
  // reuse the NB=1 epilogue for sequence b by shifting the per-b pointers
  GemvParams q = p;
  q.nb = 1;
  if constexpr (MODE == GM_STORE) {
    q.y_off = p.y_off + (long long)b * p.y_stride + (p.has_pos ? (long long)p.has_pos * p.pos[b] : 0);
    q.has_pos = 0;
  } else if constexpr (MODE == GM_QKV) {
    q.y = p.y + (long long)b * p.y_stride;
    q.kc = p.kc + (long long)b * p.kv_b_stride;
    q.vc = p.vc + (long long)b * p.kv_b_stride;
    q.pos = p.pos + b;
  } else {
    q.y = p.y + (long long)b * p.y_stride;
  }
  epilogue<MODE, 1>(q, item, v, lane);
}

}  // namespace tl
