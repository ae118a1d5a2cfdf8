// gemv_rr.hpp — the batched (4..8 sequences) decode GEMV with the activations held in
// registers ("register-resident"): the B = 8 step's weight stream, as the B = 1 kernel's.
//
// Semantics as gemv.hpp / gemv_mfma.hpp (reference src/thaBLAS.cpp:191-228 batched GEMV,
// CPU twin src/seq.cpp:40-51, with the same fused prologue and epilogues).
//
// Why: the matrix-core kernel (gemv_mfma.hpp) streams at 3.3-5.4 TB/s because every weight
// byte goes HBM -> VGPR -> LDS -> VGPR (the MFMA operand layout) and every 16-row tile
// re-reads the activations from L2; the B = 1 kernel streams at ~6.5-7 TB/s with 1-KiB
// coalesced wave-loads straight into the FMAs.  At B <= 8 the arithmetic is still tiny
// (16 packed FMAs per weight float4 against a wave-load of 1 KiB: ~4% of the VALU at the
// HBM rate), so the VALU can do it if the activations need no LDS reads:
//  * grid = one 512-thread block (8 waves) per CU; block b owns a contiguous, balanced
//    range of items (rows; 16-row tiles for the residual mode, whose epilogue leaves the
//    per-tile sums of squares of gemv_mfma.hpp for the next norm);
//  * K is cut into 1-KiB chunks (256 floats); wave w owns chunks w*CPW .. w*CPW+CPW-1 of a
//    pass and holds x'[b][chunk] for all NB sequences in VGPRs (NB*CPW*4 floats per lane,
//    RMSNorm applied as they are loaded, bit-identical to gemv_prenorm_kernel);
//  * the wave then sweeps every row of its block: one 1-KiB nt wave-load per row and chunk
//    (two batches of RB rows in flight), v_pk_fma_f32 into acc[row][seq pair];
//  * per batch the RB*NB lane partials are reduced by recursive halving (each exchange
//    step halves the values a lane carries: v_permlane32/16_swap, then DPP row_mirror,
//    row_half_mirror, quad_perm), so the 64-lane sums cost ~2 VALU per value, and land in
//    LDS as [wave][row][seq];
//  * at the end of a pass the 8 wave partials are added in wave order; K > 8*CPW chunks
//    (W2: 43 chunks) takes several passes, each reloading the wave's activations.
// Deterministic: every sum has a fixed order.  fp32 FMA order differs from the reference's
// sequential loop, within its 1e-4 logits tolerance (as the other batched kernels).
#pragma once
#include "gemv_mfma.hpp"

namespace tl {

typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kRrWaves = 8;
constexpr int kRrMaxRows = 96;   // weight rows per block (host-checked; LDS: 8 x 16 KiB x' + partials)

// One exchange step of the recursive-halving reduction: lanes whose distinguishing bit is
// set keep the upper half of the values and send the lower half (and the other way round).
template <int D>
TL_DEVICE float rr_xfer(float v) {
  if constexpr (D == 32 || D == 16) return __shfl_xor(v, D, 64);
  else if constexpr (D == 8) return dpp_f<0x140>(v);   // row_mirror: i <-> 15 - i
  else if constexpr (D == 4) return dpp_f<0x141>(v);   // row_half_mirror: i <-> 7 - i
  else if constexpr (D == 2) return dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  else return dpp_f<0xB1>(v);                          // quad_perm [1,0,3,2]
}

template <int D, int M>
TL_DEVICE void rr_stage(float (&v)[M], int lane) {
  if constexpr (D >= 1) {
    const bool hi = (lane & D) != 0;
    if constexpr (M >= 2 && (D == 32 || D == 16)) {
      // gfx950 v_permlane{32,16}_swap: odd rows (of D lanes) of a trade places with even rows of
      // b, so a' + b' holds a's pair sums in the even rows and b's in the odd ones (VALU only)
#pragma unroll
      for (int j = 0; j < M / 2; ++j) {
        const unsigned a = __float_as_uint(v[j]), b = __float_as_uint(v[j + M / 2]);
        const auto r = D == 32 ? __builtin_amdgcn_permlane32_swap(a, b, false, false)
                               : __builtin_amdgcn_permlane16_swap(a, b, false, false);
        v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      }
      (void)hi;
      float (&h)[M / 2] = *reinterpret_cast<float(*)[M / 2]>(&v[0]);
      rr_stage<D / 2, M / 2>(h, lane);
    } else if constexpr (M >= 2) {
#pragma unroll
      for (int j = 0; j < M / 2; ++j) {
        const float send = hi ? v[j] : v[j + M / 2];
        const float keep = hi ? v[j + M / 2] : v[j];
        v[j] = keep + rr_xfer<D>(send);
      }
      float (&h)[M / 2] = *reinterpret_cast<float(*)[M / 2]>(&v[0]);
      rr_stage<D / 2, M / 2>(h, lane);
    } else {
      v[0] = v[0] + rr_xfer<D>(v[0]);
      rr_stage<D / 2, 1>(v, lane);
    }
  }
}

// Sums of v[0..M) over the 64 lanes; afterwards lane l holds sum number l >> (6 - log2 M)
// (every lane of a group of 64 / M lanes holds the same one).
template <int M>
TL_DEVICE float rr_reduce(float (&v)[M], int lane) {
  rr_stage<32, M>(v, lane);
  return v[0];
}

template <int M>
struct RrLog { static constexpr int v = M <= 1 ? 0 : 1 + RrLog<M / 2>::v; };

template <int MODE, int NB, int CPW, int RB>
__global__ void __launch_bounds__(kRrWaves * 64) gemv_rr_kernel(GemvParams p) {
  constexpr int W = kRrWaves;
  constexpr int RPI = RowsPerItem<MODE>::v;
  constexpr int NP = NB / 2;           // sequence pairs (one v_pk_fma_f32 each)
  constexpr int M = RB * NB;           // values reduced per batch
  constexpr int SH = 6 - RrLog<M>::v;  // lane -> value: lane >> SH
  static_assert(M <= 64 && (M & (M - 1)) == 0, "RB * NB must be a power of two <= 64");
  // each wave's x' chunks, [j][comp][seq quad][lane] float4 (a lane's reads are 16 B apart:
  // conflict-free); only the wave that wrote them reads them, so no block barrier
  __shared__ __attribute__((aligned(16))) f4 xs[W][CPW * 4 * (NB / 4) * 64];
  __shared__ float part[W][kRrMaxRows * NB];
  __shared__ float tot[kRrMaxRows * NB];
  __shared__ float s_red[256];
  __shared__ float s_ss[16];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, bi = blockIdx.x;
  // this block's items
  int i0, i1;
  if constexpr (MODE == GM_RESID) {
    const int nt = (p.n_items + 15) >> 4;
    i0 = 16 * (int)((long long)nt * bi / G);
    i1 = 16 * (int)((long long)nt * (bi + 1) / G);
    if (i1 > p.n_items) i1 = p.n_items;
  } else {
    i0 = (int)((long long)p.n_items * bi / G);
    i1 = (int)((long long)p.n_items * (bi + 1) / G);
  }
  const int nr = (i1 - i0) * RPI;  // weight rows of this block (<= kRrMaxRows)
  const int nch = p.K >> 8;        // 1-KiB chunks per row
  const int npass = (nch + W * CPW - 1) / (W * CPW);

  const int nbat = (nr + RB - 1) / RB;  // row batches per pass
  const int nflat = npass * nbat;        // (pass, batch) in order: one software pipeline
  auto chunk0 = [&](int pass) { return pass * W * CPW + wave * CPW; };
  auto live = [&](int pass) {  // this wave's live chunks in a pass (wave-uniform)
    const int cv = nch - chunk0(pass);
    return cv < 0 ? 0 : (cv > CPW ? CPW : cv);
  };
  auto row_ptr = [&](int r) -> const f4* {
    r = r < nr ? r : nr - 1;  // past the block's rows: a valid row, result dropped
    return reinterpret_cast<const f4*>(item_row<MODE>(p, i0 + r / RPI, r % RPI));
  };
  // Every load is issued (a predicated load makes the compiler's vmcnt waits cover it too): a
  // chunk past the row re-reads the wave's first chunk, a wave with no live chunk in the pass
  // re-reads one line of the block's first row (cache hits), both against zero activations.
  auto load = [&](f4 (&wb)[RB][CPW], int g) {
    const int pass = g / nbat, bt = g - pass * nbat;
    const int cv = live(pass);
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      const f4* w = cv > 0 ? row_ptr(bt * RB + rr) + (long long)chunk0(pass) * 64 + lane : row_ptr(0) + lane;
#pragma unroll
      for (int j = 0; j < CPW; ++j) wb[rr][j] = load_w4<true>(w + (j < cv ? j : 0) * 64);
    }
  };

  // fused RMSNorm from the producer's per-tile sums of squares (gemv_mfma.hpp norm_scales,
  // same order: thread (b, j) sums tiles j, j + 16, ..., then b sums its 16 in order); the
  // first two weight batches are already in flight
  const bool fnorm = p.rms_w != nullptr;
  f4 wa[RB][CPW], wb2[RB][CPW], wc[RB][CPW];
  if (nflat > 0) load(wa, 0);
  if (nflat > 1) load(wb2, 1);
  if (nflat > 2) load(wc, 2);
  if (fnorm) {
    const int t = threadIdx.x, b = t >> 4, j = t & 15;
    if (t < 256) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        a = __fadd_rn(a, b < p.nb && j + 16 * k < p.ssq_nt ? p.ssq_in[(long long)b * p.ssq_nt + j + 16 * k] : 0.f);
      s_red[t] = a;
    }
    __syncthreads();
    if (t < p.nb) {
      float v = 0.f;
      for (int k = 0; k < 16; ++k) v = __fadd_rn(v, s_red[t * 16 + k]);
      s_ss[t] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(v, (float)p.K), 1e-5f)));  // src/seq.cpp:3-16
    }
    __syncthreads();
  }

  // activations of a pass, staged by each wave for its own chunks:
  // xs[wave][((j * 4 + comp) * NB/4 + quad) * 64 + lane] = x'[4 quad .. 4 quad + 3][k + comp],
  // k = 256 (chunk0 + j) + 4 lane
  f4* xw = xs[wave];
  auto load_x = [&](int pass) {
    const int c0 = chunk0(pass), cv = live(pass);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int k = 256 * (c0 + j) + 4 * lane;
      f4 rw = f4{1.f, 1.f, 1.f, 1.f};
      if (fnorm && j < cv) rw = *reinterpret_cast<const f4*>(p.rms_w + k);
      f4 e[NB];
#pragma unroll
      for (int s = 0; s < NB; ++s) {
        e[s] = f4{0.f, 0.f, 0.f, 0.f};
        if (j < cv && s < p.nb) {
          e[s] = *reinterpret_cast<const f4*>(p.x + (long long)s * p.x_stride + k);
          if (fnorm) {
            const float sv = s_ss[s];
            e[s] = f4{__fmul_rn(rw.x, __fmul_rn(sv, e[s].x)), __fmul_rn(rw.y, __fmul_rn(sv, e[s].y)),
                      __fmul_rn(rw.z, __fmul_rn(sv, e[s].z)), __fmul_rn(rw.w, __fmul_rn(sv, e[s].w))};
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int h = 0; h < NB / 4; ++h)
          xw[((j * 4 + c) * (NB / 4) + h) * 64 + lane] = f4{e[4 * h][c], e[4 * h + 1][c], e[4 * h + 2][c], e[4 * h + 3][c]};
    }
  };
  // the 8 wave partials of a pass, added in wave order (waves with no live chunk left none)
  auto merge = [&](int pass) {
    for (int t = threadIdx.x; t < nr * NB; t += W * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const int cw = nch - (pass * W * CPW + w * CPW);
        if (cw > 0) s = w == 0 ? part[w][t] : s + part[w][t];
      }
      tot[t] = pass == 0 ? s : tot[t] + s;
    }
  };
  auto compute = [&](const f4 (&wb)[RB][CPW], int g) {
    const int pass = g / nbat, bt = g - pass * nbat;
    if (bt == 0) {  // pass boundary (block-uniform): fold the previous pass, load this one's x'
      if (pass > 0) {
        __syncthreads();
        merge(pass - 1);
        __syncthreads();
      }
      load_x(pass);
    }
    f2v acc[RB][NP];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int q = 0; q < NP; ++q) acc[rr][q] = f2v{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < CPW; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f2v xa[NP];
#pragma unroll
        for (int h = 0; h < NB / 4; ++h) {
          const f4 t = xw[((j * 4 + c) * (NB / 4) + h) * 64 + lane];
          xa[2 * h] = f2v{t.x, t.y};
          xa[2 * h + 1] = f2v{t.z, t.w};
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
          const float w = wb[rr][j][c];
          const f2v ww = f2v{w, w};
#pragma unroll
          for (int q = 0; q < NP; ++q) acc[rr][q] = __builtin_elementwise_fma(xa[q], ww, acc[rr][q]);
        }
      }
    float v[M];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr)
#pragma unroll
      for (int s = 0; s < NB; ++s) v[rr * NB + s] = acc[rr][s >> 1][s & 1];
    const float sum = rr_reduce<M>(v, lane);
    const int idx = lane >> SH;
    const int r = bt * RB + idx / NB;
    if ((lane & ((1 << SH) - 1)) == 0 && r < nr) part[wave][r * NB + idx % NB] = sum;
  };

  // three batches in flight: the steady state issues batch g + 3 unconditionally as batch g is
  // consumed; the last (up to five) batches are peeled
  if (nflat > 0) {
    int g = 0;
    for (; g + 5 < nflat; g += 3) {
      compute(wa, g);
      load(wa, g + 3);
      compute(wb2, g + 1);
      load(wb2, g + 4);
      compute(wc, g + 2);
      load(wc, g + 5);
    }
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      if (g + t >= nflat) break;
      if (t % 3 == 0) { compute(wa, g + t); if (g + t + 3 < nflat) load(wa, g + t + 3); }
      else if (t % 3 == 1) { compute(wb2, g + t); if (g + t + 3 < nflat) load(wb2, g + t + 3); }
      else compute(wc, g + t);
    }
  }
  __syncthreads();
  if (nflat > 0) merge(npass - 1);
  __syncthreads();

  // epilogues (gemv_mfma.hpp epi_one), one thread per (item, sequence)
  const int ni = i1 - i0;
  for (int t = threadIdx.x; t < ni * NB; t += W * 64) {
    const int it = t / NB, s = t % NB;
    if (s >= p.nb) continue;
    if constexpr (MODE == GM_SWIGLU || MODE == GM_QKV) {
      epi_one<MODE>(p, i0 + it, s, tot[(2 * it) * NB + s], tot[(2 * it + 1) * NB + s]);
    } else if constexpr (MODE == GM_RESID) {
      float* y = p.y + (long long)s * p.y_stride + i0 + it;
      const float nv = __fadd_rn(*y, tot[t]);
      *y = nv;
      tot[t] = __fmul_rn(nv, nv);
    } else {
      epi_one<MODE>(p, i0 + it, s, tot[t], 0.f);
    }
  }
  if constexpr (MODE == GM_RESID) {
    if (p.ssq_out) {  // per 16-row tile and sequence: squares of its rows in order (gemv_mfma.hpp)
      __syncthreads();
      const int ntl = (ni + 15) >> 4;
      for (int t = threadIdx.x; t < ntl * NB; t += W * 64) {
        const int tl_ = t / NB, s = t % NB;
        if (s >= p.nb) continue;
        float v = 0.f;
        for (int r = 0; r < 16; ++r) {
          const int it = 16 * tl_ + r;
          v = __fadd_rn(v, it < ni ? tot[it * NB + s] : 0.f);
        }
        p.ssq_out[(long long)s * p.ssq_nt + (i0 >> 4) + tl_] = v;
      }
    }
  }
}

}  // namespace tl
