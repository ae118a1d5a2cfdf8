// gemv_mb.hpp — the batched (2..8 sequences) decode GEMV on the 16-block 4x4x1 f32 matrix cores,
// weights streamed straight into VGPRs, every wave on one contiguous run of work.
//
// Semantics as gemv.hpp / gemv_mfma.hpp: y[b][r] = sum_k W[r][k] * x'[b][k] for the reference's
// row-major [M][K] fp32 weights (src/thaBLAS.cpp:191-228 batched GEMV, CPU twin src/seq.cpp:40-51),
// x' the activation or its RMSNorm (src/seq.cpp:3-16), and the same fused epilogues (offset store,
// residual add, SwiGLU over W1/W3, QKV + RoPE + KV-cache write).
//
// Why this shape on gfx950:
//  * v_mfma_f32_4x4x1_16b_f32 is 16 independent 4x4 outer products.  Block q (lanes 4q..4q+3)
//    takes k = 4q + c of the current 64-k chunk, so lane (q, i) supplies W[row i][k] and
//    x[seq i][k]: a 4-row x 4-sequence tile per instruction with no unused columns at 4 or 8
//    sequences (the 16x16x4 form wastes half its columns at 8).  A wave-load of the weights is
//    then 4 rows x 256 contiguous bytes that land in the MFMA operand layout as they are: no LDS
//    transpose (gemv_mfma.hpp writes and reads every weight byte through LDS).
//  * The activations (every sequence's row, or one K slice of it) sit in LDS for the whole launch,
//    already normalised; the block computes the RMSNorm itself from the staged rows, so no norm
//    prologue launch and no sums of squares carried between launches.
//  * Work unit = (4-row group, 64-k chunk) = 1 KiB per weight matrix.  The units of a K slice are
//    split into equal contiguous runs, one per wave (perfect balance at any shape); each wave keeps
//    kMbDepth units in flight.  A row group cut between waves (or K slices) leaves one partial
//    4x8 tile per piece in a slab; the last piece to arrive (ticket) sums the pieces in slot
//    order (deterministic) and runs the epilogue.  Slab stores are write-through (sc1) and
//    need no release fence (a fence writing back L2 here cost 2-3x the launch: tools/probes/
//    mb_probe.hip).
#pragma once
#include <mutex>
#include <utility>
#include <vector>
#include "gemv.hpp"

namespace tl {

typedef float mb_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMbWaves = 8;      // waves per block (one block per CU: the activations fill the LDS)
constexpr int kMbDepth = 8;      // weight units in flight per wave
constexpr int kMbMaxSlices = 4;  // K slices (rows too long for the LDS)

struct MbGeom {
  int C;      // 64-k chunks per row (K / 64)
  int nsl;    // K slices; 1 = whole rows in LDS (required by the norm and the embedding prologue)
  int bps;    // blocks per slice
  int NG;     // 4-row groups
  int maxp;   // slab slots per slice and row group
  int csm;    // chunks of the largest slice
};

template <int CTRL>
TL_DEVICE float mb_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes l with equal l % 4 (the 16 k-blocks of a 4x4x1 accumulator).
TL_DEVICE float mb_red16(float r) {
  r += mb_dpp<0x124>(r);  // row_ror:4
  r += mb_dpp<0x128>(r);  // row_ror:8
  r += __shfl_xor(r, 16, 64);
  r += __shfl_xor(r, 32, 64);
  return r;
}
TL_DEVICE float mb_sel(const mb_f32x4& a, int i) { return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3]; }
// Wave g of a slice whose run holds unit u (runs: [T g / NW, T (g + 1) / NW), T >= NW).
TL_DEVICE long long mb_wave_of(long long u, long long T, long long NW) { return ((u + 1) * NW - 1) / T; }

// One output (row, sequence b).  QKV: row even, (a0, a1) = rows (row, row + 1), RoPE from the
// LDS rows rl[b][hs/2]; SWIGLU: (a0, a1) = (W1 x, W3 x).
template <int MODE>
TL_DEVICE void mb_out(const GemvParams& p, const float2* rl, const int* spos, int row, int b, float a0, float a1) {
  if constexpr (MODE == GM_STORE) {
    float* y = p.y + p.y_off + (long long)b * p.y_stride + (p.has_pos ? (long long)p.has_pos * spos[b] : 0);
    y[row] = a0;
  } else if constexpr (MODE == GM_RESID) {
    float* y = p.y + (long long)b * p.y_stride + row;
    *y = __fadd_rn(*y, a0);
  } else if constexpr (MODE == GM_SWIGLU) {
    p.y[(long long)b * p.y_stride + row] = silu_mul(a0, a1);
  } else {
    const int hh = p.head_size >> 1;
    if (row < p.dim + p.kv_dim) {
      const int i = row < p.dim ? row : row - p.dim;
      const float2 cs = rl[b * hh + ((i % p.head_size) >> 1)];
      const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
      const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
      a0 = r0; a1 = r1;
    }
    if (row < p.dim) {
      float* qd = p.y + (long long)b * p.y_stride + row;
      qd[0] = a0; qd[1] = a1;
    } else {
      int r = row - p.dim;
      float* base = p.kc;
      if (r >= p.kv_dim) { r -= p.kv_dim; base = p.vc; }
      float* dd = base + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)spos[b] * p.kv_dim + r;
      dd[0] = a0; dd[1] = a1;
    }
  }
}

template <int MODE, int NSG, bool NT>
__global__ void __launch_bounds__(kMbWaves * 64) gemv_mb_kernel(GemvParams p, MbGeom g) {
  keep_implicit_args();
  constexpr int W = kMbWaves, P = kMbDepth;
  constexpr int NR = MODE == GM_SWIGLU ? 2 : 1;
  constexpr int NS = 4 * NSG;       // sequence slots of the tile
  constexpr int SLAB = NR * NSG * 16;
  extern __shared__ __attribute__((aligned(16))) f4 xl[];  // [chunk][NSG][64 lanes], then RoPE rows
  __shared__ float s_ss[NS];
  __shared__ int s_pos[NS];
  __shared__ int s_tok[NS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bq = lane >> 2, iq = lane & 3;
  const int nb = p.nb, K = p.K;
  const long long Kl = K;
  const int slice = blockIdx.x / g.bps, bis = blockIdx.x - slice * g.bps;
  const int cs0 = (int)((long long)g.C * slice / g.nsl);
  const int Cn = (int)((long long)g.C * (slice + 1) / g.nsl) - cs0;
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
  const long long T = (long long)g.NG * Cn, NW = (long long)g.bps * W, gid = (long long)bis * W + wave;
  const long long u0 = T * gid / NW, u1 = T * (gid + 1) / NW;

  // ---- weight stream: row pointers of the issue cursor's row group, first kMbDepth units issued
  // before the activations are staged (their latency overlaps the staging)
  long long ui = u0;
  int rgi = (int)(u0 / Cn), ci = (int)(u0 - (long long)rgi * Cn);
  const float* wr[NR];
  auto set_rows = [&](int rg) {
    int row = 4 * rg + iq;
    row = row < n_rows ? row : n_rows - 1;
    if constexpr (MODE == GM_SWIGLU) {
      wr[0] = p.W0 + row * Kl + 4 * bq;
      wr[NR - 1] = p.W1 + row * Kl + 4 * bq;
    } else if constexpr (MODE == GM_QKV) {
      const float* b = row < p.dim ? p.W0 + row * Kl
                                   : row < p.dim + p.kv_dim ? p.W1 + (row - p.dim) * Kl : p.W2 + (row - p.dim - p.kv_dim) * Kl;
      wr[0] = b + 4 * bq;
    } else {
      wr[0] = p.W0 + row * Kl + 4 * bq;
    }
  };
  set_rows(rgi);
  auto issue = [&](f4 (&w)[NR]) {
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      const f4* a = reinterpret_cast<const f4*>(wr[m] + 64 * (cs0 + ci));
      if constexpr (NT) w[m] = __builtin_nontemporal_load(a);
      else w[m] = *a;
    }
    if (ui + 1 < u1) {  // past the run: the last unit again (an L2 hit, never a new line)
      ++ui;
      if (++ci == Cn) { ci = 0; set_rows(++rgi); }
    }
  };
  f4 buf[P][NR];
  if (u0 < u1) {
#pragma unroll
    for (int t = 0; t < P; ++t) issue(buf[t]);
  }

  // ---- activations: x' rows (or their slice) into LDS in the B-operand layout.  One round of
  // global loads (the embedding row's token first when there is one): the rows, the norm weights
  // and the positions together; thread t's elements all belong to sequence sb (e = t + 512 r), so
  // it keeps that sequence's partial sum of squares in a register.
  const int nx = Cn * NSG * 64;
  constexpr int XR = 16;  // activation loads in flight per thread and round
  if (p.tok) {
    if (threadIdx.x < NS) s_tok[threadIdx.x] = threadIdx.x < nb ? p.tok[threadIdx.x] : 0;
    __syncthreads();
  }
  if (threadIdx.x < NS) s_pos[threadIdx.x] = threadIdx.x < nb && p.pos ? p.pos[threadIdx.x] : 0;
  float2* rl = reinterpret_cast<float2*>(xl + g.csm * NSG * 64);
  f4* wl = reinterpret_cast<f4*>(rl + (MODE == GM_QKV ? NS * (p.head_size >> 1) : 0));  // RMSNorm weights [Cn * 16]
  if (p.rms_w) {
    const f4* w4 = reinterpret_cast<const f4*>(p.rms_w + 64LL * cs0);
    for (int j = threadIdx.x; j < Cn * 16; j += W * 64) wl[j] = w4[j];
  }
  const int sb = 4 * ((threadIdx.x >> 6) % NSG) + (threadIdx.x & 3);
  const float* src = sb >= nb ? nullptr : p.tok ? p.emb + (long long)s_tok[sb] * Kl : p.x + (long long)sb * p.x_stride;
  float sq = 0.f;
  for (int e0 = threadIdx.x; e0 < nx; e0 += XR * W * 64) {
    f4 v[XR];
#pragma unroll
    for (int r = 0; r < XR; ++r) {
      const int e = e0 + r * W * 64;
      const long long k = 64LL * (cs0 + e / (NSG * 64)) + 4 * ((e & 63) >> 2);
      v[r] = (e < nx && src) ? *reinterpret_cast<const f4*>(src + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int r = 0; r < XR; ++r) {
      const int e = e0 + r * W * 64;
      if (e < nx) {
        xl[e] = v[r];
        sq = fmaf(v[r].x, v[r].x, sq); sq = fmaf(v[r].y, v[r].y, sq);
        sq = fmaf(v[r].z, v[r].z, sq); sq = fmaf(v[r].w, v[r].w, sq);
        if (p.tok && blockIdx.x == 0 && src)  // the embedding row is also the residual stream
          *reinterpret_cast<f4*>(p.x_out + (long long)sb * p.x_stride + 64 * (e / (NSG * 64)) + 4 * ((e & 63) >> 2)) = v[r];
      }
    }
  }
  float* s_part = reinterpret_cast<float*>(wl + (p.rms_w ? g.csm * 16 : 0));  // [W][4] per-wave partial sums
  if (p.rms_w) {
    sq = mb_red16(sq);  // this wave's lanes of sequence 4 (wave % NSG) + (lane & 3)
    if (lane < 4) s_part[4 * wave + lane] = sq;
  }
  __syncthreads();
  if constexpr (MODE == GM_QKV) {
    const int hh = p.head_size >> 1;
    for (int t = threadIdx.x; t < nb * hh; t += W * 64) rl[t] = p.rope[(long long)s_pos[t / hh] * hh + t % hh];
  }
  if (p.rms_w) {
    // ss_b = 1 / sqrt(sum(x_b^2) / K + 1e-5) (src/seq.cpp:3-16), partials in thread order
    if (threadIdx.x < nb) {
      const int b = threadIdx.x, s = b >> 2, j = b & 3;
      float a = 0.f;
      for (int m = 0; m < W / NSG; ++m) a += s_part[4 * (s + NSG * m) + j];
      s_ss[b] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(a, (float)K), 1e-5f)));
    }
    __syncthreads();
    const float sv = s_ss[sb < nb ? sb : 0];
    for (int e = threadIdx.x; e < nx; e += W * 64) {
      if (sb < nb) {
        const f4 w = wl[16 * (e / (NSG * 64)) + ((e & 63) >> 2)];
        const f4 x = xl[e];
        xl[e] = f4{__fmul_rn(w.x, __fmul_rn(sv, x.x)), __fmul_rn(w.y, __fmul_rn(sv, x.y)),
                   __fmul_rn(w.z, __fmul_rn(sv, x.z)), __fmul_rn(w.w, __fmul_rn(sv, x.w))};
      }
    }
  }
  if (p.rms_w || MODE == GM_QKV) __syncthreads();
  if (u0 >= u1) return;  // (the host sizes the grid so that every wave has a run)

  // ---- stream
  mb_f32x4 acc[NR][NSG];
#pragma unroll
  for (int m = 0; m < NR; ++m)
#pragma unroll
    for (int s = 0; s < NSG; ++s) acc[m][s] = mb_f32x4{0.f, 0.f, 0.f, 0.f};
  int rgc = (int)(u0 / Cn), cc = (int)(u0 - (long long)rgc * Cn), cstart = cc;
  const long long NSLOT = (long long)g.nsl * g.maxp;
  for (long long base = u0; base < u1; base += P) {
#pragma unroll
    for (int t = 0; t < P; ++t) {
      const long long u = base + t;
      if (u < u1) {
        f4 xv[NSG];
#pragma unroll
        for (int s = 0; s < NSG; ++s) xv[s] = xl[(cc * NSG + s) * 64 + lane];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s)
              acc[m][s] = __builtin_amdgcn_mfma_f32_4x4x1f32(buf[t][m][q], xv[s][q], acc[m][s], 0, 0, 0);
        if (cc == Cn - 1 || u == u1 - 1) {  // row group rgc: this wave's piece [cstart, cc] ends
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s)
#pragma unroll
              for (int v = 0; v < 4; ++v) acc[m][s][v] = mb_red16(acc[m][s][v]);
          if (g.nsl == 1 && cstart == 0 && cc == Cn - 1) {
            // the whole row group: lane (bq < 4, iq) writes row 4 rgc + bq of sequences iq, iq + 4
            const int row = 4 * rgc + bq;
            if (bq < 4 && row < n_rows && (MODE != GM_QKV || (bq & 1) == 0)) {
#pragma unroll
              for (int s = 0; s < NSG; ++s) {
                const int b = 4 * s + iq;
                if (b < nb) {
                  const float a0 = mb_sel(acc[0][s], bq);
                  const float a1 = MODE == GM_SWIGLU ? mb_sel(acc[NR - 1][s], bq) : MODE == GM_QKV ? mb_sel(acc[0][s], bq + 1) : 0.f;
                  mb_out<MODE>(p, rl, s_pos, row, b, a0, a1);
                }
              }
            }
          } else {
            // a piece: its 4 x NS tile into slot (slice, wave - first wave of the row group)
            const long long gf = mb_wave_of((long long)rgc * Cn, T, NW);
            float* slab = p.mbpart + ((long long)rgc * NSLOT + (long long)slice * g.maxp + (gid - gf)) * SLAB;
            if (bq < 4) {
#pragma unroll
              for (int m = 0; m < NR; ++m)
#pragma unroll
                for (int s = 0; s < NSG; ++s) st1_sc1(slab + (m * NSG + s) * 16 + bq * 4 + iq, mb_sel(acc[m][s], bq));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // pieces of this row group over all slices
            int np = 0;
            for (int s2 = 0; s2 < g.nsl; ++s2) {
              const int c2 = (int)((long long)g.C * (s2 + 1) / g.nsl) - (int)((long long)g.C * s2 / g.nsl);
              const long long T2 = (long long)g.NG * c2;
              np += (int)(mb_wave_of((long long)rgc * c2 + c2 - 1, T2, NW) - mb_wave_of((long long)rgc * c2, T2, NW) + 1);
            }
            unsigned old = 0;
            if (lane == 0) old = __hip_atomic_fetch_add(p.mbcnt + rgc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            old = __builtin_amdgcn_readfirstlane(old);
            if ((int)old == np - 1) {  // last piece: sum the slots in order, then the epilogue
              if (lane == 0) __hip_atomic_store(p.mbcnt + rgc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const int s = lane >> 4, v = (lane >> 2) & 3, j = lane & 3;
              const int row = 4 * rgc + v, b = 4 * s + j;
              if (s < NSG && row < n_rows && b < nb && (MODE != GM_QKV || (v & 1) == 0)) {
                const int o0 = s * 16 + v * 4 + j;
                const int o1 = MODE == GM_SWIGLU ? (NSG + s) * 16 + v * 4 + j : o0 + 4;
                float a0 = 0.f, a1 = 0.f;
                bool first = true;
                for (int s2 = 0; s2 < g.nsl; ++s2) {
                  const int c2 = (int)((long long)g.C * (s2 + 1) / g.nsl) - (int)((long long)g.C * s2 / g.nsl);
                  const long long T2 = (long long)g.NG * c2;
                  const int n2 = (int)(mb_wave_of((long long)rgc * c2 + c2 - 1, T2, NW) - mb_wave_of((long long)rgc * c2, T2, NW) + 1);
                  const float* sl = p.mbpart + ((long long)rgc * NSLOT + (long long)s2 * g.maxp) * SLAB;
                  for (int k = 0; k < n2; ++k) {
                    const float v0 = ld1_sc1(sl + k * SLAB + o0);
                    const float v1 = MODE == GM_SWIGLU || MODE == GM_QKV ? ld1_sc1(sl + k * SLAB + o1) : 0.f;
                    a0 = first ? v0 : a0 + v0;
                    a1 = first ? v1 : a1 + v1;
                    first = false;
                  }
                }
                mb_out<MODE>(p, rl, s_pos, row, b, a0, a1);
              }
            }
          }
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s) acc[m][s] = mb_f32x4{0.f, 0.f, 0.f, 0.f};
          cstart = 0;
        }
        if (++cc == Cn) { cc = 0; ++rgc; }
      }
      issue(buf[t]);
    }
  }
}

// ------------------------------------------------------------------------------------ host side

// Dynamic LDS the kernel may use on this device (one block per CU: the rest of the CU's LDS).
inline int mb_lds_budget() {
  static const int v = [] {
    int dev = 0, lds = 160 * 1024;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    return lds - 1024;  // the static arrays
  }();
  return v;
}
inline int mb_cus() {
  static const int v = [] {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return ncu;
  }();
  return v;
}
// Largest sequence count this kernel takes: env THALLAMA_GEMV_MB (default 0 = off: measured
// slower than gemv_mfma.hpp in the 7B batch-8 step); mb_override() >= 0
// replaces it (the test hook thallama_gemv_check).
inline int& mb_override() {
  static int v = -1;
  return v;
}
inline int mb_max_nb() {
  static const int v = [] {
    const char* e = getenv("THALLAMA_GEMV_MB");
    return e ? atoi(e) : 0;
  }();
  return mb_override() >= 0 ? mb_override() : v;
}

// Epilogue modes (bit GM_*) this kernel takes (env THALLAMA_GEMV_MB_MODES, a bit mask; default all).
inline int mb_modes() {
  static const int v = [] {
    const char* e = getenv("THALLAMA_GEMV_MB_MODES");
    return e ? (int)strtol(e, nullptr, 0) : 0xF;
  }();
  return v;
}

// The launch geometry for p, or false when this kernel does not take it.
template <int MODE>
inline bool mb_plan(const GemvParams& p, MbGeom& g, size_t& lds) {
  if (p.nb < 2 || p.nb > 8 || p.nb > mb_max_nb() || !((mb_modes() >> MODE) & 1)) return false;
  if (!p.mbpart || !p.mbcnt || p.K <= 0 || (p.K & 63) || (p.x_stride & 3) || p.ssq_out) return false;
  const bool al = ((uintptr_t)p.W0 & 15) == 0 && ((uintptr_t)p.W1 & 15) == 0 && ((uintptr_t)p.W2 & 15) == 0 &&
                  ((uintptr_t)(p.tok ? p.emb : p.x) & 15) == 0 && ((uintptr_t)p.rms_w & 15) == 0 &&
                  (!p.tok || ((uintptr_t)p.x_out & 15) == 0);
  if (!al) return false;
  const int NSG = p.nb <= 4 ? 1 : 2;
  const int n_rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
  if (n_rows <= 0 || (MODE == GM_QKV && ((p.dim | p.kv_dim) & 3))) return false;
  g.C = p.K >> 6;
  g.NG = (n_rows + 3) / 4;
  const int rope_b = MODE == GM_QKV ? 4 * NSG * (p.head_size >> 1) * (int)sizeof(float2) : 0;
  const int budget = mb_lds_budget() - rope_b;
  const int per_chunk = NSG * 64 * 16 + (p.rms_w ? 256 : 0);  // activations (+ the norm weights)
  g.nsl = (g.C * per_chunk + budget - (p.rms_w ? kMbWaves * 16 : 0) - 1) / (budget - (p.rms_w ? kMbWaves * 16 : 0));
  if (g.nsl > kMbMaxSlices || ((p.rms_w || p.tok) && g.nsl > 1)) return false;
  g.csm = (g.C + g.nsl - 1) / g.nsl;
  g.bps = mb_cus() / g.nsl;
  // every wave needs a run of at least one unit in every slice
  const long long cmin = g.C / g.nsl;
  while (g.bps > 1 && (long long)g.NG * cmin < (long long)g.bps * kMbWaves) --g.bps;
  if ((long long)g.NG * cmin < (long long)g.bps * kMbWaves) return false;
  const long long umin = (long long)g.NG * cmin / ((long long)g.bps * kMbWaves);
  g.maxp = (int)((g.csm + umin - 1) / umin) + 1;
  if ((long long)g.NG * g.nsl * g.maxp * (MODE == GM_SWIGLU ? 2 : 1) * (NSG * 16) > p.mbpart_floats || g.NG > p.mbcnt_n) return false;
  lds = (size_t)g.csm * per_chunk + rope_b + (p.rms_w ? kMbWaves * 16 : 0);  // (+ the norm's partial sums)
  return true;
}

template <int MODE, int NSG, bool NT>
inline hipError_t mb_launch_t(const GemvParams& p, const MbGeom& g, size_t lds, hipStream_t s) {
  static std::mutex mu;
  static std::vector<int> done;  // devices with the raised dynamic-LDS limit
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    std::lock_guard<std::mutex> lock(mu);
    bool have = false;
    for (int d : done) have = have || d == dev;
    if (!have) {
      e = hipFuncSetAttribute((const void*)gemv_mb_kernel<MODE, NSG, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, mb_lds_budget());
      if (e != hipSuccess) return e;
      done.push_back(dev);
    }
  }
  hipLaunchKernelGGL((gemv_mb_kernel<MODE, NSG, NT>), dim3(g.nsl * g.bps), dim3(kMbWaves * 64), lds, s, p, g);
  return hipGetLastError();
}

template <int MODE>
inline hipError_t mb_launch(const GemvParams& p, const MbGeom& g, size_t lds, hipStream_t s, bool nt) {
  if (p.nb <= 4) return nt ? mb_launch_t<MODE, 1, true>(p, g, lds, s) : mb_launch_t<MODE, 1, false>(p, g, lds, s);
  return nt ? mb_launch_t<MODE, 2, true>(p, g, lds, s) : mb_launch_t<MODE, 2, false>(p, g, lds, s);
}

}  // namespace tl
