// attn_wo.hip — one launch for a layer's attention AND its Wo projection + residual (fp32, the
// batched multi-launch step at 5..8 sequences, where the two ran as separate launches).
//
// Why: at batch 8 the attention launch is latency-bound (~11 us per layer at 7B for ~33 MB of
// K/V) while HBM idles, and the Wo launch that follows pays its own ramp, tail and split-K
// reduction (~18 us for 67 MB, 3.7 TB/s).  Here every workgroup first ISSUES its share of Wo's
// weights (two 4-KiB groups per wave), then runs its attention units, then waits for exactly the
// heads its K range needs and streams the rest of its Wo rows: the first Wo bytes land while the
// attention runs, and one launch boundary per layer disappears.
//
// Grid: one 512-thread workgroup (8 waves) per 16-row tile of Wo — dim / 16 of them, at most one
// per CU, so every workgroup is resident at once (the launcher checks the tile count against the
// CU count) — and each wave owns K / 8 of the row (4 heads at 7B).  No split-K across workgroups:
// the 8 wave partials are summed in LDS in a fixed order (deterministic).
// Hand-off (MI355X_MICROARCH.md § visibility, Valid forms table row 1, one workgroup per CU): the
// wave that finishes head (b, h) stores it sc1, drains, and adds 1 to done[h]; a Wo wave polls
// done[h] with sc1 loads until it reads nb and then loads the head's columns with sc1 loads.
// Every wait is bounded: a give-up sets err (the host then disables this launch and re-runs the
// call on the two-launch step).  The workgroup whose "past every wait" ticket is the last resets
// done[] and the ticket, so the next launch starts from zero.
#include "attention.hpp"
#include "gemv_mfma.hpp"
#include "attn_wo.hpp"

namespace tl {

constexpr int kAwWaves = 8;
constexpr unsigned kAwSpinLimit = 1u << 16;  // ~65 ms of polling; a normal wait is a few us

template <int HS, int CH, int XI>
__global__ void __launch_bounds__(kAwWaves * 64) attn_wo_kernel(AttnWoParams P) {
  keep_implicit_args();
  constexpr int W = kAwWaves;
  constexpr int U = kMfmaU;       // 16-k steps per group (64 floats of K)
  constexpr int LPR = U * 4;      // lanes per row in a load: 256-B runs
  constexpr int RPI = 64 / LPR;   // rows per load instruction
  constexpr int NI = 16 / RPI;    // load instructions per 16-row tile
  constexpr int STR = U * 16 + 4; // LDS row stride (padded: conflict-free both ways)
  constexpr int TILE = 16 * STR;
  static_assert(XI >= 1 && XI <= NI, "live activation load instructions");
  __shared__ __attribute__((aligned(16))) float lds[W * 2 * TILE];
  __shared__ float s_red[256];
  __shared__ unsigned s_last;
  const GemvParams& p = P.g;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int lr = lane / LPR, lc = lane % LPR;
  const int K = p.K, nb = p.nb;
  const int tile = blockIdx.x;
  const int n_rows = p.n_items;
  const long long Kl = K;

  // this wave's K run: 16-k steps [ws, ws + per), ng groups of U steps (the launcher checks
  // K % (16 * W * U) == 0)
  const int per = (K >> 4) / W;
  const int ws = wave * per, ng = per / U;
  const float* wrow[NI];
#pragma unroll
  for (int v = 0; v < NI; ++v) {
    int R = tile * 16 + RPI * v + lr;
    R = R < n_rows ? R : n_rows - 1;
    wrow[v] = p.W0 + R * Kl;
  }
  auto wload = [&](f4 (&t)[NI], int g) {
    const int k = 16 * (ws + g * U) + 4 * lc;
#pragma unroll
    for (int v = 0; v < NI; ++v) t[v] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(wrow[v] + k));
  };
  // activations (the attention output of this launch): sc1 loads only
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(p.x);
  auto xload = [&](f4 (&t)[XI], int g) {
    const int k = 16 * (ws + g * U) + 4 * lc;
#pragma unroll
    for (int v = 0; v < XI; ++v) {
      const int r = RPI * v + lr;
      const f4 x = ld4_sc1(xr, (unsigned)(((long long)(r < nb ? r : 0) * p.x_stride + k) * 4));
      t[v] = r < nb ? x : f4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // 1. the first two groups of this wave's Wo weights, in flight through the attention
  f4 wa[NI], wb[NI];
  if (ng > 0) wload(wa, 0);
  if (ng > 1) wload(wb, 1);

  // 2. attention units (one wave each), numbered as attn_wave_kernel's blocks
  if (!(P.fault && blockIdx.x == 0))
    for (int u = blockIdx.x * W + wave; u < P.units; u += gridDim.x * W) attn_unit<HS, CH>(P.aw, u, lane);

  // 3. the heads this wave's K run covers, complete for all nb sequences (bounded wait)
  {
    const int h0 = (16 * ws) / HS, h1 = (16 * (ws + per) - 1) / HS;
    for (int h = h0; h <= h1; ++h) {
      for (unsigned spins = 0;; ++spins) {
        const unsigned v = __hip_atomic_load(as_g32(P.done + h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= (unsigned)nb) break;
        if ((spins & 255) == 255 &&
            (spins > kAwSpinLimit || __hip_atomic_load(as_g32(P.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          __hip_atomic_store(as_g32(P.err), 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }

  // 4. Wo: 16 rows x 16 sequences per wave on the matrix cores, two groups in flight
  float* wt = lds + wave * 2 * TILE;  // weight tile; activation tile right after it
  float* xt = wt + TILE;
#pragma unroll
  for (int v = XI; v < NI; ++v) *reinterpret_cast<f4*>(xt + (RPI * v + lr) * STR + 4 * lc) = f4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const f4 (&w)[NI], const f4 (&x)[XI]) {
#pragma unroll
    for (int v = 0; v < NI; ++v) *reinterpret_cast<f4*>(wt + (RPI * v + lr) * STR + 4 * lc) = w[v];
#pragma unroll
    for (int v = 0; v < XI; ++v) *reinterpret_cast<f4*>(xt + (RPI * v + lr) * STR + 4 * lc) = x[v];
    asm volatile("" ::: "memory");  // same-wave LDS ops execute in order
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 xv = *reinterpret_cast<const f4*>(xt + i * STR + 16 * u + 4 * q);
      const f4 a = *reinterpret_cast<const f4*>(wt + i * STR + 16 * u + 4 * q);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, xv.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, xv.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, xv.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, xv.w, acc, 0, 0, 0);
    }
    asm volatile("" ::: "memory");
  };
  f4 xa[XI], xb[XI];
  if (ng > 0) xload(xa, 0);
  if (ng > 1) xload(xb, 1);
  for (int g = 0; g < ng; g += 2) {
    mma(wa, xa);
    if (g + 2 < ng) {
      wload(wa, g + 2);
      xload(xa, g + 2);
    }
    if (g + 1 < ng) {
      mma(wb, xb);
      if (g + 3 < ng) {
        wload(wb, g + 3);
        xload(xb, g + 3);
      }
    }
  }

  // 5. wave partials summed in wave order, residual add, this tile's sums of squares
  __syncthreads();  // the staging tiles become the partial buffer [W][256]
  float* red = lds;
#pragma unroll
  for (int e = 0; e < 4; ++e) red[wave * 256 + (4 * q + e) * 16 + i] = acc[e];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int t = threadIdx.x, row = t >> 4, j = t & 15;
    const int R = tile * 16 + row;
    float v = red[t];
#pragma unroll
    for (int w = 1; w < W; ++w) v += red[w * 256 + t];
    float sq = 0.f;
    if (j < nb && R < n_rows) {
      float* y = p.y + (long long)j * p.y_stride + R;
      const float nv = __fadd_rn(*y, v);
      *y = nv;
      sq = __fmul_rn(nv, nv);
    }
    s_red[t] = sq;
  }
  __syncthreads();
  if (p.ssq_out && threadIdx.x < nb) {  // rows in order, as gemv_mfma_kernel's residual epilogue
    float v = 0.f;
    for (int r = 0; r < 16; ++r) v = __fadd_rn(v, s_red[r * 16 + threadIdx.x]);
    p.ssq_out[(long long)threadIdx.x * p.ssq_nt + tile] = v;
  }

  // 6. every wave of this workgroup is past its waits: the last workgroup re-arms the counters
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(P.blocks, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (s_last) {
    for (int h = threadIdx.x; h < P.aw.a.n_heads; h += blockDim.x)
      __hip_atomic_store(P.done + h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(P.blocks, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

bool attn_wo_ok(int nb, int dim, int n_heads, int head_size, int ncu) {
  const int tiles = (dim + 15) / 16;
  return nb >= 5 && nb <= 8 && (head_size == 64 || head_size == 128) && dim == n_heads * head_size &&
         dim % (16 * kAwWaves * kMfmaU) == 0 && tiles <= ncu;
}

hipError_t launch_attn_wo(const AttnWoParams& P, hipStream_t s) {
  const int tiles = (P.g.n_items + 15) / 16;
  const dim3 grid(tiles), blk(kAwWaves * 64);
  // nb 5..8: two activation load instructions (4 rows each)
  if (P.aw.a.head_size == 64) hipLaunchKernelGGL((attn_wo_kernel<64, 32, 2>), grid, blk, 0, s, P);
  else hipLaunchKernelGGL((attn_wo_kernel<128, 32, 2>), grid, blk, 0, s, P);
  return hipGetLastError();
}

}  // namespace tl
