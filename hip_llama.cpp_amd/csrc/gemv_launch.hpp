// gemv_launch.hpp — launch templates of the streaming GEMV, instantiated one epilogue
// mode per translation unit (gemv_m*.hip) so the variants compile in parallel.
#pragma once
#include <stdlib.h>
#include "gemv_dispatch.hpp"
#include "gemv_mfma.hpp"
#include "gemv_rr.hpp"

namespace tl {

// Smallest batch that takes the matrix-core GEMV.
constexpr int kMfmaMinNb = 4;

// Split K across blocks when the row tiles alone leave CUs idle: msplit = target / tiles,
// at least 2 steps per wave per split; needs the decoder's mpart/mcnt scratch, sized for
// mfma_target_blocks() tiles x splits.
// depth2: aim for half the blocks (the residual launch with K <= 4096, i.e. Wo: in the 7B B=8 step
// 18.3 us at 2 blocks per CU against 19.9-20.3 at 3-4; W2, QKV and W1/W3 keep 4, and 6-8 lost
// everywhere: tools/job_r02_depth.sh).
inline void mfma_splits(GemvParams& p, int tiles, bool depth2 = false) {
  const int nsteps = p.K >> 4;
  int ms = p.mpart && p.mcnt ? mfma_target_blocks() / (depth2 ? 2 : 1) / tiles : 1;
  const int cap = nsteps / (2 * kMfmaWaves);
  if (ms > cap) ms = cap;
  if (ms < 1) ms = 1;
  p.msteps = (nsteps + ms - 1) / ms;
  p.msplit = (nsteps + p.msteps - 1) / p.msteps;
}

// The register-resident batched GEMV (gemv_rr.hpp) when the rows fill every CU and a block's rows
// fit its LDS partials, for up to kRrMaxNb sequences (7B fp32 B=4: 740 vs 726 tok/s on the
// matrix-core kernel; at 8 sequences it measured slower, 1255-1328 vs 1408-1433,
// profiles/jobs/job_r02_t.sh).  Same ssq contract as the matrix-core kernel, so the two mix freely
// within a step.
constexpr int kRrMaxNb = 4;

inline int rr_grid() {
  static const int v = [] {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return ncu;
  }();
  return v;
}

template <int MODE>
inline bool rr_ok(const GemvParams& p) {
  const int G = rr_grid();
  if (p.nb > kRrMaxNb || p.nb > 8 || (p.K & 255) || (p.x_stride & 3)) return false;
  constexpr int RPI = RowsPerItem<MODE>::v;
  const long long rows = (long long)p.n_items * RPI;
  if (rows < 16LL * G) return false;
  const int per = MODE == GM_RESID ? 16 * (((p.n_items + 15) / 16 + G - 1) / G)
                                   : (p.n_items + G - 1) / G * RPI;
  return per <= kRrMaxRows;
}

template <int MODE, int NB, int IPW, bool NT, int WAVES, bool PF>
inline void launch_one(const GemvParams& p, hipStream_t s, int kc, size_t lds) {
  const int per_block = WAVES * IPW;
  const int blocks = (p.n_items + per_block - 1) / per_block;
  hipLaunchKernelGGL((gemv_kernel<MODE, NB, IPW, NT, WAVES, PF>), dim3(blocks), dim3(WAVES * 64), lds, s, p, kc);
}

// Variant table: NB = 1 gets the full (ipw, waves, pf, nt) space for tuning; larger NB the
// (ipw, pf, nt) space at 4 waves.
template <int MODE, int NB>
inline hipError_t launch_nb(const GemvParams& p, hipStream_t s, const GemvCfg& c) {
  int kc = (c.lds_floats / NB) & ~255;
  if (kc < 256) kc = 256;
  if (kc > p.K) kc = p.K;
  const size_t lds = 320 + (size_t)NB * kc * 4;
  if (p.n_items <= 0) return hipSuccess;
#define TL_L(IPW, NT, W, PF) launch_one<MODE, NB, IPW, NT, W, PF>(p, s, kc, lds)
  const int ipw = c.ipw >= 2 ? 2 : 1;
  bool done = false;
  if constexpr (NB == 1) {
    if (c.waves == 8) {
      done = true;
      if (ipw == 1) {
        if (c.nt) { if (c.pf) TL_L(1, true, 8, true); else TL_L(1, true, 8, false); }
        else { if (c.pf) TL_L(1, false, 8, true); else TL_L(1, false, 8, false); }
      } else {
        if (c.nt) { if (c.pf) TL_L(2, true, 8, true); else TL_L(2, true, 8, false); }
        else { if (c.pf) TL_L(2, false, 8, true); else TL_L(2, false, 8, false); }
      }
    }
  }
  if (!done) {
    if (ipw == 1) {
      if (c.nt) { if (c.pf) TL_L(1, true, 4, true); else TL_L(1, true, 4, false); }
      else { if (c.pf) TL_L(1, false, 4, true); else TL_L(1, false, 4, false); }
    } else {
      if (c.nt) { if (c.pf) TL_L(2, true, 4, true); else TL_L(2, true, 4, false); }
      else { if (c.pf) TL_L(2, false, 4, true); else TL_L(2, false, 4, false); }
    }
  }
#undef TL_L
  return hipGetLastError();
}

// The shape half of the matrix-core / register-resident selection (the norm half is the
// prologue test in launch_mode): whole 1-KiB wave-loads, 16-float k steps, aligned rows, and
// at least kMfmaMinNb sequences in every 16-sequence group launch_mode cuts.
inline bool matrix_path_ok(const GemvParams& p) {
  if (p.n_items <= 0 || p.nb <= 0 || !gemv_fast_ok(p) || (p.K & 15) || (p.x_stride & 3)) return false;
  for (int b0 = 0; b0 < p.nb; b0 += 16)
    if ((p.nb - b0 < 16 ? p.nb - b0 : 16) < kMfmaMinNb) return false;
  return true;
}

template <int MODE>
inline hipError_t launch_mode(const GemvParams& p0, hipStream_t s, const GemvCfg* cfg, bool nt) {
  if (p0.n_items <= 0 || p0.nb <= 0) return hipSuccess;
  if (!gemv_fast_ok(p0)) {
    const int blocks = (p0.n_items + 3) / 4;
    hipLaunchKernelGGL((gemv_generic_kernel<MODE>), dim3(blocks, p0.nb), dim3(256), 0, s, p0);
    return hipGetLastError();
  }
  for (int b0 = 0; b0 < p0.nb; b0 += 16) {
    GemvParams p = p0;
    p.nb = p0.nb - b0 < 16 ? p0.nb - b0 : 16;
    if (b0) {
      if (p.x) p.x += b0 * p.x_stride;
      if (p.tok) p.tok += b0;
      if (p.x_out) p.x_out += b0 * p.x_stride;
      if (p.pos) p.pos += b0;
      if (MODE == GM_STORE) p.y_off += (long long)b0 * p.y_stride;
      else p.y += (long long)b0 * p.y_stride;
      if (p.kc) p.kc += (long long)b0 * p.kv_b_stride;
      if (p.ssq_out) p.ssq_out += (long long)b0 * p.ssq_nt;
      if (p.ssq_in) p.ssq_in += (long long)b0 * p.ssq_nt;
      if (p.vc) p.vc += (long long)b0 * p.kv_b_stride;
    }
    hipError_t e;
    const GemvCfg c = cfg ? *cfg : gemv_default_cfg(MODE, p.n_items, p.K, p.nb, nt);
    const bool matrix = !cfg && matrix_path_ok(p) &&
                        ((!p.rms_w && !p.tok) || p.xn || (p.rms_w && p.ssq_in && !p.tok));
    if (!matrix) p.ssq_in = nullptr;  // the streaming kernels normalise from x themselves
    if (matrix) {
      // several sequences: the matrix-core kernel (gemv_mfma.hpp); an embedding prologue, or a
      // norm whose sums of squares the previous launch did not leave (ssq_in), runs once into
      // the scratch rows first; otherwise the kernel applies the norm itself
      if (p.tok || (p.rms_w && !p.ssq_in)) {
        p.ssq_in = nullptr;
        hipLaunchKernelGGL(gemv_prenorm_kernel<0>, dim3(p.nb), dim3(256), 0, s, p);
        p.x = p.xn;
        p.x_stride = p.K;
        p.rms_w = nullptr;
        p.tok = nullptr;
        p.x_out = nullptr;
      }
      if (rr_ok<MODE>(p)) {
        const dim3 g(rr_grid()), b(kRrWaves * 64);
        if (p.nb <= 4) hipLaunchKernelGGL((gemv_rr_kernel<MODE, 4, 2, 4>), g, b, 0, s, p);
        else hipLaunchKernelGGL((gemv_rr_kernel<MODE, 8, 2, 4>), g, b, 0, s, p);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
      const int rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
      const int tiles = (rows + 15) / 16;
      mfma_splits(p, tiles, MODE == GM_RESID && p.K <= 4096);
      const dim3 grid(tiles * p.msplit);
      // activation load instructions per 16-row group (4 rows each): only those with live rows
      const dim3 blk(kMfmaWaves * 64);
      if (p.nb <= 8) {
        if (c.nt) hipLaunchKernelGGL((gemv_mfma_kernel<MODE, true, 2>), grid, blk, 0, s, p);
        else hipLaunchKernelGGL((gemv_mfma_kernel<MODE, false, 2>), grid, blk, 0, s, p);
      } else {
        if (c.nt) hipLaunchKernelGGL((gemv_mfma_kernel<MODE, true, 4>), grid, blk, 0, s, p);
        else hipLaunchKernelGGL((gemv_mfma_kernel<MODE, false, 4>), grid, blk, 0, s, p);
      }
      e = hipGetLastError();
    } else if (p.nb == 1) e = launch_nb<MODE, 1>(p, s, c);
    else if (p.nb == 2) e = launch_nb<MODE, 2>(p, s, c);
    else if (p.nb <= 4) e = launch_nb<MODE, 4>(p, s, c);
    else if (p.nb <= 8) e = launch_nb<MODE, 8>(p, s, c);
    else e = launch_nb<MODE, 16>(p, s, c);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tl
