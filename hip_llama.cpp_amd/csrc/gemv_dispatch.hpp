// gemv_dispatch.hpp — host-side launcher for gemv.hpp (picks the NB instantiation,
// the LDS chunk and the grid; splits batches above 16 into groups of 16).
#pragma once
#include <hip/hip_runtime.h>
#include "gemv.hpp"

namespace tl {

// Launch shape of the streaming kernel.  ipw: items per wave; waves: waves per block;
// pf: prefetch the first row before staging; nt: non-temporal weight loads;
// lds_floats: activation staging budget (floats) per block.
struct GemvCfg {
  int ipw = 1;
  int waves = 4;
  bool pf = true;
  bool nt = true;
  int lds_floats = 16384;
};

// Tuned default for a shape (see tools/gemv_sweep.py and DESIGN.md §GEMV).
GemvCfg gemv_default_cfg(int mode, int n_items, int K, int nb, bool nt);

// True when the streaming kernel can take this shape: rows are a whole number of
// 1-KiB wave-loads and every base pointer is 16-B aligned.
bool gemv_fast_ok(const GemvParams& p);

// True when launch_gemv runs p (every 16-sequence group of it) on the matrix-core or the
// register-resident kernel.  Only those two read ssq_in / write ssq_out, so the decoder carries
// RMSNorm sums from a residual launch to the next normed launch only when every producer passes
// this (launch_mode and forward.hip both call it; gemv_launch.hpp matrix_path_ok).
bool gemv_matrix_path(const GemvParams& p);

// Enqueue y = W x' for p.nb sequences on `stream` with epilogue `mode`.
hipError_t launch_gemv(int mode, const GemvParams& p, hipStream_t stream, bool nt);
hipError_t launch_gemv_cfg(int mode, const GemvParams& p, hipStream_t stream, const GemvCfg& cfg);

}  // namespace tl
