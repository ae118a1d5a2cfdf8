// gemv_dispatch.hpp — host-side launcher for gemv.hpp (picks the NB instantiation,
// the LDS chunk and the grid; splits batches above 16 into groups of 16).
#pragma once
#include <hip/hip_runtime.h>
#include "gemv.hpp"

namespace tl {

// True when the streaming kernel can take this shape: rows are a whole number of
// 1-KiB wave-loads and every base pointer is 16-B aligned.
bool gemv_fast_ok(const GemvParams& p);

// Enqueue y = W x' for p.nb sequences on `stream` with epilogue `mode`.
// nt: non-temporal weight loads.  Returns hipSuccess or the launch error.
hipError_t launch_gemv(int mode, const GemvParams& p, hipStream_t stream, bool nt);

}  // namespace tl
