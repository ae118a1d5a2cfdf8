// q8_dispatch.hpp — launcher of the int8 streaming GEMV (gemv_q8.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include "gemv.hpp"

namespace tl {
bool gemv_q8_fast_ok(const GemvParams& p);
// Enqueue the Q8_0 GEMV with epilogue `mode`; p.Q*/p.S*/p.gs describe the weights.
hipError_t launch_gemv_q8(int mode, const GemvParams& p, hipStream_t stream, bool nt);
bool q8_swiglu_quant_ok(int nb, int gs, int K, int n_items);
}  // namespace tl
