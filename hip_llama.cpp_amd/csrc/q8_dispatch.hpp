// q8_dispatch.hpp — launcher of the int8 streaming GEMV (gemv_q8.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include "gemv.hpp"

namespace tl {
bool gemv_q8_fast_ok(const GemvParams& p);
// Enqueue the Q8_0 GEMV with epilogue `mode`; p.Q*/p.S*/p.gs describe the weights.
hipError_t launch_gemv_q8(int mode, const GemvParams& p, hipStream_t stream, bool nt);
// The int8 step in runq's arithmetic order for 1..8 sequences (q8_exact.hip): shape check, the
// GEMV (quantises its input first unless p.xq_ready; p.xq / p.xqs scratch required) and the
// attention (scores through att [B][H][S], output fp32 into a.out).
bool q8_exact_ok(int gs, int dim, int hidden, int hs, int seq_len);
// Kernel attributes of the exact int8 launches on the current device (decoder creation).
hipError_t q8_exact_prepare();
hipError_t launch_gemv_q8_exact(int mode, const GemvParams& p, hipStream_t stream, bool nt);
struct AttnParams;
hipError_t launch_attn_q8_exact(const AttnParams& a, int B, float* att, hipStream_t stream);
}  // namespace tl
