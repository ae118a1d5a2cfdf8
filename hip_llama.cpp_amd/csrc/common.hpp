// common.hpp — gfx950 device helpers shared by every kernel in the library.
//
// Wave64 everywhere: reductions are xor-butterflies over 64 lanes; blocks are
// multiples of 64 threads.  Nothing here is a CUDA idiom recompiled: there is
// no 32-lane warp anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TL_DEVICE __device__ __forceinline__

namespace tl {

constexpr int kWave = 64;

typedef float f4 __attribute__((ext_vector_type(4)));

TL_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

TL_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over the first `width` lanes groups (width power of two <= 64): lanes
// [g*width, (g+1)*width) end up holding their group's total.
template <int WIDTH>
TL_DEVICE float group_sum(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum; `red` must hold >= blockDim.x/64 floats of LDS.  Every
// thread returns the total.  Contains two barriers.
TL_DEVICE float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  __syncthreads();
  return t;
}

TL_DEVICE float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < nw; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Streamed-once weight load.  NT=true sets the non-temporal bit (global_load ... nt):
// once-read decode weights that would otherwise evict the KV cache / activations
// from L2 and the Infinity Cache (MI355X_MICROARCH.md, row nt-weights).
template <bool NT>
TL_DEVICE f4 load_w4(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

TL_DEVICE float dot4(f4 a, f4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  acc = fmaf(a.w, b.w, acc);
  return acc;
}

// Order-preserving float -> uint32 key (total order, -0 < +0; NaN sorts high).
TL_DEVICE uint32_t float_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Packed (value, index) for a 64-bit atomicMax argmax that resolves ties to the
// LOWEST index, like sample_argmax's strict '>' (reference src/llama.cpp:275-286).
TL_DEVICE unsigned long long argmax_pack(float v, int idx) {
  return ((unsigned long long)float_key(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}

}  // namespace tl
