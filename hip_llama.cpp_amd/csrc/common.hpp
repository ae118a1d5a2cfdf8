// common.hpp — gfx950 device helpers shared by every kernel in the library.
//
// Wave64 everywhere: reductions are xor-butterflies over 64 lanes; blocks are
// multiples of 64 threads.  Nothing here is a CUDA idiom recompiled: there is
// no 32-lane warp anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TL_DEVICE __device__ __forceinline__

// IEEE single roundings on this toolchain (clang __clang_hip_math.h): __fadd_rn / __fmul_rn /
// __fsub_rn are plain + * - (the Makefile's -ffp-contract=off keeps a*b+c two roundings) and
// __fdiv_rn and sqrtf are correctly rounded, but __fsqrt_rn is the native v_sqrt_f32 (~1 ulp):
// never use it where the reference's sqrtf must be matched.

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

// DPP lane moves (VALU, no LDS round trip; GFX9 encodings): quad_perm [1,0,3,2] = 0xB1,
// quad_perm [2,3,0,1] = 0x4E, row_half_mirror = 0x141, row_mirror = 0x140.  The __shfl_xor
// forms above lower to ds_bpermute (an LDS round trip per step); these are for latency-bound
// reductions on the decode critical path.  All 64 lanes must be active.
template <int CTRL>
TL_DEVICE float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false)); }
TL_DEVICE float lane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
// Sum over each 16-lane row; every lane of the row holds it.
TL_DEVICE float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
TL_DEVICE float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
// Wave-uniform sum / max: row reductions by DPP, the four rows combined through SGPRs.
TL_DEVICE float wave_sum_u(float v) {
  v = row16_sum(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
TL_DEVICE float wave_max_u(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// runq.c:145-171 activation quantisation, scalar pieces (gemv_q8.hpp q8_pack, the persistent
// step's staging and its attention output, the thaBLAS_q8_quantize_batch op).
TL_DEVICE int q8_round(float v) {
  // C round(): half away from zero; NaN (all-zero group, scale 0) -> 0 like the x86 reference
  const float r = roundf(v);
  return r != r ? 0 : (int)r;
}
// q = x / scale bit-identical to the IEEE division, without one: r = RN(1/scale),
// y = RN(x r), the exact remainder e = x - y scale (FMA), RN(y + r e) = RN(x / scale)
// (Markstein; equal on 1.28e9 values, tools/probes/q8div.c), valid away from under/overflow:
// scales outside [1e-30, 1e30] (an all-zero group: scale 0 -> NaN -> code 0) divide.
TL_DEVICE bool q8_fast_scale(float scale) { return scale >= 1e-30f && scale <= 1e30f; }
TL_DEVICE float q8_div_fast(float x, float scale, float r) {
  const float y = __fmul_rn(x, r);
  return __builtin_fmaf(__builtin_fmaf(-y, scale, x), r, y);
}
// The code: with scale = max|group| / 127, |x / scale| <= 127 (1 + 2^-23), and for |y| <= 200
// round-half-away-from-zero is the truncation of y + copysign(pred(0.5), y) (all 2.26e9 such
// floats: tools/probes/q8round.c).
TL_DEVICE int q8_code_fast(float x, float scale, float r) {
  const float y = q8_div_fast(x, scale, r);
  return (int)__fadd_rn(y, __builtin_copysignf(0.49999997f, y));
}
TL_DEVICE int q8_code(float x, float scale) {
  return q8_fast_scale(scale) ? q8_code_fast(x, scale, __fdiv_rn(1.0f, scale)) : q8_round(__fdiv_rn(x, scale));
}

// Exact int32 sum over aligned groups of N = 2, 4 or 8 lanes (every lane of a group gets
// it): quad DPP steps, then row_half_mirror (after the quad steps the two quads of a half-row
// each hold their sum, so the mirror pairs them).
template <int N>
TL_DEVICE int lane_group_sum_i(int v) {
  static_assert(N == 2 || N == 4 || N == 8, "group of 2, 4 or 8 lanes");
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
  if constexpr (N >= 4) v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
  if constexpr (N >= 8) v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);
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

// ---- write-through (sc1) hand-off accesses (MI355X_MICROARCH.md § visibility, Valid forms
// table row 1): data handed to another workgroup INSIDE a launch is stored sc1 and every
// load of it is an sc1 global/buffer load (never flat), so no release/acquire fence is
// needed.  Global address-space pointers keep the compiler from emitting flat_ accesses.
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
constexpr int kSC1 = 16;  // buffer-op aux bit: sc1

TL_DEVICE gu32* as_g32(const void* p) { return (gu32*)(uintptr_t)p; }
TL_DEVICE gu64* as_g64(const void* p) { return (gu64*)(uintptr_t)p; }
TL_DEVICE float ld1_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(as_g32(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
TL_DEVICE void st1_sc1(float* p, float v) {
  __hip_atomic_store(as_g32(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TL_DEVICE void st2_sc1(float* p, float a, float b) {  // p 8-byte aligned
  const unsigned long long v = ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a);
  __hip_atomic_store(as_g64(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TL_DEVICE unsigned long long ld8_sc1(const unsigned long long* p) {
  return __hip_atomic_load(as_g64(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TL_DEVICE void st8_sc1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(as_g64(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Keeps the hidden (implicit) kernel arguments in a kernel's kernarg segment.  A kernel that
// never reads them gets a segment of its explicit arguments only (gemv_mfma_kernel: 344 B instead
// of 600), and rocprofv3's counter-collection dispatch hook then faults on the host reading past
// it (SIGSEGV at a page boundary inside hipLaunchKernel, profiles/r03/pmc_sigsegv_diagnosis.md).
TL_DEVICE void keep_implicit_args() { asm volatile("" ::"s"(__builtin_amdgcn_implicitarg_ptr())); }
// Buffer resource over [base, base + 2 GiB); `base` must be wave-uniform.
TL_DEVICE __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}
TL_DEVICE f4 ld4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kSC1));
}
TL_DEVICE void st4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off, f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, byte_off, 0, kSC1);
}
// N consecutive floats (N = 1, 2, 4) at byte offset `off`, sc1.
template <int N>
TL_DEVICE void ldn_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, float* out) {
  if constexpr (N == 1) {
    out[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSC1));
  } else if constexpr (N == 2) {
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSC1);
    out[0] = __uint_as_float(v.x); out[1] = __uint_as_float(v.y);
  } else {
    const f4 v = ld4_sc1(r, off);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  }
}
// ---- data-carried hand-offs (MI355X_MICROARCH.md § visibility, R2 granules): one float
// travels as an 8-byte {value, tag} granule written by ONE 8-byte sc1 store (or both halves
// of a 16-byte sc1 store); the consumer re-reads until the tag matches.  No fence, no
// drain, no flag.  Tags are never 0 (buffers start zeroed).
TL_DEVICE unsigned long long gran(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | __float_as_uint(v);
}
constexpr unsigned kGranSpinLimit = 1u << 18;
// Pause between re-polls of a late granule: 64 cycles; with lng (the persistent step's input
// sweeps of a large model, whose phases last 6-60 us) 512 after the second re-poll and 2048 after
// the sixth, since hundreds of waves re-polling every ~1 us load the fabric the weight stream uses
// (7B fp32 +1.2%, int8 +1.3%; a model whose hand-offs are 1-3 us loses from the added latency:
// 110M -3.5% with every wait long, profiles/r05/gran_poll_ab.txt).
TL_DEVICE void gran_backoff(unsigned spins, bool lng) {
  if (lng && spins >= 6) __builtin_amdgcn_s_sleep(32);
  else if (lng && spins >= 2) __builtin_amdgcn_s_sleep(8);
  else __builtin_amdgcn_s_sleep(1);
}
// Bounded wait for one granule; a give-up (or an error already flagged) sets/keeps *err = 2.
TL_DEVICE float gran_wait(const unsigned long long* g, unsigned tag, unsigned* err, bool lng = false) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned long long x = ld8_sc1(g);
    if ((unsigned)(x >> 32) == tag) return __uint_as_float((unsigned)x);
    if ((spins & 255) == 255 &&
        (spins > kGranSpinLimit || __hip_atomic_load(as_g32(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(as_g32(err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return __uint_as_float((unsigned)x);
    }
    gran_backoff(spins, lng);
  }
}
// Four consecutive granules (a float4) at byte offset off (32-B aligned) of resource r.
TL_DEVICE bool gran4_ok(v4u a, v4u b, unsigned tag) {
  return a.y == tag && a.w == tag && b.y == tag && b.w == tag;
}
TL_DEVICE f4 gran4_val(v4u a, v4u b) {
  return f4{__uint_as_float(a.x), __uint_as_float(a.z), __uint_as_float(b.x), __uint_as_float(b.z)};
}
TL_DEVICE v4u ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1);
}
TL_DEVICE f4 gran_wait4(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned tag, unsigned* err, bool lng = false) {
  for (unsigned spins = 0;; ++spins) {
    const v4u a = ld16_sc1(r, off), b = ld16_sc1(r, off + 16);
    if (gran4_ok(a, b, tag)) return gran4_val(a, b);
    if ((spins & 255) == 255 &&
        (spins > kGranSpinLimit || __hip_atomic_load(as_g32(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(as_g32(err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return gran4_val(a, b);
    }
    gran_backoff(spins, lng);
  }
}
// Two granules {a, b} with one 16-byte sc1 store (off 16-B aligned).
TL_DEVICE void st_gran2(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned tag, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b128(v4u{__float_as_uint(a), tag, __float_as_uint(b), tag}, r, off, 0, kSC1);
}

template <int N>
TL_DEVICE void stn_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, const float* v) {
  if constexpr (N == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), r, off, 0, kSC1);
  } else if constexpr (N == 2) {
    __builtin_amdgcn_raw_buffer_store_b64(v2u{__float_as_uint(v[0]), __float_as_uint(v[1])}, r, off, 0, kSC1);
  } else {
    st4_sc1(r, off, f4{v[0], v[1], v[2], v[3]});
  }
}

}  // namespace tl
