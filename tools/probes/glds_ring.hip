// glds_ring.hip — does an LDS-DMA loader ring stream fp32 decode weights faster than register
// streaming on gfx950?  Each CU reads its own contiguous 4 MiB slab of a 1 GiB matrix once and
// dots it with an LDS-resident 4096-float vector (one "row" = 16 KiB = one ring slot).
//   A: 1 loader wave (16 x global_load_lds_dwordx4 per slot, nt) + NC consumer waves, NSLOT-deep ring
//   B: register streaming, 8 waves, 2 x 8 KiB slots in flight per wave (the persistent kernel's form)
// hipcc --offload-arch=gfx950 -O3 -o glds_ring glds_ring.hip && ./glds_ring
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int SLOTF = 4096;  // floats per slot (16 KiB)

__device__ inline float dot4(f4 a, f4 b, float c) {
  c = fmaf(a.x, b.x, c); c = fmaf(a.y, b.y, c); c = fmaf(a.z, b.z, c); return fmaf(a.w, b.w, c);
}
__device__ inline float wsum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NC, int NSLOT, int DEPTH, int NL>
__global__ void __launch_bounds__((NC + NL) * 64) ring_kernel(const float* W, int slots_per_cu, const float* x, float* out) {
  __shared__ __attribute__((aligned(16))) float ring[NSLOT][SLOTF];
  __shared__ __attribute__((aligned(16))) float xs[SLOTF];
  __shared__ unsigned full[NSLOT], freed[NSLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < SLOTF; i += blockDim.x) xs[i] = x[i];
  if (threadIdx.x < NSLOT) { full[threadIdx.x] = 0; freed[threadIdx.x] = 0; }
  __syncthreads();
  const float* base = W + (size_t)blockIdx.x * slots_per_cu * SLOTF;
  if (wave < NL) {
    // loader wave `wave`: slots wave, wave + NL, ...; DEPTH of its own slots in flight
    for (int j = 0; j * NL + wave < slots_per_cu + (DEPTH - 1) * NL; ++j) {
      const int s = j * NL + wave;
      if (s < slots_per_cu) {
        const int slot = s % NSLOT;
        const unsigned gen = s / NSLOT;  // times this slot was filled before
        while (__hip_atomic_load(&freed[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
          __builtin_amdgcn_s_sleep(1);
        const float* src = base + (size_t)s * SLOTF;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i * 256 + lane * 4),
                                           (__attribute__((address_space(3))) void*)(&ring[slot][i * 256]), 16, 0, 2);
      }
      // publish this wave's slot DEPTH - 1 back once its 16 loads have landed
      const int ps = s - (DEPTH - 1) * NL;
      if (ps >= 0 && ps < slots_per_cu) {
        if (s < slots_per_cu) {
          if constexpr (DEPTH == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else if constexpr (DEPTH == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          else if constexpr (DEPTH == 3) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) __hip_atomic_store(&full[ps % NSLOT], (unsigned)(ps / NSLOT + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  } else {
    const int c = wave - NL;
    float acc = 0.f;
    for (int s = c; s < slots_per_cu; s += NC) {
      const int slot = s % NSLOT;
      const unsigned gen = s / NSLOT + 1;
      while (__hip_atomic_load(&full[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
      const f4* r = reinterpret_cast<const f4*>(ring[slot]);
      const f4* xv = reinterpret_cast<const f4*>(xs);
      f4 w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = r[i * 64 + lane];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&freed[slot], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) a = dot4(w[i], xv[i * 64 + lane], a);
      acc += wsum(a);
    }
    if (lane == 0) out[blockIdx.x * 16 + c] = acc;
  }
}

// register streaming: 8 waves, 8-KiB slots (8 loads), A/B in flight
__global__ void __launch_bounds__(512) reg_kernel(const float* W, int slots_per_cu, const float* x, float* out) {
  __shared__ __attribute__((aligned(16))) float xs[SLOTF];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < SLOTF; i += blockDim.x) xs[i] = x[i];
  __syncthreads();
  const float* base = W + (size_t)blockIdx.x * slots_per_cu * SLOTF;
  const int n8 = slots_per_cu * 2;  // 8-KiB half slots
  f4 A[8], B[8];
  auto ld = [&](int h, f4 (&buf)[8]) {
    const f4* src = reinterpret_cast<const f4*>(base + (size_t)(h < n8 ? h : 0) * 2048);
#pragma unroll
    for (int u = 0; u < 8; ++u) buf[u] = __builtin_nontemporal_load(src + u * 64 + lane);
  };
  float acc = 0.f;
  auto use = [&](int h, const f4 (&buf)[8]) {
    const f4* xv = reinterpret_cast<const f4*>(xs + (h & 1) * 2048);
    float a = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) a = dot4(buf[u], xv[u * 64 + lane], a);
    acc += wsum(a);
  };
  int h = wave;
  ld(h, A);
  ld(h + 8, B);
  for (; h < n8; h += 16) {
    use(h, A);
    ld(h + 16, A);
    if (h + 8 < n8) use(h + 8, B);
    ld(h + 24, B);
  }
  if (lane == 0) out[blockIdx.x * 16 + wave] = acc;
}

template <int NC, int NSLOT, int DEPTH, int NL = 1>
static void launch_ring(int ncu, const float* W, int spc, const float* x, float* out) {
  hipLaunchKernelGGL((ring_kernel<NC, NSLOT, DEPTH, NL>), dim3(ncu), dim3((NC + NL) * 64), 0, 0, W, spc, x, out);
}

template <class F>
static float timeit(F f, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f(); (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int spc = 64;  // slots (16 KiB) per CU -> 1 MiB per CU per pass
  const int copies = 8;  // rotate over 8 matrices: 2 GiB, beyond the 256 MiB Infinity Cache
  const size_t per = (size_t)ncu * spc * SLOTF;
  float *W, *x, *out;
  CK(hipMalloc(&W, per * copies * 4));
  CK(hipMalloc(&x, SLOTF * 4));
  CK(hipMalloc(&out, ncu * 16 * 4));
  CK(hipMemset(W, 0, per * copies * 4));
  CK(hipMemset(x, 0, SLOTF * 4));
  const double bytes = per * 4.0;
  int it = 0;
#define RUN(NAME, ...)                                                                       \
  {                                                                                            \
    float ms = timeit([&] { const float* Wc = W + (it++ % copies) * per; __VA_ARGS__; }, 64);       \
    printf("%-28s %8.2f us  %7.0f GB/s\n", NAME, ms * 1e3, bytes / (ms * 1e-3) / 1e9);         \
  }
  RUN("register 8w 2x8KiB", hipLaunchKernelGGL(reg_kernel, dim3(ncu), dim3(512), 0, 0, Wc, spc, x, out));
  RUN("ring 3c 6slot d3 1L", launch_ring<3, 6, 3, 1>(ncu, Wc, spc, x, out));
  RUN("ring 4c 8slot d2 2L", launch_ring<4, 8, 2, 2>(ncu, Wc, spc, x, out));
  RUN("ring 4c 8slot d3 2L", launch_ring<4, 8, 3, 2>(ncu, Wc, spc, x, out));
  RUN("ring 4c 8slot d2 4L", launch_ring<4, 8, 2, 4>(ncu, Wc, spc, x, out));
  RUN("ring 6c 8slot d1 4L", launch_ring<6, 8, 1, 4>(ncu, Wc, spc, x, out));
  RUN("ring 4c 6slot d1 4L", launch_ring<4, 6, 1, 4>(ncu, Wc, spc, x, out));
  RUN("register 8w 2x8KiB", hipLaunchKernelGGL(reg_kernel, dim3(ncu), dim3(512), 0, 0, Wc, spc, x, out));
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
