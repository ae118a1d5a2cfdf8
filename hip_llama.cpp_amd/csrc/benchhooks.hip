// benchhooks.hip — in-library micro-benchmark of single GEMV launch shapes, used by
// tools/gemv_sweep.py to pick the launch shape per layer GEMV.
// Weights rotate over enough copies to defeat the 256 MiB Infinity Cache, so every
// launch streams from HBM exactly like a decode step does.
#include <math.h>
#include <vector>
#include "../../include/thallama.h"
#include "gemv_dispatch.hpp"

__global__ void __launch_bounds__(256) k_bench_fill(float* d, size_t n, uint32_t seed, float scale) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    d[i] = ((float)(h & 0xFFFF) - 32768.f) * scale;
  }
}

extern "C" int thallama_gemv_bench(int mode, int M, int K, int nb, int ipw, int waves, int pf, int nt, int iters,
                                   double* us_out) {
  if (K <= 0 || nb <= 0 || iters <= 0 || (mode != tl::GM_QKV && M <= 0)) return (int)hipErrorInvalidValue;
  const int S = 64, hs = 128;
  size_t rows;
  int n_items;
  if (mode == tl::GM_QKV) { rows = 3 * (size_t)K; n_items = 3 * K / 2; }
  else if (mode == tl::GM_SWIGLU) { rows = 2 * (size_t)M; n_items = M; }
  else { rows = M; n_items = M; }
  const size_t wfloats = rows * K;
  size_t ncopy = (size_t)ceil(1.5 * 1024 * 1024 * 1024 / (4.0 * wfloats));
  if (ncopy < 2) ncopy = 2;
  if (ncopy > 64) ncopy = 64;
  float *W = nullptr, *x = nullptr, *rw = nullptr, *y = nullptr, *kc = nullptr, *vc = nullptr;
  int* pos = nullptr;
  float *xn = nullptr, *mpart = nullptr;
  unsigned* mcnt = nullptr;
  float2* rope = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t err = hipSuccess;
#define CK(c) do { err = (c); if (err != hipSuccess) goto done; } while (0)
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMalloc(&W, wfloats * ncopy * 4));
  CK(hipMalloc(&x, (size_t)nb * (K > M ? K : M) * 4 + 64));
  CK(hipMalloc(&rw, (size_t)K * 4));
  CK(hipMalloc(&y, (size_t)nb * (K > M ? K : M) * 4 * 2 + 64));
  CK(hipMalloc(&kc, (size_t)nb * S * K * 4));
  CK(hipMalloc(&vc, (size_t)nb * S * K * 4));
  CK(hipMalloc(&pos, nb * 4));
  CK(hipMalloc(&rope, (size_t)S * hs / 2 * sizeof(float2)));
  hipLaunchKernelGGL(k_bench_fill, dim3(4096), dim3(256), 0, s, W, wfloats * ncopy, 12345u, 0.02f / 32768.f);
  hipLaunchKernelGGL(k_bench_fill, dim3(64), dim3(256), 0, s, x, (size_t)nb * (K > M ? K : M), 777u, 1.f / 32768.f);
  hipLaunchKernelGGL(k_bench_fill, dim3(16), dim3(256), 0, s, rw, (size_t)K, 99u, 1.f / 32768.f);
  hipLaunchKernelGGL(k_bench_fill, dim3(16), dim3(256), 0, s, (float*)rope, (size_t)S * hs, 5u, 1.f / 32768.f);
  CK(hipMemsetAsync(pos, 0, nb * 4, s));
  if (ipw == 0) {
    CK(hipMalloc(&xn, (size_t)16 * K * 4));
    CK(hipMalloc(&mpart, (size_t)tl::mfma_target_blocks() * 2 * 256 * 4));
    CK(hipMalloc(&mcnt, (size_t)tl::mfma_target_blocks() * 4));
    CK(hipMemsetAsync(mcnt, 0, (size_t)tl::mfma_target_blocks() * 4, s));
  }
  {
    tl::GemvParams p = {};
    p.K = K;
    p.n_items = n_items;
    p.nb = nb;
    p.x = x;
    p.x_stride = (mode == tl::GM_RESID && M != K) ? K : K;
    p.rms_w = (mode == tl::GM_QKV || mode == tl::GM_SWIGLU) ? rw : nullptr;
    p.y = y;
    p.y_stride = mode == tl::GM_QKV ? K : M;
    p.pos = pos;
    p.kc = kc;
    p.vc = vc;
    p.kv_b_stride = (long long)S * K;
    p.kv_l_off = 0;
    p.dim = K;
    p.kv_dim = K;
    p.head_size = hs;
    p.rope = rope;
    p.xn = xn;
    p.mpart = mpart;
    p.mcnt = mcnt;
    tl::GemvCfg c;
    c.ipw = ipw;
    c.waves = waves;
    c.pf = pf != 0;
    c.nt = nt != 0;
    auto launch = [&](size_t copy) {
      float* base = W + copy * wfloats;
      p.W0 = base;
      p.W1 = mode == tl::GM_SWIGLU ? base + (size_t)M * K : base + (size_t)K * K;
      p.W2 = base + 2 * (size_t)K * K;
      if (ipw == 0) return tl::launch_gemv(mode, p, s, c.nt);  // default dispatch (matrix cores at nb >= 4)
      return tl::launch_gemv_cfg(mode, p, s, c);
    };
    for (int i = 0; i < 8; ++i) CK(launch(i % ncopy));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) CK(launch(i % ncopy));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    *us_out = 1e3 * ms / iters;
  }
done:
  (void)hipStreamSynchronize(s);
  (void)hipFree(W); (void)hipFree(x); (void)hipFree(rw); (void)hipFree(y); (void)hipFree(kc); (void)hipFree(vc);
  (void)hipFree(pos); (void)hipFree(rope);
  (void)hipFree(xn); (void)hipFree(mpart); (void)hipFree(mcnt);
  (void)hipEventDestroy(e0); (void)hipEventDestroy(e1); (void)hipStreamDestroy(s);
#undef CK
  return (int)err;
}

// ---- test hook: the wave-parallel left-to-right sum (seqsum.hpp) on `count` arrays of n floats
// (device pointers), one wave each; tests/test_seqsum_gpu.py compares with the sequential chain.
#include "seqsum.hpp"
__global__ void __launch_bounds__(64) k_seqsum_check(const float* in, int n, float* out) {
  tl::keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const float* a = in + (size_t)blockIdx.x * n;
  const int ch = tl::seqsum_ch(n);
  for (int i = threadIdx.x; i < tl::seqsum_floats(n); i += 64) lds[i] = 0.f;
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += 64) lds[tl::seqsum_index(e, ch)] = a[e];
  __syncthreads();
  const float s = tl::wave_seqsum(lds, n, threadIdx.x);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

extern "C" int thallama_seqsum_check(const float* in_d, int n, int count, float* out_d) {
  if (!in_d || !out_d || n <= 0 || n > 8192 || count <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = sizeof(float) * 64 * (4 * ((n + 255) / 256) + 4);
  hipLaunchKernelGGL(k_seqsum_check, dim3(count), dim3(64), lds, 0, in_d, n, out_d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

// timing of the register form (clock cycles of one call per wave into cyc[count], low 48 bits;
// its repair rounds in the bits above)
__global__ void __launch_bounds__(64) k_seqsum_time(const float* in, int n, float* out, long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const float* a = in + (size_t)blockIdx.x * n;
  const int ch = tl::seqsum_ch(n);
  for (int i = threadIdx.x; i < tl::seqsum_floats(n); i += 64) lds[i] = 0.f;
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += 64) lds[tl::seqsum_index(e, ch)] = a[e];
  __syncthreads();
  int rounds[16] = {0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  const float s = tl::wave_seqsum_reg(lds, n, threadIdx.x, rounds);
  const long long t1 = __builtin_amdgcn_s_memtime();
  // cycles in the low 48 bits, repair rounds above
  if (threadIdx.x == 0) { out[blockIdx.x] = s; cyc[blockIdx.x] = (t1 - t0) | ((long long)rounds[0] << 48); }
  if (threadIdx.x == 0 && blockIdx.x == 0)  // diagnostics: array 0's failing lane per round
    for (int k = 1; k < 16; ++k) cyc[gridDim.x + k - 1] = rounds[k];
}

extern "C" int thallama_seqsum_time(const float* in_d, int n, int count, float* out_d, long long* cyc_d) {
  if (!in_d || !out_d || !cyc_d || n <= 0 || n > 4096 || count <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = sizeof(float) * 64 * (4 * ((n + 255) / 256) + 4);
  hipLaunchKernelGGL(k_seqsum_time, dim3(count), dim3(64), lds, 0, in_d, n, out_d, cyc_d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
