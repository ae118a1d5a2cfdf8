// mb_probe.hip — standalone probe: batched (<= 8 sequences) decode GEMV on the 16-block 4x4x1 f32
// MFMA with the weights loaded straight into VGPRs (no LDS round trip), the activations resident in
// LDS, and every wave streaming one contiguous range of (4-row group, 64-k chunk) units (perfect
// balance; a row group split between waves is combined by its last arriving piece, slot order).
// Checks y = W x against a double CPU sum, then times the launch over rotating weight copies.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_probe tools/probes/mb_probe.hip && /tmp/mb_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(c) do { hipError_t e_ = (c); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float red16(float r) {  // sum over the 16 lanes l with equal l % 4
  r += dppf<0x124>(r);  // row_ror:4
  r += dppf<0x128>(r);  // row_ror:8
  r += __shfl_xor(r, 16, 64);
  r += __shfl_xor(r, 32, 64);
  return r;
}
__device__ __forceinline__ float sel4(const f32x4& a, int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

template <int NR, int NSG, int P, int W, bool NT, bool TILED, bool XG = false>
__global__ void __launch_bounds__(W * 64) mb_kernel(const float* __restrict__ W0, const float* __restrict__ W1,
                                                    const float* __restrict__ x, int K, int M, int nb, float* y,
                                                    float* part, unsigned* cnt, int maxp) {
  extern __shared__ f4 xl[];
  const int C = K >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nx = XG ? 0 : C * NSG * 64;
  for (int e0 = threadIdx.x; e0 < nx; e0 += 8 * W * 64) {  // 8 independent loads in flight per thread
    f4 v[8];
#pragma unroll
    for (int r8 = 0; r8 < 8; ++r8) {
      const int e = e0 + r8 * W * 64;
      const int c = e / (NSG * 64), r = e - c * NSG * 64, s = r >> 6, l = r & 63;
      const int seq = 4 * s + (l & 3);
      v[r8] = (e < nx && seq < nb) ? *reinterpret_cast<const f4*>(x + (long long)seq * K + 64 * c + 4 * (l >> 2)) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int r8 = 0; r8 < 8; ++r8)
      if (e0 + r8 * W * 64 < nx) xl[e0 + r8 * W * 64] = v[r8];
  }
  __syncthreads();
  const long long NG = (M + 3) / 4, T = NG * C;
  const long long NW = (long long)gridDim.x * W, gid = (long long)blockIdx.x * W + wave;
  const long long u0 = T * gid / NW, u1 = T * (gid + 1) / NW;
  if (u0 >= u1) return;
  const int bq = lane >> 2, iq = lane & 3;
  const long long Kl = K;
  // issue cursor
  long long ui = u0;
  int rgi = (int)(u0 / C), ci = (int)(u0 - (long long)rgi * C);
  auto issue = [&](f4 (&w)[NR], f4 (&xg)[NSG]) {
    if constexpr (XG) {
#pragma unroll
      for (int s = 0; s < NSG; ++s) xg[s] = *reinterpret_cast<const f4*>(x + (long long)(4 * s + iq) * K + 64 * ci + 4 * bq);
    }
    int row = 4 * rgi + iq;
    row = row < M ? row : M - 1;
    const long long off = TILED ? ((long long)rgi * C + ci) * (NR * 256) + 4 * lane : row * Kl + 64 * ci + 4 * bq;
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      const f4* a = reinterpret_cast<const f4*>(TILED ? W0 + off + m * 256 : (m == 0 ? W0 : W1) + off);
      w[m] = NT ? __builtin_nontemporal_load(a) : *a;
    }
    if (ui + 1 < u1) {
      ++ui;
      if (++ci == C) { ci = 0; ++rgi; }
    }
  };
  f4 buf[P][NR];
  f4 xgb[P][NSG];
#pragma unroll
  for (int t = 0; t < P; ++t) issue(buf[t], xgb[t]);
  f32x4 acc[NR][NSG];
#pragma unroll
  for (int m = 0; m < NR; ++m)
#pragma unroll
    for (int s = 0; s < NSG; ++s) acc[m][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  int rgc = (int)(u0 / C), cc = (int)(u0 - (long long)rgc * C), cstart = cc;
  auto g_of = [&](long long u) { return ((u + 1) * NW - 1) / T; };
  for (long long base = u0; base < u1; base += P) {
#pragma unroll
    for (int t = 0; t < P; ++t) {
      const long long u = base + t;
      if (u < u1) {
        f4 xv[NSG];
#pragma unroll
        for (int s = 0; s < NSG; ++s) xv[s] = XG ? xgb[t][s] : xl[(cc * NSG + s) * 64 + lane];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s)
              acc[m][s] = __builtin_amdgcn_mfma_f32_4x4x1f32(buf[t][m][q], xv[s][q], acc[m][s], 0, 0, 0);
        if (cc == C - 1 || u == u1 - 1) {
          // row group rgc, chunks [cstart, cc] done by this wave
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s)
#pragma unroll
              for (int v = 0; v < 4; ++v) acc[m][s][v] = red16(acc[m][s][v]);
          if (cstart == 0 && cc == C - 1) {
            const int row = 4 * rgc + bq;
            if (bq < 4 && row < M) {
#pragma unroll
              for (int m = 0; m < NR; ++m)
#pragma unroll
                for (int s = 0; s < NSG; ++s) {
                  const int seq = 4 * s + iq;
                  if (seq < nb) y[((long long)m * nb + seq) * M + row] = sel4(acc[m][s], bq);
                }
            }
          } else {
            const long long gf = g_of((long long)rgc * C);
            const int np = (int)(g_of((long long)rgc * C + C - 1) - gf + 1);
            const int slot = (int)(gid - gf);
            float* pp = part + ((long long)rgc * maxp + slot) * (NR * NSG * 16);
            if (bq < 4) {
#pragma unroll
              for (int m = 0; m < NR; ++m)
#pragma unroll
                for (int s = 0; s < NSG; ++s)
                  __hip_atomic_store(pp + (m * NSG + s) * 16 + bq * 4 + iq, sel4(acc[m][s], bq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned old = 0;
            if (lane == 0) {
              old = __hip_atomic_fetch_add(cnt + rgc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            old = __builtin_amdgcn_readfirstlane(old);
            if ((int)old == np - 1) {
              if (lane == 0) {
                __hip_atomic_store(cnt + rgc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              if (lane < NR * NSG * 16) {
                const float* q0 = part + (long long)rgc * maxp * (NR * NSG * 16) + lane;
                float v = __hip_atomic_load(q0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (int sl = 1; sl < np; ++sl) v += __hip_atomic_load(q0 + sl * (NR * NSG * 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int m = lane / (NSG * 16), s = (lane / 16) % NSG, r = (lane >> 2) & 3, j = lane & 3;
                const int row = 4 * rgc + r, seq = 4 * s + j;
                if (row < M && seq < nb) y[((long long)m * nb + seq) * M + row] = v;
              }
            }
          }
#pragma unroll
          for (int m = 0; m < NR; ++m)
#pragma unroll
            for (int s = 0; s < NSG; ++s) acc[m][s] = f32x4{0.f, 0.f, 0.f, 0.f};
          cstart = 0;
        }
        if (++cc == C) { cc = 0; ++rgc; }
      }
      issue(buf[t], xgb[t]);
    }
  }
}

struct Shape { const char* name; int NR, M, K; };

template <int NR, int P, int W, bool NT, bool TILED = false, bool XG = false>
double run(const Shape& sh, int nb, int grid, const float* Wd, size_t wfl, int ncopy, const float* xd, float* yd,
           float* part, unsigned* cnt, int iters, bool check) {
  const int C = sh.K / 64;
  const long long NG = (sh.M + 3) / 4, T = NG * C;
  const long long NW = (long long)grid * W;
  if (T < NW) return -1;
  const int maxp = (int)((C * NW + T - 1) / T) + 2;
  const size_t lds = XG ? 0 : (size_t)C * 2 * 64 * 16;
  auto kern = mb_kernel<NR, 2, P, W, NT, TILED, XG>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const size_t mat = (size_t)sh.M * sh.K;
  auto launch = [&](int i) {
    const float* w0 = Wd + (size_t)(i % ncopy) * wfl;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(W * 64), lds, 0, w0, w0 + mat, xd, sh.K, sh.M, nb, yd, part, cnt, maxp);
  };
  if (check) {
    launch(0);
    CK(hipDeviceSynchronize());
    std::vector<float> hw(NR * mat), hx((size_t)nb * sh.K), hy((size_t)NR * nb * sh.M);
    CK(hipMemcpy(hw.data(), Wd, NR * mat * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hx.data(), xd, hx.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy.data(), yd, hy.size() * 4, hipMemcpyDeviceToHost));
    double maxe = 0;
    for (int m = 0; m < NR; ++m)
      for (int b = 0; b < nb; ++b)
        for (int r = 0; r < sh.M; r += 7) {
          double s = 0, sa = 0;
          for (int k = 0; k < sh.K; ++k) {
            size_t wi = m * mat + (size_t)r * sh.K + k;
            if (TILED) {  // element (row r, k) of matrix m in the tiled image
              const int rg = r / 4, i = r % 4, c = k / 64, bq = (k % 64) / 4, q = k % 4;
              wi = (((size_t)rg * C + c) * NR + m) * 256 + (size_t)(4 * bq + i) * 4 + q;
            }
            double t = (double)hw[wi] * hx[(size_t)b * sh.K + k]; s += t; sa += fabs(t);
          }
          const double e = fabs(s - hy[((size_t)m * nb + b) * sh.M + r]) / (sa + 1e-30);
          if (e > maxe) maxe = e;
        }
    printf("  check %s%s NR=%d nb=%d grid=%d W=%d P=%d: max rel err %.3g %s\n", sh.name, TILED ? " (tiled)" : "", NR, nb, grid, W, P, maxe, maxe < 1e-5 ? "OK" : "FAIL");
  }
  for (int i = 0; i < 3; ++i) launch(i);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 8;
  const Shape shapes[] = {{"wo", 1, 4096, 4096}, {"ffn_up", 2, 11008, 4096}, {"cls", 1, 32000, 4096}, {"qkv_as_store", 1, 12288, 4096}, {"ffn_down", 1, 4096, 11008}};
  size_t maxw = 0;
  for (auto& s : shapes) maxw = std::max(maxw, (size_t)s.NR * s.M * s.K);
  float *Wd, *xd, *yd, *part;
  unsigned* cnt;
  const size_t total = (size_t)1600 << 20;  // bytes of weights to rotate over
  CK(hipMalloc(&Wd, total));
  CK(hipMalloc(&xd, 16 * 11008 * 4));
  CK(hipMalloc(&yd, (size_t)2 * 16 * 32000 * 4));
  CK(hipMalloc(&part, (size_t)64 << 20));
  CK(hipMalloc(&cnt, (size_t)1 << 20));
  CK(hipMemset(cnt, 0, (size_t)1 << 20));
  {
    std::vector<float> h(total / 4);
    unsigned s = 12345;
    for (auto& v : h) { s = s * 1664525u + 1013904223u; v = ((int)(s >> 9) - (1 << 22)) * (0.02f / (1 << 22)); }
    CK(hipMemcpy(Wd, h.data(), total, hipMemcpyHostToDevice));
    std::vector<float> hx(16 * 11008);
    for (auto& v : hx) { s = s * 1664525u + 1013904223u; v = ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 22)); }
    CK(hipMemcpy(xd, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  }
  for (auto& sh : shapes) {
    const size_t wfl = (size_t)sh.NR * sh.M * sh.K;
    const int ncopy = (int)(total / 4 / wfl);
    const double gb = wfl * 4.0 / 1e9;
    const int iters = std::max(20, (int)(2e9 / (wfl * 4.0)));
    printf("%s (%.1f MB, %d copies)\n", sh.name, gb * 1e3, ncopy);
#define RUN(NR_, P_, W_, NT_, G_) RUNT(NR_, P_, W_, NT_, G_, false)
#define RUNX(NR_, P_, W_, G_, T_)                                                                             \
    {                                                                                                         \
      double us = run<NR_, P_, W_, true, T_, true>(sh, nb, G_, Wd, wfl, ncopy, xd, yd, part, cnt, iters, true); \
      if (us > 0) printf("    NR=%d P=%2d W=%2d grid=%d tiled=%d x-from-L2: %8.2f us  %7.1f GB/s\n", NR_, P_, W_, G_, (int)T_, us, gb / us * 1e6); \
    }
#define RUNT(NR_, P_, W_, NT_, G_, T_)                                                                        \
    {                                                                                                         \
      double us = run<NR_, P_, W_, NT_, T_>(sh, nb, G_, Wd, wfl, ncopy, xd, yd, part, cnt, iters, true);       \
      if (us > 0) printf("    NR=%d P=%2d W=%2d NT=%d grid=%d tiled=%d: %8.2f us  %7.1f GB/s\n", NR_, P_, W_, NT_, G_, (int)T_, us, gb / us * 1e6); \
    }
    if (sh.K > 4096) {
      RUNX(1, 8, 8, 256, false) RUNX(1, 8, 8, 512, false) RUNX(1, 8, 4, 512, false) RUNX(1, 8, 4, 1024, false)
    } else if (sh.NR == 1) {
      RUN(1, 8, 8, true, 256) RUN(1, 4, 8, true, 256)
      RUNX(1, 8, 8, 256, false) RUNX(1, 8, 8, 512, false) RUNX(1, 8, 4, 512, false) RUNX(1, 8, 4, 1024, false) RUNX(1, 4, 8, 512, false)
    } else {
      RUN(2, 8, 8, true, 256) RUN(2, 4, 8, true, 256)
      RUNX(2, 8, 8, 256, false) RUNX(2, 4, 8, 512, false) RUNX(2, 8, 4, 512, false) RUNX(2, 4, 4, 1024, false)
    }
  }
  return 0;
}
