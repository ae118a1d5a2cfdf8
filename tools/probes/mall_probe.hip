// mall_probe.hip — can a weight stream that the persistent step has to stall (staging, attention)
// be moved EARLIER into the Infinity Cache, so the stream that follows reads it faster than HBM?
//   stream   : every CU reads its contiguous slice of W once with nt buffer loads (the persistent
//              step's form: 16 x 16 B per lane in flight), and dots it (keeps the loads live)
//   prefetch : every CU issues default-policy LDS-DMA loads of its slice into a 1-KiB dummy LDS
//              strip per wave (no VGPRs, nothing read back) and drains them at the end
//   evict    : a 1-GiB default-policy read between trials (cold Infinity Cache)
// Prints, per size, the median of 5 trials: cold stream, stream right after a stream, prefetch
// alone, stream right after a prefetch, and prefetch + stream in one launch (waves split).
// hipcc --offload-arch=gfx950 -O3 -o mall_probe mall_probe.hip && ./mall_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NB = 256, NT = 512;

__device__ inline float dot4(f4 a, f4 b, float c) {
  c = fmaf(a.x, b.x, c); c = fmaf(a.y, b.y, c); c = fmaf(a.z, b.z, c); return fmaf(a.w, b.w, c);
}

// slice = bytes per block (multiple of 16 KiB)
__global__ void __launch_bounds__(NT) k_stream(const float* W, unsigned slice, float* out) {
  const int t = threadIdx.x;
  const char* base = reinterpret_cast<const char*>(W) + (size_t)blockIdx.x * slice;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)slice, 0x00020000);
  float a = 0.f;
  // 8 loads of 16 B per thread per round: 64 KiB per block per round
  for (unsigned off = 0; off < slice; off += NT * 16 * 8) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + (u * NT + t) * 16, 0, 2 /*nt*/));
#pragma unroll
    for (int u = 0; u < 8; ++u) a = dot4(v[u], v[u], a);
  }
  if (a == 1234.5f) out[blockIdx.x] = a;
}

__global__ void __launch_bounds__(NT) k_prefetch(const float* W, unsigned slice) {
  __shared__ __attribute__((aligned(16))) float dummy[NT / 64][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* base = reinterpret_cast<const char*>(W) + (size_t)blockIdx.x * slice;
  for (unsigned off = wave * 1024; off < slice; off += (NT / 64) * 1024)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off + lane * 16),
                                     (__attribute__((address_space(3))) void*)(&dummy[wave][0]), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// both in one launch: waves 0..3 prefetch the second half of the slice while waves 4..7 stream
// the first half, then all stream the second half
__global__ void __launch_bounds__(NT) k_overlap(const float* W, unsigned slice, float* out) {
  __shared__ __attribute__((aligned(16))) float dummy[4][256];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const char* base = reinterpret_cast<const char*>(W) + (size_t)blockIdx.x * slice;
  const unsigned half = slice / 2;
  float a = 0.f;
  if (wave < 4) {
    for (unsigned off = half + wave * 1024; off < slice; off += 4 * 1024)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off + lane * 16),
                                       (__attribute__((address_space(3))) void*)(&dummy[wave][0]), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)half, 0x00020000);
    const int tt = t - 256;
    for (unsigned off = 0; off < half; off += 256 * 16 * 8) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + (u * 256 + tt) * 16, 0, 2));
#pragma unroll
      for (int u = 0; u < 8; ++u) a = dot4(v[u], v[u], a);
    }
  }
  __syncthreads();
  const auto rs2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base + half), (short)0, (int)half, 0x00020000);
  for (unsigned off = 0; off < half; off += NT * 16 * 8) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs2, off + (u * NT + t) * 16, 0, 2));
#pragma unroll
    for (int u = 0; u < 8; ++u) a = dot4(v[u], v[u], a);
  }
  if (a == 1234.5f) out[blockIdx.x] = a;
}

__global__ void k_evict(const f4* E, size_t n, float* out) {
  float a = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a += E[i].x;
  if (a == 1234.5f) out[0] = a;
}

int main() {
  const size_t ebytes = (size_t)1 << 30;
  float *E, *W, *out;
  CK(hipMalloc(&E, ebytes));
  CK(hipMalloc(&W, (size_t)256 << 20));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(E, 0, ebytes));
  CK(hipMemset(W, 0, (size_t)256 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto tm = [&](auto f) {
    CK(hipEventRecord(e0, 0));
    f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return (int)(ms * 1000.f);
  };
  auto evict = [&] { hipLaunchKernelGGL(k_evict, dim3(2048), dim3(256), 0, 0, (const f4*)E, ebytes / 16, out); };
  printf("MB  cold_stream  stream_after_stream  prefetch  stream_after_prefetch  overlap_1launch   (us, median of 5)\n");
  for (int mb : {16, 32, 64, 128, 192}) {
    const unsigned slice = (unsigned)(((size_t)mb << 20) / NB);
    std::vector<int> r[5];
    for (int trial = 0; trial < 5; ++trial) {
      evict();
      r[0].push_back(tm([&] { hipLaunchKernelGGL(k_stream, dim3(NB), dim3(NT), 0, 0, W, slice, out); }));
      r[1].push_back(tm([&] { hipLaunchKernelGGL(k_stream, dim3(NB), dim3(NT), 0, 0, W, slice, out); }));
      evict();
      r[2].push_back(tm([&] { hipLaunchKernelGGL(k_prefetch, dim3(NB), dim3(NT), 0, 0, W, slice); }));
      r[3].push_back(tm([&] { hipLaunchKernelGGL(k_stream, dim3(NB), dim3(NT), 0, 0, W, slice, out); }));
      evict();
      r[4].push_back(tm([&] { hipLaunchKernelGGL(k_overlap, dim3(NB), dim3(NT), 0, 0, W, slice, out); }));
    }
    printf("%4d", mb);
    for (auto& v : r) {
      std::sort(v.begin(), v.end());
      printf("  %6d (%5.2f TB/s)", v[2], (double)((size_t)mb << 20) / (v[2] * 1e-6) / 1e12);
    }
    printf("\n");
  }
  CK(hipDeviceSynchronize());
  return 0;
}
