// wave_reduce_probe.hip — checks csrc/wave_reduce.hpp's transposed wave reduction on the GPU: lane l
// holds v[i] = (l + 1) * 1000 + i (exact in fp32 sums); after wave_reduce_t<NV>, every lane that
// publishes (even, < 2 NV) must hold sum over lanes of v[(l >> 1) & (NV - 1)].
// hipcc --offload-arch=gfx950 -O3 -I hip_llama.cpp_amd/csrc -o /tmp/wrp tools/probes/wave_reduce_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "wave_reduce.hpp"

template <int NV>
__global__ void k(float* out) {
  const int lane = threadIdx.x;
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = (float)((lane + 1) * 1000 + i);
  out[lane] = tl::wave_reduce_t<NV>(v, lane);
}

template <int NV>
static int check(float* d) {
  hipLaunchKernelGGL(k<NV>, dim3(1), dim3(64), 0, 0, d);
  float h[64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int l = 0; l < 64; l += 2) {
    if (l >= 2 * NV) break;
    const int i = (l >> 1) & (NV - 1);
    double want = 0;
    for (int m = 0; m < 64; ++m) want += (m + 1) * 1000 + i;
    if (h[l] != (float)want || h[l + 1] != (float)want) {
      if (bad < 4) printf("NV=%d lane %d: got %.1f / %.1f want %.1f\n", NV, l, h[l], h[l + 1], want);
      ++bad;
    }
  }
  printf("wave_reduce_t<%d>: %s\n", NV, bad ? "FAIL" : "ok");
  return bad;
}

int main() {
  float* d;
  if (hipMalloc(&d, 64 * sizeof(float)) != hipSuccess) return 2;
  const int bad = check<8>(d) + check<16>(d) + check<32>(d);
  return bad ? 1 : 0;
}
