// valu_lat.hip — TEST INFRASTRUCTURE (probe): latency of a dependent v_add_f32 chain for one wave,
// alone on its SIMD and with 1-2 busy neighbour waves on the same SIMD, in s_memtime cycles and in
// 100-MHz s_memrealtime ticks (so the shader clock too).  hipcc --offload-arch=gfx950 -O3
// tools/probes/valu_lat.hip -o /tmp/valu_lat && /tmp/valu_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_chain(const float* in, float* out, long long* cyc, int n, int busy) {
  const int w = threadIdx.x >> 6;
  float s = in[threadIdx.x & 63], a = in[64 + (threadIdx.x & 63)];
  if (w == 0) {
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 16
    for (int i = 0; i < n; ++i) s = s + a;  // dependent chain
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { cyc[blockIdx.x * 2] = t1 - t0; cyc[blockIdx.x * 2 + 1] = r1 - r0; }
  } else if (busy) {
    float b = a;
#pragma unroll 16
    for (int i = 0; i < 4 * n; ++i) b = b * 1.0000001f + a;  // a busy neighbour (independent work)
    s += b;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float *in, *out; long long* cyc;
  hipMalloc(&in, 512); hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 4096);
  hipMemset(in, 0, 512);
  const int n = 4096;
  for (int cfg = 0; cfg < 3; ++cfg) {
    // cfg 0: 1 wave per block; 1: 5 waves (wave 4 shares SIMD 0 with wave 0), busy; 2: 9 waves busy
    const int waves = cfg == 0 ? 1 : cfg == 1 ? 5 : 9;
    hipLaunchKernelGGL(k_chain, dim3(8), dim3(64 * waves), 0, 0, in, out, cyc, n, cfg > 0);
    hipDeviceSynchronize();
    long long h[16];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("waves %d: %.2f cycles per dependent add, clock %.2f GHz\n", waves, (double)h[0] / n,
           (double)h[0] / (h[1] * 10.0));
  }
  return 0;
}
