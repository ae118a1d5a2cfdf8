// run_length_probe.hip — HBM read rate vs contiguous run length per wave-load instruction, at equal
// bytes in flight: every lane loads 16 B, a wave-load covers 1 KiB made of runs of RUN bytes on
// consecutive rows of a row-major matrix (row pitch 16 KiB, llama2-7B's dim x 4 B), 8 wave-loads in
// flight per wave, 8 waves per block, one block per CU x 4; 512 MiB read once (nt loads) per launch.
//   RUN = 1024: one row per wave-load (the persistent steps' slots)
//   RUN = 256 : four rows x 256 B (gemv_mfma.hpp's load shape)
//   RUN = 64  : sixteen rows x 64 B (the MFMA lane layout loaded directly)
// hipcc --offload-arch=gfx950 -O3 -o run_length_probe run_length_probe.hip && ./run_length_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr size_t BYTES = 512ull << 20;
constexpr int PITCH = 16384;                  // row pitch (bytes)
constexpr int ROWS = (int)(BYTES / PITCH);    // 32768 rows
constexpr int NT = 512, NBLK = 1024;

// block b owns rows [b * RPB, (b + 1) * RPB) fully; a wave-load covers LPR = RUN / 16 lanes per row,
// 64 / LPR rows; the wave walks its share of the block's (row band, column) pieces
template <int RUN>
__global__ void __launch_bounds__(NT) k(const char* W, unsigned* out) {
  constexpr int LPR = RUN / 16, RPI = 64 / LPR;     // lanes per row, rows per wave-load
  constexpr int RPB = ROWS / NBLK;                  // 32 rows per block
  constexpr int PIECES = (RPB / RPI) * (PITCH / RUN);  // wave-loads per block
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W) + (size_t)blockIdx.x * RPB * PITCH, (short)0,
                                                    RPB * PITCH, 0x00020000);
  const int lr = lane / LPR, lc = lane % LPR;
  unsigned a = 0;
  for (int p0 = wave * 8; p0 < PIECES; p0 += (NT / 64) * 8) {
    v4u v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pc = p0 + i, band = pc / (PITCH / RUN), col = pc % (PITCH / RUN);
      const unsigned off = (unsigned)((band * RPI + lr) * PITCH + col * RUN + lc * 16);
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  out[blockIdx.x * NT + threadIdx.x] = a;
}

template <int RUN>
static float timeit(const char* W, unsigned* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k<RUN>, dim3(NBLK), dim3(NT), 0, 0, W, out);  // warm-up
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<RUN>, dim3(NBLK), dim3(NT), 0, 0, W, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  char* W;
  unsigned* out;
  CK(hipMalloc(&W, BYTES));
  CK(hipMalloc(&out, sizeof(unsigned) * NBLK * NT));
  CK(hipMemset(W, 1, BYTES));
  for (int rep = 0; rep < 2; ++rep) {
    const float a = timeit<1024>(W, out), b = timeit<256>(W, out), c = timeit<64>(W, out);
    printf("run 1024 B: %.1f GB/s   run 256 B: %.1f GB/s   run 64 B: %.1f GB/s\n", BYTES / a / 1e6, BYTES / b / 1e6,
           BYTES / c / 1e6);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
