// fetch_calib.hip — what rocprofv3's FETCH_SIZE reports for the read shapes the persistent steps
// use, against a known byte count (MI355X_MICROARCH.md: FETCH_SIZE is ½ of the bytes of a wide
// coalesced streaming read; other widths uncalibrated).  One kernel per shape, each reading the
// same 512 MiB buffer exactly once with nt buffer loads (the persistent steps' policy):
//   k16 : 16 B per lane, a wave-load = 1 KiB contiguous        (weights: fp32 rows, int8 rows)
//   k4  : 4 B per lane, a wave-load = 256 B contiguous         (int8 group scales: a dword a lane)
//   k8s : 8 B per lane at a 16-B stride, two loads per 1 KiB   (granule halves: ld16 at 32-B stride)
// Run under rocprofv3 --pmc FETCH_SIZE (and --kernel-trace); compare FETCH_SIZE x 1 KiB with 512 MiB.
// hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip && ./fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NB = 1024, NT = 256;
constexpr size_t BYTES = 512ull << 20;
constexpr unsigned SLICE = (unsigned)(BYTES / NB);  // 512 KiB per block

template <int E>
__device__ void k16t(const char* W, unsigned* out) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W) + (size_t)blockIdx.x * SLICE, (short)0, (int)SLICE, 0x00020000);
  unsigned a = 0;
  for (unsigned off = threadIdx.x * 16u; off < SLICE; off += NT * 16u) {
    const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
    a ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * NT + threadIdx.x] = a;
}
// k16: the measured launch; k16e: the same kernel as the cache-evicting read between launches
__global__ void __launch_bounds__(NT) k16(const char* W, unsigned* out) { k16t<0>(W, out); }
__global__ void __launch_bounds__(NT) k16e(const char* W, unsigned* out) { k16t<1>(W, out); }

__global__ void __launch_bounds__(NT) k4(const char* W, unsigned* out) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W) + (size_t)blockIdx.x * SLICE, (short)0, (int)SLICE, 0x00020000);
  unsigned a = 0;
  for (unsigned off = threadIdx.x * 4u; off < SLICE; off += NT * 4u) a ^= __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 2);
  out[blockIdx.x * NT + threadIdx.x] = a;
}

__global__ void __launch_bounds__(NT) k8s(const char* W, unsigned* out) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W) + (size_t)blockIdx.x * SLICE, (short)0, (int)SLICE, 0x00020000);
  unsigned a = 0;
  // lane l of a wave reads bytes [16 l, 16 l + 8) and then [16 l + 8, 16 l + 16) of each 1-KiB piece
  const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (unsigned base = wave * 1024u; base < SLICE; base += (NT / 64) * 1024u) {
    const v2u p = __builtin_amdgcn_raw_buffer_load_b64(rs, base + lane * 16u, 0, 2);
    const v2u q = __builtin_amdgcn_raw_buffer_load_b64(rs, base + lane * 16u + 8u, 0, 2);
    a ^= p.x ^ p.y ^ q.x ^ q.y;
  }
  out[blockIdx.x * NT + threadIdx.x] = a;
}

// write-through (sc1) stores of the hand-off shapes over 64 MiB: do they cause memory-side READS?
//   kst8  : one 8-B sc1 store per lane, a wave's 512 B contiguous   (the {value, tag} granules)
//   kst16 : one 16-B sc1 store per lane, a wave's 1 KiB contiguous  (two granules: st_gran2)
constexpr size_t SBYTES = 64ull << 20;
__global__ void __launch_bounds__(NT) kst8(char* D) {
  const size_t i = ((size_t)blockIdx.x * NT + threadIdx.x) * 8u;
  if (i < SBYTES) __builtin_amdgcn_raw_buffer_store_b64(v2u{(unsigned)i, 1u}, __builtin_amdgcn_make_buffer_rsrc(D, (short)0, 0x7ffffff0, 0x00020000), (unsigned)i, 0, 16);
}
__global__ void __launch_bounds__(NT) kst16(char* D) {
  const size_t i = ((size_t)blockIdx.x * NT + threadIdx.x) * 16u;
  if (i < SBYTES) __builtin_amdgcn_raw_buffer_store_b128(v4u{(unsigned)i, 1u, 2u, 3u}, __builtin_amdgcn_make_buffer_rsrc(D, (short)0, 0x7ffffff0, 0x00020000), (unsigned)i, 0, 16);
}

int main() {
  char* W;
  unsigned* out;
  CK(hipMalloc(&W, BYTES));
  CK(hipMalloc(&out, sizeof(unsigned) * ((1u << 30) / SLICE) * NT));  // (the largest grid: the 1-GiB read)
  CK(hipMemset(W, 1, BYTES));
  char* E;  // a 1-GiB read between kernels: every kernel starts with cold caches
  CK(hipMalloc(&E, 1ull << 30));
  CK(hipMemset(E, 2, 1ull << 30));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k16e, dim3((1u << 30) / SLICE), dim3(NT), 0, 0, (const char*)E, out);
    hipLaunchKernelGGL(k16, dim3(NB), dim3(NT), 0, 0, (const char*)W, out);
    hipLaunchKernelGGL(k16e, dim3((1u << 30) / SLICE), dim3(NT), 0, 0, (const char*)E, out);
    hipLaunchKernelGGL(k4, dim3(NB), dim3(NT), 0, 0, (const char*)W, out);
    hipLaunchKernelGGL(k16e, dim3((1u << 30) / SLICE), dim3(NT), 0, 0, (const char*)E, out);
    hipLaunchKernelGGL(k8s, dim3(NB), dim3(NT), 0, 0, (const char*)W, out);
  }
  char* D;
  CK(hipMalloc(&D, SBYTES));
  CK(hipMemset(D, 0, SBYTES));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k16e, dim3((1u << 30) / SLICE), dim3(NT), 0, 0, (const char*)E, out);
    hipLaunchKernelGGL(kst8, dim3((unsigned)(SBYTES / 8 / NT)), dim3(NT), 0, 0, D);
    hipLaunchKernelGGL(k16e, dim3((1u << 30) / SLICE), dim3(NT), 0, 0, (const char*)E, out);
    hipLaunchKernelGGL(kst16, dim3((unsigned)(SBYTES / 16 / NT)), dim3(NT), 0, 0, D);
  }
  CK(hipDeviceSynchronize());
  printf("fetch_calib: %zu bytes per k16 / k4 / k8s launch, %zu written per kst8 / kst16 launch (k16e over 1 GiB between them: cold caches)\n", BYTES, SBYTES);
  return 0;
}
