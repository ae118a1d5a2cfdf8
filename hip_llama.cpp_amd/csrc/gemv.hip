// gemv.hip — instantiations and launcher of the decode GEMV (see gemv.hpp).
#include "gemv_dispatch.hpp"

namespace tl {

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

bool gemv_fast_ok(const GemvParams& p) {
  if (p.K <= 0 || (p.K & 255)) return false;
  if (!al16(p.W0) || (p.W1 && !al16(p.W1)) || (p.W2 && !al16(p.W2))) return false;
  if (p.tok) {
    if (!al16(p.emb) || !al16(p.x_out) || (p.x_stride & 3)) return false;
  } else if (!al16(p.x) || (p.x_stride & 3)) {
    return false;
  }
  if (p.rms_w && !al16(p.rms_w)) return false;
  return true;
}

template <int MODE, int NB>
static hipError_t launch_nb(const GemvParams& p, hipStream_t s, bool nt) {
  // LDS: 320 B of reduction scratch + NB x kc floats of staged activations.
  // 64 KiB for the staged activations keeps >= 2 blocks per CU resident.
  constexpr int kBudgetFloats = 16384;
  int kc = (kBudgetFloats / NB) & ~255;
  if (kc > p.K) kc = p.K;
  const size_t lds = 320 + (size_t)NB * kc * 4;
  constexpr int IPW = 1;
  const int blocks = (p.n_items + 4 * IPW - 1) / (4 * IPW);
  if (blocks <= 0) return hipSuccess;
  if (nt)
    hipLaunchKernelGGL((gemv_kernel<MODE, NB, IPW, true>), dim3(blocks), dim3(256), lds, s, p, kc);
  else
    hipLaunchKernelGGL((gemv_kernel<MODE, NB, IPW, false>), dim3(blocks), dim3(256), lds, s, p, kc);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_mode(const GemvParams& p0, hipStream_t s, bool nt) {
  if (p0.n_items <= 0 || p0.nb <= 0) return hipSuccess;
  if (!gemv_fast_ok(p0)) {
    const int blocks = (p0.n_items + 3) / 4;
    hipLaunchKernelGGL((gemv_generic_kernel<MODE>), dim3(blocks, p0.nb), dim3(256), 0, s, p0);
    return hipGetLastError();
  }
  for (int b0 = 0; b0 < p0.nb; b0 += 16) {
    GemvParams p = p0;
    p.nb = p0.nb - b0 < 16 ? p0.nb - b0 : 16;
    if (b0) {
      if (p.x) p.x += b0 * p.x_stride;
      if (p.tok) p.tok += b0;
      if (p.x_out) p.x_out += b0 * p.x_stride;
      if (p.pos) p.pos += b0;
      if (MODE == GM_STORE) p.y_off += (long long)b0 * p.y_stride;
      else p.y += (long long)b0 * p.y_stride;
      if (p.kc) p.kc += (long long)b0 * p.kv_b_stride;
      if (p.vc) p.vc += (long long)b0 * p.kv_b_stride;
    }
    hipError_t e;
    if (p.nb == 1) e = launch_nb<MODE, 1>(p, s, nt);
    else if (p.nb == 2) e = launch_nb<MODE, 2>(p, s, nt);
    else if (p.nb <= 4) e = launch_nb<MODE, 4>(p, s, nt);
    else if (p.nb <= 8) e = launch_nb<MODE, 8>(p, s, nt);
    else e = launch_nb<MODE, 16>(p, s, nt);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_gemv(int mode, const GemvParams& p, hipStream_t s, bool nt) {
  switch (mode) {
    case GM_STORE: return launch_mode<GM_STORE>(p, s, nt);
    case GM_RESID: return launch_mode<GM_RESID>(p, s, nt);
    case GM_SWIGLU: return launch_mode<GM_SWIGLU>(p, s, nt);
    case GM_QKV: return launch_mode<GM_QKV>(p, s, nt);
  }
  return hipErrorInvalidValue;
}

}  // namespace tl
