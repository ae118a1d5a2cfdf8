// gemv.hip — instantiations and launcher of the decode GEMV (see gemv.hpp).
#include "gemv_dispatch.hpp"
#include "gemv_launch.hpp"

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

bool gemv_matrix_path(const GemvParams& p) { return matrix_path_ok(p); }

// Measured on MI355X (profiles/r01_gemv_sweep.json, llama2-7B shapes, weights streamed
// from HBM): prefetch-before-staging costs 64 VGPRs and loses occupancy everywhere
// (-2..-12 %); non-temporal weight loads win 5-10 %; at NB = 1 one item per wave is
// best except the K = 11008 down-projection (2 items, 8 waves: the 44 KiB staged
// activation is amortised over twice the rows); for NB > 1 two items per wave halve
// the LDS activation reads per weight byte.
GemvCfg gemv_default_cfg(int mode, int n_items, int K, int nb, bool nt) {
  GemvCfg c;
  c.nt = nt;
  c.pf = false;
  (void)mode;
  (void)n_items;
  if (nb == 1) {
    c.ipw = K > 8192 ? 2 : 1;
    c.waves = (K > 8192 || mode != GM_SWIGLU) ? 8 : 4;
  } else {
    c.ipw = 2;
    c.waves = 4;
  }
  return c;
}

hipError_t launch_mode_store(const GemvParams&, hipStream_t, const GemvCfg*, bool);
hipError_t launch_mode_resid(const GemvParams&, hipStream_t, const GemvCfg*, bool);
hipError_t launch_mode_swiglu(const GemvParams&, hipStream_t, const GemvCfg*, bool);
hipError_t launch_mode_qkv(const GemvParams&, hipStream_t, const GemvCfg*, bool);

static hipError_t dispatch(int mode, const GemvParams& p, hipStream_t s, const GemvCfg* cfg, bool nt) {
  switch (mode) {
    case GM_STORE: return launch_mode_store(p, s, cfg, nt);
    case GM_RESID: return launch_mode_resid(p, s, cfg, nt);
    case GM_SWIGLU: return launch_mode_swiglu(p, s, cfg, nt);
    case GM_QKV: return launch_mode_qkv(p, s, cfg, nt);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gemv(int mode, const GemvParams& p, hipStream_t s, bool nt) {
  return dispatch(mode, p, s, nullptr, nt);
}

hipError_t launch_gemv_cfg(int mode, const GemvParams& p, hipStream_t s, const GemvCfg& cfg) {
  return dispatch(mode, p, s, &cfg, cfg.nt);
}

}  // namespace tl
