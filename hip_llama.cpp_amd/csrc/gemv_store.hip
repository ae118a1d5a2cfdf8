// gemv_store.hip — GM_STORE instantiations of the streaming GEMV (gemv_launch.hpp).
#include "gemv_launch.hpp"

namespace tl {
hipError_t launch_mode_store(const GemvParams& p, hipStream_t s, const GemvCfg* cfg, bool nt) {
  return launch_mode<GM_STORE>(p, s, cfg, nt);
}
}  // namespace tl
