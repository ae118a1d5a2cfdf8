// attn_wo.hpp — a layer's attention and Wo (+ residual) in one launch (attn_wo.hip).
#pragma once
#include "attention.hpp"
#include "gemv.hpp"

namespace tl {

struct AttnWoParams {
  AttnWaveParams aw;  // the attention launch's parameters, aw.done = done
  GemvParams g;       // the Wo launch's: W0 = wo, K = n_items = dim, x = attention output, y = x, ssq_out
  unsigned* done;     // [n_heads] finished (b, h) per head; zero at launch start
  unsigned* blocks;   // workgroups past their waits (the last one re-arms done[] and this)
  unsigned* err;      // a bounded wait gave up: 3
  int units;          // attention units (nb * n_heads * NS)
  int fault;          // test hook: workgroup 0 skips its attention units, so every wait gives up
};

// Shapes the fused launch takes: 5..8 sequences (the matrix-core Wo), head size 64 / 128, K a
// multiple of 8 waves x 64 floats, at most one 16-row tile per CU.
bool attn_wo_ok(int nb, int dim, int n_heads, int head_size, int ncu);
hipError_t launch_attn_wo(const AttnWoParams& P, hipStream_t s);

}  // namespace tl
