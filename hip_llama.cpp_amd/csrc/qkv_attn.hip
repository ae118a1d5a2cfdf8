// qkv_attn.hip — RMSNorm + QKV + RoPE + K/V write and the attention of the batched multi-launch
// step (5..8 sequences, fp32, head size 64/128) as ONE launch.
//
// Semantics: the first two kernels of a layer of the reference forward (src/seq.cpp:53-136; GPU
// twin thaDNN_s_forward_batch, src/thaDNN.cpp:13-81): q/k/v = W{q,k,v} · rmsnorm(x), RoPE on (q, k),
// k/v into the cache row at pos, then per head softmax(q·K / sqrt(hs)) · V into xb.
//
// Why: at 8 sequences the attention kernel is latency-bound (11 us per layer at positions 0..255
// for ~33 MB of K/V, 0.38 of its own bytes) and its launch gap and ramp sit between
// two HBM-bound GEMVs.  Here the attention waves are blocks of the QKV launch itself: they are
// resident from the start, issue their cached K/V rows (positions < pos, written by earlier
// steps) while the QKV tiles stream, and need only q and this step's k/v row — which the QKV
// epilogue publishes as {value, tag} granules (common.hpp R2 hand-off: one 16-B sc1 store per row
// pair, no fence, no flag) — to finish.  Tile slots are dealt per kv-head group
// (gemv_mfma.hpp qkv_tile_of_slot) so a head's tiles finish together.
//
// Arithmetic: the GEMV blocks are gemv_mfma_kernel's own body (same tiles, splits, sums and
// epilogue), the attention units are attn_unit's multi-launch arithmetic (GR only changes where q
// and the new row come from: the same floats), so the step is bitwise the two-launch step.
//
// Safety: blocks [0, gemv_blocks) never wait on anything; the attention blocks come after them in
// the grid and wait with bounded granule polls (common.hpp gran_wait: a give-up sets the decoder's
// sticky error word, the host then disables this path and re-runs the call on the two-launch step,
// forward.hip check_persist).  Tags are (launch sequence << 12) + layer + 1 with the sequence word
// in device memory, advanced once per step (k_step_seq_advance), shared with the persistent steps.
#include <hip/hip_runtime.h>
#include "attention.hpp"
#include "gemv_launch.hpp"
#include "qkv_attn.hpp"

namespace tl {

template <bool NT, int HS>
__global__ void __launch_bounds__(kMfmaWaves * 64, 4) qkv_attn_kernel(GemvParams p, AttnWaveParams w, int gemv_blocks) {
  keep_implicit_args();
  const int bid = blockIdx.x;
  if (bid < gemv_blocks) {
    gemv_mfma_block<GM_QKV, NT, 2>(p, bid);
    return;
  }
  // attention: one unit per wave, head-major (the heads of the first kv groups, whose tiles come
  // first, first); unit numbering as attn_wave_kernel's (split-major over (sequence, head))
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int v = (bid - gemv_blocks) * kMfmaWaves + wave;
  const int per_h = w.B * w.NS;
  if (v >= w.a.n_heads * per_h) return;
  const int h = v / per_h, r = v - h * per_h, b = r / w.NS, s = r - b * w.NS;
  attn_unit<HS, 16, true, false>(w, s * (w.B * w.a.n_heads) + b * w.a.n_heads + h, lane);
}

__global__ void k_step_seq_advance(unsigned* seq) {
  if (threadIdx.x == 0) seq[0] = seq[0] + 1u;
}

bool qkv_attn_ok(const GemvParams& p, int n_heads, int n_kv_heads) {
  if (p.nb < 5 || p.nb > 8 || (p.head_size != 64 && p.head_size != 128)) return false;
  if ((p.dim & 15) || (p.kv_dim & 15) || n_kv_heads <= 0 || n_heads % n_kv_heads) return false;
  if (!matrix_path_ok(p) || rr_ok<GM_QKV>(p)) return false;
  return p.rms_w == nullptr || p.ssq_in != nullptr || p.xn != nullptr;
}

int qkv_attn_splits(int nb, int n_heads, int want) {
  // one attention block (4 units) per CU beside the 3 GEMV blocks the launch keeps per CU at most
  int ns = mfma_target_blocks() / (nb * n_heads);
  if (ns > want) ns = want;
  if (ns > kMaxNS) ns = kMaxNS;
  return ns < 1 ? 1 : ns;
}

hipError_t launch_qkv_attn(GemvParams p, AttnWaveParams w, hipStream_t s, bool nt) {
  if (p.tok || (p.rms_w && !p.ssq_in)) {  // embedding / norm prologue, as launch_mode
    p.ssq_in = nullptr;
    hipLaunchKernelGGL(gemv_prenorm_kernel<0>, dim3(p.nb), dim3(256), 0, s, p);
    p.x = p.xn;
    p.x_stride = p.K;
    p.rms_w = nullptr;
    p.tok = nullptr;
    p.x_out = nullptr;
  }
  p.tperm_kv_mul = w.a.kv_mul;
  const int tiles = (2 * p.n_items + 15) / 16;
  mfma_splits(p, tiles, false);
  const int gemv_blocks = tiles * p.msplit;
  const int units = w.B * w.a.n_heads * w.NS;
  const dim3 grid(gemv_blocks + (units + kMfmaWaves - 1) / kMfmaWaves), blk(kMfmaWaves * 64);
  if (p.head_size == 64) {
    if (nt) hipLaunchKernelGGL((qkv_attn_kernel<true, 64>), grid, blk, 0, s, p, w, gemv_blocks);
    else hipLaunchKernelGGL((qkv_attn_kernel<false, 64>), grid, blk, 0, s, p, w, gemv_blocks);
  } else {
    if (nt) hipLaunchKernelGGL((qkv_attn_kernel<true, 128>), grid, blk, 0, s, p, w, gemv_blocks);
    else hipLaunchKernelGGL((qkv_attn_kernel<false, 128>), grid, blk, 0, s, p, w, gemv_blocks);
  }
  return hipGetLastError();
}

hipError_t launch_step_seq_advance(unsigned* seq, hipStream_t s) {
  hipLaunchKernelGGL(k_step_seq_advance, dim3(1), dim3(64), 0, s, seq);
  return hipGetLastError();
}

}  // namespace tl
