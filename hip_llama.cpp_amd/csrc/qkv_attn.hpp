// qkv_attn.hpp — the fused QKV + attention launch of the batched multi-launch step (qkv_attn.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "attention.hpp"
#include "gemv.hpp"

namespace tl {

// p / the launch can take the fused path: 5..8 sequences on the matrix-core GEMV, head size 64 or
// 128, whole 16-row tiles per head.
bool qkv_attn_ok(const GemvParams& p, int n_heads, int n_kv_heads);
// Key splits per (sequence, head) of the fused launch: at most one block of attention units per CU.
int qkv_attn_splits(int nb, int n_heads, int want);
// p: the QKV GemvParams with gqkv / gq_stride / gseq / gtag set; w: the attention with gqkv,
// tag_seq, tag_in, err, NS set (B = p.nb).
hipError_t launch_qkv_attn(GemvParams p, AttnWaveParams w, hipStream_t s, bool nt);
// seq[0] += 1: once per step that used tagged granules (the fused launch), after its last use.
hipError_t launch_step_seq_advance(unsigned* seq, hipStream_t s);

}  // namespace tl
