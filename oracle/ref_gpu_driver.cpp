// ref_gpu_driver.cpp — TEST / MEASUREMENT INFRASTRUCTURE ONLY.  Our thin C-ABI driver around the
// REFERENCE's own GPU decode step: thaDNN_s_forward_batch (src/thaDNN.cpp:13-82) with its
// thaBLAS / thaDNN kernels (src/thaBLAS.cpp, src/thaDNN.cpp, src/thaDNN/*.cpp) and its weight
// upload / state allocation (src/models.cpp:86-125, :155-...), all compiled for gfx950 from the
// sources where they lie (oracle/Makefile -> oracle/_ref/libref_gpu.so; nothing is copied).
// Used for two things only, never linked into the product:
//   1. the reference's own decode speed on the same MI355X the bench runs on (bench.py
//      "reference_gpu"), and
//   2. the reference GPU path's own drift from its CPU forward (src/seq.cpp) over a 256-step greedy
//      decode and a 2048-step teacher-forced one — the yardstick for our own fp32 drift
//      (tests/test_golden_long_gpu.py, tests/test_golden_2048_gpu.py).
// Weights: the deterministic synthetic generator (include/thallama_synth.h), i.e. bit-identical to
// our DeviceModel(seed) and to the CPU goldens, laid out in host memory in the v0 order and
// uploaded by the reference's own copy_weight_to_device.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <vector>

#include "models.hpp"  // reference include/: Config, TransformerWeights, RunState, Transformer
#include "thaBLAS.hpp"
#include "thaDNN.hpp"
#include "../include/thallama_synth.h"

extern "C" {

// The synthetic model (v0 order in host memory) uploaded by the reference's own
// copy_weight_to_device, and its state for `batch` sequences.  Returns 0 or a nonzero status.
static int ref_setup(const int* cfg7, int shared, unsigned long long seed, int batch, Config* cfg_out,
                     TransformerWeights** wd_out, RunState** sd_out) {
  Config c;
  memcpy(&c, cfg7, sizeof(c));
  const int V = c.vocab_size < 0 ? -c.vocab_size : c.vocab_size;
  TlSynthPlan plan;
  tl_synth_plan(&plan, cfg7, shared);
  size_t total = 0;
  for (int k = 0; k < plan.n; ++k) total += plan.t[k].count;
  float* arena = (float*)malloc(total * sizeof(float));
  if (!arena) return 2;
  size_t off[16] = {0};
  for (int k = 0; k < plan.n; ++k) {
    const TlSynthTensor& e = plan.t[k];
    off[e.id] = e.offset;
    float* dst = arena + e.offset;
    if (e.kind == TL_SYNTH_NORMAL) {
      const uint64_t ts = tl_synth_tensor_seed(seed, e.id);
      const float sc = tl_synth_scale(e.stddev);
#pragma omp parallel for schedule(static)
      for (long long i = 0; i < (long long)e.count; ++i) dst[i] = tl_synth_value(ts, (uint64_t)i, sc);
    } else {
#pragma omp parallel for schedule(static)
      for (long long i = 0; i < (long long)e.count; ++i) dst[i] = e.value;
    }
  }
  Transformer t;
  memset(&t, 0, sizeof(t));
  c.vocab_size = V;
  t.config = c;
  TransformerWeights& w = t.weights;
  w.token_embedding_table = arena + off[1];
  w.rms_att_weight = arena + off[2];
  w.wq = arena + off[3];
  w.wk = arena + off[4];
  w.wv = arena + off[5];
  w.wo = arena + off[6];
  w.rms_ffn_weight = arena + off[7];
  w.w1 = arena + off[8];
  w.w2 = arena + off[9];
  w.w3 = arena + off[10];
  w.rms_final_weight = arena + off[11];
  w.wcls = shared ? w.token_embedding_table : arena + off[12];
  copy_weight_to_device(&t, *wd_out);
  alloc_state_to_device_batch(&t, *sd_out, batch);
  free(arena);
  *cfg_out = c;
  return 0;
}

static void ref_free_weights(TransformerWeights* wd) {
  for (float* p : {wd->token_embedding_table, wd->rms_att_weight, wd->rms_ffn_weight, wd->wq, wd->wk, wd->wv, wd->wo,
                   wd->w1, wd->w2, wd->w3, wd->rms_final_weight, wd->wcls})
    (void)hipFree(p);
  free(wd);
}

// Greedy decode of `batch` identical sequences from token0 at pos0 for n steps with the reference's
// forward_batch (one call per step, argmax on the host like src/llama.cpp:275-286).  cfg7: the v0
// Config (vocab_size < 0: unshared classifier).  out_tokens[n * batch] (step-major); last_logits
// [batch * V] (may be NULL): the last step's logits; *seconds: wall time of the n steps (after the
// upload).  Returns 0, or a nonzero status.
int refgpu_greedy(const int* cfg7, int shared, unsigned long long seed, int batch, int token0, int pos0, int n,
                  int* out_tokens, float* last_logits, double* seconds) {
  Config c;
  TransformerWeights* wd = nullptr;
  RunState* sd = nullptr;
  if (const int e = ref_setup(cfg7, shared, seed, batch, &c, &wd, &sd)) return e;
  const int V = c.vocab_size;
  thablasHandle_t h1, h2, h3;
  thablasCreate(&h1);
  thablasCreate(&h2);
  thablasCreate(&h3);
  float* logits = nullptr;  // the classifier writes it directly: host-mapped memory
  if (hipHostMalloc((void**)&logits, sizeof(float) * (size_t)batch * V) != hipSuccess) return 3;
  std::vector<int> tok((size_t)batch, token0), pos((size_t)batch, pos0);
  int st = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n && !st; ++i) {
    st = (int)thaDNN_s_forward_batch(h1, h2, h3, batch, &c, wd, sd, tok.data(), pos.data(), logits);
    for (int b = 0; b < batch; ++b) {
      const float* lg = logits + (size_t)b * V;
      int best = 0;
      for (int j = 1; j < V; ++j)
        if (lg[j] > lg[best]) best = j;
      out_tokens[(size_t)i * batch + b] = best;
      tok[b] = best;
      pos[b] += 1;
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  if (last_logits) memcpy(last_logits, logits, sizeof(float) * (size_t)batch * V);
  (void)hipHostFree(logits);
  ref_free_weights(wd);
  return st;
}

// Teacher-forced decode of one sequence with the reference's forward_batch: step i feeds
// tokens[i] at position pos0 + i.  probe_vals[i * k + j] = that step's logit at probe_ids[i * k + j];
// full_steps[0..n_full): steps whose whole logits vector goes to full_out[f * V].  This is the
// reference GPU path's drift from its CPU forward along a fixed token sequence (the yardstick of
// tests/test_golden_2048_gpu.py).
int refgpu_forced(const int* cfg7, int shared, unsigned long long seed, const int* tokens, int pos0, int n,
                  const int* probe_ids, int k, float* probe_vals, const int* full_steps, int n_full, float* full_out) {
  Config c;
  TransformerWeights* wd = nullptr;
  RunState* sd = nullptr;
  if (const int e = ref_setup(cfg7, shared, seed, 1, &c, &wd, &sd)) return e;
  const int V = c.vocab_size;
  thablasHandle_t h1, h2, h3;
  thablasCreate(&h1);
  thablasCreate(&h2);
  thablasCreate(&h3);
  float* logits = nullptr;
  if (hipHostMalloc((void**)&logits, sizeof(float) * (size_t)V) != hipSuccess) return 3;
  int st = 0;
  for (int i = 0; i < n && !st; ++i) {
    int tok = tokens[i], pos = pos0 + i;
    st = (int)thaDNN_s_forward_batch(h1, h2, h3, 1, &c, wd, sd, &tok, &pos, logits);
    for (int j = 0; j < k; ++j) probe_vals[(size_t)i * k + j] = logits[probe_ids[(size_t)i * k + j]];
    for (int f = 0; f < n_full; ++f)
      if (full_steps[f] == i) memcpy(full_out + (size_t)f * V, logits, sizeof(float) * (size_t)V);
  }
  (void)hipHostFree(logits);
  ref_free_weights(wd);
  return st;
}
}
