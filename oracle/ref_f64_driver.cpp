// ref_f64_driver.cpp — TEST INFRASTRUCTURE ONLY.  The REFERENCE's own CPU forward
// (/root/reference/src/seq.cpp, read in place; nothing copied) compiled with every `float` widened to
// `double` and the float libm calls to their double versions, into oracle/_ref/libref_seq_f64.so
// (oracle/Makefile): the reference's arithmetic with its rounding taken out.  It pins
// oracle/oracle.c's oracle_forward_f64 — the double restatement the GPU parity tests measure the
// GPU's and the CPU's distance from (tests/test_golden_2048_gpu.py) — to the reference's code itself
// (tests/test_oracle.py::test_forward_f64_matches_widened_reference).
// The only difference left between the two: RoPE's (cos, sin) — the reference's `float` angle
// becomes a double angle here, while oracle_forward_f64 keeps the reference's float parameters —
// about 1e-7 relative in q and k.
#include <ctype.h>
#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <fstream>
#include <iostream>
#include <vector>

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "hip_helper.hpp"  // reference include/ (#pragma once): no float state
#include "thaBLAS.hpp"     // (its float signatures stay float: declared before the widening)

#define float double
#define expf exp
#define sqrtf sqrt
#define powf pow
#define cosf cos
#define sinf sin
#include REF_SEQ_SOURCE  // seq.cpp -> utils.hpp -> models.hpp: Config / TransformerWeights / RunState in double
#undef float
#undef expf
#undef sqrtf
#undef powf
#undef cosf
#undef sinf

extern "C" {

// Teacher-forced logits of the widened reference forward for the v0 model.bin at `path`: token[i]
// at position pos0 + i (every earlier position's K/V from this same run), out_logits[n][vocab].
int ref64_forced(const char* path, const int* tokens, int pos0, int n, double* out_logits) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  Config c;
  if (fread(&c, sizeof c, 1, f) != 1) {
    fclose(f);
    return -1;
  }
  const int shared = c.vocab_size > 0;
  c.vocab_size = abs(c.vocab_size);
  const size_t dim = c.dim, hid = c.hidden_dim, L = c.n_layers, V = c.vocab_size, S = c.seq_len;
  const size_t hs = dim / c.n_heads, kvd = dim * c.n_kv_heads / c.n_heads;
  const size_t nf = V * dim + 2 * L * dim + 2 * L * dim * dim + 2 * L * dim * kvd + 3 * L * dim * hid + dim +
                    S * hs + (shared ? 0 : V * dim);
  std::vector<float> raw(nf);
  const bool ok = fread(raw.data(), sizeof(float), nf, f) == nf;
  fclose(f);
  if (!ok) return -1;
  std::vector<double> a(raw.begin(), raw.end());
  Transformer t;
  memset(&t, 0, sizeof t);
  t.config = c;
  TransformerWeights& w = t.weights;
  double* p = a.data();
  w.token_embedding_table = p; p += V * dim;
  w.rms_att_weight = p; p += L * dim;
  w.wq = p; p += L * dim * dim;
  w.wk = p; p += L * dim * kvd;
  w.wv = p; p += L * dim * kvd;
  w.wo = p; p += L * dim * dim;
  w.rms_ffn_weight = p; p += L * dim;
  w.w1 = p; p += L * dim * hid;
  w.w2 = p; p += L * dim * hid;
  w.w3 = p; p += L * dim * hid;
  w.rms_final_weight = p; p += dim;
  p += S * hs;  // freq_cis_real + imag (unused)
  w.wcls = shared ? w.token_embedding_table : p;
  std::vector<double> x(dim), xb(dim), xb2(dim), hb(hid), hb2(hid), q(dim), att(c.n_heads * S), logits(V);
  std::vector<double> kc(L * S * kvd, 0.0), vc(L * S * kvd, 0.0);
  RunState& s = t.state;
  s.x = x.data(); s.xb = xb.data(); s.xb2 = xb2.data(); s.hb = hb.data(); s.hb2 = hb2.data(); s.q = q.data();
  s.att = att.data(); s.logits = logits.data(); s.key_cache = kc.data(); s.value_cache = vc.data();
  for (int i = 0; i < n; ++i) {
    const double* lg = forward(&t, tokens[i], pos0 + i);
    memcpy(out_logits + (size_t)i * V, lg, sizeof(double) * V);
  }
  return 0;
}
}
