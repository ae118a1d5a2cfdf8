// ref_driver.cpp — TEST INFRASTRUCTURE ONLY.  Our own thin C-ABI driver around the
// REFERENCE's CPU forward, compiled together with the reference's own sources
// (/root/reference/src/seq.cpp + src/utils.cpp, headers from /root/reference/include)
// into oracle/_ref/libref_seq.so by oracle/Makefile.  Nothing from the reference is
// copied into this repository; the build reads the sources where they lie.
// Used to pin oracle/oracle.c (bit-exact logits) and to generate tests/golden/.
#include <string.h>
#include "seq.hpp"     // reference include/seq.hpp: forward(), rmsnorm(), softmax(), matmul()
#include "utils.hpp"   // reference include/utils.hpp: build_transformer(), free_transformer()

extern "C" {

// Greedy decode with the reference forward (src/seq.cpp:53-183) from model.bin `path`:
// starting from `token` at pos0, n steps; out_tokens[n]; out_logits[n*vocab] (may be NULL).
int ref_greedy(const char* path, int token, int pos0, int n, int* out_tokens, float* out_logits) {
  Transformer t;
  build_transformer(&t, (char*)path);
  const int V = t.config.vocab_size;
  for (int i = 0; i < n; ++i) {
    float* lg = forward(&t, token, pos0 + i);
    if (out_logits) memcpy(out_logits + (size_t)i * V, lg, sizeof(float) * V);
    int best = 0;  // sample_argmax semantics (src/llama.cpp:275-286)
    for (int j = 1; j < V; ++j)
      if (lg[j] > lg[best]) best = j;
    out_tokens[i] = best;
    token = best;
  }
  free_transformer(&t);
  return 0;
}

// Forced-token forward: logits for tokens[i] at position pos0+i (teacher forcing).
int ref_forced(const char* path, const int* tokens, int pos0, int n, float* out_logits) {
  Transformer t;
  build_transformer(&t, (char*)path);
  const int V = t.config.vocab_size;
  for (int i = 0; i < n; ++i) {
    float* lg = forward(&t, tokens[i], pos0 + i);
    memcpy(out_logits + (size_t)i * V, lg, sizeof(float) * V);
  }
  free_transformer(&t);
  return 0;
}

// The reference's op-level CPU functions (src/seq.cpp:3-51), exposed as-is.
void ref_rmsnorm(float* o, float* x, float* w, int size) { rmsnorm(o, x, w, size); }
void ref_softmax(float* x, int size) { softmax(x, size); }
void ref_matmul(float* xout, float* x, float* w, int n, int d) { matmul(xout, x, w, n, d); }
}
