/* runq_driver.c — TEST INFRASTRUCTURE ONLY.  Compiles the REFERENCE's runq.c in place
 * (#include of /root/reference/runq.c, its main renamed away) and exposes its int8
 * forward through a C ABI, into oracle/_ref/librunq.so (oracle/Makefile).  Nothing of
 * runq.c is copied into this repository. */
#define main runq_reference_main
#include RUNQ_SOURCE
#undef main

int ref_q8_greedy(const char* path, int token, int pos0, int n, int* out_tokens, float* out_logits) {
  Transformer t;
  build_transformer(&t, (char*)path);
  const int V = t.config.vocab_size;
  for (int i = 0; i < n; ++i) {
    float* lg = forward(&t, token, pos0 + i);
    if (out_logits) memcpy(out_logits + (size_t)i * V, lg, sizeof(float) * V);
    int best = 0;
    for (int j = 1; j < V; ++j)
      if (lg[j] > lg[best]) best = j;
    out_tokens[i] = best;
    token = best;
  }
  free_transformer(&t);
  return 0;
}
