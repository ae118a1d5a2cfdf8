// run_driver.cpp — TEST INFRASTRUCTURE ONLY.  Our thin C-ABI driver around the REFERENCE's
// tokenizer and sampler, compiled together with the reference's own run.cc (read in place,
// with TESTING defined so its main() is left out) into oracle/_ref/librun.so by
// oracle/Makefile.  run.cc's tokenizer and sampler functions are identical to
// src/llama.cpp's (checked by tests/test_host.py::test_reference_copies_identical).
// Nothing from the reference is copied into this repository.
#define TESTING
#include RUN_SOURCE

extern "C" {

void* ref_tok_load(const char* path, int vocab_size) {
  Tokenizer* t = (Tokenizer*)malloc(sizeof(Tokenizer));
  build_tokenizer(t, (char*)path, vocab_size);
  return t;
}
void ref_tok_free(void* t) {
  free_tokenizer((Tokenizer*)t);
  free(t);
}
int ref_tok_encode(void* t, const char* text, int bos, int eos, int* tokens) {
  int n = 0;
  encode((Tokenizer*)t, (char*)text, (int8_t)bos, (int8_t)eos, tokens, &n);
  return n;
}
const char* ref_tok_decode(void* t, int prev, int token) { return decode((Tokenizer*)t, prev, token); }
// append_str's filter: 1 if the piece would be appended
int ref_piece_safe(const char* piece) {
  std::string s;
  append_str((char*)piece, s);
  return s.empty() ? 0 : 1;
}

void* ref_sampler_new(int vocab, float temperature, float topp, unsigned long long seed) {
  Sampler* s = (Sampler*)malloc(sizeof(Sampler));
  build_sampler(s, vocab, temperature, topp, seed);
  return s;
}
void ref_sampler_free(void* s) {
  free_sampler((Sampler*)s);
  free(s);
}
int ref_sample(void* s, float* logits) { return sample((Sampler*)s, logits); }
unsigned long long ref_sampler_rng(void* s) { return ((Sampler*)s)->rng_state; }
int ref_sample_topp(float* p, int n, float topp, float coin) {
  ProbIndex* buf = (ProbIndex*)malloc(sizeof(ProbIndex) * (size_t)n);
  const int r = sample_topp(p, n, topp, buf, coin);
  free(buf);
  return r;
}
int ref_sample_mult(float* p, int n, float coin) { return sample_mult(p, n, coin); }
float ref_random_f32(unsigned long long* s) { return random_f32(s); }
void ref_softmax(float* x, int n) { softmax(x, n); }

}  // extern "C"
