/* thallama_host.h — the host side of the reference's CLI surface (src/llama.cpp), as a plain C
 * ABI in lib/libthallama_host.so (CPU only: no HIP dependency, so it also loads where there is
 * no GPU).  Same algorithms, same byte-level behaviour:
 *   - BPE tokenizer: build_tokenizer / encode / decode / safe_printf (src/llama.cpp:52-256);
 *   - sampler: argmax, multinomial, top-p, xorshift coin, temperature + softmax
 *     (src/llama.cpp:262-399, softmax src/seq.cpp:18-36);
 *   - test-mode request files: read_inputfile / write_outputfile (src/llama.cpp:424-505);
 *   - the test-mode scheduler of test_data_parallelism (src/llama.cpp:891-1083): one worker
 *     per GPU, each with `batch` sequence slots refilled from a shared request counter, one
 *     sampler per request (T=1.0, top-p 0.9, seed 314028).  The GPU step is a callback, so
 *     the same scheduler runs over the fused decoder (app/run.cpp) or a CPU model (tests).
 */
#ifndef THALLAMA_HOST_H
#define THALLAMA_HOST_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- tokenizer (src/llama.cpp:35-256) ---------------------------------------------------- */
typedef struct thallama_tokenizer thallama_tokenizer;
/* build_tokenizer (src/llama.cpp:52-78): NULL if the file cannot be read. */
thallama_tokenizer* thallama_tokenizer_load(const char* path, int vocab_size);
void thallama_tokenizer_free(thallama_tokenizer* t);
int thallama_tokenizer_max_token_length(const thallama_tokenizer* t);
const char* thallama_tokenizer_piece(const thallama_tokenizer* t, int id);
float thallama_tokenizer_score(const thallama_tokenizer* t, int id);
/* encode (src/llama.cpp:138-256): tokens[] must hold strlen(text)+3 ids. Returns 0. */
int thallama_tokenizer_encode(thallama_tokenizer* t, const char* text, int bos, int eos, int* tokens,
                              int* n_tokens);
/* decode (src/llama.cpp:85-96): the piece for `token` following `prev_token`. */
const char* thallama_tokenizer_decode(const thallama_tokenizer* t, int prev_token, int token);
/* The safe_printf / append_str filter (src/llama.cpp:98-126): 1 if the piece is emitted. */
int thallama_piece_is_safe(const char* piece);

/* ---- sampler (src/llama.cpp:262-399) ----------------------------------------------------- */
typedef struct thallama_sampler thallama_sampler;
thallama_sampler* thallama_sampler_create(int vocab_size, float temperature, float topp, unsigned long long seed);
void thallama_sampler_free(thallama_sampler* s);
/* sample(): like the reference it rescales and softmaxes `logits` IN PLACE when T > 0. */
int thallama_sample(thallama_sampler* s, float* logits);
unsigned long long thallama_sampler_rng_state(const thallama_sampler* s);
int thallama_sample_argmax(const float* probabilities, int n);
int thallama_sample_mult(const float* probabilities, int n, float coin);
int thallama_sample_topp(const float* probabilities, int n, float topp, float coin);
unsigned int thallama_random_u32(unsigned long long* state);
float thallama_random_f32(unsigned long long* state);
void thallama_softmax(float* x, int n);

/* ---- test-mode request files (src/llama.cpp:424-505) ------------------------------------- */
typedef struct thallama_requests thallama_requests;
/* First line: the number of requests; then one prompt per line.  NULL if unreadable. */
thallama_requests* thallama_requests_read(const char* path, int max_token_len, int max_seq_len);
void thallama_requests_free(thallama_requests* r);
int thallama_requests_count(const thallama_requests* r);
const char* thallama_requests_prompt(const thallama_requests* r, int i);
const char* thallama_requests_output(const thallama_requests* r, int i);
/* Sampling of every request (default: the reference's temperature 1.0, top-p 0.9, seed
 * 314028 per request, src/llama.cpp:897-900).  temperature 0 = greedy (argmax), an addition
 * for token-exact runs; the seed stays 314028. */
void thallama_requests_set_sampling(thallama_requests* r, float temperature, float topp);
/* write_outputfile: the count, then every generated string followed by "\n". 0 on success. */
int thallama_requests_write(const thallama_requests* r, const char* path);

/* ---- test-mode scheduler (src/llama.cpp:891-1083) ----------------------------------------- */
/* One decode step for `batch` slots of worker `worker`: token[b] at pos[b] -> logits[b*V..].
 * Slots without a request carry token 0 / pos 0 (as in the reference).  Returns 0 on success. */
typedef int (*thallama_step_fn)(void* ctx, int worker, int batch, const int* token, const int* pos, float* logits);
/* Runs every request of r over n_workers workers (threads) with `batch` slots each, writing
 * each request's generated text into r.  seq_len bounds every sequence (max_seq_len).
 * *gen_tokens = the reference's num_gen_tokens.  Returns 0, or the first nonzero step status. */
int thallama_serve_requests(thallama_requests* r, const char* tokenizer_path, int vocab_size, int n_workers,
                            int batch, thallama_step_fn step, void* ctx, long long* gen_tokens);
/* Prompt processing for slot `slot` of worker `worker`: tokens[0..n) at positions pos0.. into
 * that slot's KV cache, logits not needed.  Returns 0 when done, > 0 when the replica cannot
 * (the scheduler then steps through the prompt), < 0 on error. */
typedef int (*thallama_prefill_fn)(void* ctx, int worker, int slot, const int* tokens, int n, int pos0);
/* thallama_serve_requests with batched prompts: a newly admitted request's prompt tokens
 * 0..n-2 go through `prefill` (when non-null) instead of n-1 decode steps; the outputs and
 * *gen_tokens are those of thallama_serve_requests (identical up to the logits tolerance). */
int thallama_serve_requests_prefill(thallama_requests* r, const char* tokenizer_path, int vocab_size,
                                    int n_workers, int batch, thallama_step_fn step, thallama_prefill_fn prefill,
                                    void* ctx, long long* gen_tokens);
/* A greedy decode step that samples on the device: token[b] at pos[b] -> next[b] = the argmax of
 * slot b's logits with sample_argmax's rule (first index of the maximum, src/llama.cpp:275-286).
 * Only B ids cross to the host instead of B x V logits.  Returns 0 on success. */
typedef int (*thallama_argmax_step_fn)(void* ctx, int worker, int batch, const int* token, const int* pos, int* next);
/* thallama_serve_requests_prefill where, for greedy sampling (temperature 0), `argmax_step` (when
 * non-null) replaces `step`: same outputs and *gen_tokens, since greedy sampling is that argmax.
 * With another temperature `step` runs as before (it must then be non-null). */
int thallama_serve_requests_greedy(thallama_requests* r, const char* tokenizer_path, int vocab_size, int n_workers,
                                   int batch, thallama_step_fn step, thallama_argmax_step_fn argmax_step,
                                   thallama_prefill_fn prefill, void* ctx, long long* gen_tokens);
/* thallama_serve_requests_greedy with per-worker accounting (each array n_workers long, any may be
 * NULL): worker w's share of *gen_tokens, the requests it finished, and the seconds from the
 * common start to its last step — one worker per GPU, so these are the per-GPU numbers of a
 * multi-GPU run.  logits_bufs (NULL, or n_workers pointers, each NULL or batch x vocab floats):
 * the buffer worker w's step callback writes its logits into — pinned host memory lets the device
 * copy them at the link rate, like the reference's hipHostMalloc'd logits_host. */
int thallama_serve_requests_stats(thallama_requests* r, const char* tokenizer_path, int vocab_size, int n_workers,
                                  int batch, thallama_step_fn step, thallama_argmax_step_fn argmax_step,
                                  thallama_prefill_fn prefill, void* ctx, long long* gen_tokens,
                                  long long* worker_tokens, double* worker_seconds, int* worker_requests,
                                  float* const* logits_bufs);

#ifdef __cplusplus
}
#endif
#endif
