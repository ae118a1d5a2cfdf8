// runtime.hip — model.bin v0 loader, device residency, synthetic weights and
// small device-memory helpers.
//
// Loader semantics follow the reference exactly (src/utils.cpp:119-177:
// 28-byte Config header, negative vocab_size = unshared classifier, mmap,
// v0 tensor order, freq_cis block skipped).  Device residency differs by
// design: the reference issues 12 hipMalloc + 12 blocking H2D copies per GPU
// (src/models.cpp:86-125); here the payload is ONE arena with the file's own
// layout, so upload is one copy and replication to other GPUs is one RCCL
// broadcast (apps/batch_manager.cpp).
#include <fcntl.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include "../../include/hip_helper.hpp"
#include "../../include/thallama.h"
#include "synth.hpp"
#include "api_lock.hpp"

// ------------------------------------------------------------------ layout
extern "C" size_t thallama_v0_payload_floats(const Config* p, int shared_weights) {
  const size_t dim = p->dim, hid = p->hidden_dim, L = p->n_layers, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  const size_t hs = p->dim / p->n_heads, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  size_t n = V * dim;              // token_embedding_table
  n += L * dim;                    // rms_att
  n += L * dim * dim;              // wq
  n += 2 * L * dim * kvd;          // wk, wv
  n += L * dim * dim;              // wo
  n += L * dim;                    // rms_ffn
  n += 3 * L * dim * hid;          // w1, w2, w3
  n += dim;                        // rms_final
  n += (size_t)p->seq_len * hs;    // freq_cis_real + freq_cis_imag (unused)
  if (!shared_weights) n += V * dim;
  return n;
}

// reference src/utils.cpp:119-148
extern "C" void thallama_map_weights(TransformerWeights* w, const Config* p, float* ptr, int shared_weights) {
  const int head_size = p->dim / p->n_heads;
  const unsigned long long n_layers = p->n_layers;
  const unsigned long long V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  w->token_embedding_table = ptr;
  ptr += V * p->dim;
  w->rms_att_weight = ptr;
  ptr += n_layers * p->dim;
  w->wq = ptr;
  ptr += n_layers * p->dim * (p->n_heads * head_size);
  w->wk = ptr;
  ptr += n_layers * p->dim * (p->n_kv_heads * head_size);
  w->wv = ptr;
  ptr += n_layers * p->dim * (p->n_kv_heads * head_size);
  w->wo = ptr;
  ptr += n_layers * (p->n_heads * head_size) * p->dim;
  w->rms_ffn_weight = ptr;
  ptr += n_layers * p->dim;
  w->w1 = ptr;
  ptr += n_layers * p->dim * p->hidden_dim;
  w->w2 = ptr;
  ptr += n_layers * p->hidden_dim * p->dim;
  w->w3 = ptr;
  ptr += n_layers * p->dim * p->hidden_dim;
  w->rms_final_weight = ptr;
  ptr += p->dim;
  ptr += (unsigned long long)p->seq_len * head_size / 2;
  ptr += (unsigned long long)p->seq_len * head_size / 2;
  w->wcls = shared_weights ? w->token_embedding_table : ptr;
}

extern "C" void memory_map_weights(TransformerWeights* w, Config* p, float* ptr, int shared_weights) {
  thallama_map_weights(w, p, ptr, shared_weights);
}

// ------------------------------------------------------------------ host loader
// reference src/utils.cpp:85-104
extern "C" void malloc_run_state(RunState* s, Config* p) {
  const int kv_dim = (p->dim * p->n_kv_heads) / p->n_heads;
  memset(s, 0, sizeof(*s));
  s->x = (float*)calloc(p->dim, sizeof(float));
  s->xb = (float*)calloc(p->dim, sizeof(float));
  s->xb2 = (float*)calloc(p->dim, sizeof(float));
  s->hb = (float*)calloc(p->hidden_dim, sizeof(float));
  s->hb2 = (float*)calloc(p->hidden_dim, sizeof(float));
  s->q = (float*)calloc(p->dim, sizeof(float));
  s->key_cache = (float*)calloc((size_t)p->n_layers * p->seq_len * kv_dim, sizeof(float));
  s->value_cache = (float*)calloc((size_t)p->n_layers * p->seq_len * kv_dim, sizeof(float));
  s->att = (float*)calloc((size_t)p->n_heads * p->seq_len, sizeof(float));
  s->logits = (float*)calloc(p->vocab_size, sizeof(float));
  if (!s->x || !s->xb || !s->xb2 || !s->hb || !s->hb2 || !s->q || !s->key_cache || !s->value_cache || !s->att ||
      !s->logits) {
    fprintf(stderr, "malloc failed!\n");
    exit(EXIT_FAILURE);
  }
}

extern "C" void free_run_state(RunState* s) {
  free(s->x);
  free(s->xb);
  free(s->xb2);
  free(s->hb);
  free(s->hb2);
  free(s->q);
  free(s->att);
  free(s->logits);
  free(s->key_cache);
  free(s->value_cache);
}

// reference src/utils.cpp:150-170
extern "C" void read_checkpoint(char* checkpoint, Config* config, TransformerWeights* weights, int* fd, float** data,
                                ssize_t* file_size) {
  FILE* file = fopen(checkpoint, "rb");
  if (!file) {
    fprintf(stderr, "Couldn't open file %s\n", checkpoint);
    exit(EXIT_FAILURE);
  }
  if (fread(config, sizeof(Config), 1, file) != 1) exit(EXIT_FAILURE);
  const int shared_weights = config->vocab_size > 0 ? 1 : 0;
  config->vocab_size = abs(config->vocab_size);
  fseek(file, 0, SEEK_END);
  *file_size = ftell(file);
  fclose(file);
  *fd = open(checkpoint, O_RDONLY);
  if (*fd == -1) {
    fprintf(stderr, "open failed!\n");
    exit(EXIT_FAILURE);
  }
  *data = (float*)mmap(NULL, *file_size, PROT_READ, MAP_PRIVATE, *fd, 0);
  if (*data == MAP_FAILED) {
    fprintf(stderr, "mmap failed!\n");
    exit(EXIT_FAILURE);
  }
  float* weights_ptr = *data + sizeof(Config) / sizeof(float);
  thallama_map_weights(weights, config, weights_ptr, shared_weights);
}

// reference src/utils.cpp:106-117
extern "C" void print_transformer(Transformer* t) {
  printf("---------Model Information----------\n");
  printf("dim: %d\n", t->config.dim);
  printf("hidden_dim: %d\n", t->config.hidden_dim);
  printf("n_layers: %d\n", t->config.n_layers);
  printf("n_heads: %d\n", t->config.n_heads);
  printf("n_kv_heads: %d\n", t->config.n_kv_heads);
  printf("vocab_size: %d\n", t->config.vocab_size);
  printf("seq_len: %d\n", t->config.seq_len);
  printf("weights_size: %lu MB\n", (unsigned long)((t->file_size - sizeof(Config)) / (1024L * 1024L)));
  printf("------------------------------------\n");
}

extern "C" void build_transformer(Transformer* t, char* checkpoint_path) {
  read_checkpoint(checkpoint_path, &t->config, &t->weights, &t->fd, &t->data, &t->file_size);
  malloc_run_state(&t->state, &t->config);
  print_transformer(t);
}

extern "C" void free_transformer(Transformer* t) {
  if (t->data != MAP_FAILED && t->data) munmap(t->data, t->file_size);
  if (t->fd != -1) close(t->fd);
  free_run_state(&t->state);
}

// ------------------------------------------------------------------ device residency
// A host-to-device copy outside the process lock: ordered on a private non-blocking stream, so it
// neither disturbs another thread's capture nor blocks the other threads for its duration (a 7B
// model is 27 GB; the reference uploads from one host thread per GPU at once, src/llama.cpp:919-943).
// Only the stream's creation and destruction take the lock.
static void h2d_private(void* dst, const void* src, size_t bytes) {
  hipStream_t st = nullptr;
  {
    tl::ApiLock lock(tl::api_mu());
    CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  }
  CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
  CHECK_HIP(hipStreamSynchronize(st));
  tl::ApiLock lock(tl::api_mu());
  CHECK_HIP(hipStreamDestroy(st));
}

static void* dev_alloc(size_t bytes) {
  void* a = nullptr;
  tl::ApiLock lock(tl::api_mu());
  CHECK_HIP(hipMalloc(&a, bytes));
  return a;
}

// reference src/models.cpp:86-127: one arena, one copy (the payload is contiguous after the
// header in a v0 file, src/utils.cpp:119-177)
extern "C" void copy_weight_to_device(Transformer* t_h, TransformerWeights*& w_d) {
  const Config* p = &t_h->config;
  const int shared = t_h->weights.wcls == t_h->weights.token_embedding_table;
  const size_t n = thallama_v0_payload_floats(p, shared);
  float* arena = (float*)dev_alloc(n * sizeof(float));
  h2d_private(arena, t_h->weights.token_embedding_table, n * sizeof(float));
  w_d = (TransformerWeights*)malloc(sizeof(TransformerWeights));
  thallama_map_weights(w_d, p, arena, shared);
}

// reference src/models.cpp:9-84: a host Transformer whose weights and (one-sequence) state are
// on the device
extern "C" void copy_transformer_to_device(thablasHandle_t handle, Transformer* t_h, Transformer*& t_d) {
  (void)handle;
  t_d = (Transformer*)calloc(1, sizeof(Transformer));
  t_d->config = t_h->config;
  TransformerWeights* w = nullptr;
  copy_weight_to_device(t_h, w);
  t_d->weights = *w;
  free(w);
  RunState* s = nullptr;
  alloc_state_to_device_batch(t_h, s, 1);
  t_d->state = *s;
  free(s);
  t_d->fd = -1;
}

// reference src/models.cpp:129-153
extern "C" void alloc_state_to_device(Transformer* t_h, RunState*& s_d) { alloc_state_to_device_batch(t_h, s_d, 1); }

extern "C" void free_weight_device(TransformerWeights* w_d) {
  if (!w_d) return;
  tl::ApiLock lock(tl::api_mu());
  CHECK_HIP(hipFree(w_d->token_embedding_table));
  free(w_d);
}

// reference src/models.cpp:155-179 (same buffers and shapes, 64-bit sizes)
extern "C" void alloc_state_to_device_batch(Transformer* t_h, RunState*& s_d_batch, int batch_size) {
  const Config* p = &t_h->config;
  const size_t dim = p->dim, V = p->vocab_size, L = p->n_layers, H = p->n_heads, S = p->seq_len;
  const size_t hid = p->hidden_dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads, B = batch_size;
  RunState* s = (RunState*)calloc(1, sizeof(RunState));
  tl::ApiLock lock(tl::api_mu());
  CHECK_HIP(hipMalloc(&s->x, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->xb, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->xb2, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->hb, hid * B * 4));
  CHECK_HIP(hipMalloc(&s->hb2, hid * B * 4));
  CHECK_HIP(hipMalloc(&s->q, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->att, H * S * B * 4));
  CHECK_HIP(hipMalloc(&s->logits, V * B * 4));
  CHECK_HIP(hipMalloc(&s->key_cache, L * S * kvd * B * 4));
  CHECK_HIP(hipMalloc(&s->value_cache, L * S * kvd * B * 4));
  CHECK_HIP(hipMemset(s->key_cache, 0, L * S * kvd * B * 4));
  CHECK_HIP(hipMemset(s->value_cache, 0, L * S * kvd * B * 4));
  s_d_batch = s;
}

extern "C" void free_state_device(RunState* s) {
  if (!s) return;
  tl::ApiLock lock(tl::api_mu());
  float* bufs[] = {s->x,         s->xb,          s->xb2,        s->hb,         s->hb2,
                   s->q,         s->att,         s->logits,     s->key_cache,  s->value_cache,
                   s->key_matmul, s->value_matmul, s->key_layer_cache, s->value_layer_cache};
  for (float* b : bufs)
    if (b) CHECK_HIP(hipFree(b));
  free(s);
}

// ------------------------------------------------------------------ pipeline / 70B residency (§8(f4))
// The reference's staging for its pipeline and layer-streaming drivers (src/models.cpp:181-758),
// with the same signatures and what they hand the drivers (forward.hip: pipeline_forward,
// thaDNN_s_forward_70B).  Each device's share is ONE arena and the copies are ranges of the
// mmapped payload; the run states use the decoder's cache layout [batch][layers][seq][kv_dim].

// (layers [pipe_id * pipe_size, +pipe_size) of t_h) -> one device arena: embedding | rms_att |
// rms_ffn | wq | wk | wv | wo | w1 | w2 | w3 | rms_final | wcls (a shared classifier points at the
// embedding)
static TransformerWeights* upload_pipeline_weights(const Transformer* t_h, int pipe_size, int pipe_id) {
  const Config* p = &t_h->config;
  const size_t dim = p->dim, hid = p->hidden_dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads, P = pipe_size, l0 = (size_t)pipe_id * pipe_size;
  const TransformerWeights& h = t_h->weights;
  const bool shared = h.wcls == h.token_embedding_table;
  const struct { const float* src; size_t n; } part[12] = {
      {h.token_embedding_table, V * dim}, {h.rms_att_weight + l0 * dim, P * dim}, {h.rms_ffn_weight + l0 * dim, P * dim},
      {h.wq + l0 * dim * dim, P * dim * dim}, {h.wk + l0 * dim * kvd, P * dim * kvd}, {h.wv + l0 * dim * kvd, P * dim * kvd},
      {h.wo + l0 * dim * dim, P * dim * dim}, {h.w1 + l0 * dim * hid, P * dim * hid}, {h.w2 + l0 * dim * hid, P * dim * hid},
      {h.w3 + l0 * dim * hid, P * dim * hid}, {h.rms_final_weight, dim}, {h.wcls, shared ? 0 : V * dim}};
  size_t total = 0;
  for (const auto& e : part) total += e.n;
  float* arena = (float*)dev_alloc(total * sizeof(float));
  float* dst[12];
  size_t off = 0;
  for (int i = 0; i < 12; ++i) {
    dst[i] = arena + off;
    if (part[i].n) h2d_private(dst[i], part[i].src, part[i].n * sizeof(float));
    off += part[i].n;
  }
  TransformerWeights* w = (TransformerWeights*)calloc(1, sizeof(TransformerWeights));
  w->token_embedding_table = dst[0];
  w->rms_att_weight = dst[1]; w->rms_ffn_weight = dst[2];
  w->wq = dst[3]; w->wk = dst[4]; w->wv = dst[5]; w->wo = dst[6]; w->w1 = dst[7]; w->w2 = dst[8]; w->w3 = dst[9];
  w->rms_final_weight = dst[10];
  w->wcls = shared ? dst[0] : dst[11];
  return w;
}

// A run state for `batch` sequences over `layers` layers (the decoder's layout); key/value_matmul
// are the reference pipeline's per-step K/V rows (kept for the struct's users; the decoder writes
// K/V straight into the cache).
static RunState* alloc_stage_state(const Config* p, int layers, int batch) {
  const size_t dim = p->dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size, H = p->n_heads, S = p->seq_len;
  const size_t hid = p->hidden_dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads, B = batch, L = layers;
  RunState* s = (RunState*)calloc(1, sizeof(RunState));
  tl::ApiLock lock(tl::api_mu());
  CHECK_HIP(hipMalloc(&s->x, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->xb, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->xb2, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->hb, hid * B * 4));
  CHECK_HIP(hipMalloc(&s->hb2, hid * B * 4));
  CHECK_HIP(hipMalloc(&s->q, dim * B * 4));
  CHECK_HIP(hipMalloc(&s->att, H * S * B * 4));
  CHECK_HIP(hipMalloc(&s->logits, V * B * 4));
  CHECK_HIP(hipMalloc(&s->key_cache, L * S * kvd * B * 4));
  CHECK_HIP(hipMalloc(&s->value_cache, L * S * kvd * B * 4));
  CHECK_HIP(hipMemset(s->key_cache, 0, L * S * kvd * B * 4));
  CHECK_HIP(hipMemset(s->value_cache, 0, L * S * kvd * B * 4));
  CHECK_HIP(hipMalloc(&s->key_matmul, kvd * B * 4));
  CHECK_HIP(hipMalloc(&s->value_matmul, kvd * B * 4));
  return s;
}

extern "C" void set_transformer(void) {}

// reference src/models.cpp:327-372
extern "C" void copy_transformer_weight_pipeline_to_device_batch(Transformer* t_h, TransformerWeights*& w_d, int pipe_size,
                                                                 int pipe_id, int batch_size) {
  (void)batch_size;
  w_d = upload_pipeline_weights(t_h, pipe_size, pipe_id);
}

// reference src/models.cpp:374-408
extern "C" void alloc_run_state_to_device_batch(thablasHandle_t, Transformer* t_h, RunState*& s_d, int pipe_size, int pipe_id,
                                                int batch_size) {
  (void)pipe_id;
  s_d = alloc_stage_state(&t_h->config, pipe_size, batch_size);
}

// reference src/models.cpp:255-325: weights and state of one stage in a device Transformer (its
// config stays the whole model's)
extern "C" void copy_transformer_pipeline_to_device_batch(thablasHandle_t, Transformer* t_h, Transformer*& t_d, int pipe_size,
                                                          int pipe_id, int batch_size) {
  t_d = (Transformer*)calloc(1, sizeof(Transformer));
  t_d->config = t_h->config;
  TransformerWeights* w = upload_pipeline_weights(t_h, pipe_size, pipe_id);
  t_d->weights = *w;
  free(w);
  RunState* s = alloc_stage_state(&t_h->config, pipe_size, batch_size);
  t_d->state = *s;
  free(s);
  t_d->fd = -1;
}

// reference src/models.cpp:181-253
extern "C" void copy_transformer_pipeline_to_device(thablasHandle_t handle, Transformer* t_h, Transformer*& t_d, int pipe_size,
                                                    int pipe_id) {
  copy_transformer_pipeline_to_device_batch(handle, t_h, t_d, pipe_size, pipe_id, 1);
}

// reference src/models.cpp:410-440: the host half of the layer-swapped cache.  An MI355X keeps the
// whole cache on the device (below), so the host state holds no buffers.
extern "C" void alloc_swap_run_state_on_host_batch(thablasHandle_t, Transformer*, RunState*& s_h, int, int, int, int) {
  s_h = (RunState*)calloc(1, sizeof(RunState));
}

// reference src/models.cpp:442-476: the device half, n_buffer_words positions there and the rest
// swapped to host per layer; here every position (seq_len) lives on the device.
extern "C" void alloc_swap_run_state_to_device_batch(thablasHandle_t, Transformer* t_h, RunState*& s_d, int pipe_size, int,
                                                     int batch_size, int n_buffer_words) {
  (void)n_buffer_words;
  s_d = alloc_stage_state(&t_h->config, pipe_size, batch_size);
}

// reference src/models.cpp:511-692: every layer's weights in pinned host memory (H2D copies at the
// link's full rate), h_w[l] per layer.  The K/V cache stays on the device (alloc_state_to_device_
// 70B), so the per-device host states hold no buffers.
extern "C" void copy_transformer_to_host_70B(Transformer* storage_t, TransformerWeights* h_w[], RunState* h_s[], int n_devices) {
  const Config* p = &storage_t->config;
  const size_t dim = p->dim, hid = p->hidden_dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const TransformerWeights& s = storage_t->weights;
  const size_t layer = 2 * dim + 2 * dim * dim + 2 * dim * kvd + 3 * dim * hid;
  for (int l = 0; l < p->n_layers; ++l) {
    float* h = nullptr;
    {
      tl::ApiLock lock(tl::api_mu());
      CHECK_HIP(hipHostMalloc(&h, layer * sizeof(float), hipHostMallocDefault));
    }
    const size_t L = l;
    TransformerWeights* w = (TransformerWeights*)calloc(1, sizeof(TransformerWeights));
    const struct { float** dst; const float* src; size_t n; } t[9] = {
        {&w->rms_att_weight, s.rms_att_weight + L * dim, dim}, {&w->rms_ffn_weight, s.rms_ffn_weight + L * dim, dim},
        {&w->wq, s.wq + L * dim * dim, dim * dim}, {&w->wk, s.wk + L * dim * kvd, dim * kvd},
        {&w->wv, s.wv + L * dim * kvd, dim * kvd}, {&w->wo, s.wo + L * dim * dim, dim * dim},
        {&w->w1, s.w1 + L * dim * hid, dim * hid}, {&w->w2, s.w2 + L * dim * hid, dim * hid},
        {&w->w3, s.w3 + L * dim * hid, dim * hid}};
    for (const auto& e : t) {
      *e.dst = h;
      memcpy(h, e.src, e.n * sizeof(float));
      h += e.n;
    }
    h_w[l] = w;
  }
  for (int g = 0; g < n_devices; ++g) h_s[g] = (RunState*)calloc(1, sizeof(RunState));
}

// reference src/models.cpp:694-717: one sequence's state; every layer's K/V rows live here
extern "C" void alloc_state_to_device_70B(Transformer* t_h, RunState*& d_s) {
  d_s = alloc_stage_state(&t_h->config, t_h->config.n_layers, 1);
}

// reference src/models.cpp:719-758: embedding, final norm and classifier on the device, plus two
// staging slots for the streamed layers (rms_att | rms_ffn | wq | wk | wv | wo | w1 | w2 | w3 each,
// slot 1 right after slot 0; the per-layer fields point at slot 0)
extern "C" void alloc_weight_to_device_70B(Transformer* h_t, TransformerWeights*& d_w) {
  const Config* p = &h_t->config;
  const size_t dim = p->dim, hid = p->hidden_dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t layer = 2 * dim + 2 * dim * dim + 2 * dim * kvd + 3 * dim * hid;
  const TransformerWeights& h = h_t->weights;
  const bool shared = h.wcls == h.token_embedding_table;
  float* a = (float*)dev_alloc((V * dim + dim + (shared ? 0 : V * dim) + 2 * layer) * sizeof(float));
  d_w = (TransformerWeights*)calloc(1, sizeof(TransformerWeights));
  d_w->token_embedding_table = a;
  h2d_private(a, h.token_embedding_table, V * dim * sizeof(float));
  a += V * dim;
  d_w->rms_final_weight = a;
  h2d_private(a, h.rms_final_weight, dim * sizeof(float));
  a += dim;
  if (shared) {
    d_w->wcls = d_w->token_embedding_table;
  } else {
    d_w->wcls = a;
    h2d_private(a, h.wcls, V * dim * sizeof(float));
    a += V * dim;
  }
  float** f[9] = {&d_w->rms_att_weight, &d_w->rms_ffn_weight, &d_w->wq, &d_w->wk, &d_w->wv, &d_w->wo, &d_w->w1,
                  &d_w->w2, &d_w->w3};
  const size_t n[9] = {dim, dim, dim * dim, dim * kvd, dim * kvd, dim * dim, dim * hid, dim * hid, dim * hid};
  for (int i = 0; i < 9; ++i) {
    *f[i] = a;
    a += n[i];
  }
}

extern "C" void free_transformer_device(void) {}

// ------------------------------------------------------------------ synthetic weights
__global__ void __launch_bounds__(256) k_synth(float* dst, size_t n, uint64_t tseed, float scale) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = tl_synth_value(tseed, i, scale);
}

__global__ void __launch_bounds__(256) k_fill(float* dst, size_t n, float v) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = v;
}

extern "C" int thallama_synth_arena(float* arena, const Config* cfg, int shared_weights, uint64_t seed,
                                    hipStream_t stream) {
  TlSynthPlan plan;
  tl_synth_plan(&plan, cfg, shared_weights);
  tl::ApiLock lock(tl::api_mu());  // (launches on the legacy stream when stream is null)
  for (int t = 0; t < plan.n; ++t) {
    const TlSynthTensor& e = plan.t[t];
    if (!e.count) continue;
    float* dst = arena + e.offset;
    int blocks = (int)((e.count + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    if (e.kind == TL_SYNTH_NORMAL) {
      hipLaunchKernelGGL(k_synth, dim3(blocks), dim3(256), 0, stream, dst, e.count, tl_synth_tensor_seed(seed, e.id),
                         tl_synth_scale(e.stddev));
    } else {
      hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, stream, dst, e.count, e.value);
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return (int)err;
  }
  return 0;
}

// ------------------------------------------------------------------ helpers
extern "C" int thallama_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
extern "C" int thallama_set_device(int dev) { return (int)hipSetDevice(dev); }
extern "C" void* thallama_malloc(size_t bytes) {
  tl::ApiLock lock(tl::api_mu());
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  return p;
}
extern "C" int thallama_free(void* p) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipFree(p);
}
extern "C" int thallama_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
}
extern "C" int thallama_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
}
extern "C" int thallama_memcpy_d2d(void* dst, const void* src, size_t bytes) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice);
}
extern "C" int thallama_memset(void* dst, int value, size_t bytes) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipMemset(dst, value, bytes);
}
extern "C" int thallama_sync(void) {
  tl::ApiLock lock(tl::api_mu());
  return (int)hipDeviceSynchronize();
}

namespace tl {
std::recursive_mutex& api_mu() {
  static std::recursive_mutex m;
  return m;
}
}  // namespace tl
