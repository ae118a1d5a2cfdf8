/* oracle.c — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (hip_llama.cpp_amd/).  Only tests/, the smoke check
 * in __graft_entry__.py and bench.py's cpu_baseline leg use it, and only as the
 * checker / CPU baseline.
 *
 * A plain-C restatement of the reference's CPU decode path:
 *   fp32 : /root/reference/src/seq.cpp  (rmsnorm :3-16, softmax :18-36,
 *          matmul :40-51, forward :53-183)
 *   int8 : /root/reference/runq.c       (quantize :145-171, matmul :317-342,
 *          forward :344-481; weight Q8_0 quantisation per train/export.py:46-70)
 * Every floating-point operation is done in the reference's order with no
 * contraction (build with -ffp-contract=off), so the fp32 forward is
 * bit-identical to the reference compiled for x86-64 — checked against the
 * reference itself (oracle/_ref, built by oracle/Makefile from the reference
 * sources) by tests/test_oracle.py and pinned by tests/golden/.
 * The matmul row loop may run on several OpenMP threads: each row's sum is
 * still sequential, so results do not depend on the thread count.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/thallama_synth.h"

typedef struct {
  int dim, hidden_dim, n_layers, n_heads, n_kv_heads, vocab_size, seq_len;
} OCfg;

typedef struct {
  int8_t* q;
  float* s;
} OQT; /* runq.c:34-37 QuantizedTensor */

typedef struct {
  OCfg c;
  int shared;
  float* arena; /* v0 payload (owned) */
  size_t n;
  float *emb, *rms_att, *wq, *wk, *wv, *wo, *rms_ffn, *w1, *w2, *w3, *rms_final, *wcls;
  /* RunState (reference include/models.hpp:41-60, single sequence) */
  float *x, *xb, *xb2, *hb, *hb2, *q, *att, *logits, *kc, *vc;
  /* int8 twin (runq.c) */
  int gs;
  unsigned char* q8arena; /* v2 payload after the 256-B header (owned) */
  size_t q8bytes;
  float* q8_emb;          /* dequantised embedding (runq.c:199-201) */
  OQT *q_tok, *q_wq, *q_wk, *q_wv, *q_wo, *q_w1, *q_w2, *q_w3, *q_wcls;
  OQT xq, hq;
  float *k, *v;
  int view; /* 1: a second decoder over another model's weights (owns its RunState only) */
  double *kc64, *vc64; /* forward_f64's own K/V rows (flag kF64OwnCache), lazily allocated */
} OModel;

static int g_threads = 1;
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int oracle_get_threads(void) { return g_threads; }

/* ------------------------------------------------------------ fp32 ops */
/* seq.cpp:3-16 */
void oracle_rmsnorm(float* o, const float* x, const float* weight, int size) {
  float ss = 0.0f;
  for (int j = 0; j < size; j++) ss += x[j] * x[j];
  ss /= size;
  ss += 1e-5f;
  ss = 1.0f / sqrtf(ss);
  for (int j = 0; j < size; j++) o[j] = weight[j] * (ss * x[j]);
}

/* seq.cpp:18-36 */
void oracle_softmax(float* x, int size) {
  float max_val = x[0];
  for (int i = 1; i < size; i++)
    if (x[i] > max_val) max_val = x[i];
  float sum = 0.0f;
  for (int i = 0; i < size; i++) {
    x[i] = expf(x[i] - max_val);
    sum += x[i];
  }
  for (int i = 0; i < size; i++) x[i] /= sum;
}

/* seq.cpp:40-51: W (d,n) @ x (n,) -> xout (d,) */
void oracle_matmul(float* xout, const float* x, const float* w, int n, int d) {
  int i;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1 && (long)n * d > 65536) schedule(static)
  for (i = 0; i < d; i++) {
    float val = 0.0f;
    const float* wr = w + (size_t)i * n;
    for (int j = 0; j < n; j++) val += wr[j] * x[j];
    xout[i] = val;
  }
}

/* seq.cpp:87-101 (rotates q for i < dim, k for i < kv_dim) */
void oracle_rope(float* q, float* k, int dim, int head_size, int kv_dim, int pos) {
  for (int i = 0; i < dim; i += 2) {
    int head_dim = i % head_size;
    float freq = 1.0f / powf(10000.0f, head_dim / (float)head_size);
    float val = pos * freq;
    float fcr = cosf(val);
    float fci = sinf(val);
    int rotn = i < kv_dim ? 2 : 1;
    for (int v = 0; v < rotn; v++) {
      float* vec = v == 0 ? q : k;
      float v0 = vec[i];
      float v1 = vec[i + 1];
      vec[i] = v0 * fcr - v1 * fci;
      vec[i + 1] = v0 * fci + v1 * fcr;
    }
  }
}

/* seq.cpp:159-166 */
void oracle_swiglu(float* hb, const float* hb2, int n) {
  for (int i = 0; i < n; i++) {
    float val = hb[i];
    val *= (1.0f / (1.0f + expf(-val)));
    val *= hb2[i];
    hb[i] = val;
  }
}

/* The 3-kernel attention API (src/thaDNN/thaDNN_mha.cpp) for one sequence, layer offset
 * already applied: scores, softmax, weighted V sum; seq.cpp:103-136. */
void oracle_attention(float* xb, float* att, const float* q, const float* kc, const float* vc, int pos, int n_heads,
                      int head_size, int kv_dim, int kv_mul, int seq_len) {
  for (int h = 0; h < n_heads; h++) {
    const float* qh = q + h * head_size;
    float* a = att + (size_t)h * seq_len;
    for (int t = 0; t <= pos; t++) {
      const float* k = kc + (size_t)t * kv_dim + (h / kv_mul) * head_size;
      float score = 0.0f;
      for (int i = 0; i < head_size; i++) score += qh[i] * k[i];
      score /= sqrtf(head_size);
      a[t] = score;
    }
    oracle_softmax(a, pos + 1);
    float* o = xb + h * head_size;
    memset(o, 0, head_size * sizeof(float));
    for (int t = 0; t <= pos; t++) {
      const float* v = vc + (size_t)t * kv_dim + (h / kv_mul) * head_size;
      float w = a[t];
      for (int i = 0; i < head_size; i++) o[i] += w * v[i];
    }
  }
}

/* ------------------------------------------------------------ model */
static void map_v0(OModel* m) {
  const OCfg* p = &m->c;
  const size_t L = p->n_layers, dim = p->dim, hs = p->dim / p->n_heads;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads, V = p->vocab_size;
  float* ptr = m->arena;
  m->emb = ptr; ptr += V * dim;
  m->rms_att = ptr; ptr += L * dim;
  m->wq = ptr; ptr += L * dim * dim;
  m->wk = ptr; ptr += L * dim * kvd;
  m->wv = ptr; ptr += L * dim * kvd;
  m->wo = ptr; ptr += L * dim * dim;
  m->rms_ffn = ptr; ptr += L * dim;
  m->w1 = ptr; ptr += L * dim * p->hidden_dim;
  m->w2 = ptr; ptr += L * dim * p->hidden_dim;
  m->w3 = ptr; ptr += L * dim * p->hidden_dim;
  m->rms_final = ptr; ptr += dim;
  ptr += (size_t)p->seq_len * hs; /* freq_cis_real + imag */
  m->wcls = m->shared ? m->emb : ptr;
}

size_t oracle_payload_floats(const OCfg* p, int shared) {
  const size_t L = p->n_layers, dim = p->dim, hs = p->dim / p->n_heads;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads, V = p->vocab_size;
  size_t n = V * dim + 2 * L * dim + 2 * L * dim * dim + 2 * L * dim * kvd + 3 * L * dim * p->hidden_dim + dim +
             (size_t)p->seq_len * hs;
  if (!shared) n += V * dim;
  return n;
}

static int alloc_state(OModel* m) {
  const OCfg* p = &m->c;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  m->x = calloc(p->dim, 4); m->xb = calloc(p->dim, 4); m->xb2 = calloc(p->dim, 4);
  m->hb = calloc(p->hidden_dim, 4); m->hb2 = calloc(p->hidden_dim, 4); m->q = calloc(p->dim, 4);
  m->att = calloc((size_t)p->n_heads * p->seq_len, 4); m->logits = calloc(p->vocab_size, 4);
  m->kc = calloc((size_t)p->n_layers * p->seq_len * kvd, 4);
  m->vc = calloc((size_t)p->n_layers * p->seq_len * kvd, 4);
  m->k = calloc(kvd, 4); m->v = calloc(kvd, 4);
  return m->x && m->xb && m->xb2 && m->hb && m->hb2 && m->q && m->att && m->logits && m->kc && m->vc && m->k && m->v;
}

/* Build a model over a copy of a v0 payload (or the synthetic generator when arena == NULL). */
OModel* oracle_model_new(const OCfg* c, int shared, const float* arena, uint64_t seed) {
  OModel* m = calloc(1, sizeof(OModel));
  if (!m) return NULL;
  m->c = *c;
  if (m->c.vocab_size < 0) m->c.vocab_size = -m->c.vocab_size;
  m->shared = shared;
  m->n = oracle_payload_floats(&m->c, shared);
  m->arena = malloc(m->n * sizeof(float));
  if (!m->arena) { free(m); return NULL; }
  if (arena) {
    memcpy(m->arena, arena, m->n * sizeof(float));
  } else {
    TlSynthPlan plan;
    tl_synth_plan(&plan, &m->c, shared);
    for (int t = 0; t < plan.n; ++t) {
      const TlSynthTensor* e = &plan.t[t];
      float* dst = m->arena + e->offset;
      if (e->kind == TL_SYNTH_NORMAL) {
        const uint64_t ts = tl_synth_tensor_seed(seed, e->id);
        const float sc = tl_synth_scale(e->stddev);
        long long i;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
        for (i = 0; i < (long long)e->count; ++i) dst[i] = tl_synth_value(ts, (uint64_t)i, sc);
      } else {
        for (size_t i = 0; i < e->count; ++i) dst[i] = e->value;
      }
    }
  }
  map_v0(m);
  if (!alloc_state(m)) return NULL;
  return m;
}

float* oracle_model_arena(OModel* m) { return m->arena; }
size_t oracle_model_arena_floats(OModel* m) { return m->n; }
float* oracle_model_logits(OModel* m) { return m->logits; }
float* oracle_model_kcache(OModel* m) { return m->kc; }
float* oracle_model_vcache(OModel* m) { return m->vc; }
float* oracle_model_x(OModel* m) { return m->x; }
/* RunState buffers after a forward (diagnostics): 0 x, 1 xb, 2 xb2, 3 hb, 4 hb2, 5 q, 6 k, 7 v */
float* oracle_model_buf(OModel* m, int which) {
  float* b[8] = {m->x, m->xb, m->xb2, m->hb, m->hb2, m->q, m->k, m->v};
  return which >= 0 && which < 8 ? b[which] : NULL;
}

void oracle_model_reset_kv(OModel* m) {
  const OCfg* p = &m->c;
  const size_t kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  memset(m->kc, 0, (size_t)p->n_layers * p->seq_len * kvd * 4);
  memset(m->vc, 0, (size_t)p->n_layers * p->seq_len * kvd * 4);
}

/* Write a llama2.c v0 model.bin (28-byte Config header, negative vocab = unshared). */
int oracle_write_v0(OModel* m, const char* path) {
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  OCfg h = m->c;
  if (!m->shared) h.vocab_size = -h.vocab_size;
  int ok = fwrite(&h, sizeof(h), 1, f) == 1 && fwrite(m->arena, sizeof(float), m->n, f) == m->n;
  fclose(f);
  return ok ? 0 : -1;
}

void oracle_model_free(OModel* m) {
  if (!m) return;
  free(m->kc64);
  free(m->vc64);
  if (m->view) {
    free(m->x); free(m->xb); free(m->xb2); free(m->hb); free(m->hb2); free(m->q);
    free(m->att); free(m->logits); free(m->kc); free(m->vc); free(m->k); free(m->v);
    free(m->xq.q); free(m->xq.s); free(m->hq.q); free(m->hq.s);
    free(m);
    return;
  }
  free(m->arena);
  free(m->x); free(m->xb); free(m->xb2); free(m->hb); free(m->hb2); free(m->q);
  free(m->att); free(m->logits); free(m->kc); free(m->vc); free(m->k); free(m->v);
  free(m->q8arena); free(m->q8_emb);
  free(m->q_tok); free(m->q_wq); free(m->q_wk); free(m->q_wv); free(m->q_wo);
  free(m->q_w1); free(m->q_w2); free(m->q_w3);
  if (m->q_wcls && !m->shared) free(m->q_wcls);
  free(m->xq.q); free(m->xq.s); free(m->hq.q); free(m->hq.s);
  free(m);
}

/* seq.cpp:53-183 */
float* oracle_forward(OModel* m, int token, int pos) {
  const OCfg* p = &m->c;
  float* x = m->x;
  const int dim = p->dim;
  const int kv_dim = (p->dim * p->n_kv_heads) / p->n_heads;
  const int kv_mul = p->n_heads / p->n_kv_heads;
  const int hidden_dim = p->hidden_dim;
  const int head_size = dim / p->n_heads;
  memcpy(x, m->emb + (size_t)token * dim, dim * sizeof(*x));
  for (unsigned long long l = 0; l < (unsigned long long)p->n_layers; l++) {
    oracle_rmsnorm(m->xb, x, m->rms_att + l * dim, dim);
    const size_t loff = l * p->seq_len * (size_t)kv_dim;
    float* k = m->kc + loff + (size_t)pos * kv_dim;
    float* v = m->vc + loff + (size_t)pos * kv_dim;
    oracle_matmul(m->q, m->xb, m->wq + l * dim * dim, dim, dim);
    oracle_matmul(k, m->xb, m->wk + l * dim * kv_dim, dim, kv_dim);
    oracle_matmul(v, m->xb, m->wv + l * dim * kv_dim, dim, kv_dim);
    oracle_rope(m->q, k, dim, head_size, kv_dim, pos);
    oracle_attention(m->xb, m->att, m->q, m->kc + loff, m->vc + loff, pos, p->n_heads, head_size, kv_dim, kv_mul,
                     p->seq_len);
    oracle_matmul(m->xb2, m->xb, m->wo + l * dim * dim, dim, dim);
    for (int i = 0; i < dim; i++) x[i] += m->xb2[i];
    oracle_rmsnorm(m->xb, x, m->rms_ffn + l * dim, dim);
    oracle_matmul(m->hb, m->xb, m->w1 + l * dim * hidden_dim, dim, hidden_dim);
    oracle_matmul(m->hb2, m->xb, m->w3 + l * dim * hidden_dim, dim, hidden_dim);
    oracle_swiglu(m->hb, m->hb2, hidden_dim);
    oracle_matmul(m->xb, m->hb, m->w2 + l * dim * hidden_dim, hidden_dim, dim);
    for (int i = 0; i < dim; i++) x[i] += m->xb[i];
  }
  oracle_rmsnorm(x, x, m->rms_final, dim);
  oracle_matmul(m->logits, x, m->wcls, p->dim, p->vocab_size);
  return m->logits;
}

/* The same forward (seq.cpp:53-183) with every accumulation, product, norm, softmax and SwiGLU in
 * double precision: the exact value of the reference's arithmetic up to ~1e-16, used only to
 * attribute a GPU-vs-CPU logit difference (which side carries the rounding error).  Reads the
 * fp32 weights and the K/V rows 0..pos-1 of m's cache (as float); the current position's K/V
 * are kept in double and m is not modified.  The RoPE (cos, sin) are the reference's float values
 * (powf/cosf/sinf of the float angle, seq.cpp:88-92): parameters, not accumulations. */
static void matmul_f64(double* xout, const double* x, const float* w, int n, int d) {
  int i;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1 && (long)n * d > 65536) schedule(static)
  for (i = 0; i < d; i++) {
    double val = 0.0;
    const float* wr = w + (size_t)i * n;
    for (int j = 0; j < n; j++) val += (double)wr[j] * x[j];
    xout[i] = val;
  }
}

static void rmsnorm_f64(double* o, const double* x, const float* weight, int size) {
  double ss = 0.0;
  for (int j = 0; j < size; j++) ss += x[j] * x[j];
  ss = 1.0 / sqrt(ss / size + (double)1e-5f);
  for (int j = 0; j < size; j++) o[j] = (double)weight[j] * (ss * x[j]);
}

/* flags: kF64RopeDouble — RoPE's (cos, sin) computed in double like every other quantity (default:
 * the reference's float values, which its fp32 forward and the GPU use); kF64OwnCache — the K/V rows
 * of earlier positions from this function's own double cache (written at every call) instead of the
 * fp32 cache.  With both, this is the reference's src/seq.cpp widened to double, which
 * oracle/ref_f64_driver.cpp builds from the reference source itself
 * (tests/test_oracle.py::test_forward_f64_matches_widened_reference). */
enum { kF64RopeDouble = 1, kF64OwnCache = 2 };
static int forward_f64_impl(OModel* m, int token, int pos, double* logits, int flags);
int oracle_forward_f64(OModel* m, int token, int pos, double* logits) { return forward_f64_impl(m, token, pos, logits, 0); }
int oracle_forward_f64_ex(OModel* m, int token, int pos, double* logits, int flags) {
  return forward_f64_impl(m, token, pos, logits, flags);
}

static int forward_f64_impl(OModel* m, int token, int pos, double* logits, int flags) {
  const int rope_double = flags & kF64RopeDouble;
  const size_t cache_n = (size_t)m->c.n_layers * m->c.seq_len * ((size_t)m->c.dim * m->c.n_kv_heads / m->c.n_heads);
  if ((flags & kF64OwnCache) && !m->kc64) {
    m->kc64 = (double*)calloc(cache_n, sizeof(double));
    m->vc64 = (double*)calloc(cache_n, sizeof(double));
    if (!m->kc64 || !m->vc64) return -1;
  }
  const double* kc64 = (flags & kF64OwnCache) ? m->kc64 : NULL;
  const double* vc64 = (flags & kF64OwnCache) ? m->vc64 : NULL;
  const OCfg* p = &m->c;
  const int dim = p->dim, hid = p->hidden_dim, hs = dim / p->n_heads;
  const int kvd = (p->dim * p->n_kv_heads) / p->n_heads, kv_mul = p->n_heads / p->n_kv_heads;
  const size_t big = (size_t)(hid > dim ? hid : dim);
  double* x = (double*)malloc(sizeof(double) * dim);
  double* xb = (double*)malloc(sizeof(double) * big);
  double* xb2 = (double*)malloc(sizeof(double) * dim);
  double* q = (double*)malloc(sizeof(double) * dim);
  double* k = (double*)malloc(sizeof(double) * kvd);
  double* v = (double*)malloc(sizeof(double) * kvd);
  double* hb = (double*)malloc(sizeof(double) * hid);
  double* hb2 = (double*)malloc(sizeof(double) * hid);
  double* att = (double*)malloc(sizeof(double) * (pos + 1));
  if (!x || !xb || !xb2 || !q || !k || !v || !hb || !hb2 || !att) return -1;
  for (int i = 0; i < dim; i++) x[i] = m->emb[(size_t)token * dim + i];
  for (int l = 0; l < p->n_layers; l++) {
    const size_t L = l;
    rmsnorm_f64(xb, x, m->rms_att + L * dim, dim);
    matmul_f64(q, xb, m->wq + L * dim * dim, dim, dim);
    matmul_f64(k, xb, m->wk + L * dim * kvd, dim, kvd);
    matmul_f64(v, xb, m->wv + L * dim * kvd, dim, kvd);
    for (int i = 0; i < dim; i += 2) {
      const int head_dim = i % hs;
      double fcr, fci;
      if (rope_double) {
        const double freq = 1.0 / pow(10000.0, head_dim / (double)hs), val = pos * freq;
        fcr = cos(val);
        fci = sin(val);
      } else {
        const float freq = 1.0f / powf(10000.0f, head_dim / (float)hs);
        const float val = pos * freq;
        fcr = cosf(val);
        fci = sinf(val);
      }
      for (int r = 0; r < (i < kvd ? 2 : 1); r++) {
        double* vec = r == 0 ? q : k;
        const double v0 = vec[i], v1 = vec[i + 1];
        vec[i] = v0 * fcr - v1 * fci;
        vec[i + 1] = v0 * fci + v1 * fcr;
      }
    }
    const size_t loff = L * p->seq_len * (size_t)kvd;
    if (flags & kF64OwnCache) {
      memcpy(m->kc64 + loff + (size_t)pos * kvd, k, sizeof(double) * kvd);
      memcpy(m->vc64 + loff + (size_t)pos * kvd, v, sizeof(double) * kvd);
    }
    for (int h = 0; h < p->n_heads; h++) {
      const double* qh = q + h * hs;
      const int off = (h / kv_mul) * hs;
      double mx = -1e300, sum = 0.0;
      for (int t = 0; t <= pos; t++) {
        double sc = 0.0;
        for (int i = 0; i < hs; i++)
          sc += qh[i] * (t < pos ? (kc64 ? kc64[loff + (size_t)t * kvd + off + i]
                                         : (double)m->kc[loff + (size_t)t * kvd + off + i])
                                 : k[off + i]);
        att[t] = sc / sqrt((double)hs);
        if (att[t] > mx) mx = att[t];
      }
      for (int t = 0; t <= pos; t++) {
        att[t] = exp(att[t] - mx);
        sum += att[t];
      }
      double* o = xb + h * hs;
      for (int i = 0; i < hs; i++) o[i] = 0.0;
      for (int t = 0; t <= pos; t++) {
        const double w = att[t] / sum;
        for (int i = 0; i < hs; i++)
          o[i] += w * (t < pos ? (vc64 ? vc64[loff + (size_t)t * kvd + off + i]
                                       : (double)m->vc[loff + (size_t)t * kvd + off + i])
                               : v[off + i]);
      }
    }
    matmul_f64(xb2, xb, m->wo + L * dim * dim, dim, dim);
    for (int i = 0; i < dim; i++) x[i] += xb2[i];
    rmsnorm_f64(xb, x, m->rms_ffn + L * dim, dim);
    matmul_f64(hb, xb, m->w1 + L * dim * hid, dim, hid);
    matmul_f64(hb2, xb, m->w3 + L * dim * hid, dim, hid);
    for (int i = 0; i < hid; i++) hb[i] = hb[i] * (1.0 / (1.0 + exp(-hb[i]))) * hb2[i];
    matmul_f64(xb, hb, m->w2 + L * dim * hid, hid, dim);
    for (int i = 0; i < dim; i++) x[i] += xb[i];
  }
  rmsnorm_f64(xb, x, m->rms_final, dim);
  matmul_f64(logits, xb, m->wcls, dim, p->vocab_size);
  free(x); free(xb); free(xb2); free(q); free(k); free(v); free(hb); free(hb2); free(att);
  return 0;
}

/* ------------------------------------------------------------ lockstep batch (fixture generation) */
/* B independent sequences over ONE copy of the weights, each a view (oracle_model_view_cap) with
 * its own RunState and K/V cache, stepped together: every per-sequence value is computed exactly
 * as oracle_forward computes it — each matmul row is the same left-to-right chain from 0.0f, with
 * no contraction — so views[b]->logits after a call is bit-identical to
 * oracle_forward(views[b], tokens[b], pos[b]) (tests/test_oracle.py checks it).  Only the loop
 * nest differs: a tile of 8 rows x 16 sequences walks j once, so the weights are read once per
 * step instead of once per sequence and 8 independent chains keep the adders busy.  Used to make
 * the 7B request-workload fixture (tests/golden/make_golden_requests.py). */
typedef float ov16 __attribute__((vector_size(64)));
#define OM_R 8  /* rows per tile */
#define OM_S 16 /* sequences per tile (one ov16) */

__attribute__((target_clones("avx512f", "avx2", "default")))
static void matmul_tile(float* acc_out, const float* w, const float* xt, int n, int rows) {
  /* acc_out [OM_R][OM_S]; w rows r < rows of length n; xt [n][OM_S] */
  ov16 acc[OM_R];
  for (int r = 0; r < OM_R; r++) acc[r] = (ov16){0};
  const float* wr[OM_R];
  for (int r = 0; r < OM_R; r++) wr[r] = w + (size_t)(r < rows ? r : 0) * n;
  for (int j = 0; j < n; j++) {
    ov16 xv;
    memcpy(&xv, xt + (size_t)j * OM_S, sizeof xv);
    for (int r = 0; r < OM_R; r++) {
      const ov16 p = wr[r][j] * xv; /* -ffp-contract=off: a separate multiply and add */
      acc[r] = acc[r] + p;
    }
  }
  memcpy(acc_out, acc, sizeof acc);
}

/* xout[b][i] = sum_j w[i][j] * x[b][j], i < d, in seq.cpp:40-51's order for every b */
static void matmul_multi(float* const* xout, float* const* x, const float* w, int n, int d, int B, float* xt) {
  for (int s0 = 0; s0 < B; s0 += OM_S) {
    const int ns = B - s0 < OM_S ? B - s0 : OM_S;
    for (int j = 0; j < n; j++)
      for (int s = 0; s < OM_S; s++) xt[(size_t)j * OM_S + s] = s < ns ? x[s0 + s][j] : 0.0f;
    const int tiles = (d + OM_R - 1) / OM_R;
    int t;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(dynamic, 4)
    for (t = 0; t < tiles; t++) {
      const int i0 = t * OM_R, rows = d - i0 < OM_R ? d - i0 : OM_R;
      float acc[OM_R][OM_S];
      matmul_tile(&acc[0][0], w + (size_t)i0 * n, xt, n, rows);
      for (int r = 0; r < rows; r++)
        for (int s = 0; s < ns; s++) xout[s0 + s][i0 + r] = acc[r][s];
    }
  }
}

OModel* oracle_model_view_cap(OModel* m, int seq_cap);

int oracle_forward_multi(OModel** ms, int B, const int* tokens, const int* pos) {
  if (B <= 0) return 0;
  const OCfg* p = &ms[0]->c;
  const int dim = p->dim, hid = p->hidden_dim, hs = dim / p->n_heads;
  const int kvd = (p->dim * p->n_kv_heads) / p->n_heads, kv_mul = p->n_heads / p->n_kv_heads;
  for (int b = 0; b < B; b++)
    if (pos[b] < 0 || pos[b] >= ms[b]->c.seq_len || ms[b]->emb != ms[0]->emb) return -1;
  float** in = malloc(sizeof(float*) * B);
  float** out = malloc(sizeof(float*) * B);
  float** out2 = malloc(sizeof(float*) * B);
  float* xt = malloc(sizeof(float) * (size_t)(hid > dim ? hid : dim) * OM_S);
  if (!in || !out || !out2 || !xt) { free(in); free(out); free(out2); free(xt); return -1; }
  const OModel* w = ms[0];
  int b;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
  for (b = 0; b < B; b++) memcpy(ms[b]->x, w->emb + (size_t)tokens[b] * dim, dim * sizeof(float));
  for (unsigned long long l = 0; l < (unsigned long long)p->n_layers; l++) {
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
    for (b = 0; b < B; b++) oracle_rmsnorm(ms[b]->xb, ms[b]->x, w->rms_att + l * dim, dim);
    for (b = 0; b < B; b++) in[b] = ms[b]->xb, out[b] = ms[b]->q;
    matmul_multi(out, in, w->wq + l * dim * dim, dim, dim, B, xt);
    for (b = 0; b < B; b++) out[b] = ms[b]->kc + l * ms[b]->c.seq_len * (size_t)kvd + (size_t)pos[b] * kvd;
    matmul_multi(out, in, w->wk + l * dim * kvd, dim, kvd, B, xt);
    for (b = 0; b < B; b++) out2[b] = ms[b]->vc + l * ms[b]->c.seq_len * (size_t)kvd + (size_t)pos[b] * kvd;
    matmul_multi(out2, in, w->wv + l * dim * kvd, dim, kvd, B, xt);
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(dynamic, 1)
    for (b = 0; b < B; b++) {
      OModel* m = ms[b];
      const size_t loff = l * m->c.seq_len * (size_t)kvd;
      oracle_rope(m->q, m->kc + loff + (size_t)pos[b] * kvd, dim, hs, kvd, pos[b]);
      oracle_attention(m->xb, m->att, m->q, m->kc + loff, m->vc + loff, pos[b], p->n_heads, hs, kvd, kv_mul,
                       m->c.seq_len);
    }
    for (b = 0; b < B; b++) out[b] = ms[b]->xb2;
    matmul_multi(out, in, w->wo + l * dim * dim, dim, dim, B, xt);
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
    for (b = 0; b < B; b++) {
      OModel* m = ms[b];
      for (int i = 0; i < dim; i++) m->x[i] += m->xb2[i];
      oracle_rmsnorm(m->xb, m->x, w->rms_ffn + l * dim, dim);
    }
    for (b = 0; b < B; b++) out[b] = ms[b]->hb, out2[b] = ms[b]->hb2;
    matmul_multi(out, in, w->w1 + l * dim * hid, dim, hid, B, xt);
    matmul_multi(out2, in, w->w3 + l * dim * hid, dim, hid, B, xt);
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
    for (b = 0; b < B; b++) oracle_swiglu(ms[b]->hb, ms[b]->hb2, hid);
    for (b = 0; b < B; b++) in[b] = ms[b]->hb, out[b] = ms[b]->xb;
    matmul_multi(out, in, w->w2 + l * dim * hid, hid, dim, B, xt);
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
    for (b = 0; b < B; b++)
      for (int i = 0; i < dim; i++) ms[b]->x[i] += ms[b]->xb[i];
  }
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1)
  for (b = 0; b < B; b++) oracle_rmsnorm(ms[b]->x, ms[b]->x, w->rms_final, dim);
  for (b = 0; b < B; b++) in[b] = ms[b]->x, out[b] = ms[b]->logits;
  matmul_multi(out, in, w->wcls, dim, p->vocab_size, B, xt);
  free(in); free(out); free(out2); free(xt);
  return 0;
}

/* llama.cpp:275-286 */
int oracle_argmax(const float* v, int n) {
  int max_i = 0;
  float max_p = v[0];
  for (int i = 1; i < n; i++)
    if (v[i] > max_p) { max_i = i; max_p = v[i]; }
  return max_i;
}

/* Greedy decode: tokens[0] = first token at pos0; writes n generated ids into out. */
int oracle_greedy(OModel* m, int token, int pos0, int n, int* out) {
  for (int i = 0; i < n; ++i) {
    float* lg = oracle_forward(m, token, pos0 + i);
    token = oracle_argmax(lg, m->c.vocab_size);
    out[i] = token;
  }
  return 0;
}

/* ------------------------------------------------------------ int8 (runq.c) */
/* runq.c:145-171: activation quantisation, round() = half away from zero */
void oracle_q8_quantize(int8_t* q, float* s, const float* x, int n, int gs) {
  const int num_groups = n / gs;
  const float Q_MAX = 127.0f;
  for (int group = 0; group < num_groups; group++) {
    float wmax = 0.0;
    for (int i = 0; i < gs; i++) {
      float val = fabsf(x[group * gs + i]);
      if (val > wmax) wmax = val;
    }
    float scale = wmax / Q_MAX;
    s[group] = scale;
    for (int i = 0; i < gs; i++) {
      float quant_value = x[group * gs + i] / scale;
      int8_t quantized = (int8_t)round(quant_value);
      q[group * gs + i] = quantized;
    }
  }
}

/* train/export.py:46-70 weight quantisation: scale = max|w|/127 (fp32), q = torch.round(w/scale)
 * (round half to EVEN, unlike the activation path). */
void oracle_q8_quantize_weights(int8_t* q, float* s, const float* w, size_t n, int gs) {
  const size_t ng = n / gs;
  long long g;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
  for (g = 0; g < (long long)ng; ++g) {
    float wmax = 0.f;
    for (int i = 0; i < gs; ++i) {
      float a = fabsf(w[g * gs + i]);
      if (a > wmax) wmax = a;
    }
    float scale = wmax / 127.0f;
    s[g] = scale;
    for (int i = 0; i < gs; ++i) q[g * gs + i] = (int8_t)rintf(w[g * gs + i] / scale);
  }
}

/* runq.c:317-342 */
void oracle_q8_matmul(float* xout, const int8_t* xq, const float* xs, const int8_t* wq, const float* ws, int n, int d,
                      int gs) {
  int i;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1 && (long)n * d > 65536) schedule(static)
  for (i = 0; i < d; i++) {
    float val = 0.0f;
    int32_t ival = 0;
    const size_t in = (size_t)i * n;
    for (int j = 0; j <= n - gs; j += gs) {
      for (int k = 0; k < gs; k++) ival += ((int32_t)xq[j + k]) * ((int32_t)wq[in + j + k]);
      val += ((float)ival) * ws[(in + j) / gs] * xs[j / gs];
      ival = 0;
    }
    xout[i] = val;
  }
}

size_t oracle_q8_payload_bytes(const OCfg* p, int shared, int gs) {
  const size_t L = p->n_layers, dim = p->dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t hid = p->hidden_dim, V = p->vocab_size;
  size_t b = 4 * (2 * L * dim + dim);
#define QT(N) ((N) + 4 * ((N) / gs))
  b += QT(V * dim);
  b += L * QT(dim * dim) * 2 + L * QT(dim * kvd) * 2 + L * QT(dim * hid) * 3;
  if (!shared) b += QT(V * dim);
#undef QT
  return b;
}

static OQT* map_qt(unsigned char** ptr, int n, size_t size_each, int gs) {
  OQT* r = malloc(n * sizeof(OQT));
  unsigned char* p = *ptr;
  for (int i = 0; i < n; i++) {
    r[i].q = (int8_t*)p;
    p += size_each;
    r[i].s = (float*)p;
    p += 4 * (size_each / gs);
  }
  *ptr = p;
  return r;
}

/* Build the runq v2 payload (export.py version2_export order, after the 256-B header) from the
 * model's fp32 weights and map it like runq.c:189-217. */
int oracle_q8_build(OModel* m, int gs) {
  const OCfg* p = &m->c;
  const size_t L = p->n_layers, dim = p->dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t hid = p->hidden_dim, V = p->vocab_size;
  m->gs = gs;
  m->q8bytes = oracle_q8_payload_bytes(p, m->shared, gs);
  m->q8arena = malloc(m->q8bytes);
  if (!m->q8arena) return -1;
  unsigned char* ptr = m->q8arena;
  memcpy(ptr, m->rms_att, 4 * L * dim); ptr += 4 * L * dim;
  memcpy(ptr, m->rms_ffn, 4 * L * dim); ptr += 4 * L * dim;
  memcpy(ptr, m->rms_final, 4 * dim); ptr += 4 * dim;
  struct { const float* src; size_t each; int n; } list[8] = {
      {m->emb, V * dim, 1}, {m->wq, dim * dim, (int)L}, {m->wk, dim * kvd, (int)L}, {m->wv, dim * kvd, (int)L},
      {m->wo, dim * dim, (int)L}, {m->w1, dim * hid, (int)L}, {m->w2, dim * hid, (int)L}, {m->w3, dim * hid, (int)L}};
  for (int t = 0; t < 8; ++t)
    for (int i = 0; i < list[t].n; ++i) {
      int8_t* q = (int8_t*)ptr;
      float* s = (float*)(ptr + list[t].each);
      oracle_q8_quantize_weights(q, s, list[t].src + i * list[t].each, list[t].each, gs);
      ptr += list[t].each + 4 * (list[t].each / gs);
    }
  if (!m->shared) {
    int8_t* q = (int8_t*)ptr;
    float* s = (float*)(ptr + V * dim);
    oracle_q8_quantize_weights(q, s, m->wcls, V * dim, gs);
  }
  /* map (runq.c:189-217) */
  ptr = m->q8arena + 4 * (2 * L * dim + dim);
  m->q_tok = map_qt(&ptr, 1, V * dim, gs);
  m->q8_emb = malloc(4 * V * dim);
  for (size_t i = 0; i < V * dim; i++) m->q8_emb[i] = m->q_tok[0].q[i] * m->q_tok[0].s[i / gs];
  m->q_wq = map_qt(&ptr, (int)L, dim * dim, gs);
  m->q_wk = map_qt(&ptr, (int)L, dim * kvd, gs);
  m->q_wv = map_qt(&ptr, (int)L, dim * kvd, gs);
  m->q_wo = map_qt(&ptr, (int)L, dim * dim, gs);
  m->q_w1 = map_qt(&ptr, (int)L, dim * hid, gs);
  m->q_w2 = map_qt(&ptr, (int)L, hid * dim, gs);
  m->q_w3 = map_qt(&ptr, (int)L, dim * hid, gs);
  m->q_wcls = m->shared ? m->q_tok : map_qt(&ptr, 1, dim * V, gs);
  m->xq.q = calloc(dim, 1); m->xq.s = calloc(dim, 4);
  m->hq.q = calloc(hid, 1); m->hq.s = calloc(hid, 4);
  return 0;
}

unsigned char* oracle_q8_payload(OModel* m) { return m->q8arena; }
size_t oracle_q8_payload_size(OModel* m) { return m->q8bytes; }

/* Write a runq v2 ("ak42") file: 256-B header (magic, version 2, Config, shared flag, group size). */
int oracle_write_v2(OModel* m, const char* path) {
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  unsigned char hdr[256];
  memset(hdr, 0, sizeof hdr);
  uint32_t magic = 0x616b3432;
  int version = 2;
  memcpy(hdr, &magic, 4);
  memcpy(hdr + 4, &version, 4);
  memcpy(hdr + 8, &m->c, sizeof(OCfg));
  hdr[8 + sizeof(OCfg)] = (unsigned char)m->shared;
  memcpy(hdr + 9 + sizeof(OCfg), &m->gs, 4);
  int ok = fwrite(hdr, 1, 256, f) == 256 && fwrite(m->q8arena, 1, m->q8bytes, f) == m->q8bytes;
  fclose(f);
  return ok ? 0 : -1;
}

/* runq.c:344-481 */
float* oracle_q8_forward(OModel* m, int token, int pos) {
  const OCfg* p = &m->c;
  float* x = m->x;
  const int dim = p->dim, gs = m->gs;
  const int kv_dim = (p->dim * p->n_kv_heads) / p->n_heads;
  const int kv_mul = p->n_heads / p->n_kv_heads;
  const int hidden_dim = p->hidden_dim;
  const int head_size = dim / p->n_heads;
  memcpy(x, m->q8_emb + (size_t)token * dim, dim * sizeof(float));
  for (int l = 0; l < p->n_layers; l++) {
    oracle_rmsnorm(m->xb, x, m->rms_att + (size_t)l * dim, dim);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    oracle_q8_matmul(m->q, m->xq.q, m->xq.s, m->q_wq[l].q, m->q_wq[l].s, dim, dim, gs);
    oracle_q8_matmul(m->k, m->xq.q, m->xq.s, m->q_wk[l].q, m->q_wk[l].s, dim, kv_dim, gs);
    oracle_q8_matmul(m->v, m->xq.q, m->xq.s, m->q_wv[l].q, m->q_wv[l].s, dim, kv_dim, gs);
    oracle_rope(m->q, m->k, dim, head_size, kv_dim, pos);
    const size_t loff = (size_t)l * p->seq_len * kv_dim;
    memcpy(m->kc + loff + (size_t)pos * kv_dim, m->k, kv_dim * sizeof(float));
    memcpy(m->vc + loff + (size_t)pos * kv_dim, m->v, kv_dim * sizeof(float));
    oracle_attention(m->xb, m->att, m->q, m->kc + loff, m->vc + loff, pos, p->n_heads, head_size, kv_dim, kv_mul,
                     p->seq_len);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    oracle_q8_matmul(m->xb2, m->xq.q, m->xq.s, m->q_wo[l].q, m->q_wo[l].s, dim, dim, gs);
    for (int i = 0; i < dim; i++) x[i] += m->xb2[i];
    oracle_rmsnorm(m->xb, x, m->rms_ffn + (size_t)l * dim, dim);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    oracle_q8_matmul(m->hb, m->xq.q, m->xq.s, m->q_w1[l].q, m->q_w1[l].s, dim, hidden_dim, gs);
    oracle_q8_matmul(m->hb2, m->xq.q, m->xq.s, m->q_w3[l].q, m->q_w3[l].s, dim, hidden_dim, gs);
    oracle_swiglu(m->hb, m->hb2, hidden_dim);
    oracle_q8_quantize(m->hq.q, m->hq.s, m->hb, hidden_dim, gs);
    oracle_q8_matmul(m->xb, m->hq.q, m->hq.s, m->q_w2[l].q, m->q_w2[l].s, hidden_dim, dim, gs);
    for (int i = 0; i < dim; i++) x[i] += m->xb[i];
  }
  oracle_rmsnorm(x, x, m->rms_final, dim);
  oracle_q8_quantize(m->xq.q, m->xq.s, x, dim, gs);
  oracle_q8_matmul(m->logits, m->xq.q, m->xq.s, m->q_wcls[0].q, m->q_wcls[0].s, dim, p->vocab_size, gs);
  return m->logits;
}

int oracle_q8_greedy(OModel* m, int token, int pos0, int n, int* out) {
  for (int i = 0; i < n; ++i) {
    float* lg = oracle_q8_forward(m, token, pos0 + i);
    token = oracle_argmax(lg, m->c.vocab_size);
    out[i] = token;
  }
  return 0;
}

/* ------------------------------------------------------------ CPU baseline, aggregate mode */
/* BASELINE.md CPU-baseline plan (ii): P independent single-threaded decoders, one per core, over
 * disjoint sequences (decoder i starts from token 1 + i at pos 0), sharing one copy of the
 * weights; each is the unchanged single-sequence forward above with its own RunState. */
OModel* oracle_model_view(OModel* m) { return oracle_model_view_cap(m, 0); }

/* A view whose K/V cache holds positions 0..seq_cap-1 only (seq_cap <= 0: the model's seq_len).
 * The cache stride is the only thing seq_len sets in the forward (RoPE and attention read
 * positions 0..pos), so a capped view computes the same values for every pos < seq_cap. */
OModel* oracle_model_view_cap(OModel* m, int seq_cap) {
  OModel* v = calloc(1, sizeof(OModel));
  if (!v) return NULL;
  *v = *m; /* weight pointers */
  if (seq_cap > 0 && seq_cap < v->c.seq_len) v->c.seq_len = seq_cap;
  v->view = 1;
  v->x = v->xb = v->xb2 = v->hb = v->hb2 = v->q = v->att = v->logits = v->kc = v->vc = v->k = v->v = NULL;
  v->kc64 = v->vc64 = NULL;
  v->xq.q = v->hq.q = NULL;
  v->xq.s = v->hq.s = NULL;
  if (!alloc_state(v)) { oracle_model_free(v); return NULL; }
  if (m->q8arena) {
    v->xq.q = calloc(m->c.dim, 1); v->xq.s = calloc(m->c.dim, 4);
    v->hq.q = calloc(m->c.hidden_dim, 1); v->hq.s = calloc(m->c.hidden_dim, 4);
  }
  return v;
}

#include <pthread.h>
#include <sched.h>
#include <time.h>

typedef struct {
  OModel* m;
  int q8, cpu, start, n;
  int* out;
} OAggJob;

static void* agg_worker(void* a) {
  OAggJob* j = (OAggJob*)a;
  if (j->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(j->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof set, &set);
  }
  if (j->q8) oracle_q8_greedy(j->m, j->start, 0, j->n, j->out);
  else oracle_greedy(j->m, j->start, 0, j->n, j->out);
  return NULL;
}

/* Runs P decoders of n greedy tokens each at once (decoder i pinned to cpus[i % ncpu], or
 * unpinned when ncpu == 0); out[P][n] receives the tokens.  Returns the wall time in seconds,
 * or -1 on an allocation failure. */
double oracle_aggregate(OModel* m, int q8, int P, const int* cpus, int ncpu, int n, int* out) {
  OAggJob* jobs = calloc(P, sizeof(OAggJob));
  pthread_t* th = calloc(P, sizeof(pthread_t));
  const int saved = g_threads;
  double secs = -1.0;
  int ok = jobs && th;
  for (int i = 0; ok && i < P; ++i) {
    jobs[i].m = oracle_model_view(m);
    ok = jobs[i].m != NULL;
    jobs[i].q8 = q8; jobs[i].cpu = ncpu > 0 ? cpus[i % ncpu] : -1;
    jobs[i].start = 1 + i % (m->c.vocab_size - 1); jobs[i].n = n; jobs[i].out = out + (size_t)i * n;
  }
  if (ok) {
    g_threads = 1; /* each decoder single-threaded, like seq.cpp */
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int started = 0;
    for (; started < P; ++started)
      if (pthread_create(&th[started], NULL, agg_worker, &jobs[started]) != 0) break;
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    g_threads = saved;
    if (started == P) secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  }
  for (int i = 0; jobs && i < P; ++i) oracle_model_free(jobs[i].m);
  free(jobs);
  free(th);
  return secs;
}

/* The synthetic generator, exposed so tests can check the device filler bit-for-bit. */
void oracle_synth_fill(float* dst, size_t n, uint64_t seed, int id, double stddev, size_t offset) {
  const uint64_t ts = tl_synth_tensor_seed(seed, id);
  const float sc = tl_synth_scale(stddev);
  for (size_t i = 0; i < n; ++i) dst[i] = tl_synth_value(ts, offset + i, sc);
}
