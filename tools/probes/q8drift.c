/* q8drift.c — TEST INFRASTRUCTURE (a measurement probe, never shipped).
 *
 * How far does an int8 (runq.c) greedy decode drift when individual fp32 reductions are taken
 * in another order than runq's sequential one?  Runs the oracle's runq restatement
 * (oracle/oracle.c, pinned to runq.c) on a synthetic model, greedy from BOS, then re-runs it
 * teacher-forced along the same tokens with some reductions replaced by GPU-like orders:
 *   bit 1  GEMV: per 4096-wide chunk a pairwise tree over the 64 group products (the wave sum),
 *          chunks added in order (runq.c:330-338 is one sequential chain over all groups)
 *   bit 2  RMSNorm sum of squares: 576 fma chains over strided float4s, wave trees, waves in
 *          order (runq.c:282-295 is sequential)
 *   bit 4  attention dot products, softmax sum and att.V sums as pairwise trees (runq.c:405-433)
 *   bit 8  expf -> exp2f(x * log2(e)) (an ~1-ulp device exp) in softmax and SwiGLU
 * and reports per step the reference's top-2 margin, the max |dlogit| and whether the argmax
 * differs.  Build: gcc -O2 -fopenmp -ffp-contract=off tools/probes/q8drift.c -o /tmp/q8drift -lm
 * Run: THREADS=8 /tmp/q8drift <dim> <hidden> <layers> <heads> <kv_heads> <vocab> <seq> <steps> <mask>...
 */
#include "../../oracle/oracle.c"

static int g_mask = 0;

static float tree(const float* v, int n) {
  if (n == 1) return v[0];
  int h = n / 2;
  return tree(v, h) + tree(v + h, n - h);
}

static float dexpf(float x) { return (g_mask & 8) ? exp2f(x * 1.44269504f) : expf(x); }

static void d_rmsnorm(float* o, const float* x, const float* w, int size) {
  float ss;
  if (g_mask & 2) {
    float part[576];
    for (int t = 0; t < 576; ++t) {
      float s = 0.f;
      for (int j = t; j < size / 4; j += 576)
        for (int u = 0; u < 4; ++u) s = fmaf(x[4 * j + u], x[4 * j + u], s);
      part[t] = s;
    }
    ss = 0.f;
    for (int wv = 0; wv < 9; ++wv) ss += tree(part + 64 * wv, 64);
  } else {
    ss = 0.f;
    for (int j = 0; j < size; j++) ss += x[j] * x[j];
  }
  ss /= size;
  ss += 1e-5f;
  ss = 1.0f / sqrtf(ss);
  for (int j = 0; j < size; j++) o[j] = w[j] * (ss * x[j]);
}

static void d_matmul(float* xout, const int8_t* xq, const float* xs, const int8_t* wq, const float* ws, int n, int d,
                     int gs) {
  if (!(g_mask & 1)) { oracle_q8_matmul(xout, xq, xs, wq, ws, n, d, gs); return; }
  int i;
#pragma omp parallel for num_threads(g_threads) schedule(static)
  for (i = 0; i < d; i++) {
    const size_t in = (size_t)i * n;
    const int ng = n / gs;
    float val = 0.f, prod[64];
    for (int c0 = 0; c0 < ng; c0 += 64) {
      for (int g = 0; g < 64; ++g) {
        prod[g] = 0.f;
        if (c0 + g >= ng) continue;
        const int j = (c0 + g) * gs;
        int32_t ival = 0;
        for (int k = 0; k < gs; k++) ival += ((int32_t)xq[j + k]) * ((int32_t)wq[in + j + k]);
        prod[g] = ((float)ival) * ws[(in + j) / gs] * xs[j / gs];
      }
      const float t = tree(prod, 64);
      val = c0 == 0 ? t : val + t;
    }
    xout[i] = val;
  }
}

static void d_attention(OModel* m, int l, int pos) {
  const OCfg* p = &m->c;
  const int dim = p->dim, hs = dim / p->n_heads, kvd = dim * p->n_kv_heads / p->n_heads;
  const int kv_mul = p->n_heads / p->n_kv_heads;
  const size_t loff = (size_t)l * p->seq_len * kvd;
  const int tr = g_mask & 4;
  float tmp[4096];
  for (int h = 0; h < p->n_heads; h++) {
    const float* q = m->q + h * hs;
    float* att = m->att + (size_t)h * p->seq_len;
    for (int t = 0; t <= pos; t++) {
      const float* k = m->kc + loff + (size_t)t * kvd + (h / kv_mul) * hs;
      float score = 0.f;
      if (tr) { for (int i = 0; i < hs; i++) tmp[i] = q[i] * k[i]; score = tree(tmp, hs); }
      else for (int i = 0; i < hs; i++) score += q[i] * k[i];
      att[t] = score / sqrtf(hs);
    }
    float mx = att[0];
    for (int t = 1; t <= pos; t++) if (att[t] > mx) mx = att[t];
    float sum = 0.f;
    for (int t = 0; t <= pos; t++) { att[t] = dexpf(att[t] - mx); if (!tr) sum += att[t]; }
    if (tr) sum = tree(att, pos + 1);
    for (int t = 0; t <= pos; t++) att[t] /= sum;
    float* xb = m->xb + h * hs;
    for (int i = 0; i < hs; i++) {
      if (tr) {
        for (int t = 0; t <= pos; t++) tmp[t] = att[t] * m->vc[loff + (size_t)t * kvd + (h / kv_mul) * hs + i];
        xb[i] = tree(tmp, pos + 1);
      } else {
        float s = 0.f;
        for (int t = 0; t <= pos; t++) s += att[t] * m->vc[loff + (size_t)t * kvd + (h / kv_mul) * hs + i];
        xb[i] = s;
      }
    }
  }
}

static float* d_forward(OModel* m, int token, int pos) {
  const OCfg* p = &m->c;
  float* x = m->x;
  const int dim = p->dim, gs = m->gs, kv_dim = dim * p->n_kv_heads / p->n_heads, hid = p->hidden_dim;
  const int head_size = dim / p->n_heads;
  memcpy(x, m->q8_emb + (size_t)token * dim, dim * sizeof(float));
  for (int l = 0; l < p->n_layers; l++) {
    d_rmsnorm(m->xb, x, m->rms_att + (size_t)l * dim, dim);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    d_matmul(m->q, m->xq.q, m->xq.s, m->q_wq[l].q, m->q_wq[l].s, dim, dim, gs);
    d_matmul(m->k, m->xq.q, m->xq.s, m->q_wk[l].q, m->q_wk[l].s, dim, kv_dim, gs);
    d_matmul(m->v, m->xq.q, m->xq.s, m->q_wv[l].q, m->q_wv[l].s, dim, kv_dim, gs);
    oracle_rope(m->q, m->k, dim, head_size, kv_dim, pos);
    const size_t loff = (size_t)l * p->seq_len * kv_dim;
    memcpy(m->kc + loff + (size_t)pos * kv_dim, m->k, kv_dim * sizeof(float));
    memcpy(m->vc + loff + (size_t)pos * kv_dim, m->v, kv_dim * sizeof(float));
    d_attention(m, l, pos);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    d_matmul(m->xb2, m->xq.q, m->xq.s, m->q_wo[l].q, m->q_wo[l].s, dim, dim, gs);
    for (int i = 0; i < dim; i++) x[i] += m->xb2[i];
    d_rmsnorm(m->xb, x, m->rms_ffn + (size_t)l * dim, dim);
    oracle_q8_quantize(m->xq.q, m->xq.s, m->xb, dim, gs);
    d_matmul(m->hb, m->xq.q, m->xq.s, m->q_w1[l].q, m->q_w1[l].s, dim, hid, gs);
    d_matmul(m->hb2, m->xq.q, m->xq.s, m->q_w3[l].q, m->q_w3[l].s, dim, hid, gs);
    for (int i = 0; i < hid; i++) {
      float v = m->hb[i];
      v *= (1.0f / (1.0f + dexpf(-v)));
      m->hb[i] = v * m->hb2[i];
    }
    oracle_q8_quantize(m->hq.q, m->hq.s, m->hb, hid, gs);
    d_matmul(m->xb, m->hq.q, m->hq.s, m->q_w2[l].q, m->q_w2[l].s, hid, dim, gs);
    for (int i = 0; i < dim; i++) x[i] += m->xb[i];
  }
  d_rmsnorm(x, x, m->rms_final, dim);
  oracle_q8_quantize(m->xq.q, m->xq.s, x, dim, gs);
  d_matmul(m->logits, m->xq.q, m->xq.s, m->q_wcls[0].q, m->q_wcls[0].s, dim, p->vocab_size, gs);
  return m->logits;
}

int main(int argc, char** argv) {
  if (argc < 10) { fprintf(stderr, "usage: see header\n"); return 2; }
  OCfg c = {atoi(argv[1]), atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7])};
  const int steps = atoi(argv[8]);
  oracle_set_threads(getenv("THREADS") ? atoi(getenv("THREADS")) : 8);
  OModel* m = oracle_model_new(&c, 0, NULL, 7);
  oracle_q8_build(m, 64);
  /* the int8 forward reads the v2 payload only (its norms lead the payload) */
  m->rms_att = (float*)m->q8arena;
  m->rms_ffn = m->rms_att + (size_t)c.n_layers * c.dim;
  m->rms_final = m->rms_ffn + (size_t)c.n_layers * c.dim;
  free(m->arena); m->arena = NULL;
  const int V = c.vocab_size;
  int* tok = malloc(sizeof(int) * (steps + 1));
  float* ref = malloc(sizeof(float) * (size_t)steps * V);
  tok[0] = 1;
  for (int s = 0; s < steps; ++s) {
    float* lg = oracle_q8_forward(m, tok[s], s);
    memcpy(ref + (size_t)s * V, lg, sizeof(float) * V);
    tok[s + 1] = oracle_argmax(lg, V);
  }
  for (int ai = 9; ai < argc; ++ai) {
  const int mask = atoi(argv[ai]);
  oracle_model_reset_kv(m);
  g_mask = mask;
  int first_flip = -1;
  for (int s = 0; s < steps; ++s) {
    float* lg = d_forward(m, tok[s], s);
    const float* r = ref + (size_t)s * V;
    int a = oracle_argmax(r, V), b = oracle_argmax(lg, V);
    float top1 = r[a], top2 = -1e30f, dmax = 0.f;
    for (int j = 0; j < V; ++j) {
      if (j != a && r[j] > top2) top2 = r[j];
      float d = fabsf(lg[j] - r[j]);
      if (d > dmax) dmax = d;
    }
    if (a != b && first_flip < 0) first_flip = s;
    printf("step %3d tok %5d margin %.3e dmax %.3e %s\n", s, tok[s + 1], top1 - top2, dmax, a != b ? "FLIP" : "");
    fflush(stdout);
  }
  printf("mask %d first_flip %d\n", mask, first_flip);
  }
  return 0;
}
