/* thallama_synth.h — the deterministic synthetic-weight generator, shared by the
 * device filler (hip_llama.cpp_amd/csrc/runtime.hip) and the host oracle
 * (oracle/oracle.c) so both sides see bit-identical weights.
 *
 * Distribution: train/model.py:232-247 of the reference — every linear and the
 * embedding ~ N(0, 0.02); wo and w3 ~ N(0, 0.02/sqrt(2*n_layers)); RMSNorm
 * weights = 1.  The normal is approximated by an Irwin-Hall sum of four
 * uniform 16-bit integers from one splitmix64 draw per element:
 *     v = (float)(u0+u1+u2+u3 - 131070) * scale,   scale = (float)(sigma*sqrt(3)/65536)
 * All arithmetic is integer except one int->float conversion and one float
 * multiply, so host and device agree exactly (no libm, no contraction).
 * Layout of the arena: llama2.c v0 payload order (reference src/utils.cpp:119-148).
 */
#ifndef THALLAMA_SYNTH_H
#define THALLAMA_SYNTH_H
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __HIPCC__
#define TL_HD __host__ __device__
#else
#define TL_HD
#endif

static inline TL_HD uint64_t tl_mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

static inline TL_HD uint64_t tl_synth_tensor_seed(uint64_t seed, int id) {
  return tl_mix64(seed ^ (0xD1B54A32D192ED03ULL * (uint64_t)(id + 1)));
}

static inline TL_HD float tl_synth_value(uint64_t tseed, uint64_t i, float scale) {
  const uint64_t r = tl_mix64(tseed + i * 0x9E3779B97F4A7C15ULL);
  const int32_t s = (int32_t)((r & 0xFFFF) + ((r >> 16) & 0xFFFF) + ((r >> 32) & 0xFFFF) + (r >> 48));
  return (float)(s - 131070) * scale;
}

static inline float tl_synth_scale(double stddev) { return (float)(stddev * sqrt(3.0) / 65536.0); }

enum { TL_SYNTH_NORMAL = 0, TL_SYNTH_CONST = 1 };

typedef struct {
  int id;        /* generator stream id */
  int kind;      /* TL_SYNTH_NORMAL / TL_SYNTH_CONST */
  double stddev; /* NORMAL */
  float value;   /* CONST */
  size_t offset; /* floats from the arena start */
  size_t count;  /* floats */
} TlSynthTensor;

typedef struct {
  int n;
  TlSynthTensor t[16];
} TlSynthPlan;

/* cfg points at a struct whose first 7 ints are the v0 Config. */
static inline void tl_synth_plan(TlSynthPlan* plan, const void* cfgv, int shared_weights) {
  const int* c = (const int*)cfgv;
  const size_t dim = c[0], hid = c[1], L = c[2], H = c[3], KVH = c[4];
  const size_t V = c[5] < 0 ? (size_t)(-c[5]) : (size_t)c[5], S = c[6];
  const size_t hs = dim / H, kvd = dim * KVH / H;
  const double sd = 0.02, sd_res = 0.02 / sqrt(2.0 * (double)L);
  size_t off = 0;
  int n = 0;
#define TL_ADD(ID, KIND, SD, VAL, CNT)                                  \
  do {                                                                  \
    TlSynthTensor e_;                                                   \
    e_.id = (ID); e_.kind = (KIND); e_.stddev = (SD); e_.value = (VAL); \
    e_.offset = off; e_.count = (CNT);                                  \
    plan->t[n++] = e_;                                                  \
    off += (CNT);                                                       \
  } while (0)
  TL_ADD(1, TL_SYNTH_NORMAL, sd, 0.f, V * dim);        /* token_embedding_table */
  TL_ADD(2, TL_SYNTH_CONST, 0.0, 1.f, L * dim);        /* rms_att_weight */
  TL_ADD(3, TL_SYNTH_NORMAL, sd, 0.f, L * dim * dim);  /* wq */
  TL_ADD(4, TL_SYNTH_NORMAL, sd, 0.f, L * dim * kvd);  /* wk */
  TL_ADD(5, TL_SYNTH_NORMAL, sd, 0.f, L * dim * kvd);  /* wv */
  TL_ADD(6, TL_SYNTH_NORMAL, sd_res, 0.f, L * dim * dim); /* wo */
  TL_ADD(7, TL_SYNTH_CONST, 0.0, 1.f, L * dim);        /* rms_ffn_weight */
  TL_ADD(8, TL_SYNTH_NORMAL, sd, 0.f, L * dim * hid);  /* w1 */
  TL_ADD(9, TL_SYNTH_NORMAL, sd, 0.f, L * dim * hid);  /* w2 */
  TL_ADD(10, TL_SYNTH_NORMAL, sd_res, 0.f, L * dim * hid); /* w3 */
  TL_ADD(11, TL_SYNTH_CONST, 0.0, 1.f, dim);           /* rms_final_weight */
  TL_ADD(13, TL_SYNTH_CONST, 0.0, 0.f, S * hs);        /* freq_cis (unused) */
  if (!shared_weights) TL_ADD(12, TL_SYNTH_NORMAL, sd, 0.f, V * dim); /* wcls */
#undef TL_ADD
  plan->n = n;
}

#endif
