/* seqsum.c — TEST INFRASTRUCTURE (probe): the wave-parallel sequential fp32 sum of csrc/seqsum.hpp
 * emulated on the CPU (64 lanes x CH consecutive elements) against the plain left-to-right chain
 * s = fl(s + a[k]) (runq.c:284-287 / src/seq.cpp:5-8, the RMSNorm sum of squares; runq.c:306-310,
 * the softmax sum): bit-identical results and the number of repair rounds on typical and
 * adversarial data.  Build: gcc -O2 -ffp-contract=off tools/probes/seqsum.c -o /tmp/seqsum -lm */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float chain(const float* a, int n, float s) {
  for (int k = 0; k < n; ++k) s = s + a[k];
  return s;
}

/* returns the sum; *rounds = repair rounds used */
static float wave_seqsum(const float* a, int n, int* rounds) {
  const int CH = (n + 63) / 64;
  float pad[64 * 256];
  memset(pad, 0, sizeof(float) * 64 * CH);
  memcpy(pad, a, sizeof(float) * n);
  double part[64], pre[65];
  for (int L = 0; L < 64; ++L) { double d = 0; for (int k = 0; k < CH; ++k) d += pad[L * CH + k]; part[L] = d; }
  pre[0] = 0; for (int L = 0; L < 64; ++L) pre[L + 1] = pre[L] + part[L];
  float start[64];
  double inc[64];
  for (int L = 0; L < 64; ++L) {
    start[L] = L ? (float)pre[L] : 0.f;  /* guess */
    inc[L] = (double)chain(pad + L * CH, CH, start[L]) - (double)start[L];
  }
  int lo = 0;          /* lanes < lo are final: start[lo] is the true value */
  *rounds = 0;
  for (;;) {
    /* scan from lane lo */
    double s = start[lo];
    for (int L = lo; L < 64; ++L) { start[L] = (float)s; s += inc[L]; }
    const float total = (float)s;
    /* verify */
    int bad = -1;
    float endv[64];
    for (int L = lo; L < 64; ++L) {
      endv[L] = chain(pad + L * CH, CH, start[L]);
      const float next = L + 1 < 64 ? start[L + 1] : total;
      if (bad < 0 && endv[L] != next) bad = L;
      inc[L] = (double)endv[L] - (double)start[L];
    }
    ++*rounds;
    if (bad < 0) return total;
    if (bad == 63) return endv[63];
    start[bad + 1] = endv[bad];
    lo = bad + 1;
  }
}

/* the variant with one prefix of the guessed increments for every round (csrc/seqsum.hpp
 * wave_seqsum_reg) */
static float wave_seqsum_1p(const float* a, int n, int* rounds) {
  const int CH = (n + 63) / 64;
  float pad[64 * 256];
  memset(pad, 0, sizeof(float) * 64 * CH);
  memcpy(pad, a, sizeof(float) * n);
  double part[64], pre[65], inc[64];
  float start[64], e[64];
  for (int L = 0; L < 64; ++L) part[L] = chain(pad + L * CH, CH, 0.f);
  pre[0] = 0; for (int L = 0; L < 64; ++L) pre[L + 1] = pre[L] + part[L];
  for (int L = 0; L < 64; ++L) {
    start[L] = L ? (float)pre[L] : 0.f;
    inc[L] = (double)chain(pad + L * CH, CH, start[L]) - (double)start[L];
  }
  pre[0] = 0; for (int L = 0; L < 64; ++L) pre[L + 1] = pre[L] + inc[L];
  int lo = 0; float slo = 0.f; double plo = 0.0;
  *rounds = 0;
  for (;;) {
    for (int L = lo + 1; L < 64; ++L) start[L] = (float)((double)slo + (pre[L] - plo));
    const float total = (float)((double)slo + (pre[64] - plo));
    int bad = -1;
    for (int L = lo; L < 64; ++L) {
      e[L] = chain(pad + L * CH, CH, start[L]);
      const float next = L + 1 < 64 ? start[L + 1] : total;
      if (bad < 0 && e[L] != next) bad = L;
    }
    ++*rounds;
    if (bad < 0) return total;
    if (bad == 63) return e[63];
    lo = bad + 1; slo = e[bad]; plo = pre[lo]; start[lo] = slo;
  }
}

static unsigned long long rs = 88172645463325252ull;
static double urand(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (rs >> 11) * (1.0 / 9007199254740992.0); }
static double nrand(void) { double u = urand() + 1e-300, v = urand(); return sqrt(-2 * log(u)) * cos(6.283185307179586 * v); }

int main(void) {
  static float a[4096];
  int kinds = 6, trials = 2000, worst = 0;
  long long bad = 0, hist[70] = {0};
  for (int kind = 0; kind < kinds; ++kind)
    for (int t = 0; t < trials; ++t) {
      int n = kind == 5 ? 1 + (int)(urand() * 4096) : 4096;
      for (int i = 0; i < n; ++i) {
        double x;
        switch (kind) {
          case 0: x = nrand(); break;                                /* residual stream */
          case 1: x = nrand() * exp(3 * nrand()); break;             /* heavy tails */
          case 2: x = (int)(nrand() * 8); break;                     /* small integers: many ties */
          case 3: x = ldexp(1.0, (int)(urand() * 20) - 10); break;   /* powers of two */
          case 4: x = i < 8 ? 1000 * nrand() : nrand() * 1e-3; break;/* a few huge first */
          default: x = nrand(); break;                               /* ragged lengths */
        }
        float xf = (float)x;
        a[i] = xf * xf;
      }
      int r, r1;
      float got = wave_seqsum(a, n, &r), want = chain(a, n, 0.f), got1 = wave_seqsum_1p(a, n, &r1);
      if (memcmp(&got, &want, 4)) ++bad;
      if (memcmp(&got1, &want, 4)) ++bad;
      if (r1 > r) r = r1;
      hist[r < 69 ? r : 69]++;
      if (r > worst) worst = r;
    }
  printf("mismatches %lld of %d; repair rounds histogram:", bad, kinds * trials);
  for (int i = 0; i < 70; ++i) if (hist[i]) printf(" %d:%lld", i, hist[i]);
  printf(" (worst %d)\n", worst);
  return bad != 0;
}
