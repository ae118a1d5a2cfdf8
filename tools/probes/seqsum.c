/* seqsum.c — TEST INFRASTRUCTURE (probe): the wave-parallel sequential fp32 sum of csrc/seqsum.hpp
 * emulated on the CPU (64 lanes x CH consecutive elements) against the plain left-to-right chain
 * s = fl(s + a[k]) (runq.c:284-287 / src/seq.cpp:5-8, the RMSNorm sum of squares; runq.c:306-310,
 * the softmax sum): bit-identical results and the number of repair rounds on typical and
 * adversarial data.  Build: gcc -O2 -ffp-contract=off tools/probes/seqsum.c -o /tmp/seqsum -lm */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifndef NV
#define NV 2
#endif

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

/* The parity-resolved variant (csrc/seqsum.hpp wave_seqsum_par): each lane also chains its chunk
 * from its guess plus one ulp, so a chunk whose increment depends on its start's parity (a binade
 * crossing, a tie) has both increments; the starts are then resolved in ONE ordered pass over
 * those lanes, and one verification chain proves the result.  A failed verification falls back
 * to the repair rounds (from the first failing lane).  *rounds = 1 + fallback rounds. */
static float wave_seqsum_par(const float* a, int n, int* rounds) {
  const int CH = (n + 63) / 64;
  float pad[64 * 256];
  memset(pad, 0, sizeof(float) * 64 * CH);
  memcpy(pad, a, sizeof(float) * n);
  double part[64], pre[65], D[64][NV];
  float G[64], S[65];
  int dep[64];
  for (int L = 0; L < 64; ++L) part[L] = chain(pad + L * CH, CH, 0.f);
  pre[0] = 0; for (int L = 0; L < 64; ++L) pre[L + 1] = pre[L] + part[L];
  for (int L = 0; L < 64; ++L) {
    G[L] = L ? (float)pre[L] : 0.f;
    float g = G[L];
    dep[L] = 0;
    for (int k = 0; k < NV; ++k) {  /* starts G, G + u, G + 2u, ... (same binade assumed) */
      D[L][k] = (double)chain(pad + L * CH, CH, g) - (double)g;
      if (L && D[L][k] != D[L][0]) dep[L] = 1;
      g = L ? nextafterf(g, INFINITY) : 0.f;
    }
  }
  double acc = 0, P = 0;
  for (int L = 0; L < 64; ++L) {
    S[L] = (float)(P + acc);
    if (dep[L]) {
      unsigned sb, gb;
      memcpy(&sb, &S[L], 4); memcpy(&gb, &G[L], 4);
      if ((sb >> 23) == (gb >> 23)) acc += D[L][(sb - gb) & (NV - 1)] - D[L][0];
    }
    P += D[L][0];
  }
  S[64] = (float)(P + acc);
  *rounds = 1;
  for (int L = 0; L < 64; ++L)
    if (chain(pad + L * CH, CH, S[L]) != S[L + 1]) {
      int r;
      const float v = wave_seqsum_1p(a, n, &r);  /* (the kernel continues from lane L instead) */
      *rounds += r;
      return v;
    }
  return S[64];
}

static unsigned long long rs = 88172645463325252ull;
static double urand(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (rs >> 11) * (1.0 / 9007199254740992.0); }
static double nrand(void) { double u = urand() + 1e-300, v = urand(); return sqrt(-2 * log(u)) * cos(6.283185307179586 * v); }

int main(void) {
  static float a[4096];
  int kinds = 6, trials = 2000, worst = 0;
  long long bad = 0, hist[70] = {0}, par_hist[6][2] = {{0}}, par_r1[6] = {0};
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
      int r, r1, rp;
      float got = wave_seqsum(a, n, &r), want = chain(a, n, 0.f), got1 = wave_seqsum_1p(a, n, &r1);
      float gotp = wave_seqsum_par(a, n, &rp);
      if (memcmp(&got, &want, 4)) ++bad;
      if (memcmp(&got1, &want, 4)) ++bad;
      if (memcmp(&gotp, &want, 4)) ++bad;
      par_hist[kind][rp == 1 ? 0 : 1]++;
      par_r1[kind] += r1;
      if (r1 > r) r = r1;
      hist[r < 69 ? r : 69]++;
      if (r > worst) worst = r;
    }
  printf("mismatches %lld of %d; repair rounds histogram:", bad, kinds * trials);
  for (int i = 0; i < 70; ++i) if (hist[i]) printf(" %d:%lld", i, hist[i]);
  printf(" (worst %d)\n", worst);
  for (int k = 0; k < kinds; ++k)
    printf("kind %d: parity-resolved pass proves the sum in %lld of %lld (fallback %lld); repair rounds mean %.2f\n", k,
           par_hist[k][0], par_hist[k][0] + par_hist[k][1], par_hist[k][1], (double)par_r1[k] / trials);
  return bad != 0;
}
