// libm_exact.hpp — the host C library's expf, restated bit for bit, for host and device.
//
// Why: the reference's CPU paths call libm expf in the softmax (src/seq.cpp:18-36, runq.c:297-315)
// and the SwiGLU (src/seq.cpp:159-166, runq.c:455-462).  The int8 (runq) path re-quantises every
// activation vector, so one last-bit difference in an exp result can move an int8 code and the
// greedy decode then leaves runq's (tools/probes/q8drift.c: an ~1-ulp device exp alone diverges
// within ~10 steps).  A device exp that is merely accurate is not enough: the host's expf is not
// correctly rounded (max error ~0.502 ulp), so the int8 path must compute what it computes.
//
// What: glibc >= 2.27 expf (the algorithm of Szabolcs Nagy's optimized-routines expf, glibc
// sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c; here glibc 2.35, x86-64, whose ifunc picks the
// FMA build on FMA/AVX2 hosts): with N = 32,
//   z = x * (N / ln 2) in double;  k = round-to-nearest-int(z) via the 0x1.8p52 shift;  r = z - k;
//   s = 2^(k/N) = bits(T[k % N] + (k << 47));  y = s * (C2 r + 1 + (C0 r + C1) r^2)  rounded once to
//   float; |x| >= 88 and NaN go through the special cases below.
// The table T[i] = bits(2^(i/N)) - (i << 47) holds the correctly rounded doubles 2^(i/32)
// (tests/test_libm_exact.py recomputes them); C0..C2 are the published degree-3 coefficients
// (scaled by N^-3, N^-2, N^-1).  The FMA build contracts the three a*b+c of the polynomial and
// r = z - k (into fma(x, N/ln2, -k)); k itself comes from the rounded product z.
// tools/probes/expf_exact.cpp checks this restatement against the host's expf on all 2^32 inputs:
// 0 mismatches (glibc 2.35, the CPU container and, through tests/test_libm_exact.py on a sample,
// every host the CPU suite runs on).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define TL_LIBM_HD __host__ __device__
#else
#define TL_LIBM_HD
#endif

namespace tl {

// bits(2^(i/32)) - (i << 47), i = 0..31 (the correctly rounded doubles)
#define TL_EXPF_TABLE                                                                                          \
  {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,             \
   0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,             \
   0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,             \
   0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,             \
   0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,             \
   0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,             \
   0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,             \
   0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}

TL_LIBM_HD inline double libm_asdouble(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return d;
}
TL_LIBM_HD inline uint64_t libm_asu64(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}
TL_LIBM_HD inline uint32_t libm_asu32(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

// fma(a, b, c) with one rounding, on both sides
TL_LIBM_HD inline double libm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// T: the table above (expf_libm passes the constant; a kernel may pass a copy in LDS, which a
// lane reads without a memory round trip)
TL_LIBM_HD inline float expf_libm_tab(float x, const uint64_t* T) {
#if defined(__clang__)
#pragma clang fp contract(off)  // only the explicit fma below fuse (HIP compiles with contraction on)
#endif
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double Shift = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const uint32_t ux = libm_asu32(x);
  const uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= (libm_asu32(88.0f) >> 20)) {  // |x| >= 88 or NaN
    if (ux == libm_asu32(-__builtin_inff())) return 0.0f;
    if (abstop >= (libm_asu32(__builtin_inff()) >> 20)) return x + x;
    if (x > 0x1.62e42ep6f) return __builtin_inff();  // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;             // underflow
  }
  const double xd = (double)x;
  double z = InvLn2N * xd;
  double kd = z + Shift;
  const uint64_t ki = libm_asu64(kd);
  kd -= Shift;
  const double r = libm_fma(InvLn2N, xd, -kd);  // the FMA build contracts z - kd (z's product fused)
  uint64_t t = T[ki % 32];
  t += ki << 47;
  const double s = libm_asdouble(t);
  z = libm_fma(C0, r, C1);
  const double r2 = r * r;
  double y = libm_fma(C2, r, 1.0);
  y = libm_fma(z, r2, y);
  y = y * s;
  return (float)y;
}

TL_LIBM_HD inline float expf_libm(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr uint64_t T[32] = TL_EXPF_TABLE;
#else
  static const uint64_t T[32] = TL_EXPF_TABLE;
#endif
  return expf_libm_tab(x, T);
}

}  // namespace tl
