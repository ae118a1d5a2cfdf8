// expf_exact.cpp — TEST INFRASTRUCTURE (probe): hip_llama.cpp_amd/csrc/libm_exact.hpp's expf_libm
// against the host C library's expf on ALL 2^32 float inputs (bit patterns; NaNs compared as NaN).
// Build: g++ -O2 -fopenmp -ffp-contract=off -I hip_llama.cpp_amd/csrc tools/probes/expf_exact.cpp -o /tmp/expf_exact
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "libm_exact.hpp"

#include <stdlib.h>
int main(int argc, char** argv) {
  const long long stride = argc > 1 ? atoll(argv[1]) : 1;  // 1: every input
  long long bad = 0, nan_bad = 0;
  uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad, nan_bad) schedule(static, 1 << 16)
  for (long long i = 0; i < (1ll << 32); i += stride) {
    float x;
    uint32_t u = (uint32_t)i;
    memcpy(&x, &u, 4);
    volatile float xv = x;
    const float a = expf(xv), b = tl::expf_libm(x);
    uint32_t ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    if (ua != ub) {
      if (a != a && b != b) { ++nan_bad; continue; }
      ++bad;
#pragma omp critical
      if (!first) first = u ? u : 1;
    }
  }
  printf("mismatches %lld (nan-payload only %lld), first input bits 0x%08x\n", bad, nan_bad, first);
  return bad != 0;
}
