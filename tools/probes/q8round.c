#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
int main(void){
  const float c = 0.49999997f;  /* pred(0.5) */
  long bad = 0, n = 0;
  for (uint64_t u = 0; u < 0x100000000ull; ++u) {
    uint32_t b = (uint32_t)u; float x; memcpy(&x, &b, 4);
    if (!(fabsf(x) <= 200.0f)) continue;
    ++n;
    int r0 = (int)roundf(x);
    int r1 = (int)(x + copysignf(c, x));
    if (r0 != r1) { if (bad < 5) printf("x=%a r0=%d r1=%d\n", x, r0, r1); ++bad; }
  }
  printf("c=%a n=%ld bad=%ld\n", c, n, bad);
}
