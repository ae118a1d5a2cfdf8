#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static uint32_t rs = 12345;
static uint32_t xr(void){ rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; }
static float rnd(void){ float f; uint32_t u; do { u = xr(); memcpy(&f,&u,4);} while(!isfinite(f)); return f; }
int main(void){
  long bad = 0, n = 0;
  for (long it = 0; it < 20000000; ++it) {
    float g[64]; float m = 0.f;
    int mode = it % 4;
    float sc = ldexpf(1.f, (int)(xr() % 60) - 40);
    for (int i = 0; i < 64; ++i) {
      float v = mode == 0 ? rnd() : ((float)(int32_t)xr() / 2147483648.f) * sc;
      if (mode == 3 && (i & 1)) v = (float)((int)(xr() % 255) - 127) * (sc / 127.f);  // exact multiples: ties
      g[i] = v; m = fmaxf(m, fabsf(v));
    }
    float scale = m / 127.0f;
    if (!(scale > 1e-30f) || !isfinite(scale)) continue;
    float r = 1.0f / scale;
    for (int i = 0; i < 64; ++i) {
      float q0 = g[i] / scale;
      float d1 = g[i] * r;
      float e = fmaf(-d1, scale, g[i]);
      float q1 = fmaf(e, r, d1);
      ++n;
      if (roundf(q0) != roundf(q1) || (q0 != q1 && isfinite(q0))) { if (bad < 10) printf("x=%a s=%a q0=%a q1=%a\n", g[i], scale, q0, q1); ++bad; }
    }
  }
  printf("n=%ld bad=%ld\n", n, bad);
}
