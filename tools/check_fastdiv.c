// Empirical check of the Markstein division used by trace.hip (RT_FASTDIV): q = fma(fma(-n*r, d, n), r, n*r)
// with r = RN(1/d) equals RN(n/d).  gcc -O2 -ffp-contract=off tools/check_fastdiv.c -lm && ./a.out 2000000000
#include <stdlib.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>
#include <string.h>
// xorshift
static uint64_t s = 88172645463325252ull;
static inline uint64_t nx(void){ s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float uf(void){ return (nx() >> 40) * (1.0f/16777216.0f); }
static inline float bits(uint32_t u){ float f; memcpy(&f,&u,4); return f; }
int main(int argc, char** argv){
  long long N = atoll(argv[1]); long long bad = 0;
  for (long long i = 0; i < N; ++i) {
    float d, n;
    int mode = i & 3;
    if (mode == 0) { d = uf(); if (fabsf(d) < 1e-4f) d = 1e-4f; }
    else if (mode == 1) { d = bits(0x38D1B717u + (uint32_t)(nx() % (0x3F800000u - 0x38D1B717u + 1))); } // [1e-4,1] all bit patterns
    else if (mode == 2) { d = 1e-4f; }
    else { d = bits(0x3F7FFFFFu - (uint32_t)(nx()%64)); } // near 1 with all-ones significand
    if (nx() & 1) d = -d;
    // numerator: split - o, values of varied magnitude
    float e = (float)((int)(nx() % 40) - 20);
    n = (uf() * 2.0f - 1.0f) * ldexpf(1.0f, (int)e);
    if ((i & 7) == 5) n = bits((uint32_t)nx()) ; // arbitrary bit patterns
    if (!isfinite(n) || fabsf(n) > 1e30f || (n != 0 && fabsf(n) < 1e-30f)) continue;
    float q = n / d;
    float zh = 1.0f / d;
    float q0 = n * zh;
    float r = fmaf(-q0, d, n);
    float q1 = fmaf(r, zh, q0);
    if (memcmp(&q, &q1, 4) != 0) { if (bad < 10) printf("mismatch n=%a d=%a q=%a q1=%a\n", n, d, q, q1); ++bad; }
  }
  printf("N=%lld bad=%lld\n", N, bad);
  return 0;
}
