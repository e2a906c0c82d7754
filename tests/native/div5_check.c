/* div5_check.c -- test infrastructure: the kernel's correctly rounded x / 5 (csrc/kvc.hip
 * div5_rn: q0 = x * RN(1/5), exact FMA residual, one FMA correction; q0 when the residual is 0
 * or q0 is infinite) against IEEE x / 5.0f, bit for bit (NaN payloads aside).
 *   div5_check [STRIDE]   checks every STRIDE-th of the 2^32 fp32 patterns (default 1: all) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float div5_rn(float x) {
  const float q0 = x * 0.2f;
  const float r = fmaf(-q0, 5.0f, x);
  return (r == 0.0f || isinf(q0)) ? q0 : fmaf(r, 0.2f, q0);
}

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], NULL, 10) : 1;
  uint64_t bad = 0, n = 0;
  for (uint64_t u = 0; u < (1ull << 32); u += stride, ++n) {
    const float x = fbits((uint32_t)u);
    const float ref = x / 5.0f, got = div5_rn(x);
    if (ubits(ref) != ubits(got) && !(isnan(ref) && isnan(got))) {
      if (bad < 8) printf("x=0x%08x ref=0x%08x got=0x%08x\n", (uint32_t)u, ubits(ref), ubits(got));
      ++bad;
    }
  }
  printf("div5_check: %llu patterns, %llu mismatches\n", (unsigned long long)n,
         (unsigned long long)bad);
  return bad != 0;
}
