/* markstein_check.c -- the sphere hit normal's division (p - c) / r as a
 * Markstein division by RN(1/r) (rtp_kernels.hip shade_hit, RTP_SPH_NORMAL_MK;
 * rtp_device.hpp div_markstein) against IEEE float division, on the host:
 *   q = RN(a * ri); rem = fma(-q, r, a); q' = fma(rem, ri, q).
 * usage: markstein_check exhaustive <r>      every float a, |a| in [2^-40, 2^40] (both signs)
 *        markstein_check sampled <n> <seed>  n random (a, r): |a| in [2^-40, 2^40], r in [2^-20, 2^20]
 * Prints "OK <count>" or the first mismatch and exits 1. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static int check(float a, float r, float ri) {
  const volatile float want = a / r;
  const float q = a * ri;
  const float rem = fmaf(-q, r, a);
  const float got = fmaf(rem, ri, q);
  if (u_of(got) != u_of(want)) {
    printf("MISMATCH a=%a r=%a got=%a want=%a\n", a, r, got, want);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "exhaustive")) {
    const float r = strtof(argv[2], NULL), ri = 1.0f / r;
    uint64_t n = 0;
    for (uint32_t u = u_of(0x1p-40f); u <= u_of(0x1p40f); u++) {
      const float a = f_of(u);
      if (check(a, r, ri) || check(-a, r, ri)) return 1;
      n += 2;
    }
    printf("OK %llu\n", (unsigned long long)n);
    return 0;
  }
  if (argc >= 4 && !strcmp(argv[1], "sampled")) {
    const long n = atol(argv[2]);
    uint64_t s = strtoull(argv[3], NULL, 10) * 0x9E3779B97F4A7C15ull + 1;
    for (long i = 0; i < n; i++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      const uint32_t ua = u_of(0x1p-40f) + (uint32_t)((s & 0xffffffffu) % (u_of(0x1p40f) - u_of(0x1p-40f) + 1));
      const uint32_t ur = u_of(0x1p-20f) + (uint32_t)((s >> 32) % (u_of(0x1p20f) - u_of(0x1p-20f) + 1));
      const float a = (i & 1) ? -f_of(ua) : f_of(ua), r = f_of(ur);
      if (check(a, r, 1.0f / r)) return 1;
    }
    printf("OK %ld\n", n);
    return 0;
  }
  fprintf(stderr, "usage: markstein_check exhaustive <r> | sampled <n> <seed>\n");
  return 2;
}
