/* Bit-exactness check of the divide used by the open-case SOR kernels
 * (kernels.hpp div_denom): x / d computed as q = RN(x*y), y = RN(1/d), then two
 * FMA corrections q <- RN(q + RN(x - q*d)*y), sign of x. Compared with the
 * IEEE divide (x / d) on random numerators over +-100 binades, for the
 * denominators of the BASELINE configs and random / adversarial ones
 * (significands with long runs of ones). Prints mismatches; exit 1 if any.
 * usage: division_check SAMPLES_PER_DENOMINATOR RANDOM_DENOMINATORS */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xr(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}
static double bits(uint64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}
static double div_denom(double x, double d, double y) {
  double q = x * y;
  q = fma(fma(-q, d, x), y, q);
  q = fma(fma(-q, d, x), y, q);
  return copysign(q, x);
}
static double denom_of(int nx, int ny, double lx, double ly) {
  const double dx = lx / nx, dy = ly / ny;
  const double idx2 = 1.0 / (dx * dx), idy2 = 1.0 / (dy * dy);
  return 2.0 * (idx2 + idy2);
}

int main(int argc, char** argv) {
  const long per = argc > 1 ? atol(argv[1]) : 100000;
  const int nrand = argc > 2 ? atoi(argv[2]) : 200;
  /* channel (length 8 x height 1?) and step geometries at the config sizes and
   * the reference's own; the exact lengths do not matter for the check */
  double fixed[] = {denom_of(4096, 512, 8.0, 1.0), denom_of(8192, 512, 8.0, 2.0), denom_of(93, 31, 3.0, 1.0),
                    denom_of(256, 32, 8.0, 1.0), 3.0, 7.0, 10.0, 0.1, 1.0 / 3.0, bits(0x3fffffffffffffffull),
                    bits(0x3ff0000000000001ull)};
  const int nf = (int)(sizeof fixed / sizeof fixed[0]);
  long bad = 0, n = 0;
  for (int k = 0; k < nf + nrand; ++k) {
    double d;
    if (k < nf) {
      d = fixed[k];
    } else {
      uint64_t b = (xr() & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
      if (k % 3 == 0) b |= 0x000ffffffffff000ull; /* long runs of ones */
      d = ldexp(bits(b), (int)(xr() % 60) - 30);
    }
    const double y = 1.0 / d;
    for (long t = 0; t < per; ++t) {
      const uint64_t b = (xr() & 0x800fffffffffffffull) | ((uint64_t)(1023 + (int)(xr() % 200) - 100) << 52);
      const double x = bits(b);
      const double a = x / d, m = div_denom(x, d, y);
      if (memcmp(&a, &m, 8) != 0) {
        if (bad < 5) printf("mismatch d=%a x=%a div=%a fma=%a\n", d, x, a, m);
        ++bad;
      }
      ++n;
    }
    const double zs[2] = {0.0, -0.0};
    for (int z = 0; z < 2; ++z) {
      const double a = zs[z] / d, m = div_denom(zs[z], d, y);
      if (memcmp(&a, &m, 8) != 0) ++bad;
    }
  }
  printf("%ld mismatches of %ld\n", bad, n);
  return bad != 0;
}
