/* Bit-exactness check of the divides used by the open-case SOR kernels
 * (device.hpp div_denom), y = RN(1/d), sign of x restored at the end:
 *  - two:   q = RN(x*y), then two FMA corrections q <- RN(q + RN(x - q*d)*y);
 *  - split: q = RN(x*y + RN(x*ylo)) with ylo = RN((1 - y*d)/d) (a faithful
 *           quotient), then one correction;
 *  - one:   q = RN(x*y), one correction - only for denominators with
 *           |1 - y*d| <= 2^-54 (RN(x*y) is then faithful).
 * Compared with the IEEE divide (x / d) on random numerators over +-100
 * binades and on numerators whose quotient lies next to a rounding midpoint,
 * for the denominators of the BASELINE configs and random / adversarial ones
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
static double div_split(double x, double d, double y, double ylo) {
  double q = fma(x, y, x * ylo);
  q = fma(fma(-q, d, x), y, q);
  return copysign(q, x);
}
static double div_one(double x, double d, double y) {
  double q = x * y;
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
  long bad = 0, n = 0, n_one = 0;
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
    const double r = fma(-y, d, 1.0); /* exact */
    const double ylo = r / d;
    const int one_ok = fabs(r) <= 0x1p-54;
    n_one += one_ok;
    for (long t = 0; t < per; ++t) {
      double x;
      if (t % 4 == 3) { /* quotient next to a midpoint: x = RN(m*d), m = odd 54-bit significand */
        const uint64_t mm = (xr() & 0x1fffffffffffffull) | 0x20000000000000ull | 1ull;
        const int k = (int)(xr() % 120) - 60 - 53;
        x = fma((double)(mm >> 1), ldexp(d, k + 1), ldexp(d, k)); /* RN(mm * 2^k * d), one rounding */
        if (xr() & 1) x = -x;
      } else {
        const uint64_t b = (xr() & 0x800fffffffffffffull) | ((uint64_t)(1023 + (int)(xr() % 200) - 100) << 52);
        x = bits(b);
      }
      const double a = x / d;
      const double m[3] = {div_denom(x, d, y), div_split(x, d, y, ylo), one_ok ? div_one(x, d, y) : a};
      for (int v = 0; v < 3; ++v)
        if (memcmp(&a, &m[v], 8) != 0) {
          if (bad < 5) printf("mismatch (variant %d) d=%a x=%a div=%a fma=%a\n", v, d, x, a, m[v]);
          ++bad;
        }
      ++n;
    }
    const double zs[2] = {0.0, -0.0};
    for (int z = 0; z < 2; ++z) {
      const double a = zs[z] / d, m0 = div_denom(zs[z], d, y), m1 = div_split(zs[z], d, y, ylo),
                   m2 = div_one(zs[z], d, y);
      if (memcmp(&a, &m0, 8) != 0 || memcmp(&a, &m1, 8) != 0 || memcmp(&a, &m2, 8) != 0) ++bad;
    }
  }
  printf("one-correction denominators: %ld of %d\n", n_one, nf + nrand);
  printf("%ld mismatches of %ld\n", bad, n);
  return bad != 0;
}
