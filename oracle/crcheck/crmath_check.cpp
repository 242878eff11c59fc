// Host check of cr_math.h (the device's correctly rounded atan / sin / cos / tan) against the
// host libm (glibc, the functions the reference's numba code calls): counts of bitwise
// mismatches over random and structured arguments from the solver's domains.
//   crmath_check N  ->  one JSON line
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../ali-fmm-and-ray-tracing_amd/csrc/cr_math.h"

static uint64_t bits(double v) {
  uint64_t b;
  memcpy(&b, &v, 8);
  return b;
}

struct Count {
  long n = 0, bad = 0;
  double worst = 0;
  double arg = 0;
  void check(double x, double mine, double ref) {
    n++;
    if (bits(mine) != bits(ref)) {
      bad++;
      if (bad <= 1) arg = x;
    }
  }
};

int main(int argc, char** argv) {
  const long N = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  Count at, at_int, s, c, t, s_deg, c_deg, t_deg;
  for (long i = 0; i < N; i++) {
    // atan: log-uniform magnitude over [2^-40, 2^40], both signs
    double x = ldexp(1.0 + U(g), (int)(U(g) * 80) - 40) * (U(g) < 0.5 ? -1 : 1);
    at.check(x, crm::atan(x), atan(x));
    // atan of ratios (wavefront directions dz/dx, slopes of ray segments)
    double y = (U(g) - 0.5) * 20, z = (U(g) - 0.5) * 20;
    if (z != 0) at.check(y / z, crm::atan(y / z), atan(y / z));
    // sin / cos / tan on [-7, 7]
    double a = (U(g) - 0.5) * 14;
    s.check(a, crm::sin(a), sin(a));
    c.check(a, crm::cos(a), cos(a));
    t.check(a, crm::tan(a), tan(a));
    // angles in degrees times pi/180 (the Christoffel forms' arguments)
    double e = U(g) * 360 - 90;
    double r = e * (M_PI / 180);
    s_deg.check(r, crm::sin(r), sin(r));
    c_deg.check(r, crm::cos(r), cos(r));
    t_deg.check(r, crm::tan(r), tan(r));
  }
  // integer ratios (source-init stencil angles, atan(i / j)) and whole degrees
  for (int i = -200; i <= 200; i++)
    for (int j = 1; j <= 200; j++) at_int.check((double)i / j, crm::atan((double)i / j), atan((double)i / j));
  for (int d = -3600; d <= 3600; d++) {
    double r = d * 0.1 * (M_PI / 180);
    s_deg.check(r, crm::sin(r), sin(r));
    c_deg.check(r, crm::cos(r), cos(r));
    t_deg.check(r, crm::tan(r), tan(r));
  }
  printf("{");
  const char* names[] = {"atan", "atan_int_ratio", "sin", "cos", "tan", "sin_deg", "cos_deg", "tan_deg"};
  Count* cs[] = {&at, &at_int, &s, &c, &t, &s_deg, &c_deg, &t_deg};
  for (int k = 0; k < 8; k++)
    printf("%s\"%s\": {\"n\": %ld, \"mismatch\": %ld, \"first_arg\": %.17g}", k ? ", " : "", names[k], cs[k]->n,
           cs[k]->bad, cs[k]->arg);
  printf("}\n");
  return 0;
}
