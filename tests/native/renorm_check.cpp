// Host check of rtk::renormalized (csrc/rt_device.h): normalized(a) with the
// fast path for |a| within a few ulps of 1.  The same arithmetic is restated
// here with std::fma (-ffp-contract=off) and compared bit for bit with the
// reference's normalisation (vec3.h:26-29: len = sqrt((x*x + y*y) + z*z),
// x/len, y/len, z/len) on
//   * random unit vectors normalised once (the shadow and camera directions,
//     scene.h:72 / camera.h:24 + ray.h:12),
//   * reflections d - 2 (d.n) n of unit vectors (main.cpp:46),
//   * vectors scaled by 1 + k 2^-53 for small k (every length class),
//   * components 0, -0, tiny, subnormal and at binade edges,
// and the quotient step alone on random numerators over the exponent range.
//   renorm_check N   -> prints "checked N fast F mismatches M"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {

struct V {
  double x, y, z;
};

V normalized(V a) {
  const double len = std::sqrt((a.x * a.x + a.y * a.y) + a.z * a.z);
  return {a.x / len, a.y / len, a.z / len};
}

// rt_device.h renormalized(), restated; fast = took the fast path
V renormalized(V a, bool &fast) {
  constexpr double u = 0x1p-53;
  const double s = (a.x * a.x + a.y * a.y) + a.z * a.z;
  const double t = (s - 1.0) * 0x1p53;
  auto usable = [](double x) { return std::fabs(x) >= 0x1p-959 || x == 0.0; };
  fast = t >= -4.0 && t <= 6.0 && usable(a.x) && usable(a.y) && usable(a.z);
  if (!fast) return normalized(a);
  const double len = t > 3.0 ? 1.0 + 2.0 * u : (t > -0.5 ? 1.0 : (t > -2.5 ? 1.0 - u : 1.0 - 2.0 * u));
  const double rcp = t > 3.0 ? 1.0 - 2.0 * u : (t > -0.5 ? 1.0 : 1.0 + 2.0 * u);
  auto q = [&](double x) {
    const double q0 = x * rcp;
    return std::copysign(std::fma(std::fma(-q0, len, x), rcp, q0), x);
  };
  return {q(a.x), q(a.y), q(a.z)};
}

uint64_t st = 0x9E3779B97F4A7C15ull;
uint64_t next() {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}
double uni() { return (double)(next() >> 11) * 0x1p-53 * 2.0 - 1.0; }

bool same(double a, double b) { return std::memcmp(&a, &b, sizeof a) == 0; }

}  // namespace

int main(int argc, char **argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
  long checked = 0, fast_n = 0, bad = 0;
  auto check = [&](V a) {
    bool fast;
    const V got = renormalized(a, fast), want = normalized(a);
    ++checked;
    fast_n += fast;
    if (!same(got.x, want.x) || !same(got.y, want.y) || !same(got.z, want.z)) {
      if (bad < 5) std::printf("mismatch %a %a %a\n", a.x, a.y, a.z);
      ++bad;
    }
  };
  const double special[] = {0.0, -0.0, 0x1p-1074, -0x1p-1000, 0x1p-960, 0x1p-959, 1e-300, 0x1.fffffffffffffp-1,
                            0x1p-1, 0x1.0000000000001p-1};
  for (long k = 0; k < n; ++k) {
    const double sc = std::ldexp(1.0, (int)(next() % 40) - 20);
    V v{uni() * sc, uni() * sc * (next() & 1 ? 1.0 : 1e-3), uni() * sc};
    if (next() % 16 == 0) v.x = special[next() % 10];
    if (next() % 32 == 0) v.y = special[next() % 10];
    const V d = normalized(v);
    check(d);  // a renormalised unit vector
    V nn = normalized(V{uni(), uni(), uni()});
    const double dn = 2.0 * ((d.x * nn.x + d.y * nn.y) + d.z * nn.z);
    check(V{d.x - nn.x * dn, d.y - nn.y * dn, d.z - nn.z * dn});  // a reflection (main.cpp:46 order)
    const double f = 1.0 + (double)((int)(next() % 17) - 8) * 0x1p-53;
    check(V{d.x * f, d.y * f, d.z * f});  // lengths across (and beyond) the fast classes
    check(V{special[next() % 10], d.y, d.z});
  }
  // the quotient step alone: random numerators over the usable exponent range
  const double lens[4] = {1.0 - 0x1p-52, 1.0 - 0x1p-53, 1.0, 1.0 + 0x1p-52};
  const double rcps[4] = {1.0 + 0x1p-52, 1.0 + 0x1p-52, 1.0, 1.0 - 0x1p-52};
  for (long k = 0; k < n; ++k) {
    uint64_t b = next();
    const int e = (int)(next() % 1920) + 64;
    b = (b & 0x800fffffffffffffull) | ((uint64_t)e << 52);
    double x;
    std::memcpy(&x, &b, sizeof x);
    const int i = (int)(next() & 3);
    const double q0 = x * rcps[i];
    const double q = std::copysign(std::fma(std::fma(-q0, lens[i], x), rcps[i], q0), x);
    ++checked;
    if (!same(q, x / lens[i])) ++bad;
  }
  for (int i = 0; i < 4; ++i)
    if (!same(1.0 / lens[i], rcps[i])) ++bad;  // rcp = RN(1/len)
  std::printf("checked %ld fast %ld mismatches %ld\n", checked, fast_n, bad);
  return bad != 0;
}
