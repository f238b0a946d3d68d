// Host check of rtk::shadow_quiet's bound (rt_device.h): for random shaded
// points hp and lights L over many scales and offsets from the origin, the
// shadow line the reference builds (scene.h:65-86: o = hp + ldir*EPS,
// d = normalized(ldir), ldir = normalized(L - hp)) passes within
// reach * 2^-45 of L, reach = |L - hp| + |hp|_1 + |L|_1 + 1, measured as the
// device's shadow_cells measures it (off = |(L - o) x d|_1).  fp64 with no
// contraction, the same operation order as rt_device.h.  Prints the number of
// rays, the largest off / bound ratio and the number of violations.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#pragma STDC FP_CONTRACT OFF

struct V { double x, y, z; };
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V scale(V a, double t) { return {a.x * t, a.y * t, a.z * t}; }
static double length(V a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static V normalized(V a) { double l = length(a); return {a.x / l, a.y / l, a.z / l}; }

static uint64_t s = 0x9E3779B97F4A7C15ull;
static double uni() {  // splitmix64 -> [0, 1)
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * 0x1p-53;
}
static double sym() { return 2.0 * uni() - 1.0; }

int main(int argc, char **argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 10000000;
  long bad = 0;
  double worst = 0.0;
  for (long i = 0; i < n; i++) {
    const double off0 = std::pow(10.0, 7.0 * uni() - 1.0) * (uni() < 0.5 ? 0.0 : 1.0);  // 0 or 0.1 .. 1e6
    const double sc = std::pow(10.0, 7.0 * uni() - 3.0);                                // 1e-3 .. 1e4
    const V c = {off0 * sym(), off0 * sym(), off0 * sym()};
    const V hp = add(c, {sc * sym(), sc * sym(), sc * sym()});
    const V lp = add(c, {sc * sym(), sc * sym(), sc * sym()});
    const V to_light = sub(lp, hp);
    const double dist = length(to_light);
    const V ldir = normalized(to_light);
    const V o = add(hp, scale(ldir, 0.001));
    const V d = normalized(ldir);
    const V w = sub(lp, o);
    const double off = std::fabs(w.y * d.z - w.z * d.y) + std::fabs(w.z * d.x - w.x * d.z) +
                       std::fabs(w.x * d.y - w.y * d.x);
    const double reach = dist + (std::fabs(hp.x) + std::fabs(hp.y) + std::fabs(hp.z)) +
                         (std::fabs(lp.x) + std::fabs(lp.y) + std::fabs(lp.z)) + 1.0;
    if (!(dist > 0.0)) continue;
    const double bound = reach * 0x1p-45;
    const double r = off / bound;
    if (r > worst) worst = r;
    if (!(off <= bound)) bad++;
  }
  std::printf("checked %ld worst_ratio %.3e violations %ld\n", n, worst, bad);
  return bad ? 1 : 0;
}
