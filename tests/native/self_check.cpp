// Host check of shadow_cells' own-sphere pre-test (rt_device.h): for random
// shaded points on spheres (hit points computed as the reference computes
// them: a camera-like ray, Sphere::intersect, o + d t), random lights and
// the reference's shadow ray (scene.h:65-86: o = p + ldir * EPSILON,
// d = normalized(ldir)), the pre-test's two decisions must agree with the
// reference's own test of that sphere (sphere.h:26-59):
//   "in shadow" (origin inside, dist^2 > 6 r^2) => the sphere reports t < dist
//   "skip"      (both roots provably negative)  => the sphere reports no t < dist
// Radii 1e-4 .. 1e5 (and negative), grazing hits, lights on, near and inside
// the sphere.  Prints "checked <n> shadow <k> skip <m> wrong <w>".
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

namespace {
struct V {
  double x, y, z;
};
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V scl(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V unit(V a) {
  const double l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return {a.x / l, a.y / l, a.z / l};
}
// sphere.h:26-59
bool ref_hit(V c, double rr, V o, V d, double &t) {
  const V oc = sub(o, c);
  const double a = dot(d, d), b = 2.0 * dot(oc, d), cc = dot(oc, oc) - rr;
  const double disc = b * b - 4 * a * cc;
  if (disc < 0) return false;
  if (disc == 0) {
    t = -b / (2 * a);
    return true;
  }
  const double t1 = (-b - std::sqrt(disc)) / (2 * a), t2 = (-b + std::sqrt(disc)) / (2 * a);
  if ((t1 < t2 ? t2 : t1) < 0) return false;
  t = (t2 < t1) ? t2 : t1;
  if (t < 0) t = (t1 < t2) ? t2 : t1;
  return true;
}
}  // namespace

int main(int argc, char **argv) {
  const long N = argc > 1 ? std::atol(argv[1]) : 1000000;
  std::mt19937_64 rng(1234567);
  std::uniform_real_distribution<double> U(-1.0, 1.0), U01(0.0, 1.0);
  auto rdir = [&] {
    V v;
    do v = {U(rng), U(rng), U(rng)};
    while (dot(v, v) > 1.0 || dot(v, v) < 1e-6);
    return unit(v);
  };
  long checked = 0, shadow = 0, skip = 0, wrong = 0;
  for (long it = 0; it < N; ++it) {
    const double r = std::pow(10.0, -4.0 + 9.0 * U01(rng)) * (U01(rng) < 0.05 ? -1.0 : 1.0);
    const V c = scl({U(rng), U(rng), U(rng)}, std::pow(10.0, 3.0 * U01(rng)));
    const double rr = r * r;
    // a ray from outside towards a point near the sphere (grazing sometimes)
    const V n0 = rdir();
    const double far = std::fabs(r) * std::pow(10.0, 3.0 * U01(rng)) + 1.0;
    const V o0 = add(c, scl(n0, far));
    const double graze = U01(rng) < 0.3 ? 1.0 - std::pow(10.0, -12.0 * U01(rng)) : U01(rng);
    const V target = add(c, scl(rdir(), std::fabs(r) * graze));
    const V d0 = unit(unit(sub(target, o0)));
    double t0;
    if (!ref_hit(c, rr, o0, d0, t0)) continue;
    const V hp = add(o0, scl(d0, t0));
    // a light: anywhere, close to the surface, or inside the sphere
    V L;
    const double mode = U01(rng);
    if (mode < 0.2) L = add(c, scl(rdir(), std::fabs(r) * (0.5 + U01(rng))));
    else if (mode < 0.4) L = add(hp, scl(rdir(), std::fabs(r) * std::pow(10.0, -6.0 + 6.0 * U01(rng))));
    else L = add(hp, scl(rdir(), std::fabs(r) * std::pow(10.0, 4.0 * U01(rng))));
    const V to_light = sub(L, hp);
    const double dist = std::sqrt(to_light.x * to_light.x + to_light.y * to_light.y + to_light.z * to_light.z);
    const V ldir = unit(to_light);
    const V o = add(hp, scl(ldir, 0.001)), d = unit(ldir);
    // the pre-test, as shadow_cells computes it
    const double a = (d.x * d.x + d.y * d.y) + d.z * d.z, a4 = 4.0 * a, a2 = 2.0 * a;
    const double T = dist < 1e20 ? dist : 1e20;
    const bool fast = a2 >= 0x1p-60 && a2 <= 0x1p60 && dist == dist && T >= 0x1p-900;
    bool pre_shadow = false, pre_skip = false;
    if (fast) {
      const double ocx = o.x - c.x, ocy = o.y - c.y, ocz = o.z - c.z;
      const double cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rr;
      if (cc < 0.0) {
        pre_shadow = dist * dist > 6.0 * rr && rr < 1e38 && rr > 1e-200;
      } else if (cc > 0.0) {
        const double b = 2.0 * ((ocx * d.x + ocy * d.y) + ocz * d.z);
        const double p = b * b, disc = p - a4 * cc;
        pre_skip = b > 0.0 && (disc < 0.0 || (disc > 0.0 && p > 1e-290 && disc < p * (1.0 - 0x1p-50)));
      }
    }
    double t;
    const bool occ = ref_hit(c, rr, o, d, t) && t < 1e20 && t < dist;  // scene.h:78-82 for this sphere
    ++checked;
    shadow += pre_shadow;
    skip += pre_skip;
    if ((pre_shadow && !occ) || (pre_skip && occ)) {
      if (++wrong <= 5)
        std::printf("wrong: r %.17g c (%.17g %.17g %.17g) L (%.17g %.17g %.17g) shadow %d skip %d occ %d\n", r, c.x,
                    c.y, c.z, L.x, L.y, L.z, pre_shadow, pre_skip, occ);
    }
  }
  std::printf("checked %ld shadow %ld skip %ld wrong %ld\n", checked, shadow, skip, wrong);
  return wrong ? 1 : 0;
}
