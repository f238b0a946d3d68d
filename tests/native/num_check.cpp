// Check of intersect_num's square-root-free decisions (rt_device.h, the code
// the kernels run, here on the CPU) against the reference's test
// (sphere.h:26-59):
//  * shadow queries (scene.h:65-86: o = p + ldir * EPSILON, d =
//    normalized(ldir), occluded when the sphere reports t < dist): shaded
//    points on a first sphere, lights far, near and on it, and second spheres
//    placed along the query's line -- between the point and the light, beyond
//    either, through the origin, grazing the line (distance |r| (1 +- 10^-k))
//    and exactly tangent (axis-aligned lines) -- radii 1e-4 .. 1e5, some
//    negative.  intersect_num with the caller's bound qocc = q(1 - 2^-48)
//    and shadow_cells' decision around it must give the reference's
//    "occluded" for every pair;
//  * closest hits (qocc < 0): a returned numerator gives the reference's t
//    exactly (fl(num / a2)), a miss is a miss.
// Also the bound behind shadow_cells' off_free (below).  Prints "shadow
// <pairs> occluded <k> early <e> skipped <s> wrong <w>", "closest <pairs> hits
// <h> skipped <s> wrong <w>" and "off <queries> max_ratio <r> wrong <w>".
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I csrc num_check.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "rt_device.h"

using rtk::D3;
using rtk::SphGeo;

namespace {
struct V {
  double x, y, z;
};
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V scl(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
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
D3 d3(V v) { return D3{v.x, v.y, v.z}; }
}  // namespace

int main(int argc, char **argv) {
  const long N = argc > 1 ? std::atol(argv[1]) : 1000000;
  std::mt19937_64 rng(7654321);
  std::uniform_real_distribution<double> U(-1.0, 1.0), U01(0.0, 1.0);
  auto rdir = [&] {
    V v;
    do v = {U(rng), U(rng), U(rng)};
    while (dot(v, v) > 1.0 || dot(v, v) < 1e-6);
    return unit(v);
  };
  auto rrad = [&] { return std::pow(10.0, -4.0 + 9.0 * U01(rng)) * (U01(rng) < 0.05 ? -1.0 : 1.0); };
  long sh = 0, sh_occ = 0, sh_early = 0, sh_skip = 0, sh_wrong = 0;
  long cl = 0, cl_hit = 0, cl_skip = 0, cl_wrong = 0;
  for (long it = 0; it < N; ++it) {
    // the shaded point: a camera-like ray's hit on a first sphere
    const double r0 = rrad();
    const V c0 = scl({U(rng), U(rng), U(rng)}, std::pow(10.0, 3.0 * U01(rng)));
    const V n0 = rdir();
    const V o0 = add(c0, scl(n0, std::fabs(r0) * std::pow(10.0, 3.0 * U01(rng)) + 1.0));
    const V d0 = unit(unit(sub(add(c0, scl(rdir(), std::fabs(r0) * U01(rng))), o0)));
    double t0;
    if (!ref_hit(c0, r0 * r0, o0, d0, t0)) continue;
    const V hp = add(o0, scl(d0, t0));
    V L;
    const double mode = U01(rng);
    if (mode < 0.1) L = add(c0, scl(rdir(), std::fabs(r0) * (0.5 + U01(rng))));
    else if (mode < 0.3) L = add(hp, scl(rdir(), std::fabs(r0) * std::pow(10.0, -6.0 + 6.0 * U01(rng))));
    else L = add(hp, scl(rdir(), std::fabs(r0) * std::pow(10.0, 4.0 * U01(rng))));
    // axis-aligned shadow rays now and then: exact tangents below
    const bool axis = U01(rng) < 0.1;
    if (axis) {
      const int ax = (int)(U01(rng) * 3.0) % 3;
      const double len = std::pow(10.0, -2.0 + 5.0 * U01(rng)) * (U01(rng) < 0.5 ? -1.0 : 1.0);
      L = hp;
      (ax == 0 ? L.x : ax == 1 ? L.y : L.z) += len;
    }
    const V to_light = sub(L, hp);
    const double dist = std::sqrt(dot(to_light, to_light));
    const V ldir = unit(to_light);
    const V o = add(hp, scl(ldir, 0.001)), d = unit(ldir);
    const double a = (d.x * d.x + d.y * d.y) + d.z * d.z, a4 = 4.0 * a, a2 = 2.0 * a;
    const double T = dist < rtk::kInf ? dist : rtk::kInf;
    const bool fast = rtk::a2_ok(a2) && dist == dist && T >= 0x1p-900;
    const double q = a2 * T, qlo = q * (1.0 - 0x1p-48), qhi = q * (1.0 + 0x1p-48);
    // a perpendicular for offsets from the line
    V perp = cross(d, rdir());
    if (dot(perp, perp) < 1e-12) continue;
    perp = unit(perp);
    for (int k = 0; k < 8; ++k) {
      const double r = rrad();
      const double rr = r * r;
      // the centre's position along the line: behind the origin, between, beyond the light
      const double u = U01(rng);
      const double tc = u < 0.3 ? -dist * std::pow(10.0, -3.0 + 4.0 * U01(rng)) - std::fabs(r) * U01(rng)
                        : u < 0.75 ? dist * U01(rng)
                                   : dist * (1.0 + std::pow(10.0, -3.0 + 4.0 * U01(rng)));
      const double hm = U01(rng);
      double h;
      if (hm < 0.3) h = std::fabs(r) * (1.0 + (U01(rng) < 0.5 ? -1.0 : 1.0) * std::pow(10.0, -15.0 * U01(rng)));
      else if (hm < 0.4) h = 0.0;
      else h = std::fabs(r) * 2.0 * U01(rng);
      V c = add(add(o, scl(d, tc)), scl(perp, h));
      if (axis && U01(rng) < 0.5) {  // exactly tangent to the axis-aligned line: offset along another axis
        const V pc = add(o, scl(d, tc));
        c = pc;
        if (std::fabs(d.x) < 0.5) c.x += std::fabs(r);
        else c.y += std::fabs(r);
      }
      const SphGeo s{c.x, c.y, c.z, rr};
      double t;
      const bool want = ref_hit(c, rr, o, d, t) && t < rtk::kInf && t < dist;  // scene.h:78-82
      // shadow_cells' test(i)
      bool occ = false;
      double num = 0.0;
      const int res = fast ? rtk::intersect_num(s, d3(o), d3(d), a4, num, qlo) : 2;
      if (res == 3) {
        occ = true;
        ++sh_early;
      } else if (res == 1) {
        if (num < qlo) occ = true;
        else if (!(num > qhi)) {
          const double tt = num / a2;
          occ = tt < rtk::kInf && tt < dist;
        }
      } else if (res == 2) {
        double tt;
        occ = rtk::intersect(s, d3(o), d3(d), a4, a2, tt) && tt < rtk::kInf && tt < dist;
      }
      ++sh;
      sh_occ += want;
      if (res == 0 && fast) {  // a miss with disc > 0: decided without the square root
        const V oc = sub(o, c);
        const double b = 2.0 * ((oc.x * d.x + oc.y * d.y) + oc.z * d.z);
        const double cc = ((oc.x * oc.x + oc.y * oc.y) + oc.z * oc.z) - rr;
        sh_skip += b * b - a4 * cc > 0.0;
      }
      if (occ != want && ++sh_wrong <= 5)
        std::printf("shadow wrong: c (%.17g %.17g %.17g) r %.17g o (%.17g %.17g %.17g) d (%.17g %.17g %.17g) "
                    "dist %.17g res %d want %d\n",
                    c.x, c.y, c.z, r, o.x, o.y, o.z, d.x, d.y, d.z, dist, res, want);
      // closest hit semantics on the same pair and on the camera-like ray
      for (int w = 0; w < 2; ++w) {
        const V ro = w ? o : o0, rd = w ? d : d0;
        const double ra = (rd.x * rd.x + rd.y * rd.y) + rd.z * rd.z, ra4 = 4.0 * ra, ra2 = 2.0 * ra;
        if (!rtk::a2_ok(ra2)) continue;
        double rt;
        const bool hit = ref_hit(c, rr, ro, rd, rt);
        double rn = 0.0;
        const int rc = rtk::intersect_num(s, d3(ro), d3(rd), ra4, rn);
        ++cl;
        bool bad = false;
        if (rc == 1) {
          ++cl_hit;
          bad = !hit || !(rn / ra2 == rt);
        } else if (rc == 0) {
          bad = hit;
        } else if (rc == 2) {
          ++cl_skip;
        } else {
          bad = true;
        }
        if (bad && ++cl_wrong <= 5)
          std::printf("closest wrong: c (%.17g %.17g %.17g) r %.17g rc %d hit %d\n", c.x, c.y, c.z, r, rc, hit);
      }
    }
  }
  // shadow_cells' off_free bound: for scenes at scales 1e-3 .. 1e5, centred
  // up to 1e6 scene sizes from the origin, hit points on spheres (a ray's
  // hit, o + d t) and lights in the box, the line's distance from its light as
  // shadow_cells computes it stays below 2^-41 (1.01 B + 0.01), B the box's
  // largest |coordinate| (the host then skips the per-ray check when that is
  // <= max_off)
  long off_n = 0, off_wrong = 0;
  double off_ratio = 0.0;
  for (long it = 0; it < N / 4; ++it) {
    const double scale = std::pow(10.0, -3.0 + 8.0 * U01(rng));
    const V ctr = scl(rdir(), scale * std::pow(10.0, 6.0 * U01(rng)) * (U01(rng) < 0.3 ? 0.0 : 1.0));
    const V c = add(ctr, scl({U(rng), U(rng), U(rng)}, scale));
    const double r = scale * std::pow(10.0, -3.0 * U01(rng));
    const V L = add(ctr, scl({U(rng), U(rng), U(rng)}, scale * 2.0));
    // the box of the sphere and the light
    double B = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double ck = k == 0 ? c.x : k == 1 ? c.y : c.z, lk = k == 0 ? L.x : k == 1 ? L.y : L.z;
      B = std::max(B, std::max(std::fabs(ck) + r, std::fabs(lk)));
    }
    const V o0 = add(c, scl(rdir(), r * (1.0 + 10.0 * U01(rng))));
    const V d0 = unit(sub(add(c, scl(rdir(), r * U01(rng))), o0));
    double t0;
    if (!ref_hit(c, r * r, o0, d0, t0) || !(t0 > 0)) continue;
    const V hp = add(o0, scl(d0, t0));
    const V to_light = sub(L, hp);
    const double len = std::sqrt((to_light.x * to_light.x + to_light.y * to_light.y) + to_light.z * to_light.z);
    if (!(len > 0)) continue;
    const V ldir = {to_light.x / len, to_light.y / len, to_light.z / len};
    const V o = add(hp, scl(ldir, 0.001)), d = unit(ldir);  // Ray(): direction normalised again
    const V w = sub(L, o);
    const double off = std::fabs(w.y * d.z - w.z * d.y) + std::fabs(w.z * d.x - w.x * d.z) +
                       std::fabs(w.x * d.y - w.y * d.x);
    const double bound = 0x1p-41 * (1.01 * B + 0.01);
    ++off_n;
    off_ratio = std::max(off_ratio, off / bound);
    if (!(off <= bound) && ++off_wrong <= 5)
      std::printf("off wrong: B %.17g off %.17g bound %.17g\n", B, off, bound);
  }
  std::printf("shadow %ld occluded %ld early %ld skipped %ld wrong %ld\n", sh, sh_occ, sh_early, sh_skip, sh_wrong);
  std::printf("closest %ld hits %ld skipped %ld wrong %ld\n", cl, cl_hit, cl_skip, cl_wrong);
  std::printf("off %ld max_ratio %.3g wrong %ld\n", off_n, off_ratio, off_wrong);
  return (sh_wrong || cl_wrong || off_wrong) ? 1 : 0;
}
