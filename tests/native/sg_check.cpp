// Check of the sphere grids (rt_lightgrid.h build_sphere_grids): for random
// scenes (scales 0.1 .. 1000, far from the origin, negative and tiny radii,
// overlapping spheres) and reflection rays built as the renderer builds them
// (main.cpp:32-46: a camera ray's closest hit, the normal, origin hit point +
// normal * 0.001, the reflected direction normalised by Ray()), plus rays from
// those origins aimed at sphere silhouettes ahead and behind (discriminant
// near 0): when the origin passes the device's check against the ball of the
// grid of the sphere it leaves (rt_device.h sg_usable), every sphere the
// reference's test (sphere.h:26-59) reports a hit for -- whatever the sign of
// t -- must be on the list of the cell the device looks up, under the device's
// binning and its +-2^-22 quotient errors, with an entry bound tlo <= t, and
// the early-exit scan of that list (rt_device.h grid_closest) must give the
// reference's find_intersection result (scene.h:41-61).  Prints
// "checked <rays> <hit pairs> fallback <rays> missed <count> wrong <count>".
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rt_lightgrid.h"

namespace {
struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V scl(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V nrm(V a) {
  const double l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
bool hit(V c, double r, V o, V d, double &t) {  // sphere.h:26-59
  V oc = sub(o, c);
  double a = dot(d, d), b = 2.0 * dot(oc, d), cc = dot(oc, oc) - r * r;
  double disc = b * b - 4 * a * cc;
  if (disc < 0) return false;
  if (disc == 0) {
    t = -b / (2 * a);
    return true;
  }
  double t1 = (-b - std::sqrt(disc)) / (2 * a), t2 = (-b + std::sqrt(disc)) / (2 * a);
  if (std::fmax(t1, t2) < 0) return false;
  t = std::fmin(t1, t2);
  if (t < 0) t = std::fmax(t1, t2);
  return true;
}
}  // namespace

int main(int argc, char **argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 20;
  long rays = 0, pairs = 0, fallback = 0, missed = 0, wrong = 0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(5000 + seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const double scale = std::pow(10.0, (int)(rng() % 5) - 1);  // 0.1 .. 1000
    const double shift = (rng() % 3 == 0) ? 1e4 * scale : 0.0;
    const int n = 20 + (int)(rng() % 300);
    const int N = (int[]){1, 3, 8, 16, 32, 64}[rng() % 6];
    std::vector<double> cx(n), cy(n), cz(n), r(n);
    for (int i = 0; i < n; i++) {
      cx[i] = shift + scale * 10 * U(rng);
      cy[i] = shift + scale * 10 * U(rng);
      cz[i] = shift + scale * 10 * U(rng);
      const int kind = (int)(rng() % 10);
      r[i] = scale * (kind == 0 ? 1e-4 : kind == 1 ? 5.0 : 0.05 + 1.5 * std::fabs(U(rng)));
      if (kind == 2) r[i] = -r[i];  // the parser accepts negative radii
    }
    if (rng() % 2) {  // a ground sphere under the scene (the synth scenes' r = 100 at y = -102)
      cx[0] = shift, cy[0] = shift - scale * 110.0, cz[0] = shift, r[0] = scale * 100.0;
    }
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int i = 0; i < n; i++) {
      const double p[3] = {cx[i], cy[i], cz[i]};
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], p[k] - std::fabs(r[i]));
        hi[k] = std::fmax(hi[k], p[k] + std::fabs(r[i]));
      }
    }
    double d2 = 0;
    for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    const double diam = std::sqrt(d2);
    // the ball radii of rt_kernel.hip sphere_grids()
    std::vector<double> rho(n);
    for (int i = 0; i < n; i++)
      rho[i] = (std::fabs(r[i]) + 0.001) * (1.0 + 1e-6) + 1e-12 * (std::fabs(cx[i]) + std::fabs(cy[i]) + std::fabs(cz[i])) +
               1e-9 * diam;
    std::vector<int32_t> start, ent;
    std::vector<uint8_t> ok;
    if (rtk::build_sphere_grids(cx.data(), cy.data(), cz.data(), r.data(), n, rho.data(), diam, N, 32,
                                size_t(64) << 20, start, ent, ok) == 0)
      continue;  // no grids: the device sweeps as before
    const size_t stride = (size_t)6 * N * N + 1;
    V P{shift + scale * 14 * U(rng), shift + scale * 14 * U(rng), shift + scale * 14 * U(rng)};
    for (int q = 0; q < 4000; q++) {
      // a camera ray and its closest hit (scene.h:41-61)
      V d0 = nrm(nrm({U(rng), U(rng), U(rng)}));
      if (q % 2) {  // aimed at a random sphere
        const int s = (int)(rng() % n);
        d0 = nrm(nrm(sub(add({cx[s], cy[s], cz[s]}, scl({U(rng), U(rng), U(rng)}, 0.7 * std::fabs(r[s]))), P)));
      }
      int hs = -1;
      double ht = 1e20;
      for (int i = 0; i < n; i++) {
        double t;
        if (hit({cx[i], cy[i], cz[i]}, r[i], P, d0, t) && t < ht) ht = t, hs = i;
      }
      if (hs < 0 || !ok[hs]) continue;
      const V C{cx[hs], cy[hs], cz[hs]};
      const V hp = add(P, scl(d0, ht));                       // main.cpp:32
      const V nm = nrm(sub(hp, C));                           // sphere.h:62-64
      const V o = add(hp, scl(nm, 0.001));                    // main.cpp:46
      V d = nrm(sub(d0, scl(scl(nm, 2.0), dot(d0, nm))));    // reflect(), then Ray() normalises
      if (q % 4 >= 2) {  // from that origin towards a point just on/off a silhouette, ahead or behind
        const int s = (int)(rng() % n);
        V c{cx[s], cy[s], cz[s]};
        V w = sub(c, o);
        V perp = nrm({w.y - w.z, w.z - w.x, w.x - w.y});
        if (!(dot(perp, perp) > 0.5)) perp = nrm({1.0, 2.0, 3.0});
        const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
        V dir = sub(add(c, scl(perp, std::fabs(r[s]) * f)), o);
        if (q % 4 == 3) dir = scl(dir, -1.0);
        d = nrm(dir);
      }
      rays++;
      // the device's origin check (sg_usable)
      const V oc = sub(o, C);
      if (!((oc.x * oc.x + oc.y * oc.y) + oc.z * oc.z <= rho[hs] * rho[hs])) {
        fallback++;
        continue;
      }
      int bi_ref = -1;
      double bt_ref = 1e20;
      for (int i = 0; i < n; i++) {
        double t;
        if (hit({cx[i], cy[i], cz[i]}, r[i], o, d, t) && t < bt_ref) bt_ref = t, bi_ref = i;
      }
      const float fx = (float)d.x, fy = (float)d.y, fz = (float)d.z;
      for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
        const int cc = rtk::lg_cell(fx, fy, fz, N, rel);
        if (cc < 0) continue;  // the device tests every sphere
        const int32_t *st = start.data() + stride * (size_t)hs;
        std::vector<float> tlo(n, NAN);
        for (int k = st[cc]; k < st[cc + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          float &m = tlo[ent[2 * k]];  // a sphere listed twice (ahead and behind): its lower bound
          m = m != m ? b : std::fmin(m, b);
        }
        for (int i = 0; i < n; i++) {
          double t;
          if (!hit({cx[i], cy[i], cz[i]}, r[i], o, d, t)) continue;
          if (rel == 0.0f) pairs++;
          if (!((double)tlo[i] <= t) && !(t != t)) {
            if (++missed < 10)
              std::printf("MISS seed %d N %d leaving %d sphere %d t %.17g tlo %.9g\n", seed, N, hs, i, t, (double)tlo[i]);
          }
        }
        double bt = 1e20;
        int bi = -1;
        for (int k = st[cc]; k < st[cc + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          if ((double)b > bt) break;
          const int i = ent[2 * k];
          double t;
          if (hit({cx[i], cy[i], cz[i]}, r[i], o, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
        }
        if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
          if (++wrong < 10) std::printf("WRONG seed %d N %d got %d %.17g want %d %.17g\n", seed, N, bi, bt, bi_ref, bt_ref);
        }
      }
    }
  }
  std::printf("checked %ld %ld fallback %ld missed %ld wrong %ld\n", rays, pairs, fallback, missed, wrong);
  return (missed != 0 || wrong != 0) ? 1 : 0;
}
