// Check of the camera grid (rt_lightgrid.h build_point_grid): for random
// scenes, camera positions (inside spheres, next to their surfaces, far from
// the origin) and camera-ray directions (uniform, and aimed at sphere
// silhouettes so the discriminant is near 0), every sphere the reference's
// test (sphere.h:26-59) reports a hit for -- whatever the sign of t -- must be
// on the list of the cell the device looks up, under the device's binning
// and its +-2^-22 quotient errors, with an entry bound tlo <= t; and the
// device's early-exit scan of that list (rt_device.h cam_closest) must give
// the reference's find_intersection result (scene.h:41-61).  Prints
// "checked <rays> <hit pairs> missed <count> wrong <count>".
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
  long rays = 0, pairs = 0, missed = 0, wrong = 0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(1000 + seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const double scale = std::pow(10.0, (int)(rng() % 5) - 1);  // 0.1 .. 1000
    const double shift = (rng() % 3 == 0) ? 1e5 * scale : 0.0;
    const int n = 20 + (int)(rng() % 300);
    const int N = (int[]){1, 3, 16, 64, 256, 512}[rng() % 6];
    std::vector<double> cx(n), cy(n), cz(n), r(n);
    for (int i = 0; i < n; i++) {
      cx[i] = shift + scale * 10 * U(rng);
      cy[i] = shift + scale * 10 * U(rng);
      cz[i] = shift + scale * 10 * U(rng);
      const int kind = (int)(rng() % 10);
      r[i] = scale * (kind == 0 ? 1e-4 : kind == 1 ? 5.0 : 0.05 + 1.5 * std::fabs(U(rng)));
      if (kind == 2) r[i] = -r[i];  // the parser accepts negative radii
    }
    // the camera: free, inside a sphere, or on (just off) a sphere's surface
    V P{shift + scale * 12 * U(rng), shift + scale * 12 * U(rng), shift + scale * 12 * U(rng)};
    const int pk = (int)(rng() % 4);
    if (pk == 1) {
      const int s = (int)(rng() % n);
      P = add({cx[s], cy[s], cz[s]}, scl(nrm({U(rng), U(rng), U(rng)}), 0.5 * std::fabs(r[s])));
    } else if (pk == 2) {
      const int s = (int)(rng() % n);
      P = add({cx[s], cy[s], cz[s]}, scl(nrm({U(rng), U(rng), U(rng)}), std::fabs(r[s]) * (1.0 + 1e-12)));
    }
    double lo[3] = {P.x, P.y, P.z}, hi[3] = {P.x, P.y, P.z};
    for (int i = 0; i < n; i++) {
      const double p[3] = {cx[i], cy[i], cz[i]};
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], p[k] - std::fabs(r[i]));
        hi[k] = std::fmax(hi[k], p[k] + std::fabs(r[i]));
      }
    }
    double d2 = 0;
    for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    std::vector<int32_t> start, ent;
    if (!rtk::build_point_grid(cx.data(), cy.data(), cz.data(), r.data(), n, P.x, P.y, P.z, std::sqrt(d2), N, 32,
                               size_t(64) << 20, start, ent))
      continue;  // the device then sweeps as before
    for (int q = 0; q < 3000; q++) {
      V dir;
      if (q % 3 == 0) {
        dir = {U(rng), U(rng), U(rng)};
      } else {  // towards a point just on/off a sphere's silhouette
        const int s = (int)(rng() % n);
        V c{cx[s], cy[s], cz[s]};
        V w = sub(c, P);
        V perp = nrm({w.y - w.z, w.z - w.x, w.x - w.y});
        if (!(dot(perp, perp) > 0.5)) perp = nrm({1.0, 2.0, 3.0});
        const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
        dir = sub(add(c, scl(perp, std::fabs(r[s]) * f)), P);
        if (q % 3 == 2) dir = scl(dir, -1.0);  // a silhouette behind the camera
      }
      V d = nrm(nrm(dir));  // camera.h:24 then ray.h:12
      int bi_ref = -1;
      double bt_ref = 1e20;
      for (int i = 0; i < n; i++) {  // scene.h:41-61
        double t;
        if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && t < bt_ref) bt_ref = t, bi_ref = i;
      }
      rays++;
      const float fx = (float)d.x, fy = (float)d.y, fz = (float)d.z;
      for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
        const int c = rtk::lg_cell(fx, fy, fz, N, rel);
        if (c < 0) continue;  // the device tests every sphere
        std::vector<float> tlo(n, NAN);
        for (int k = start[c]; k < start[c + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          tlo[ent[2 * k]] = b;
        }
        for (int i = 0; i < n; i++) {
          double t;
          if (!hit({cx[i], cy[i], cz[i]}, r[i], P, d, t)) continue;
          if (rel == 0.0f) pairs++;
          if (!((double)tlo[i] <= t) && !(t != t)) {
            if (++missed < 10)
              std::printf("MISS seed %d N %d sphere %d t %.17g tlo %.9g\n", seed, N, i, t, (double)tlo[i]);
          }
        }
        // cam_closest's scan: ascending tlo, stop at the first tlo > best t
        double bt = 1e20;
        int bi = -1;
        for (int k = start[c]; k < start[c + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          if ((double)b > bt) break;
          const int i = ent[2 * k];
          double t;
          if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
        }
        if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
          if (++wrong < 10) std::printf("WRONG seed %d N %d got %d %.17g want %d %.17g\n", seed, N, bi, bt, bi_ref, bt_ref);
        }
      }
    }
  }
  std::printf("checked %ld %ld missed %ld wrong %ld\n", rays, pairs, missed, wrong);
  return (missed != 0 || wrong != 0) ? 1 : 0;
}
