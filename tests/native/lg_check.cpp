// Conservativeness check of the per-light direction grids (rt_lightgrid.h):
// for random scenes and random shaded points, every sphere the exact fp64
// shadow test of the reference reports as occluding must be on the global list
// or on the list of the cell the device would look up -- half the lights just
// outside a sphere, where the shadow ray's EPSILON overshoot past the light
// (scene.h:72-82) reaches into it from any direction; every fifth scene small
// (diameter 0.2 .. 20) and 1e6 .. 1e10 from the origin, where the rounding
// of the shadow ray's origin and distance is far above kLgOvershoot's
// absolute slack and must be covered by the relative margins.  Prints
// "checked <queries> <occluding pairs> missed <count>".
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
V nrm(V a) { return scl(a, 1.0 / std::sqrt(dot(a, a))); }
// sphere.h:26-59 as the reference computes it
bool hit(V c, double r, V o, V d, double &t) {
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
  long queries = 0, pairs = 0, missed = 0, far_q = 0, far_p = 0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    double scale = std::pow(10.0, (int)(rng() % 5) - 1);   // 0.1 .. 1000
    double shift = (rng() % 3 == 0) ? 1e5 * scale : 0.0;  // far from the origin
    if (seed % 5 == 4) {  // small scenes very far from the origin: |coords| / diameter up to 1e10
      scale = std::pow(10.0, -(double)(rng() % 3));             // 1 .. 0.01
      shift = std::pow(10.0, 6.0 + 2.0 * (double)(rng() % 3));  // 1e6 .. 1e10
    }
    const int n = 20 + (int)(rng() % 200), nl = 1 + (int)(rng() % 4);
    const int N = (int[]){1, 2, 7, 32, 64}[rng() % 5];
    std::vector<double> cx(n), cy(n), cz(n), r(n), lx(nl), ly(nl), lz(nl);
    for (int i = 0; i < n; i++) {
      cx[i] = shift + scale * 10 * U(rng);
      cy[i] = shift + scale * 10 * U(rng);
      cz[i] = shift + scale * 10 * U(rng);
      const int kind = (int)(rng() % 10);
      r[i] = scale * (kind == 0 ? 1e-4 : kind == 1 ? 5.0 : 0.05 + 1.5 * std::fabs(U(rng)));
    }
    for (int l = 0; l < nl; l++) {
      lx[l] = shift + scale * 10 * U(rng);
      ly[l] = shift + scale * 10 * U(rng);
      lz[l] = shift + scale * 10 * U(rng);
      if (rng() % 2 == 0) {  // just outside a sphere, within the shadow rays' EPSILON overshoot (or a bit beyond)
        const int s = (int)(rng() % n);
        const V u = nrm({U(rng), U(rng), U(rng)});
        const double gap = 0.0015 * std::fabs(U(rng));
        lx[l] = cx[s] + u.x * (r[s] + gap), ly[l] = cy[s] + u.y * (r[s] + gap), lz[l] = cz[s] + u.z * (r[s] + gap);
      }
    }
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    auto grow = [&](double x, double y, double z, double rr) {
      const double p[3] = {x, y, z};
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], p[k] - rr);
        hi[k] = std::fmax(hi[k], p[k] + rr);
      }
    };
    for (int i = 0; i < n; i++) grow(cx[i], cy[i], cz[i], r[i]);
    for (int l = 0; l < nl; l++) grow(lx[l], ly[l], lz[l], 0.0);
    double d2 = 0;
    for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    const double diam = std::sqrt(d2);
    std::vector<int32_t> start, ids;
    rtk::build_light_grid(cx.data(), cy.data(), cz.data(), r.data(), n, lx.data(), ly.data(), lz.data(), nl, diam, N,
                          start, ids);
    const int cells = 6 * N * N;
    const double max_off = 1e-7 * diam;
    for (int q = 0; q < 4000; q++) {
      // shaded point on a random sphere's surface (as hit points are)
      const int s0 = (int)(rng() % n);
      V dir = nrm({U(rng), U(rng), U(rng)});
      V hp = add({cx[s0], cy[s0], cz[s0]}, scl(dir, r[s0]));
      const int l = (int)(rng() % nl);
      V L{lx[l], ly[l], lz[l]};
      V tl = sub(L, hp);
      const double dist = std::sqrt(dot(tl, tl));
      V ld = nrm(tl);
      V so = add(hp, scl(ld, 0.001)), sd = nrm(ld);  // EPSILON, absolute (ray_math_constants.h:22)
      V w = sub(L, so);
      const double off = std::fabs(w.y * sd.z - w.z * sd.y) + std::fabs(w.z * sd.x - w.x * sd.z) +
                         std::fabs(w.x * sd.y - w.y * sd.x);
      if (!(off <= max_off)) continue;  // the device tests every sphere for such rays
      // the device bins with quotients within 2^-22 of the IEEE ones (lg_cell_rcp):
      // a sphere must be listed in the cell of every such binning
      const int c = rtk::lg_cell((float)-sd.x, (float)-sd.y, (float)-sd.z, N);
      const int cm = rtk::lg_cell((float)-sd.x, (float)-sd.y, (float)-sd.z, N, -0x1p-22f);
      const int cp = rtk::lg_cell((float)-sd.x, (float)-sd.y, (float)-sd.z, N, 0x1p-22f);
      if (c < 0) continue;
      const int32_t *st = start.data() + (size_t)l * (cells + 2);
      std::vector<char> listed(n, 0), in_c(n, 0), in_m(n, 0), in_p(n, 0);
      for (int k = st[c]; k < st[c + 1]; k++) in_c[ids[k]] = 1;
      for (int k = st[cm]; k < st[cm + 1]; k++) in_m[ids[k]] = 1;
      for (int k = st[cp]; k < st[cp + 1]; k++) in_p[ids[k]] = 1;
      for (int i = 0; i < n; i++) listed[i] = in_c[i] && in_m[i] && in_p[i];
      for (int k = st[cells]; k < st[cells + 1]; k++) listed[ids[k]] = 1;
      queries++;
      far_q += seed % 5 == 4;
      for (int i = 0; i < n; i++) {
        double t;
        if (hit({cx[i], cy[i], cz[i]}, r[i], so, sd, t) && t < 1e20 && t < dist) {
          pairs++;
          far_p += seed % 5 == 4;
          if (!listed[i]) {
            missed++;
            if (missed < 10)
              std::printf("MISS seed %d N %d light %d sphere %d t %.17g dist %.17g\n", seed, N, l, i, t, dist);
          }
        }
      }
    }
  }
  std::printf("far %ld %ld\n", far_q, far_p);  // the 1e6 .. 1e10 scenes' queries and occluding pairs
  std::printf("checked %ld %ld missed %ld\n", queries, pairs, missed);
  return missed != 0;
}
