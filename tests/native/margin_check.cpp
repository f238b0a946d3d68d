// Near-boundary proofs of the culling structures (round 6): geometry placed
// within 2 EPSILON of every margin the structures rely on, run through the
// product's own builders (rt_lightgrid.cpp, rt_bvh.cpp) and the kernels' own
// host-callable lookup / walk arithmetic (rt_lightgrid.h lg_cell, rt_device.h
// walk4_ray / box4_hit / pf_keep / behind_cells / grid_closest_line), against
// the reference's test (sphere.h:26-59) and find_intersection (scene.h:41-61).
// EPSILON = 0.001 is absolute in the reference (ray_math_constants.h:22): a
// reflection ray starts at hit + n * EPSILON (main.cpp:46), a shadow ray
// EPSILON past its point (scene.h:76-82; the light grids' proof is
// tests/native/lg_check.cpp).
//
// Scenes: scales 0.01 .. 100, 0 .. 1e7 from the origin, contact pairs whose
// surfaces are -EPSILON .. +2 EPSILON apart (a reflection off one near the
// contact starts inside, on or just outside the other), cameras within
// +-2 EPSILON of a sphere surface, negative radii.
//
//  camgrid    -- build_point_grid around the camera P: rays at silhouettes
//                (+-1e-12), along cube-map cell EDGES (a minor coordinate
//                exactly on a cell boundary; spheres placed grazing those
//                directions within 2 EPSILON), binned with the device's
//                +-2^-22 quotient errors: every sphere the reference hits
//                (either sign of t) is listed with tlo <= t and the early-exit
//                scan returns find_intersection's (t, index).
//  spheregrid -- build_sphere_grids: reflection rays off points next to a
//                contact, and rays from those origins at the neighbour's
//                silhouette and along cell edges; the device's origin-ball
//                check (sg_usable), then the same list / scan conditions.
//  ugrid      -- build_ugrid (1,500 spheres): lines tangent to a sphere at a
//                point ON a cell plane (up to rounding) behind the origin, and
//                origins within 2 EPSILON of a cell plane: behind_cells hands
//                every backward-tangent / disc == 0 sphere to the exact test
//                and grid_closest_line returns find_intersection's (t, index).
//  bvh        -- build_bvh / build_bvh4 as rt_upload_scene builds them (fp32
//                boxes relative to the bounds' centre, leaves of 2, 1 above
//                1,024 spheres), the render's margins (bvh_args): every sphere
//                the reference hits, either sign of t, is reachable through
//                boxes that pass box4_hit and a leaf prefilter that passes
//                pf_keep; and the walk pruned at float_up(best t) finds
//                find_intersection's (t, index).
// Prints one line per structure:
//   "<name> <rays> <hit pairs> <targeted> ... missed <count> wrong <count>".
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I csrc -I include margin_check.cpp
//         csrc/rt_bvh.cpp csrc/rt_lightgrid.cpp
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rt_device.h"
#include "rt_lightgrid.h"

using rtk::BvhArgs;
using rtk::D3;

namespace {
constexpr double kEps = 0.001;  // ray_math_constants.h:22
struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V scl(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V nrm(V a) {
  const double l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
double comp(V a, int k) { return k == 0 ? a.x : (k == 1 ? a.y : a.z); }
// sphere.h:26-59: 1 = hit through disc == 0 (t set), 2 = other hit, 0 = miss
int ref_test(V c, double r, V o, V d, double &t) {
  V oc = sub(o, c);
  double a = dot(d, d), b = 2.0 * dot(oc, d), cc = dot(oc, oc) - r * r;
  double disc = b * b - 4 * a * cc;
  if (disc < 0) return 0;
  if (disc == 0) {
    t = -b / (2 * a);
    return 1;
  }
  double t1 = (-b - std::sqrt(disc)) / (2 * a), t2 = (-b + std::sqrt(disc)) / (2 * a);
  if (std::fmax(t1, t2) < 0) return 0;
  t = std::fmin(t1, t2);
  if (t < 0) t = std::fmax(t1, t2);
  return 2;
}

struct Scene {
  std::vector<V> C;
  std::vector<double> R;
  std::vector<int> contact;  // contact[i] = j: i was placed touching j (-1: free)
  double scale = 1, shift = 0;
  int n() const { return (int)C.size(); }
  // find_intersection (scene.h:41-61)
  int closest(V o, V d, double &bt) const {
    int bi = -1;
    bt = 1e20;
    for (int i = 0; i < n(); i++) {
      double t;
      if (ref_test(C[i], R[i], o, d, t) && t < bt) bt = t, bi = i;
    }
    return bi;
  }
};

V rand_unit(std::mt19937_64 &rng) {
  std::normal_distribution<double> G(0.0, 1.0);
  for (;;) {
    V u{G(rng), G(rng), G(rng)};
    const double l = dot(u, u);
    if (l > 1e-6) return nrm(u);
  }
}

// A random scene with contact pairs (gaps -EPSILON .. +2 EPSILON, absolute).
// cloud: a flat synth10k-like cloud (80 x 13.5 x 105, radii 0.15 .. 0.6).
Scene make_scene(std::mt19937_64 &rng, int n, double scale, double shift, bool cloud = false) {
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  static const double kGaps[] = {-1.0, -0.5, 0.0, 0.5, 0.999, 1.0, 1.001, 1.5, 2.0};
  Scene s;
  s.scale = scale;
  s.shift = shift;
  const V off{shift, -0.5 * shift, shift};
  for (int i = 0; i < n; i++) {
    if (i > 0 && rng() % 3 == 0) {  // touching sphere j
      const int j = (int)(rng() % i);
      const V u = rand_unit(rng);
      const double r = scale * (cloud ? 0.15 + 0.45 * std::fabs(U(rng)) : 0.1 + 1.2 * std::fabs(U(rng)));
      const double g = kGaps[rng() % 9] * kEps;
      s.C.push_back(add(s.C[j], scl(u, std::fabs(s.R[j]) + r + g)));
      s.R.push_back(r);
      s.contact.push_back(j);
      continue;
    }
    if (cloud) {
      s.C.push_back(add(off, scl(V{U(rng) * 40, U(rng) * 6.75 + 5.25, U(rng) * 52.5 - 67.5}, scale)));
      s.R.push_back(scale * (0.15 + 0.45 * std::fabs(U(rng))));
      s.contact.push_back(-1);
      continue;
    }
    s.C.push_back(add(off, scl(V{U(rng) * 10, U(rng) * 10, U(rng) * 10}, scale)));
    const int kind = (int)(rng() % 10);
    double r = scale * (kind == 0 ? 0.01 : kind == 1 ? 4.0 : 0.1 + 1.5 * std::fabs(U(rng)));
    if (kind == 2) r = -r;  // the parser accepts negative radii
    s.R.push_back(r);
    s.contact.push_back(-1);
  }
  return s;
}

// A camera within +-2 EPSILON of a sphere surface (or free)
V make_camera(std::mt19937_64 &rng, const Scene &s) {
  static const double kGaps[] = {-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 2.0};
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  if (rng() % 4 == 0)
    return add(V{s.shift, -0.5 * s.shift, s.shift}, scl(V{U(rng) * 14, U(rng) * 14, U(rng) * 14}, s.scale));
  const int i = (int)(rng() % s.n());
  return add(s.C[i], scl(rand_unit(rng), std::fabs(s.R[i]) + kGaps[rng() % 7] * kEps));
}

// A direction whose minor coordinate lies exactly on a cell boundary of an
// N x N cube map (lg_cell: (p/m + 1) N / 2 an integer), the other random.
V edge_dir(std::mt19937_64 &rng, int N) {
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const int face = (int)(rng() % 6), axis = face / 2;
  const double sg = (face & 1) ? -1.0 : 1.0;
  const double p = -1.0 + 2.0 * (double)(rng() % (N + 1)) / (double)N;
  const double q = (rng() % 3 == 0) ? -1.0 + 2.0 * (double)(rng() % (N + 1)) / (double)N : U(rng);
  double v[3];
  v[axis] = sg;
  const bool swap = rng() & 1;
  v[(axis + 1) % 3] = swap ? q : p;
  v[(axis + 2) % 3] = swap ? p : q;
  return V{v[0], v[1], v[2]};
}

// A point at distance |r| + g from C in a direction perpendicular to u (the
// line P + t u then grazes the sphere of radius |r| around C at distance g).
V graze_centre(std::mt19937_64 &rng, V P, V u, double t, double r, double g) {
  V w = cross(u, rand_unit(rng));
  w = nrm(w);
  return add(add(P, scl(u, t)), scl(w, std::fabs(r) + g));
}

struct Stat {
  long rays = 0, pairs = 0, targeted = 0, extra = 0, missed = 0, wrong = 0;
};

// One looked-up list of a point grid (camera grid or a sphere's grid): every
// sphere hit (either sign of t) listed with tlo <= t; the early-exit scan ==
// find_intersection.  start/ent as build_point_grid / build_sphere_grids.
void check_list(const Scene &s, V o, V d, const int32_t *st, const std::vector<int32_t> &ent, int N, Stat &S,
                const char *what, int seed) {
  double bt_ref;
  const int bi_ref = s.closest(o, d, bt_ref);
  const float fx = (float)d.x, fy = (float)d.y, fz = (float)d.z;
  for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
    const int c = rtk::lg_cell(fx, fy, fz, N, rel);
    if (c < 0) continue;  // the device tests every sphere
    std::vector<float> tlo(s.n(), NAN);
    for (int k = st[c]; k < st[c + 1]; k++) {
      float b;
      std::memcpy(&b, &ent[2 * k + 1], sizeof b);
      float &m = tlo[ent[2 * k]];
      m = m != m ? b : std::fmin(m, b);
    }
    for (int i = 0; i < s.n(); i++) {
      double t;
      if (!ref_test(s.C[i], s.R[i], o, d, t)) continue;
      if (rel == 0.0f) S.pairs++;
      if (!((double)tlo[i] <= t) && !(t != t)) {
        if (++S.missed <= 10)
          std::printf("MISS %s seed %d N %d sphere %d t %.17g tlo %.9g\n", what, seed, N, i, t, (double)tlo[i]);
      }
    }
    double bt = 1e20;
    int bi = -1;
    for (int k = st[c]; k < st[c + 1]; k++) {
      float b;
      std::memcpy(&b, &ent[2 * k + 1], sizeof b);
      if ((double)b > bt) break;
      const int i = ent[2 * k];
      double t;
      if (ref_test(s.C[i], s.R[i], o, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
    }
    if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
      if (++S.wrong <= 10)
        std::printf("WRONG %s seed %d N %d got %d %.17g want %d %.17g\n", what, seed, N, bi, bt, bi_ref, bt_ref);
    }
  }
}

double diameter(const Scene &s, const V *P) {
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int i = 0; i < s.n(); i++)
    for (int k = 0; k < 3; k++) {
      lo[k] = std::fmin(lo[k], comp(s.C[i], k) - std::fabs(s.R[i]));
      hi[k] = std::fmax(hi[k], comp(s.C[i], k) + std::fabs(s.R[i]));
    }
  double d2 = 0;
  for (int k = 0; k < 3; k++) {
    const double l = P ? std::fmin(lo[k], comp(*P, k)) : lo[k], h = P ? std::fmax(hi[k], comp(*P, k)) : hi[k];
    d2 += (h - l) * (h - l);
  }
  return std::sqrt(d2);
}

// ---------------------------------------------------------------- camera grid
void camgrid(int seeds, Stat &S) {
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(61000 + seed);
    const double scale = std::pow(10.0, (double)(seed % 3) * 2.0 - 2.0);
    const double shift = (double[]){0.0, 1e3, 1e5, 1e7}[seed % 4] * (seed % 8 < 4 ? 1.0 : scale);
    const int N = (int[]){1, 3, 16, 64, 256}[rng() % 5];
    Scene s = make_scene(rng, 30 + (int)(rng() % 200), scale, shift);
    const V P = make_camera(rng, s);
    // spheres grazing cell-edge directions from P within 2 EPSILON
    std::vector<V> edges;
    for (int e = 0; e < 24; e++) {
      const V u = nrm(nrm(edge_dir(rng, N)));
      const double r = scale * (0.05 + (double)(rng() % 100) / 50.0);
      const double t = ((rng() & 1) ? 1.0 : -1.0) * scale * (1.0 + (double)(rng() % 20));  // ahead or behind
      const double g = ((double)(rng() % 5) - 1.0) * kEps;                                 // -1 .. 3 EPSILON
      s.C.push_back(graze_centre(rng, P, u, t, r, std::fmin(g, 2.0 * kEps)));
      s.R.push_back(r);
      s.contact.push_back(-1);
      edges.push_back(u);
    }
    std::vector<int32_t> start, ent;
    std::vector<double> cx, cy, cz;
    for (const V &c : s.C) cx.push_back(c.x), cy.push_back(c.y), cz.push_back(c.z);
    if (!rtk::build_point_grid(cx.data(), cy.data(), cz.data(), s.R.data(), s.n(), P.x, P.y, P.z, diameter(s, &P), N,
                               32, size_t(64) << 20, start, ent))
      continue;  // the device then sweeps
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (int q = 0; q < 1500; q++) {
      V d;
      if (q % 3 == 0) {  // along a cell edge (one of the grazing spheres' directions, or a new one)
        d = (q % 6 == 0) ? edges[rng() % edges.size()] : nrm(nrm(edge_dir(rng, N)));
        S.targeted++;
      } else {  // at a silhouette (+-1e-12), ahead or behind
        const int i = (int)(rng() % s.n());
        V w = sub(s.C[i], P);
        V perp = nrm(cross(w, rand_unit(rng)));
        const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
        V dir = sub(add(s.C[i], scl(perp, std::fabs(s.R[i]) * f)), P);
        if (q % 3 == 2) dir = scl(dir, -1.0);
        d = nrm(nrm(dir));  // camera.h:24 then ray.h:12
      }
      S.rays++;
      check_list(s, P, d, start.data(), ent, N, S, "camgrid", seed);
    }
  }
}

// --------------------------------------------------------------- sphere grids
void spheregrid(int seeds, Stat &S) {
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(62000 + seed);
    const double scale = std::pow(10.0, (double)(seed % 3) * 2.0 - 2.0);
    const double shift = (double[]){0.0, 1e3, 1e5, 1e7}[seed % 4] * (seed % 8 < 4 ? 1.0 : scale);
    const int N = (int[]){1, 3, 8, 16, 32}[rng() % 5];
    Scene s = make_scene(rng, 30 + (int)(rng() % 200), scale, shift);
    const int n = s.n();
    std::vector<double> cx(n), cy(n), cz(n), rho(n);
    for (int i = 0; i < n; i++) cx[i] = s.C[i].x, cy[i] = s.C[i].y, cz[i] = s.C[i].z;
    const double diam = diameter(s, nullptr);
    for (int i = 0; i < n; i++)  // the ball radii of rt_kernel.hip sphere_grids()
      rho[i] = (std::fabs(s.R[i]) + 0.001) * (1.0 + 1e-6) +
               1e-12 * (std::fabs(cx[i]) + std::fabs(cy[i]) + std::fabs(cz[i])) + 1e-9 * diam;
    std::vector<int32_t> start, ent;
    std::vector<uint8_t> ok;
    if (rtk::build_sphere_grids(cx.data(), cy.data(), cz.data(), s.R.data(), n, rho.data(), diam, N, 32,
                                size_t(64) << 20, start, ent, ok) == 0)
      continue;
    const size_t stride = (size_t)6 * N * N + 1;
    std::vector<int> touching;
    for (int i = 0; i < n; i++)
      if (s.contact[i] >= 0) touching.push_back(i);
    if (touching.empty()) continue;
    for (int q = 0; q < 1500; q++) {
      // a camera ray at a point next to a contact: towards the contact point
      // of pair (i, j), from outside, nudged so it hits one of them near it
      const int i = touching[rng() % touching.size()], j = s.contact[i];
      const V u = nrm(sub(s.C[i], s.C[j]));
      const V cp = add(s.C[j], scl(u, std::fabs(s.R[j])));  // j's surface towards i
      const V side = nrm(cross(u, rand_unit(rng)));
      const double back = std::fabs(s.R[j]) + std::fabs(s.R[i]) + 5.0 * s.scale;
      const V P = add(cp, scl(side, back));
      const V aim = add(cp, scl(rand_unit(rng), kEps * (double)(rng() % 4)));
      const V d0 = nrm(nrm(sub(aim, P)));
      double ht;
      const int hs = s.closest(P, d0, ht);
      if (hs < 0 || !ok[hs]) continue;
      const V hp = add(P, scl(d0, ht));                                       // main.cpp:32
      const V nm = nrm(sub(hp, s.C[hs]));                                     // sphere.h:62-64
      const V o = add(hp, scl(nm, kEps));                                     // main.cpp:46
      V d = nrm(sub(d0, scl(scl(nm, 2.0), dot(d0, nm))));                     // reflect(), then Ray()
      if (q % 3 == 1) {  // from that origin at the neighbour's silhouette, ahead or behind
        const int k = (hs == i) ? j : i;
        V w = sub(s.C[k], o);
        V perp = nrm(cross(w, rand_unit(rng)));
        const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
        V dir = sub(add(s.C[k], scl(perp, std::fabs(s.R[k]) * f)), o);
        if (rng() & 1) dir = scl(dir, -1.0);
        d = nrm(dir);
      } else if (q % 3 == 2) {  // along a cell edge of the grid of the sphere it leaves
        d = nrm(edge_dir(rng, N));
      }
      S.rays++;
      S.targeted += std::fabs(std::sqrt(dot(sub(o, s.C[hs == i ? j : i]), sub(o, s.C[hs == i ? j : i]))) -
                              std::fabs(s.R[hs == i ? j : i])) <= 2.0 * kEps;
      const V oc = sub(o, s.C[hs]);  // the device's origin check (sg_usable)
      if (!((oc.x * oc.x + oc.y * oc.y) + oc.z * oc.z <= rho[hs] * rho[hs])) {
        S.extra++;  // falls back to the sweep
        continue;
      }
      check_list(s, o, d, start.data() + stride * (size_t)hs, ent, N, S, "spheregrid", seed);
    }
  }
}

// ---------------------------------------------------------------- uniform grid
void ugrid(int seeds, Stat &S) {
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(63000 + seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const double scale = std::pow(10.0, (double)(seed % 3) - 1.0);
    const double shift = (double[]){0.0, 1e3, 1e5}[seed % 3] * scale;
    Scene s = make_scene(rng, 1500, scale, shift, true);
    // a ground sphere (global)
    s.C.push_back({shift, -0.5 * shift - 110.0 * scale, shift});
    s.R.push_back(100.0 * scale);
    s.contact.push_back(-1);
    const int N = s.n();
    const V cam = add(V{shift, -0.5 * shift, shift}, V{0.0, 3.0 * scale, 12.0 * scale});
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, rmax = 0.0;
    for (int i = 0; i < N; i++) {
      const double a = std::fabs(s.R[i]);
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], comp(s.C[i], k) - a);
        hi[k] = std::fmax(hi[k], comp(s.C[i], k) + a);
      }
      rmax = std::fmax(rmax, a);
    }
    double c0[3];
    for (int k = 0; k < 3; k++) c0[k] = 0.5 * (lo[k] + hi[k]);
    const double diam = diameter(s, &cam) + 0.01;
    std::vector<double> bx(N), by(N), bz(N);
    for (int i = 0; i < N; i++) bx[i] = s.C[i].x - c0[0], by[i] = s.C[i].y - c0[1], bz[i] = s.C[i].z - c0[2];
    rtk::UgridHost ug;
    if (!rtk::build_ugrid(bx.data(), by.data(), bz.data(), s.R.data(), N, (size_t)64 << 20, ug, 2.0)) {
      std::printf("ugrid seed %d: no grid\n", seed);
      continue;
    }
    BvhArgs bv{};
    bv.c0x = c0[0], bv.c0y = c0[1], bv.c0z = c0[2];
    const float margin = (float)(1e-6 * (diam + rmax) * (1.0 + 1e-6));
    bv.pmargin = 4.0f * margin;
    if (!((double)bv.pmargin + 1e-4 * (double)ug.extent <= (double)ug.reg_margin)) {  // the device keeps the BVH then
      std::printf("ugrid seed %d: margin %g + %g > %g\n", seed, (double)bv.pmargin, 1e-4 * ug.extent, ug.reg_margin);
      continue;
    }
    bv.ug = rtk::UgArgs{reinterpret_cast<const float4 *>(ug.rec.data()), ug.rid.data(),
                        reinterpret_cast<const float4 *>(ug.q.data()), ug.ids.data(), ug.glob.data(),
                        (int)ug.glob.size(), ug.nx, ug.ny, ug.nz, ug.gx, ug.gy, ug.gz, ug.cs, 1, 1,
                        (float)(1e-4 * (double)ug.extent)};
    bv.tf_min = 0.0f;
    const double g0[3] = {(double)ug.gx + c0[0], (double)ug.gy + c0[1], (double)ug.gz + c0[2]};
    const int ncell[3] = {ug.nx, ug.ny, ug.nz};
    const double cs = (double)ug.cs, tol = 1e-7 * diam;
    std::vector<char> seen(N);
    for (int li = 0; li < 3000; li++) {
      const int si = (int)(rng() % (N - 1));
      const V C = s.C[si];
      const double r = std::fabs(s.R[si]);
      // the tangent point on a cell plane: axis k, a plane crossing the sphere
      const int k = (int)(rng() % 3);
      const double ck = comp(C, k);
      const double p0 = std::ceil((ck - r - g0[k]) / cs), p1 = std::floor((ck + r - g0[k]) / cs);
      V nn;
      if (p1 >= p0 && p0 >= 0 && p1 <= ncell[k]) {
        const double plane = g0[k] + cs * (p0 + (double)(rng() % (long)(p1 - p0 + 1)));
        const double nk = std::fmax(-1.0, std::fmin(1.0, (plane - ck) / r));
        const double rest = std::sqrt(std::fmax(0.0, 1.0 - nk * nk)), phi = 6.283185307179586 * U(rng);
        double v[3];
        v[k] = nk;
        v[(k + 1) % 3] = rest * std::cos(phi);
        v[(k + 2) % 3] = rest * std::sin(phi);
        nn = V{v[0], v[1], v[2]};
        S.targeted++;
      } else {
        nn = rand_unit(rng);
      }
      const V P = add(C, scl(nn, r));
      const V d = nrm(cross(nn, rand_unit(rng)));
      double back = (0.01 + 30.0 * U(rng) * U(rng)) * scale;
      if (li % 2) {  // the origin within 2 EPSILON of a cell plane of axis k2
        const int k2 = (int)(rng() % 3);
        const double dk = comp(d, k2);
        if (std::fabs(dk) > 0.05) {
          const double ok = comp(P, k2) + dk * back;
          const double plane = g0[k2] + cs * std::round((ok - g0[k2]) / cs);
          const double g = ((double)(rng() % 5) - 2.0) * kEps;
          const double b2 = (plane + g - comp(P, k2)) / dk;
          if (b2 > 0) back = b2, S.extra++;
        }
      }
      const V o = add(P, scl(d, back));
      S.rays++;
      std::fill(seen.begin(), seen.end(), 0);
      rtk::Work work;
      rtk::behind_cells(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z}, work, [&](int i) { seen[i] = 1; });
      {
        double bt = 1e20, rt;
        int bi = -1;
        auto fold = [&](int i) {
          double t;
          if (ref_test(s.C[i], s.R[i], o, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
        };
        rtk::Work w2;
        rtk::grid_closest_line(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z}, w2, fold, [&] { return bt; });
        const int ri = s.closest(o, d, rt);
        if (bi != ri || (ri >= 0 && bt != rt)) {
          if (++S.wrong <= 10)
            std::printf("WRONG ugrid seed %d line %d grid (%d, %.17g) reference (%d, %.17g)\n", seed, li, bi, bt, ri,
                        rt);
        }
      }
      for (int i = 0; i < N; i++) {
        const long double ox = (long double)o.x - s.C[i].x, oy = (long double)o.y - s.C[i].y,
                          oz = (long double)o.z - s.C[i].z;
        const long double dd = (long double)d.x * d.x + (long double)d.y * d.y + (long double)d.z * d.z;
        const long double tf = -(ox * d.x + oy * d.y + oz * d.z) / dd;
        const long double px = ox + tf * d.x, py = oy + tf * d.y, pz = oz + tf * d.z;
        const long double dist = std::sqrt(px * px + py * py + pz * pz);
        const bool tangent_behind = std::fabs((double)(dist - std::fabs((long double)s.R[i]))) <= tol && tf <= 0;
        double t = 0.0;
        const bool disc0 = ref_test(s.C[i], s.R[i], o, d, t) == 1 && t <= 0.0;
        if (!tangent_behind && !disc0) continue;
        S.pairs++;
        if (!seen[i]) {
          if (++S.missed <= 10)
            std::printf("MISS ugrid seed %d line %d sphere %d disc0 %d\n", seed, li, i, (int)disc0);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------ BVH
void bvh(int seeds, Stat &S) {
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(64000 + seed);
    const double scale = std::pow(10.0, (double)(seed % 3) * 2.0 - 2.0);
    const double shift = (double[]){0.0, 1e3, 1e5, 1e7}[seed % 4] * (seed % 8 < 4 ? 1.0 : scale);
    const int n = (seed % 5 == 4) ? 1100 : 30 + (int)(rng() % 300);
    Scene s = make_scene(rng, n, scale, shift);
    const V P = make_camera(rng, s);
    // rt_upload_scene: bounds of the spheres, centre c0, BVH relative to it
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, rmax = 0.0;
    for (int i = 0; i < n; i++) {
      const double a = std::fabs(s.R[i]);
      for (int k = 0; k < 3; k++) {
        lo[k] = std::min(lo[k], comp(s.C[i], k) - a);
        hi[k] = std::max(hi[k], comp(s.C[i], k) + a);
      }
      if (a > rmax) rmax = a;
    }
    double c0[3];
    for (int k = 0; k < 3; k++) c0[k] = 0.5 * (lo[k] + hi[k]);
    std::vector<double> bx(n), by(n), bz(n), br(n);
    for (int i = 0; i < n; i++)
      bx[i] = s.C[i].x - c0[0], by[i] = s.C[i].y - c0[1], bz[i] = s.C[i].z - c0[2], br[i] = s.R[i];
    std::vector<rtk::BvhNode> nodes;
    std::vector<int32_t> prims;
    rtk::build_bvh(bx.data(), by.data(), bz.data(), br.data(), n, n > 1024 ? 1 : 2, nodes, prims);
    std::vector<float4> pf(prims.size());
    for (size_t k = 0; k < prims.size(); k++) {
      const int id = prims[k];
      float rr = (float)std::fabs(br[id]);
      if ((double)rr < std::fabs(br[id])) rr = std::nextafter(rr, INFINITY);
      pf[k] = make_float4((float)bx[id], (float)by[id], (float)bz[id], rr);
    }
    std::vector<rtk::BvhNode4> n4;
    int stack4 = 0;
    const int32_t root4 = rtk::build_bvh4(nodes, n4, stack4);
    // bvh_args: the extent with the camera, margin = 1e-6 (diameter + largest radius)
    double d2 = 0.0;
    for (int k = 0; k < 3; k++) {
      const double l = std::min(lo[k], comp(P, k)), h = std::max(hi[k], comp(P, k));
      d2 += (h - l) * (h - l);
    }
    BvhArgs bv{};
    bv.c0x = c0[0], bv.c0y = c0[1], bv.c0z = c0[2];
    bv.diam = std::sqrt(d2) + 0.01;
    bv.margin = (float)(1e-6 * (bv.diam + rmax) * (1.0 + 1e-6));
    bv.pmargin = 4.0f * bv.margin;
    bv.tf_min = -INFINITY;
    // the walk's visit set for prune bound tmf: every sphere reached through
    // boxes that pass box4_hit (exit >= tf_min below the root) and pf_keep
    std::vector<char> reach(n);
    auto walk = [&](V o, V d, float tmf, auto &&leaf) {
      const rtk::Walk4Ray r = rtk::walk4_ray(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z});
      float tn, tf;
      if (!rtk::box4_hit(r, nodes[0].lo[0], nodes[0].lo[1], nodes[0].lo[2], nodes[0].hi[0], nodes[0].hi[1],
                         nodes[0].hi[2], tmf, tn, tf))
        return;
      std::vector<int32_t> todo{root4};
      while (!todo.empty()) {
        const int32_t ref = todo.back();
        todo.pop_back();
        if (ref >= 0) {
          const rtk::BvhNode4 &nd = n4[ref];
          for (int k = 0; k < 4; k++)
            if (rtk::box4_hit(r, nd.lox[k], nd.loy[k], nd.loz[k], nd.hix[k], nd.hiy[k], nd.hiz[k], tmf, tn, tf) &&
                tf >= r.tfm)
              todo.push_back(nd.c[k]);
        } else {
          const int lf = -(ref + 1), first = lf >> 4, cnt = lf & 15;
          for (int k = 0; k < cnt; k++)
            if (rtk::pf_keep(r, pf[first + k].x, pf[first + k].y, pf[first + k].z, pf[first + k].w, bv.pmargin))
              leaf(prims[first + k]);
        }
      }
    };
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (int q = 0; q < 2000; q++) {
      V o = P, d;
      if (q % 4 == 3) {  // a reflection off a contact: origin hit + n EPSILON (main.cpp:46)
        const int i = (int)(rng() % n);
        const int j = s.contact[i] >= 0 ? s.contact[i] : i;
        const V cp = add(s.C[j], scl(nrm(sub(s.C[i], s.C[j])), std::fabs(s.R[j])));
        const V d0 = nrm(nrm(sub(add(cp, scl(rand_unit(rng), 2.0 * kEps)), P)));
        double ht;
        const int hs = s.closest(P, d0, ht);
        if (hs < 0) continue;
        const V hp = add(P, scl(d0, ht)), nm = nrm(sub(hp, s.C[hs]));
        o = add(hp, scl(nm, kEps));
        d = nrm(sub(d0, scl(scl(nm, 2.0), dot(d0, nm))));
        S.extra++;
      } else {  // at a silhouette (+-1e-12 relative), ahead of or behind the origin
        const int i = (int)(rng() % n);
        V w = sub(s.C[i], o);
        V perp = nrm(cross(w, rand_unit(rng)));
        const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
        V dir = sub(add(s.C[i], scl(perp, std::fabs(s.R[i]) * f)), o);
        if (q % 4 == 2) dir = scl(dir, -1.0);
        d = nrm(nrm(dir));
        S.targeted++;
      }
      S.rays++;
      std::fill(reach.begin(), reach.end(), 0);
      walk(o, d, INFINITY, [&](int i) { reach[i] = 1; });
      double bt_ref;
      const int bi_ref = s.closest(o, d, bt_ref);
      for (int i = 0; i < n; i++) {
        double t;
        if (!ref_test(s.C[i], s.R[i], o, d, t)) continue;
        S.pairs++;
        if (!reach[i] && !(t != t)) {
          if (++S.missed <= 10) std::printf("MISS bvh seed %d ray %d sphere %d t %.17g\n", seed, q, i, t);
        }
      }
      // pruned at float_up(best t): the walk's bound never drops below it
      double bt = 1e20;
      int bi = -1;
      walk(o, d, rtk::float_up(bt_ref), [&](int i) {
        double t;
        if (ref_test(s.C[i], s.R[i], o, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
      });
      if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
        if (++S.wrong <= 10)
          std::printf("WRONG bvh seed %d ray %d got %d %.17g want %d %.17g\n", seed, q, bi, bt, bi_ref, bt_ref);
      }
    }
  }
}
}  // namespace

int main(int argc, char **argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 24;
  Stat cg, sg, ugs, bv;
  camgrid(seeds, cg);
  std::printf("camgrid %ld %ld edge %ld missed %ld wrong %ld\n", cg.rays, cg.pairs, cg.targeted, cg.missed, cg.wrong);
  spheregrid(seeds, sg);
  std::printf("spheregrid %ld %ld contact %ld fallback %ld missed %ld wrong %ld\n", sg.rays, sg.pairs, sg.targeted,
              sg.extra, sg.missed, sg.wrong);
  ugrid(std::max(3, seeds / 4), ugs);
  std::printf("ugrid %ld %ld plane %ld origin_plane %ld missed %ld wrong %ld\n", ugs.rays, ugs.pairs, ugs.targeted,
              ugs.extra, ugs.missed, ugs.wrong);
  bvh(seeds, bv);
  std::printf("bvh %ld %ld silhouette %ld reflection %ld missed %ld wrong %ld\n", bv.rays, bv.pairs, bv.targeted,
              bv.extra, bv.missed, bv.wrong);
  return (cg.missed || cg.wrong || sg.missed || sg.wrong || ugs.missed || ugs.wrong || bv.missed || bv.wrong) ? 1 : 0;
}
