// Check of the behind grid (rt_bvh.h build_ugrid + rt_device.h behind_cells,
// the same code the kernels run, here on the CPU): for random scenes (uniform
// clouds with a ground sphere, dense clusters with overlapping and negative
// radii, tiny spheres, far from the origin; scales 0.01 .. 100) and lines
// (random origins just outside sphere surfaces as reflection rays start,
// random directions; and lines built tangent to a sphere at a point BEHIND
// their origin), every sphere whose surface the backward half-line
// {o + t d, t <= 0} passes within 1e-7 of the scene diameter of -- which
// includes every sphere for which the reference's test (sphere.h:26-59)
// takes its disc == 0 branch with t <= 0 -- must be handed to the exact test
// by behind_cells.  Scenes whose listing margin does not cover the prefilter
// margin are counted (the device does not use the grid for them).
// grid_closest_line (the grid walk of the whole line, early exit) must give
// find_intersection's (t, index) exactly, for the same lines.
// argv: seeds, cells per listed sphere.  Prints "overflow cells <count>",
// "closest <lines> hits <count> wrong <count>" and "checked <lines>
// <near-tangent pairs> <exact disc0 pairs> scenes <used>/<built> cells/line
// <mean> missed <count>".
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I csrc -I include ug_check.cpp csrc/rt_bvh.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "rt_device.h"

using rtk::BvhArgs;
using rtk::D3;

namespace {
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
}  // namespace

int main(int argc, char **argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 24;
  const double cps = argc > 2 ? std::atof(argv[2]) : 2.0;  // cells per listed sphere (build_ugrid)
  long overflow = 0;  // cells with more than four entries (their lists continue in the overflow list)
  long lines = 0, near = 0, exact0 = 0, missed = 0, built = 0, used = 0, wrong = 0, hits = 0;
  double cells = 0.0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(9100 + seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const int kind = seed % 4;
    const double scale = std::pow(10.0, (double)(seed / 4 % 5) - 2.0);  // 0.01 .. 100
    const double shift = (seed % 7 == 3) ? 1e4 * scale : 0.0;
    std::vector<V> C;
    std::vector<double> R;
    const int n = kind == 0 ? 3000 : (kind == 1 ? 800 : (kind == 2 ? 1500 : 400));
    for (int i = 0; i < n; i++) {
      V c;
      double r;
      if (kind == 0) {  // a flat cloud like synth10k
        c = {(U(rng) * 80 - 40) * scale, (U(rng) * 13.5 - 1.5) * scale, (U(rng) * 105 - 120) * scale};
        r = (0.15 + 0.45 * U(rng)) * scale;
      } else if (kind == 1) {  // a dense cluster: overlapping spheres, some negative radii
        c = {(U(rng) * 10 - 5) * scale, (U(rng) * 10 - 5) * scale, (U(rng) * 10 - 5) * scale};
        r = (0.2 + 1.3 * U(rng)) * scale * (U(rng) < 0.1 ? -1.0 : 1.0);
      } else if (kind == 2) {  // tiny spheres spread wide
        c = {(U(rng) * 200 - 100) * scale, (U(rng) * 200 - 100) * scale, (U(rng) * 200 - 100) * scale};
        r = (1e-3 + 1e-2 * U(rng)) * scale;
      } else {  // mixed sizes, with a few large ones
        c = {(U(rng) * 40 - 20) * scale, (U(rng) * 40 - 20) * scale, (U(rng) * 40 - 20) * scale};
        r = (U(rng) < 0.03 ? 8.0 : 0.1 + U(rng)) * scale;
      }
      C.push_back(add(c, {shift, -shift, shift}));
      R.push_back(r);
    }
    if (kind == 0 || kind == 3) {  // a ground sphere (global: listed in no cell)
      C.push_back({shift, -102.0 * scale - shift, -20.0 * scale + shift});
      R.push_back(100.0 * scale);
    }
    const int N = (int)C.size();
    const V cam = add({0.0, 3.0 * scale, 12.0 * scale}, {shift, -shift, shift});
    // the upload's centre and the render's margins (rt_kernel.hip rt_upload_scene, bvh_args)
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, rmax = 0.0;
    for (int i = 0; i < N; i++) {
      const double p[3] = {C[i].x, C[i].y, C[i].z}, a = std::fabs(R[i]);
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], p[k] - a);
        hi[k] = std::fmax(hi[k], p[k] + a);
      }
      rmax = std::fmax(rmax, a);
    }
    double c0[3], d2 = 0.0;
    for (int k = 0; k < 3; k++) c0[k] = 0.5 * (lo[k] + hi[k]);
    const double cp[3] = {cam.x, cam.y, cam.z};
    for (int k = 0; k < 3; k++) {
      const double l = std::fmin(lo[k], cp[k]), h = std::fmax(hi[k], cp[k]);
      d2 += (h - l) * (h - l);
    }
    const double diam = std::sqrt(d2) + 0.01;
    std::vector<double> bx(N), by(N), bz(N);
    for (int i = 0; i < N; i++) {
      bx[i] = C[i].x - c0[0];
      by[i] = C[i].y - c0[1];
      bz[i] = C[i].z - c0[2];
    }
    rtk::UgridHost ug;
    if (!rtk::build_ugrid(bx.data(), by.data(), bz.data(), R.data(), N, (size_t)64 << 20, ug, cps)) {
      std::printf("scene %d: no grid\n", seed);  // (the pytest requires every scene at the default density)
      continue;
    }
    built++;
    BvhArgs bv{};
    bv.c0x = c0[0];
    bv.c0y = c0[1];
    bv.c0z = c0[2];
    const float margin = (float)(1e-6 * (diam + rmax) * (1.0 + 1e-6));
    bv.pmargin = 4.0f * margin;
    if (!((double)bv.pmargin + 1e-4 * (double)ug.extent <= (double)ug.reg_margin)) continue;  // the device keeps the full walks
    used++;
    bv.ug = rtk::UgArgs{reinterpret_cast<const float4 *>(ug.rec.data()), ug.rid.data(),
                        reinterpret_cast<const float4 *>(ug.q.data()), ug.ids.data(), ug.glob.data(),
                        (int)ug.glob.size(), ug.nx, ug.ny, ug.nz, ug.gx, ug.gy, ug.gz, ug.cs, 1, 1,
                        (float)(1e-4 * (double)ug.extent)};
    for (size_t c = 0; c + 1 < ug.start.size(); c++) overflow += ug.start[c + 1] - ug.start[c] > 4;
    bv.tf_min = 0.0f;
    std::vector<char> seen(N);
    const double tol = 1e-7 * diam;
    for (int li = 0; li < 4000; li++) {
      V o, d;
      if (li % 2 == 0) {  // a reflection-like origin: just outside a random sphere, a random direction
        const int s = (int)(rng() % N);
        const V nn = nrm({U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5});
        o = add(add(C[s], scl(nn, std::fabs(R[s]))), scl(nn, 0.001 * scale));
        d = nrm({U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5});
      } else {  // a line tangent to sphere s at a point P behind the origin
        const int s = (int)(rng() % N);
        const V nn = nrm({U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5});
        const V P = add(C[s], scl(nn, std::fabs(R[s])));
        V tdir = cross(nn, nrm({U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5}));
        d = nrm(tdir);
        const double back = (0.01 + 60.0 * U(rng) * U(rng)) * scale;
        o = add(P, scl(d, back));
      }
      lines++;
      std::fill(seen.begin(), seen.end(), 0);
      rtk::Work work;
      rtk::behind_cells(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z}, work, [&](int i) { seen[i] = 1; });
      cells += (double)work.cull;
      {  // the grid's closest hit along the whole line == find_intersection (scene.h:41-61)
        double bt = 1e20, rt = 1e20;
        int bi = -1, ri = -1;
        auto fold = [&](int i) {
          double t;
          if (ref_test(C[i], R[i], o, d, t) && (t < bt || (t == bt && i < bi))) {
            bt = t;
            bi = i;
          }
        };
        rtk::Work w2;
        rtk::grid_closest_line(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z}, w2, fold, [&] { return bt; });
        for (int i = 0; i < N; i++) {
          double t;
          if (ref_test(C[i], R[i], o, d, t) && t < rt) {
            rt = t;
            ri = i;
          }
        }
        if (bi != ri || (ri >= 0 && bt != rt)) {
          if (++wrong <= 10)
            std::printf("WRONG scene %d line %d grid (%d, %.17g) reference (%d, %.17g)\n", seed, li, bi, bt, ri, rt);
        }
        hits += ri >= 0;
      }
      for (int i = 0; i < N; i++) {
        // long double geometry: distance of the line to the centre, the foot point's t
        const long double ox = (long double)o.x - C[i].x, oy = (long double)o.y - C[i].y,
                          oz = (long double)o.z - C[i].z;
        const long double dd = (long double)d.x * d.x + (long double)d.y * d.y + (long double)d.z * d.z;
        const long double tf = -(ox * d.x + oy * d.y + oz * d.z) / dd;
        const long double px = ox + tf * d.x, py = oy + tf * d.y, pz = oz + tf * d.z;
        const long double dist = std::sqrt(px * px + py * py + pz * pz);
        const bool tangent_behind = std::fabs((double)(dist - std::fabs((long double)R[i]))) <= tol && tf <= 0;
        double t = 0.0;
        const bool disc0 = ref_test(C[i], R[i], o, d, t) == 1 && t <= 0.0;
        if (!tangent_behind && !disc0) continue;
        near += tangent_behind;
        exact0 += disc0;
        if (!seen[i]) {
          if (++missed <= 10)
            std::printf("MISS scene %d line %d sphere %d r %.17g dist-r %.3Lg t %.6Lg disc0 %d\n", seed, li, i, R[i],
                        dist - std::fabs((long double)R[i]), tf, (int)disc0);
        }
      }
    }
  }
  std::printf("overflow cells %ld\n", overflow);
  std::printf("closest %ld hits %ld wrong %ld\n", lines, hits, wrong);
  std::printf("checked %ld %ld %ld scenes %ld/%ld cells/line %.1f missed %ld\n", lines, near, exact0, used, built,
              cells / (double)(lines ? lines : 1), missed);
  return (missed || wrong) ? 2 : 0;
}
