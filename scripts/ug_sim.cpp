// Walk coherence of cfg 5's reflection rays (planning tool for the round-3
// review's item 3, not a test): the uniform-grid closest-hit walk the
// kernels run (rt_device.h grid_closest_line, host-callable) for the level-1
// reflection rays of a scene's camera view, and the SIMD efficiency of 64-ray
// waves -- sum of per-ray cost / (64 x the costliest ray of each wave),
// summed over waves -- for different ways of packing the rays into waves:
//   tile    the kernel's order: the reflection rays of 8x8-pixel tiles, in
//           tile order, packed 64 at a time (merge_tiles' LDS queue);
//   oct+cell  sorted by (direction octant, origin's grid cell);
//   cell+oct  sorted by (origin's grid cell, octant);
//   cost    sorted by the cost itself (an oracle bound: the best any
//           ordering can do).
// Cost = grid cells visited (the walk loop's iterations) or exact tests.
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I cs420-ray-tracer_amd/csrc -I include scripts/ug_sim.cpp \
//       cs420-ray-tracer_amd/csrc/rt_bvh.cpp -o /tmp/ug_sim && /tmp/ug_sim cs420-ray-tracer_amd/scenes/synth10k.txt 960 540
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <numeric>
#include <sstream>
#include <string>
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
bool ref_test(V c, double r, V o, V d, double &t) {  // sphere.h:26-59
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
struct Ray {
  V o, d;
  int tile, pix;
  long cells, tests, behind;
  unsigned key_oc, key_co;
};
double efficiency(const std::vector<Ray> &rays, const std::vector<int> &order, bool by_cells) {
  double sum = 0, lanes = 0;
  for (size_t w = 0; w < order.size(); w += 64) {
    long mx = 0;
    const size_t e = std::min(order.size(), w + 64);
    for (size_t k = w; k < e; k++) {
      const Ray &r = rays[order[k]];
      const long c = by_cells ? r.cells : r.tests;
      sum += c;
      mx = std::max(mx, c);
    }
    lanes += 64.0 * mx;
  }
  return sum / lanes;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: ug_sim scene.txt W H\n");
    return 2;
  }
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
  std::vector<V> C;
  std::vector<double> R, refl;
  V cam{0, 0, 0}, look{0, 0, -1};
  double fov = 60;
  {
    std::ifstream in(argv[1]);
    std::string line;
    while (std::getline(in, line)) {
      std::istringstream is(line);
      std::string k;
      is >> k;
      if (k == "sphere") {
        double x, y, z, r, cr, cg, cb, m, rough, sh;
        if (is >> x >> y >> z >> r >> cr >> cg >> cb >> m >> rough >> sh) {
          C.push_back({x, y, z});
          R.push_back(r);
          refl.push_back(m);
        }
      } else if (k == "camera") {
        is >> cam.x >> cam.y >> cam.z >> look.x >> look.y >> look.z >> fov;
      }
    }
  }
  const int N = (int)C.size();
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
  for (int i = 0; i < N; i++) bx[i] = C[i].x - c0[0], by[i] = C[i].y - c0[1], bz[i] = C[i].z - c0[2];
  rtk::UgridHost ug;
  if (!rtk::build_ugrid(bx.data(), by.data(), bz.data(), R.data(), N, (size_t)64 << 20, ug, 2.0)) {
    std::printf("no grid\n");
    return 1;
  }
  BvhArgs bv{};
  bv.c0x = c0[0], bv.c0y = c0[1], bv.c0z = c0[2];
  const float margin = (float)(1e-6 * (diam + rmax) * (1.0 + 1e-6));
  bv.pmargin = 4.0f * margin;
  bv.ug = rtk::UgArgs{reinterpret_cast<const float4 *>(ug.rec.data()), ug.rid.data(),
                      reinterpret_cast<const float4 *>(ug.q.data()), ug.ids.data(), ug.glob.data(),
                      (int)ug.glob.size(), ug.nx, ug.ny, ug.nz, ug.gx, ug.gy, ug.gz, ug.cs, 1, 1,
                      (float)(1e-4 * (double)ug.extent)};
  bv.tf_min = 0.0f;
  // camera (camera.h: forward, right = forward x up, up; scale = tan(fov / 2))
  const V fw = nrm(sub(look, cam));
  const V rt = nrm(cross(fw, {0, 1, 0}));
  const V up = cross(rt, fw);
  const double sc = std::tan(fov * M_PI / 360.0), aspect = (double)W / H;
  auto closest = [&](V o, V d, long &cells, long &tests) {
    double bt = 1e20;
    int bi = -1;
    rtk::Work w;
    rtk::grid_closest_line(bv, D3{o.x, o.y, o.z}, D3{d.x, d.y, d.z}, w,
                           [&](int i) {
                             double t;
                             if (ref_test(C[i], R[i], o, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
                           },
                           [&] { return bt; });
    cells = (long)w.cull;
    tests = (long)w.exact;
    return std::make_pair(bi, bt);
  };
  std::vector<Ray> rays;
  const int ntx = (W + 7) / 8;
  long cam_cells = 0;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const double u = (double)x / (W - 1), v = (double)(H - 1 - y) / (H - 1);
      const V d = nrm(add(fw, add(scl(rt, (u - 0.5) * sc * aspect), scl(up, (v - 0.5) * sc))));
      long c, t;
      const auto h = closest(cam, d, c, t);
      cam_cells += c;
      if (h.first < 0 || !(refl[h.first] > 0)) continue;
      const V p = add(cam, scl(d, h.second));
      const V n = nrm(sub(p, C[h.first]));
      const V rd = sub(d, scl(n, 2.0 * dot(d, n)));
      Ray r;
      r.o = add(p, scl(n, 1e-3));
      r.d = rd;
      r.tile = (y / 8) * ntx + x / 8;
      r.pix = y * W + x;
      rays.push_back(r);
    }
  for (Ray &r : rays) {
    closest(r.o, r.d, r.cells, r.tests);
    const unsigned oct = (r.d.x < 0) | (r.d.y < 0) << 1 | (r.d.z < 0) << 2;
    const int cx = std::clamp((int)std::floor(((float)(r.o.x - c0[0]) - ug.gx) / ug.cs), 0, ug.nx - 1);
    const int cy = std::clamp((int)std::floor(((float)(r.o.y - c0[1]) - ug.gy) / ug.cs), 0, ug.ny - 1);
    const int cz = std::clamp((int)std::floor(((float)(r.o.z - c0[2]) - ug.gz) / ug.cs), 0, ug.nz - 1);
    const unsigned cell = (unsigned)((cz * ug.ny + cy) * ug.nx + cx);
    r.key_oc = oct << 24 | cell;
    r.key_co = cell << 3 | oct;
    {  // the cells of the line behind its origin (where the whole-line walk starts): the behind walk's count
      rtk::Work w;
      rtk::behind_cells(bv, D3{r.o.x, r.o.y, r.o.z}, D3{r.d.x, r.d.y, r.d.z}, w, [](int) {});
      r.behind = (long)w.cull;
    }
  }
  std::vector<int> tile(rays.size());
  std::iota(tile.begin(), tile.end(), 0);
  std::stable_sort(tile.begin(), tile.end(), [&](int a, int b) { return rays[a].tile < rays[b].tile; });
  auto sorted = [&](auto key) {
    std::vector<int> o(rays.size());
    std::iota(o.begin(), o.end(), 0);
    std::stable_sort(o.begin(), o.end(), [&](int a, int b) { return key(rays[a]) < key(rays[b]); });
    return o;
  };
  const auto oc = sorted([](const Ray &r) { return r.key_oc; });
  const auto co = sorted([](const Ray &r) { return r.key_co; });
  const auto bycells = sorted([](const Ray &r) { return r.cells; });
  const auto bytests = sorted([](const Ray &r) { return r.tests; });
  const auto bybehind = sorted([](const Ray &r) { return r.behind; });
  // the kernel's packing, then each 8-wave window (512 rays, ~ the rays of a few tiles) sorted by the
  // behind count: a local sort a workgroup could do in LDS
  std::vector<int> local = tile;
  for (size_t w = 0; w < local.size(); w += 512)
    std::stable_sort(local.begin() + w, local.begin() + std::min(local.size(), w + 512),
                     [&](int a, int b) { return rays[a].behind < rays[b].behind; });
  double mb = 0;
  for (const Ray &r : rays) mb += r.behind;
  double mc = 0, mt = 0;
  for (const Ray &r : rays) mc += r.cells, mt += r.tests;
  std::printf("scene %s %dx%d: %d spheres, grid %dx%dx%d, camera rays %d (cells/ray %.1f), level-1 rays %zu: "
              "cells/ray %.1f, exact tests/ray %.1f\n",
              argv[1], W, H, N, ug.nx, ug.ny, ug.nz, W * H, (double)cam_cells / (W * H), rays.size(),
              mc / rays.size(), mt / rays.size());
  std::printf("SIMD efficiency (cells | tests): tile %.3f | %.3f  oct+cell %.3f | %.3f  cell+oct %.3f | %.3f  "
              "cost-sorted bound %.3f | %.3f\n",
              efficiency(rays, tile, true), efficiency(rays, tile, false), efficiency(rays, oc, true),
              efficiency(rays, oc, false), efficiency(rays, co, true), efficiency(rays, co, false),
              efficiency(rays, bycells, true), efficiency(rays, bytests, false));
  std::printf("behind-origin cells/ray %.1f (%.0f %% of the walk); sorted by that count: %.3f | %.3f; "
              "512-ray windows of the tile order sorted by it: %.3f | %.3f\n",
              mb / rays.size(), 100.0 * mb / mc, efficiency(rays, bybehind, true), efficiency(rays, bybehind, false),
              efficiency(rays, local, true), efficiency(rays, local, false));
  return 0;
}
