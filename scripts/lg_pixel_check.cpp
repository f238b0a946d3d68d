// Debugging tool (not a test): the shadow queries of one pixel on the CPU.
// Reads "W H D" and a scene text, puts the camera at (px, py, pz) with the
// scene camera's basis, traces pixel (x, row) to its closest hit
// (scene.h:41-61), and for every light prints the reference's in_shadow
// (scene.h:65-86, the occluding spheres), the light grid's cell for the
// query (rt_lightgrid.h build_light_grid, lg_cell at 0 and +-2^-22), whether
// each occluder is on that cell's list or the light's global list, and the
// line's computed distance from the light against max_off and the off_free
// bound.
//   g++ -O2 -std=c++17 -ffp-contract=off -I cs420-ray-tracer_amd/csrc scripts/lg_pixel_check.cpp \
//       cs420-ray-tracer_amd/csrc/rt_lightgrid.cpp -lpthread -o /tmp/lgp
//   /tmp/lgp scene.txt px py pz x row N
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
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
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double len(V a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
V nrm(V a) {
  const double l = len(a);
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
  if ((t1 < t2 ? t2 : t1) < 0) return false;
  t = (t2 < t1) ? t2 : t1;
  if (t < 0) t = (t1 < t2) ? t2 : t1;
  return true;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 8) return 2;
  std::ifstream f(argv[1]);
  int W, H, D;
  f >> W >> H >> D;
  std::string line;
  std::vector<double> cx, cy, cz, r;
  std::vector<V> lights;
  V pos{0, 0, 0}, look{0, 0, -1};
  double fov = 60;
  while (std::getline(f, line)) {
    std::istringstream s(line);
    std::string k;
    s >> k;
    double v[10];
    if (k == "sphere") {
      for (double &x : v) s >> x;
      cx.push_back(v[0]), cy.push_back(v[1]), cz.push_back(v[2]), r.push_back(v[3]);
    } else if (k == "light") {
      for (int i = 0; i < 7; i++) s >> v[i];
      lights.push_back({v[0], v[1], v[2]});
    } else if (k == "camera") {
      for (int i = 0; i < 7; i++) s >> v[i];
      pos = {v[0], v[1], v[2]}, look = {v[3], v[4], v[5]}, fov = v[6];
    }
  }
  const int n = (int)cx.size(), nl = (int)lights.size(), x = std::atoi(argv[5]), y = std::atoi(argv[6]),
            N = std::atoi(argv[7]);
  const V fwd = nrm(sub(look, pos)), right = nrm(cross(fwd, {0, 1, 0})), up = nrm(cross(right, fwd));
  const double scale = std::tan(fov * 0.5 * M_PI / 180.0);
  const V P{std::strtod(argv[2], nullptr), std::strtod(argv[3], nullptr), std::strtod(argv[4], nullptr)};
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  auto grow = [&](V p, double rr) {
    const double q[3] = {p.x, p.y, p.z};
    for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], q[k] - rr), hi[k] = std::max(hi[k], q[k] + rr);
  };
  for (int i = 0; i < n; i++) grow({cx[i], cy[i], cz[i]}, std::fabs(r[i]));
  for (V L : lights) grow(L, 0.0);
  double d2 = 0, B = 0;
  for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]), B = std::max(B, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
  const double diam = std::sqrt(d2), max_off = 1e-7 * diam;
  std::printf("scene diam %.9g B %.9g max_off %.3g off_free bound %.3g\n", diam, B, max_off,
              0x1p-41 * (1.01 * B + 0.01));
  std::vector<double> lx, ly, lz;
  for (V L : lights) lx.push_back(L.x), ly.push_back(L.y), lz.push_back(L.z);
  std::vector<int32_t> start, ids;
  rtk::build_light_grid(cx.data(), cy.data(), cz.data(), r.data(), n, lx.data(), ly.data(), lz.data(), nl, diam, N,
                        start, ids);
  const long long cells = 6LL * N * N;
  const int j = H - 1 - y;
  const double u = (double)x / (W - 1), v = (double)j / (H - 1);
  const double su = ((u - 0.5) * scale) * 1.0, sv = (v - 0.5) * scale;
  const V d = nrm(nrm(add(add(fwd, scl(right, su)), scl(up, sv))));
  int bi = -1;
  double bt = 1e20;
  for (int i = 0; i < n; i++) {
    double t;
    if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && t < bt) bt = t, bi = i;
  }
  if (bi < 0) {
    std::printf("miss\n");
    return 0;
  }
  const V hp = add(P, scl(d, bt));
  std::printf("hit sphere %d t %.17g hp (%.17g %.17g %.17g)\n", bi, bt, hp.x, hp.y, hp.z);
  for (int l = 0; l < nl; l++) {
    const V L = lights[l];
    const V to = sub(L, hp);
    const double dist = len(to);
    const V ldir = nrm(to);
    const V o = add(hp, scl(ldir, 0.001)), dd = nrm(ldir);  // scene.h:72-76, ray.h:12
    std::vector<int> occ;
    for (int i = 0; i < n; i++) {
      double t;
      if (hit({cx[i], cy[i], cz[i]}, r[i], o, dd, t) && t < dist) occ.push_back(i);
    }
    const V w = sub(L, o);
    const double off = std::fabs(w.y * dd.z - w.z * dd.y) + std::fabs(w.z * dd.x - w.x * dd.z) +
                       std::fabs(w.x * dd.y - w.y * dd.x);
    std::printf("light %d dist %.9g occluders %zu off %.3g", l, dist, occ.size(), off);
    const V q = sub(hp, L);
    for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
      const int c = rtk::lg_cell((float)q.x, (float)q.y, (float)q.z, N, rel);
      std::printf(" | cell %d", c);
      if (c < 0) continue;
      const int32_t *st = start.data() + (size_t)l * (cells + 2);
      for (int i : occ) {
        bool on = false;
        for (int k = st[c]; k < st[c + 1]; k++) on = on || ids[k] == i;
        for (int k = st[cells]; k < st[cells + 1]; k++) on = on || ids[k] == i;
        std::printf(" occ %d listed %d", i, (int)on);
      }
    }
    std::printf("\n");
  }
  return 0;
}
