// Debugging tool (not a test): one scene's camera grid on the CPU.  Reads
// "W H D" and a scene text (scripts/fuzz_repro.py's gpurun_out/
// fuzz_repro_scene.txt), puts the scene camera at the point (px, py, pz)
// -- the basis stays, as bench.py's and the fuzz's moving cameras do -- builds
// the host camera grid (rt_lightgrid.h build_point_grid) at that point with
// the launch's N, and for every pixel compares the reference's closest hit
// (scene.h:41-61) with the grid's early-exit scan at the device's cell and at
// +-2^-22 quotient errors.  Prints the pixels that differ.
//   g++ -O2 -std=c++17 -ffp-contract=off -I cs420-ray-tracer_amd/csrc scripts/cg_scene_check.cpp \
//       cs420-ray-tracer_amd/csrc/rt_lightgrid.cpp -lpthread -o /tmp/cgs
//   /tmp/cgs scene.txt px py pz N
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
V nrm(V a) {
  const double l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
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
  if (argc < 6) return 2;
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
  const int n = (int)cx.size(), N = std::atoi(argv[5]);
  const V fwd = nrm(sub(look, pos)), right = nrm(cross(fwd, {0, 1, 0})), up = nrm(cross(right, fwd));
  const double scale = std::tan(fov * 0.5 * M_PI / 180.0);
  const V P{std::strtod(argv[2], nullptr), std::strtod(argv[3], nullptr), std::strtod(argv[4], nullptr)};  // the moved position
  // the device's extent: the scene box (spheres and lights) with the point
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  auto grow = [&](V p, double rr) {
    const double q[3] = {p.x, p.y, p.z};
    for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], q[k] - rr), hi[k] = std::max(hi[k], q[k] + rr);
  };
  for (int i = 0; i < n; i++) grow({cx[i], cy[i], cz[i]}, std::fabs(r[i]));
  for (V L : lights) grow(L, 0.0);
  grow(P, 0.0);
  double d2 = 0;
  for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
  std::vector<int32_t> start, ent;
  if (!rtk::build_point_grid(cx.data(), cy.data(), cz.data(), r.data(), n, P.x, P.y, P.z, std::sqrt(d2), N, 32,
                             size_t(256) << 20, start, ent)) {
    std::printf("grid refused\n");
    return 0;
  }
  long bad = 0;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const int j = H - 1 - y;
      const double u = (double)x / (W - 1), v = (double)j / (H - 1);
      const double su = ((u - 0.5) * scale) * 1.0, sv = (v - 0.5) * scale;
      const V d = nrm(nrm(add(add(fwd, scl(right, su)), scl(up, sv))));
      int bi_ref = -1;
      double bt_ref = 1e20;
      for (int i = 0; i < n; i++) {
        double t;
        if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && t < bt_ref) bt_ref = t, bi_ref = i;
      }
      for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
        const int c = rtk::lg_cell((float)d.x, (float)d.y, (float)d.z, N, rel);
        if (c < 0) continue;
        double bt = 1e20;
        int bi = -1, len = start[c + 1] - start[c];
        for (int k = start[c]; k < start[c + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          if ((double)b > bt) break;
          const int i = ent[2 * k];
          double t;
          if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
        }
        bool listed = bi_ref < 0;
        for (int k = start[c]; k < start[c + 1] && !listed; k++) listed = ent[2 * k] == bi_ref;
        if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
          if (++bad <= 20)
            std::printf("pixel x %d row %d rel %g cell %d len %d: grid %d %.17g ref %d %.17g listed %d\n", x, y,
                        (double)rel, c, len, bi, bt, bi_ref, bt_ref, (int)listed);
        }
      }
    }
  std::printf("spheres %d N %d pixels %d differ %ld\n", n, N, W * H, bad);
  return 0;
}
