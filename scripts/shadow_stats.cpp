// Shadow-query statistics of a frame on the CPU (a design tool, not a test):
// the camera rays' hits (level 0 only), and for each hit and light the list
// the device's shadow_cells would test (its direction-grid cell + the light's
// global list, rt_lightgrid.cpp, N as rt_upload_scene picks it), tested in
// list order with early exit, with the reference's fp64 test (sphere.h:26-59,
// scene.h:65-86).  Per 8x8 tile (one level-0 wave) and light it reports the
// loop trips of the current per-lane loop (max over lanes of the tests each
// lane executes), the union of the lanes' lists (a wave-uniform loop over it,
// stopping when every lane is occluded), and how the tested entries split:
// the lane's own sphere, the occluder, a sphere whose whole extent lies
// behind the ray origin, a line that misses the sphere, other.
//   g++ -O2 -std=c++17 -I cs420-ray-tracer_amd/csrc -I include scripts/shadow_stats.cpp \
//       cs420-ray-tracer_amd/csrc/rt_lightgrid.cpp -L cs420-ray-tracer_amd -lrt_hip -o /tmp/ss
//   /tmp/ss scene.txt W H
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#include "rt_hip.h"
#include "rt_lightgrid.h"

namespace {
struct V {
  double x, y, z;
};
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V operator*(V a, double t) { return {a.x * t, a.y * t, a.z * t}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V unit(V a) {
  double l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
struct S {
  V c;
  double r;
};
bool hit(const S &s, V o, V d, double &t) {
  V oc = o - s.c;
  double a = dot(d, d), b = 2.0 * dot(oc, d), c = dot(oc, oc) - s.r * s.r;
  double disc = b * b - 4 * a * c;
  if (disc < 0) return false;
  if (disc == 0) {
    t = -b / (2 * a);
    return true;
  }
  double t1 = (-b - std::sqrt(disc)) / (2 * a), t2 = (-b + std::sqrt(disc)) / (2 * a);
  if (std::max(t1, t2) < 0) return false;
  t = std::min(t1, t2);
  if (t < 0) t = std::max(t1, t2);
  return true;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  rt_scene sc;
  if (rt_scene_load(argv[1], &sc, 0) != RT_OK) return 3;
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
  rt_camera cam;
  rt_camera_from_scene(&sc, &cam);
  const int n = sc.num_spheres, nl = sc.num_lights;
  std::vector<S> sp(n);
  std::vector<double> cx(n), cy(n), cz(n), br(n), lx(nl), ly(nl), lz(nl);
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int i = 0; i < n; i++) {
    const rt_sphere &q = sc.spheres[i];
    sp[i] = {{q.center[0], q.center[1], q.center[2]}, q.radius};
    cx[i] = q.center[0], cy[i] = q.center[1], cz[i] = q.center[2], br[i] = std::fabs(q.radius);
    for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], q.center[k] - br[i]), hi[k] = std::max(hi[k], q.center[k] + br[i]);
  }
  std::vector<V> L(nl);
  for (int l = 0; l < nl; l++) {
    const rt_light &q = sc.lights[l];
    L[l] = {q.position[0], q.position[1], q.position[2]};
    lx[l] = L[l].x, ly[l] = L[l].y, lz[l] = L[l].z;
    for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], q.position[k]), hi[k] = std::max(hi[k], q.position[k]);
  }
  double d2 = 0;
  for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
  const double diam = std::sqrt(d2);
  const int N = n > 1024 ? 384 : 128;
  std::vector<int32_t> start, ids;
  rtk::build_light_grid(cx.data(), cy.data(), cz.data(), br.data(), n, lx.data(), ly.data(), lz.data(), nl, diam, N,
                        start, ids);
  const size_t stride = 6 * (size_t)N * N + 2;
  const V P{cam.position[0], cam.position[1], cam.position[2]}, F{cam.forward[0], cam.forward[1], cam.forward[2]},
      R{cam.right[0], cam.right[1], cam.right[2]}, U{cam.up[0], cam.up[1], cam.up[2]};
  long long trips_lane2 = 0, lane_tests2 = 0, n_self_occ = 0, n_self_miss = 0;
  long long queries = 0, lane_tests = 0, trips_lane = 0, trips_union = 0, wave_lights = 0;
  long long c_self = 0, c_occ = 0, c_behind = 0, c_miss = 0, c_other = 0, len_sum = 0, occl = 0;
  long long hist[10] = {0};
  for (int ty = 0; ty < H; ty += 8)
    for (int tx = 0; tx < W; tx += 8) {
      struct Lane {
        V hp;
        int idx;
      };
      std::vector<Lane> lanes;
      for (int yy = ty; yy < std::min(ty + 8, H); yy++)
        for (int xx = tx; xx < std::min(tx + 8, W); xx++) {
          const int j = H - 1 - yy;
          const double u = double(xx) / (W - 1), v = double(j) / (H - 1);
          V d = unit(unit(F + R * ((u - 0.5) * cam.scale * 1.0) + U * ((v - 0.5) * cam.scale)));
          double bt = 1e20;
          int bi = -1;
          for (int i = 0; i < n; i++) {
            double t;
            if (hit(sp[i], P, d, t) && t < bt) bt = t, bi = i;
          }
          if (bi >= 0) lanes.push_back({P + d * bt, bi});
        }
      if (lanes.empty()) continue;
      for (int l = 0; l < nl; l++) {
        ++wave_lights;
        int maxt = 0, maxt2 = 0;
        std::set<int> uni;
        std::vector<char> occ_by_union(lanes.size(), 0);
        std::vector<std::vector<int>> lists(lanes.size());
        for (size_t k = 0; k < lanes.size(); k++) {
          const V hp = lanes[k].hp;
          const V tl = L[l] - hp;
          const double dist = std::sqrt(dot(tl, tl));
          const V ld = unit(tl);
          const V so = hp + ld * 0.001, sd = unit(ld);
          const V dir = hp - L[l];
          const int c = rtk::lg_cell((float)dir.x, (float)dir.y, (float)dir.z, N);
          std::vector<int> &lst = lists[k];
          const int32_t *st = start.data() + (size_t)l * stride;
          if (c >= 0)
            for (int32_t e = st[c]; e < st[c + 1]; e++) lst.push_back(ids[(size_t)e]);
          for (int32_t e = st[stride - 2]; e < st[stride - 1]; e++) lst.push_back(ids[(size_t)e]);
          len_sum += (long long)lst.size();
          ++queries;
          // the self pre-test (shadow_cells): own sphere decided without sqrt
          int tests = 0, tests2 = 0;
          bool occ = false, self_occ = false, self_miss = false;
          {
            const S &q = sp[lanes[k].idx];
            const V oc = so - q.c;
            const double rr = q.r * q.r, c = dot(oc, oc) - rr, b = 2.0 * dot(oc, sd);
            if (c < 0) self_occ = dist * dist > 6.0 * rr;
            else if (c > 0 && b > 0) {
              const double p = b * b, disc = p - 4 * dot(sd, sd) * c;
              self_miss = disc < 0 || (disc > 0 && disc < p * (1 - 0x1p-50));
            }
          }
          if (!self_occ)
            for (int i : lst) {
              if (self_miss && i == lanes[k].idx) continue;
              ++tests2;
              double t;
              if (hit(sp[i], so, sd, t) && t < 1e20 && t < dist) break;
            }
          maxt2 = std::max(maxt2, tests2);
          lane_tests2 += tests2;
          n_self_occ += self_occ;
          n_self_miss += self_miss;
          for (int i : lst) {
            ++tests;
            double t;
            const bool h = hit(sp[i], so, sd, t) && t < 1e20 && t < dist;
            const V co = sp[i].c - so;
            const double tc = dot(co, sd), ld2 = dot(co, co) - tc * tc, r = std::fabs(sp[i].r);
            if (i == lanes[k].idx) ++c_self;
            else if (h) ++c_occ;
            else if (ld2 > r * r) ++c_miss;
            else if (tc < -r) ++c_behind;
            else ++c_other;
            if (h) {
              occ = true;
              break;
            }
          }
          occl += occ;
          lane_tests += tests;
          maxt = std::max(maxt, tests);
          hist[std::min(tests, 9)]++;
          for (int i : lst) uni.insert(i);
        }
        trips_lane += maxt;
        trips_lane2 += maxt2;
        // union in ascending order until every lane is occluded
        int ut = 0;
        std::vector<char> done(lanes.size(), 0);
        size_t ndone = 0;
        for (int i : uni) {
          if (ndone == lanes.size()) break;
          ++ut;
          for (size_t k = 0; k < lanes.size(); k++) {
            if (done[k]) continue;
            const V hp = lanes[k].hp, tl = L[l] - hp;
            const double dist = std::sqrt(dot(tl, tl));
            const V ld = unit(tl), so = hp + ld * 0.001, sd = unit(ld);
            double t;
            if (hit(sp[i], so, sd, t) && t < 1e20 && t < dist) done[k] = 1, ++ndone;
          }
        }
        trips_union += ut;
      }
    }
  std::printf("queries %lld (waves x lights %lld), mean list %.2f, lane tests %lld (%.2f per query), occluded %.1f%%\n",
              queries, wave_lights, (double)len_sum / queries, lane_tests, (double)lane_tests / queries,
              100.0 * occl / queries);
  std::printf("wave loop trips: per-lane loop %lld (%.2f per wave-light), union loop %lld (%.2f)\n", trips_lane,
              (double)trips_lane / wave_lights, trips_union, (double)trips_union / wave_lights);
  std::printf("with the self pre-test: self occluded %lld, self miss proven %lld; list tests %lld, wave trips %lld (%.2f)\n",
              n_self_occ, n_self_miss, lane_tests2, trips_lane2, (double)trips_lane2 / wave_lights);
  std::printf("tested entries: self %lld, occluder %lld, line misses %lld, behind origin %lld, other %lld\n", c_self,
              c_occ, c_miss, c_behind, c_other);
  std::printf("tests per query histogram:");
  for (int i = 0; i < 10; i++) std::printf(" %d:%lld", i, hist[i]);
  std::printf("\n");
  return 0;
}
