// bvh_sim.cpp -- CPU model of the render loop's BVH traversal cost (tuning
// tool, not part of the product).  Traces a frame in fp64, groups lanes into
// 8x8-pixel waves as the megakernel does, and for every closest-hit / shadow
// query counts per-lane node visits and sphere tests under several traversal
// strategies; the "wave trips" column is the per-query maximum over the
// wave's lanes (what a divergent SIMD loop pays).
//
//   g++ -O2 -std=c++17 -I include -o /tmp/bvh_sim scripts/bvh_sim.cpp \
//       cs420-ray-tracer_amd/csrc/rt_bvh.cpp cs420-ray-tracer_amd/csrc/rt_host.cpp
//   /tmp/bvh_sim scene.txt W H depth [max_leaf]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cs420-ray-tracer_amd/csrc/rt_bvh.h"
#include "rt_hip.h"

using rtk::BvhNode;
struct V {
  double x, y, z;
};
static V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V operator*(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V nrmz(V a) { return a * (1.0 / std::sqrt(dot(a, a))); }

struct Scene {
  std::vector<V> c;
  std::vector<double> r, refl;
  std::vector<V> lights;
};

static bool hit_sphere(const Scene &s, int i, V o, V d, double &t) {
  V oc = o - s.c[i];
  double a = dot(d, d), b = 2 * dot(oc, d), cc = dot(oc, oc) - s.r[i] * s.r[i];
  double disc = b * b - 4 * a * cc;
  if (disc < 0) return false;
  double sq = std::sqrt(disc), t1 = (-b - sq) / (2 * a), t2 = (-b + sq) / (2 * a);
  if (std::max(t1, t2) < 0) return false;
  t = t1 < 0 ? t2 : t1;
  return true;
}

struct Stats {
  double lane_nodes = 0, lane_tests = 0, wave_nodes = 0, wave_tests = 0, wave_trips = 0;
  long queries = 0, wq = 0;
};

// one strategy; returns per-lane (nodes, tests) for a query
struct Strategy {
  const char *name;
  int kind;      // 0 stackless preorder, 1 ordered stack BVH2, 2 ordered BVH4
  bool forward;  // prune boxes wholly behind the origin
};

struct Bvh4 {
  struct Node {
    float lo[4][3], hi[4][3];
    int child[4];  // >=0 inner node, <0: leaf -(first<<4|count)-1, INT_MIN empty
  };
  std::vector<Node> n;
};

static long g_maxstk[3] = {0, 0, 0};
struct QR {
  V o, d;
  int lev;
};
static std::vector<QR> g_deep;  // rays of level >= 2 in the order the tiles spawn them
static double g_zero[4][4];  // per class: lane queries, zero-term lanes, wave queries, all-zero waves
static const std::vector<BvhNode> *g_nodes;
static const std::vector<int32_t> *g_prims;

static bool box(const float *lo, const float *hi, V o, V inv, double &tn, double &tf) {
  double a[3] = {(lo[0] - o.x) * inv.x, (lo[1] - o.y) * inv.y, (lo[2] - o.z) * inv.z};
  double b[3] = {(hi[0] - o.x) * inv.x, (hi[1] - o.y) * inv.y, (hi[2] - o.z) * inv.z};
  tn = std::max({std::min(a[0], b[0]), std::min(a[1], b[1]), std::min(a[2], b[2])});
  tf = std::min({std::max(a[0], b[0]), std::max(a[1], b[1]), std::max(a[2], b[2])});
  return tn <= tf;
}

// Children of BVH2 node i (preorder + skip): left = i+1, right = nodes[i+1].skip
static void walk2(const Scene &s, const Strategy &st, V o, V d, bool shadow, double T, double &bt, int &bi,
                  long &nodes, long &tests) {
  const auto &N = *g_nodes;
  const auto &P = *g_prims;
  V inv{1 / d.x, 1 / d.y, 1 / d.z};
  auto leaf = [&](const BvhNode &nd) -> bool {
    int first = nd.leaf >> 4, cnt = nd.leaf & 15;
    for (int k = 0; k < cnt; k++) {
      int i = P[first + k];
      tests++;
      double t;
      if (hit_sphere(s, i, o, d, t)) {
        if (shadow) {
          if (t < T) return false;
        } else if (t < bt || (t == bt && i < bi)) {
          bt = t;
          bi = i;
        }
      }
    }
    return true;
  };
  auto lim = [&]() { return shadow ? T : bt; };
  if (st.kind == 0) {
    int i = 0, n = (int)N.size();
    while (i < n) {
      nodes++;
      double tn, tf;
      bool in = box(N[i].lo, N[i].hi, o, inv, tn, tf) && !(tn > lim()) && (!st.forward || tf >= 0);
      if (in && N[i].leaf >= 0) {
        if (!leaf(N[i])) return;
        i = N[i].skip;
      } else
        i = in ? i + 1 : N[i].skip;
    }
    return;
  }
  // ordered: stack of (node, tn)
  std::vector<std::pair<int, double>> stk;
  double tn0, tf0;
  nodes++;
  if (!box(N[0].lo, N[0].hi, o, inv, tn0, tf0)) return;
  stk.push_back({0, tn0});
  while (!stk.empty()) {
    auto [i, tn] = stk.back();
    stk.pop_back();
    if (tn > lim()) continue;
    if (N[i].leaf >= 0) {
      if (!leaf(N[i])) return;
      continue;
    }
    int l = i + 1, r = N[i + 1].skip;
    if (st.kind == 2) {  // 4-wide: the grandchildren of i (a leaf child stands for itself)
      int cand[4], nc = 0;
      for (int c : {l, r}) {
        if (N[c].leaf >= 0) cand[nc++] = c;
        else {
          cand[nc++] = c + 1;
          cand[nc++] = N[c + 1].skip;
        }
      }
      nodes++;
      std::pair<double, int> hits[4];
      int nh = 0;
      for (int k = 0; k < nc; k++) {
        double a, b;
        if (box(N[cand[k]].lo, N[cand[k]].hi, o, inv, a, b) && !(a > lim()) && (!st.forward || b >= 0))
          hits[nh++] = {a, cand[k]};
      }
      std::sort(hits, hits + nh, [](auto &x, auto &y) { return x.first > y.first; });  // far first
      for (int k = 0; k < nh; k++) stk.push_back({hits[k].second, hits[k].first});
      g_maxstk[2] = std::max(g_maxstk[2], (long)stk.size());
      continue;
    }
    double tnl, tfl, tnr, tfr;
    nodes++;  // one visit tests both children (child boxes stored in the parent)
    bool hl = box(N[l].lo, N[l].hi, o, inv, tnl, tfl) && !(tnl > lim()) && (!st.forward || tfl >= 0);
    bool hr = box(N[r].lo, N[r].hi, o, inv, tnr, tfr) && !(tnr > lim()) && (!st.forward || tfr >= 0);
    if (hl && hr) {
      if (tnl <= tnr) {
        stk.push_back({r, tnr});
        stk.push_back({l, tnl});
      } else {
        stk.push_back({l, tnl});
        stk.push_back({r, tnr});
      }
      if (st.kind == 1) g_maxstk[1] = std::max(g_maxstk[1], (long)stk.size());
    } else if (hl)
      stk.push_back({l, tnl});
    else if (hr)
      stk.push_back({r, tnr});
  }
}

int main(int argc, char **argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: bvh_sim scene W H depth [max_leaf]\n");
    return 2;
  }
  rt_scene sc;
  if (rt_scene_load(argv[1], &sc, 0) != 0) return 1;
  rt_camera cam;
  rt_camera_from_scene(&sc, &cam);
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), D = std::atoi(argv[4]);
  const int max_leaf = argc > 5 ? std::atoi(argv[5]) : 4;
  Scene s;
  std::vector<double> cx, cy, cz, rr;
  for (int i = 0; i < sc.num_spheres; i++) {
    const rt_sphere &q = sc.spheres[i];
    s.c.push_back({q.center[0], q.center[1], q.center[2]});
    s.r.push_back(q.radius);
    s.refl.push_back(q.reflectivity);
    cx.push_back(q.center[0]);
    cy.push_back(q.center[1]);
    cz.push_back(q.center[2]);
    rr.push_back(q.radius);
  }
  for (int l = 0; l < sc.num_lights; l++)
    s.lights.push_back({sc.lights[l].position[0], sc.lights[l].position[1], sc.lights[l].position[2]});
  std::vector<BvhNode> nodes;
  std::vector<int32_t> prims;
  rtk::build_bvh(cx.data(), cy.data(), cz.data(), rr.data(), (int)s.r.size(), max_leaf, nodes, prims);
  g_nodes = &nodes;
  g_prims = &prims;
  std::printf("spheres %zu nodes %zu\n", s.r.size(), nodes.size());
  const Strategy strats[] = {{"preorder-line", 0, false}, {"ordered-line", 1, false}, {"ordered4-line", 2, false}};
  const int NS = 3;
  // stats[strategy][class]: class 0 primary closest, 1 primary shadow, 2 secondary closest, 3 secondary shadow
  Stats stats[NS][4];
  V P{cam.position[0], cam.position[1], cam.position[2]};
  V F{cam.forward[0], cam.forward[1], cam.forward[2]}, R{cam.right[0], cam.right[1], cam.right[2]},
      U{cam.up[0], cam.up[1], cam.up[2]};
  for (int ty = 0; ty < H; ty += 8)
    for (int tx = 0; tx < W; tx += 8) {
      // lanes
      V o[64], d[64];
      bool alive[64];
      for (int l = 0; l < 64; l++) {
        int x = tx + (l & 7), y = ty + (l >> 3);
        alive[l] = x < W && y < H;
        if (!alive[l]) continue;
        int j = H - 1 - y;
        double u = (double)x / (W - 1), v = (double)j / (H - 1);
        V dir = F + R * ((u - 0.5) * cam.scale) + U * ((v - 0.5) * cam.scale);
        d[l] = nrmz(dir);
        o[l] = P;
      }
      for (int lev = 0; lev < D; lev++) {
        int cls = lev == 0 ? 0 : 2;
        double bt[64];
        int bi[64];
        // closest per strategy (results must agree; use strategy 0's)
        for (int k = 0; k < NS; k++) {
          long mx_n = 0, mx_t = 0, any = 0;
          for (int l = 0; l < 64; l++) {
            if (!alive[l]) continue;
            any = 1;
            long nn = 0, nt = 0;
            double t = INFINITY;
            int b = -1;
            walk2(s, strats[k], o[l], d[l], false, 0, t, b, nn, nt);
            if (k == 0) {
              bt[l] = t;
              bi[l] = b;
            }
            stats[k][cls].lane_nodes += nn;
            stats[k][cls].lane_tests += nt;
            stats[k][cls].queries++;
            mx_n = std::max(mx_n, nn);
            mx_t = std::max(mx_t, nt);
          }
          if (any) {
            stats[k][cls].wave_nodes += mx_n;
            stats[k][cls].wave_tests += mx_t;
            stats[k][cls].wq++;
          }
        }
        bool hit[64];
        V hp[64], nrm[64];
        for (int l = 0; l < 64; l++) {
          hit[l] = alive[l] && bi[l] >= 0;
          if (!hit[l]) continue;
          hp[l] = o[l] + d[l] * bt[l];
          nrm[l] = nrmz(hp[l] - s.c[bi[l]]);
        }
        for (size_t L = 0; L < s.lights.size(); L++) {
          // shadow queries whose Phong term is exactly zero (n.l <= 0 and r.v <= 0)
          {
            int nh = 0, nz = 0;
            for (int l = 0; l < 64; l++) {
              if (!hit[l]) continue;
              nh++;
              V ld = nrmz(s.lights[L] - hp[l]);
              V view = nrmz(o[l] - hp[l]);
              V nl2 = ld * -1.0;
              V r = nl2 - nrm[l] * (2.0 * dot(nl2, nrm[l]));
              if (dot(nrm[l], ld) <= 0 && dot(r, view) <= 0) nz++;
            }
            if (nh) {
              g_zero[cls][0] += nh;
              g_zero[cls][1] += nz;
              g_zero[cls][2] += 1;
              g_zero[cls][3] += nz == nh;
            }
          }
          for (int k = 0; k < NS; k++) {
            long mx_n = 0, mx_t = 0, any = 0;
            for (int l = 0; l < 64; l++) {
              if (!hit[l]) continue;
              any = 1;
              V tl = s.lights[L] - hp[l];
              double dist = std::sqrt(dot(tl, tl));
              V ld = nrmz(tl);
              long nn = 0, nt = 0;
              double t = 0;
              int b = 0;
              walk2(s, strats[k], hp[l] + ld * 0.001, ld, true, dist, t, b, nn, nt);
              stats[k][cls + 1].lane_nodes += nn;
              stats[k][cls + 1].lane_tests += nt;
              stats[k][cls + 1].queries++;
              mx_n = std::max(mx_n, nn);
              mx_t = std::max(mx_t, nt);
            }
            if (any) {
              stats[k][cls + 1].wave_nodes += mx_n;
              stats[k][cls + 1].wave_tests += mx_t;
              stats[k][cls + 1].wq++;
            }
          }
        }
        for (int l = 0; l < 64; l++) {
          if (!hit[l] || s.refl[bi[l]] <= 0 || lev + 1 >= D) {
            alive[l] = false;
            continue;
          }
          V rd = d[l] - nrm[l] * (2 * dot(d[l], nrm[l]));
          o[l] = hp[l] + nrm[l] * 0.001;
          d[l] = nrmz(rd);
          if (lev + 1 == 2) g_deep.push_back({o[l], d[l], lev + 1});
        }
      }
    }
  const char *cn[4] = {"primary", "prim-shadow", "secondary", "sec-shadow"};
  for (int c = 0; c < 4; c++) {
    std::printf("%-12s queries %ld waves %ld\n", cn[c], stats[0][c].queries, stats[0][c].wq);
    for (int k = 0; k < NS; k++) {
      const Stats &q = stats[k][c];
      std::printf("   %-15s lane nodes/q %6.2f tests/q %6.2f | wave-max nodes/wq %7.2f tests/wq %6.2f | tot wave "
                  "node-trips %.3g test-trips %.3g\n",
                  strats[k].name, q.lane_nodes / q.queries, q.lane_tests / q.queries, q.wave_nodes / q.wq,
                  q.wave_tests / q.wq, q.wave_nodes, q.wave_tests);
    }
  }
  for (int c = 0; c < 4; c += 2)
    std::printf("zero-term shadow queries, %s: lanes %.1f %%, whole waves %.1f %%\n", c ? "secondary" : "primary",
                100 * g_zero[c][1] / g_zero[c][0], 100 * g_zero[c][3] / g_zero[c][2]);
  std::printf("max stack: ordered %ld ordered4 %ld\n", g_maxstk[1], g_maxstk[2]);
  // level-2 rays packed 64 per wave in spawn order (the deferred queue): the
  // ordered4 closest walk's lane utilisation per wave (sum of lane node visits
  // / 64 x the wave's max) against a walk whose finished lanes refill
  {
    std::vector<long> nodes_of(g_deep.size());
    double sum = 0;
    for (size_t k = 0; k < g_deep.size(); k++) {
      long nn = 0, nt = 0;
      double t = INFINITY;
      int b = -1;
      walk2(s, strats[2], g_deep[k].o, g_deep[k].d, false, 0, t, b, nn, nt);
      nodes_of[k] = nn + nt;
      sum += nn + nt;
    }
    double wsum = 0;
    for (size_t k = 0; k < g_deep.size(); k += 64) {
      long mx = 0;
      for (size_t j = k; j < std::min(g_deep.size(), k + 64); j++) mx = std::max(mx, nodes_of[j]);
      wsum += 64.0 * mx;
    }
    // the same rays sorted by direction octant, then a coarse origin grid cell
    {
      V lo{1e300, 1e300, 1e300}, hi{-1e300, -1e300, -1e300};
      for (auto &q : g_deep)
        lo = {std::min(lo.x, q.o.x), std::min(lo.y, q.o.y), std::min(lo.z, q.o.z)},
        hi = {std::max(hi.x, q.o.x), std::max(hi.y, q.o.y), std::max(hi.z, q.o.z)};
      for (int bits : {0, 1, 2, 3, 4}) {
        std::vector<std::pair<long, size_t>> key(g_deep.size());
        for (size_t k = 0; k < g_deep.size(); k++) {
          const QR &q = g_deep[k];
          long oct = (q.d.x < 0) | ((q.d.y < 0) << 1) | ((q.d.z < 0) << 2);
          const int G = 1 << bits;
          auto cell = [&](double v, double a, double b) {
            int c = (int)((v - a) / std::max(1e-300, b - a) * G);
            return (long)std::min(std::max(c, 0), G - 1);
          };
          long m = (cell(q.o.x, lo.x, hi.x) * G + cell(q.o.y, lo.y, hi.y)) * G + cell(q.o.z, lo.z, hi.z);
          key[k] = {oct * 100000 + m, k};
        }
        std::stable_sort(key.begin(), key.end());
        double ws = 0;
        for (size_t k = 0; k < key.size(); k += 64) {
          long mx = 0;
          for (size_t j = k; j < std::min(key.size(), k + 64); j++) mx = std::max(mx, nodes_of[key[j].second]);
          ws += 64.0 * mx;
        }
        std::printf("  sorted by octant + %d^3 origin cells: lane util %.3f\n", 1 << bits, sum / std::max(1.0, ws));
      }
    }
    if (const char *dump = std::getenv("BVH_SIM_DUMP")) {  // per-ray walk steps, spawn order
      if (FILE *f = std::fopen(dump, "w")) {
        for (long v : nodes_of) std::fprintf(f, "%ld\n", v);
        std::fclose(f);
      }
    }
    std::vector<long> srt = nodes_of;
    std::sort(srt.begin(), srt.end());
    auto pct = [&](double p) { return srt.empty() ? 0L : srt[(size_t)(p * (srt.size() - 1))]; };
    std::printf("level-2 rays %zu: node+leaf steps mean %.1f p50 %ld p90 %ld p99 %ld max %ld; wave-packed lane util %.3f\n",
                g_deep.size(), sum / std::max<size_t>(1, g_deep.size()), pct(0.5), pct(0.9), pct(0.99),
                srt.empty() ? 0L : srt.back(), sum / std::max(1.0, wsum));
  }
  return 0;
}
