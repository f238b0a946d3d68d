// rt_bvh.cpp -- host-side binned-SAH BVH builder for the sphere list.
#include "rt_bvh.h"

#include <algorithm>
#include <cfloat>
#include <cmath>

namespace rtk {
namespace {

struct Box {
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  void grow(const double *l, const double *h) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], l[k]);
      hi[k] = std::max(hi[k], h[k]);
    }
  }
  double area() const {
    if (lo[0] > hi[0]) return 0.0;
    double e[3];
    for (int k = 0; k < 3; k++) e[k] = hi[k] - lo[k];
    return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
  }
};

struct Prim {
  double lo[3], hi[3], c[3];
  int32_t id;
};

float round_down(double v) {
  float f = (float)v;
  if ((double)f > v) f = std::nextafter(f, -FLT_MAX);
  return f;
}
float round_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = std::nextafter(f, FLT_MAX);
  return f;
}

struct Builder {
  std::vector<Prim> &p;
  int max_leaf;
  std::vector<BvhNode> &nodes;
  std::vector<int32_t> &prims;

  void emit_box(BvhNode &nd, const Box &b) {
    for (int k = 0; k < 3; k++) {
      nd.lo[k] = round_down(b.lo[k]);
      nd.hi[k] = round_up(b.hi[k]);
    }
  }

  // Builds [begin, end) in preorder; returns nothing, fills skip pointers.
  void build(int begin, int end) {
    Box b, cb;
    for (int i = begin; i < end; i++) {
      b.grow(p[i].lo, p[i].hi);
      cb.grow(p[i].c, p[i].c);
    }
    const int me = (int)nodes.size();
    nodes.push_back(BvhNode{});
    emit_box(nodes[me], b);
    const int count = end - begin;
    int split = -1;
    if (count > max_leaf || count > 15) {
      // binned SAH over the centroid bounds
      int axis = 0;
      double ext = -1.0;
      for (int k = 0; k < 3; k++)
        if (cb.hi[k] - cb.lo[k] > ext) {
          ext = cb.hi[k] - cb.lo[k];
          axis = k;
        }
      if (ext > 0.0 && std::isfinite(ext)) {
        constexpr int kBins = 16;
        Box bins[kBins];
        int cnt[kBins] = {};
        auto bin_of = [&](const Prim &q) {
          int bi = (int)((q.c[axis] - cb.lo[axis]) / ext * kBins);
          return std::min(std::max(bi, 0), kBins - 1);
        };
        for (int i = begin; i < end; i++) {
          int bi = bin_of(p[i]);
          cnt[bi]++;
          bins[bi].grow(p[i].lo, p[i].hi);
        }
        double best = DBL_MAX;
        int best_bin = -1;
        for (int s = 1; s < kBins; s++) {
          Box l, r;
          int nl = 0, nr = 0;
          for (int i = 0; i < s; i++)
            if (cnt[i]) l.grow(bins[i].lo, bins[i].hi), nl += cnt[i];
          for (int i = s; i < kBins; i++)
            if (cnt[i]) r.grow(bins[i].lo, bins[i].hi), nr += cnt[i];
          if (!nl || !nr) continue;
          double cost = l.area() * nl + r.area() * nr;
          if (cost < best) {
            best = cost;
            best_bin = s;
          }
        }
        if (best_bin > 0) {
          auto mid = std::partition(p.begin() + begin, p.begin() + end,
                                    [&](const Prim &q) { return bin_of(q) < best_bin; });
          split = (int)(mid - p.begin());
        }
      }
      if (split <= begin || split >= end) {  // degenerate centroids: median by index
        split = begin + count / 2;
      }
    }
    if (split < 0) {
      nodes[me].leaf = ((int32_t)prims.size() << 4) | count;
      for (int i = begin; i < end; i++) prims.push_back(p[i].id);
    } else {
      nodes[me].leaf = -1;
      build(begin, split);
      build(split, end);
    }
    nodes[me].skip = (int32_t)nodes.size();
  }
};

}  // namespace

void build_bvh(const double *cx, const double *cy, const double *cz, const double *r, int n, int max_leaf,
               std::vector<BvhNode> &nodes, std::vector<int32_t> &prims) {
  nodes.clear();
  prims.clear();
  if (n <= 0) return;
  std::vector<Prim> p((size_t)n);
  for (int i = 0; i < n; i++) {
    const double c[3] = {cx[i], cy[i], cz[i]};
    const double rr = std::fabs(r[i]);
    for (int k = 0; k < 3; k++) {
      p[i].c[k] = c[k];
      p[i].lo[k] = c[k] - rr;
      p[i].hi[k] = c[k] + rr;
      if (!std::isfinite(p[i].lo[k]) || !std::isfinite(p[i].hi[k])) {  // NaN/inf: a box that always hits
        p[i].lo[k] = -DBL_MAX;
        p[i].hi[k] = DBL_MAX;
        p[i].c[k] = 0.0;
      }
    }
    p[i].id = i;
  }
  Builder b{p, std::max(1, std::min(max_leaf, 15)), nodes, prims};
  nodes.reserve(2 * (size_t)n);
  b.build(0, n);
}

int32_t build_bvh2(const std::vector<BvhNode> &nodes, std::vector<BvhNode2> &out, int &depth) {
  out.clear();
  depth = 0;
  if (nodes.empty()) return -1;
  // preorder index of each internal node -> its BvhNode2 index
  std::vector<int32_t> map(nodes.size(), -1);
  for (size_t i = 0; i < nodes.size(); i++)
    if (nodes[i].leaf < 0) {
      map[i] = (int32_t)out.size();
      out.push_back(BvhNode2{});
    }
  auto ref = [&](int i) { return nodes[i].leaf >= 0 ? -(nodes[i].leaf + 1) : map[i]; };
  std::vector<std::pair<int, int>> todo{{0, 0}};  // (preorder index, depth)
  while (!todo.empty()) {
    const auto [i, dep] = todo.back();
    todo.pop_back();
    depth = std::max(depth, dep);
    if (nodes[i].leaf >= 0) continue;
    const int l = i + 1, r = nodes[l].skip;
    BvhNode2 &b = out[map[i]];
    for (int k = 0; k < 3; k++) {
      b.lo0[k] = nodes[l].lo[k];
      b.hi0[k] = nodes[l].hi[k];
      b.lo1[k] = nodes[r].lo[k];
      b.hi1[k] = nodes[r].hi[k];
    }
    b.c0 = ref(l);
    b.c1 = ref(r);
    todo.push_back({l, dep + 1});
    todo.push_back({r, dep + 1});
  }
  return ref(0);
}

int32_t build_bvh4(const std::vector<BvhNode> &nodes, std::vector<BvhNode4> &out, int &stack) {
  out.clear();
  stack = 0;
  if (nodes.empty()) return -1;
  if (nodes[0].leaf >= 0) return -(nodes[0].leaf + 1);
  // the 4-wide nodes are the binary root and every internal grandchild reached
  // from one; `kids` lists the up-to-4 preorder children of binary node i
  auto kids = [&](int i, int *c) {
    int n = 0;
    const int l = i + 1, r = nodes[l].skip;
    for (int x : {l, r}) {
      if (nodes[x].leaf >= 0) {
        c[n++] = x;
      } else {
        c[n++] = x + 1;
        c[n++] = nodes[x + 1].skip;
      }
    }
    return n;
  };
  std::vector<int32_t> map(nodes.size(), -1);
  std::vector<int> order{0};  // breadth of 4-wide nodes, in creation order
  map[0] = 0;
  for (size_t q = 0; q < order.size(); q++) {
    int c[4];
    const int n = kids(order[q], c);
    for (int k = 0; k < n; k++)
      if (nodes[c[k]].leaf < 0 && map[c[k]] < 0) {
        map[c[k]] = (int32_t)order.size();
        order.push_back(c[k]);
      }
  }
  out.resize(order.size());
  const float qnan = __builtin_nanf("");
  std::vector<int> need(order.size(), 0);  // worst pending entries below each node
  for (size_t q = order.size(); q-- > 0;) {
    int c[4];
    const int n = kids(order[q], c);
    BvhNode4 &b = out[q];
    int worst = 0;
    for (int k = 0; k < 4; k++) {
      const bool on = k < n;
      b.lox[k] = on ? nodes[c[k]].lo[0] : qnan;
      b.loy[k] = on ? nodes[c[k]].lo[1] : qnan;
      b.loz[k] = on ? nodes[c[k]].lo[2] : qnan;
      b.hix[k] = on ? nodes[c[k]].hi[0] : qnan;
      b.hiy[k] = on ? nodes[c[k]].hi[1] : qnan;
      b.hiz[k] = on ? nodes[c[k]].hi[2] : qnan;
      b.c[k] = !on ? 0 : nodes[c[k]].leaf >= 0 ? -(nodes[c[k]].leaf + 1) : map[c[k]];
      if (on && nodes[c[k]].leaf < 0) worst = std::max(worst, need[map[c[k]]]);
      b.pad[k] = 0;
    }
    // entering the nearest child leaves at most n - 1 pending here
    need[q] = n - 1 + worst;
  }
  stack = need[0];
  return 0;
}

}  // namespace rtk
