// rt_bvh.cpp -- host-side binned-SAH BVH builder for the sphere list.
#include "rt_bvh.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstddef>
#include <cstring>

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

bool build_ugrid(const double *cx, const double *cy, const double *cz, const double *r, int n, size_t max_entries,
                 UgridHost &out, double cells_per_sphere) {
  out = UgridHost{};
  if (n <= 0) return false;
  double clo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, chi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i = 0; i < n; i++) {
    const double c[3] = {cx[i], cy[i], cz[i]};
    if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]) || !std::isfinite(r[i])) return false;
    for (int k = 0; k < 3; k++) {
      clo[k] = std::min(clo[k], c[k]);
      chi[k] = std::max(chi[k], c[k]);
    }
  }
  // first cell size from the centres' box (two cells per sphere); spheres
  // wider than two such cells are global
  const double cps = std::isfinite(cells_per_sphere) && cells_per_sphere > 1e-3 ? cells_per_sphere : 2.0;
  auto cell_for = [cps](const double *lo, const double *hi, int m) {
    double vol = 1.0, emax = 0.0;
    for (int k = 0; k < 3; k++) emax = std::max(emax, hi[k] - lo[k]);
    const double floor_e = std::max(emax * 1e-3, 1e-9);
    for (int k = 0; k < 3; k++) vol *= std::max(hi[k] - lo[k], floor_e);
    return std::cbrt(vol / (cps * std::max(1, m)));
  };
  const double cs0 = cell_for(clo, chi, n);
  std::vector<int32_t> small;
  small.reserve((size_t)n);
  for (int i = 0; i < n; i++) {
    if (std::fabs(r[i]) > 2.0 * cs0) out.glob.push_back(i);
    else small.push_back(i);
  }
  if (out.glob.size() > 64) return false;  // every line would test them all
  if (small.empty()) {  // only global spheres: one empty cell
    out.cs = 1.0f;
    out.nx = out.ny = out.nz = 1;
    out.reg_margin = FLT_MAX;
    out.start.assign(2, 0);
    out.rec.assign(4, UgRec{0.0f, 0.0f, 0.0f, -1.0f});
    out.rid.assign(4, 0);
    out.q.assign(1, UgRec{0.0f, 0.0f, 0.0f, -1.0f});
    return true;
  }
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i : small) {
    const double c[3] = {cx[i], cy[i], cz[i]}, a = std::fabs(r[i]);
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], c[k] - a);
      hi[k] = std::max(hi[k], c[k] + a);
    }
  }
  double E = 0.0;
  for (int k = 0; k < 3; k++) E = std::max(E, hi[k] - lo[k]);
  double cs = cell_for(lo, hi, (int)small.size());
  // listing margin: the device's prefilter margin plus the DDA's fp32 error
  // (both checked against it per launch, rt_kernel.hip bvh_args)
  const double mg = 1e-3 * cs + 2e-4 * E;
  for (int k = 0; k < 3; k++) {
    lo[k] -= mg;
    hi[k] += mg;
  }
  E += 2.0 * mg;
  int dim[3];
  constexpr double kMaxCells = 16.0 * (1 << 20);
  bool fits = false;
  for (int it = 0; it < 8 && !fits; it++) {  // at most 512 cells per axis and 16 M cells
    double cells = 1.0;
    for (int k = 0; k < 3; k++) {
      dim[k] = (int)std::min(512.0, std::max(1.0, std::ceil((hi[k] - lo[k]) / cs)));
      cells *= dim[k];
    }
    fits = cells <= kMaxCells;
    if (!fits) cs *= std::cbrt(cells / kMaxCells) * 1.01;
  }
  if (!fits) return false;  // the cap still fails: no grid (the BVH walks stay)
  for (int k = 0; k < 3; k++) cs = std::max(cs, (hi[k] - lo[k]) / dim[k] * (1.0 + 1e-6));
  if (!(cs > 0.0) || !std::isfinite(cs)) return false;
  // fp32 origin and cell size, rounded so that the fp32 grid still covers [lo, hi]
  out.gx = round_down(lo[0]);
  out.gy = round_down(lo[1]);
  out.gz = round_down(lo[2]);
  out.cs = round_up(cs);
  out.nx = dim[0];
  out.ny = dim[1];
  out.nz = dim[2];
  out.reg_margin = round_down(mg);
  out.extent = round_up(E);
  const double g0[3] = {out.gx, out.gy, out.gz}, fcs = out.cs;
  const size_t ncell = (size_t)dim[0] * dim[1] * dim[2];
  std::vector<uint32_t> count(ncell + 1, 0u);
  auto range = [&](int i, int (&a)[3], int (&b)[3]) {
    const double c[3] = {cx[i], cy[i], cz[i]}, rr = std::fabs(r[i]) + mg;
    for (int k = 0; k < 3; k++) {
      a[k] = std::max(0, std::min(dim[k] - 1, (int)std::floor((c[k] - rr - g0[k]) / fcs)));
      b[k] = std::max(0, std::min(dim[k] - 1, (int)std::floor((c[k] + rr - g0[k]) / fcs)));
    }
  };
  size_t total = 0;
  for (int i : small) {
    int a[3], b[3];
    range(i, a, b);
    total += (size_t)(b[0] - a[0] + 1) * (b[1] - a[1] + 1) * (b[2] - a[2] + 1);
    if (total > max_entries) return false;
    for (int z = a[2]; z <= b[2]; z++)
      for (int y = a[1]; y <= b[1]; y++)
        for (int x = a[0]; x <= b[0]; x++) count[((size_t)z * dim[1] + y) * dim[0] + x]++;
  }
  out.start.assign(ncell + 1, 0);
  for (size_t c = 0; c < ncell; c++) out.start[c + 1] = out.start[c] + (int32_t)count[c];
  out.ids.assign(total, 0);
  std::vector<int32_t> fill(out.start.begin(), out.start.end() - 1);
  for (int i : small) {  // ascending sphere index within every cell
    int a[3], b[3];
    range(i, a, b);
    for (int z = a[2]; z <= b[2]; z++)
      for (int y = a[1]; y <= b[1]; y++)
        for (int x = a[0]; x <= b[0]; x++) out.ids[(size_t)fill[((size_t)z * dim[1] + y) * dim[0] + x]++] = i;
  }
  // the device records: slot data (centre - c0 and |radius| rounded up, fp32)
  out.q.resize(total + 1);
  for (size_t k = 0; k < total; k++) {
    const int i = out.ids[k];
    float rr = (float)std::fabs(r[i]);
    if ((double)rr < std::fabs(r[i])) rr = std::nextafter(rr, INFINITY);
    out.q[k] = UgRec{(float)cx[i], (float)cy[i], (float)cz[i], rr};
  }
  out.q[total] = UgRec{0.0f, 0.0f, 0.0f, -1.0f};
  out.rec.assign(ncell * 4, UgRec{0.0f, 0.0f, 0.0f, -1.0f});
  out.rid.assign(ncell * 4, 0);
  for (size_t c = 0; c < ncell; c++) {
    const int32_t k0 = out.start[c], k1 = out.start[c + 1];
    const int m = k1 - k0;
    const int inl = m <= 4 ? m : 3;
    for (int j = 0; j < inl; j++) {
      out.rec[4 * c + j] = out.q[(size_t)k0 + j];
      out.rid[4 * c + j] = out.ids[(size_t)k0 + j];
    }
    if (m > 4) {
      UgRec o{};
      const int32_t a0 = k0 + 3;
      std::memcpy(&o.x, &a0, sizeof(float));
      std::memcpy(&o.y, &k1, sizeof(float));
      o.w = -2.0f;
      out.rec[4 * c + 3] = o;
    }
  }
  return true;
}

}  // namespace rtk
