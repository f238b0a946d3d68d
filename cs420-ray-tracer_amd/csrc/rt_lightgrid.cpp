// rt_lightgrid.cpp -- host builder of the per-light direction grids (see rt_lightgrid.h).
#include "rt_lightgrid.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>

namespace rtk {
namespace {

struct Dir {
  double x, y, z;
};

Dir face_dir(int face, double a, double b) {
  Dir d;
  switch (face) {
    case 0: d = {1.0, a, b}; break;
    case 1: d = {-1.0, a, b}; break;
    case 2: d = {a, 1.0, b}; break;
    case 3: d = {a, -1.0, b}; break;
    case 4: d = {a, b, 1.0}; break;
    default: d = {a, b, -1.0}; break;
  }
  const double l = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
  return {d.x / l, d.y / l, d.z / l};
}

double angle(const Dir &u, const Dir &v) {  // robust for small angles
  const double cx = u.y * v.z - u.z * v.y, cy = u.z * v.x - u.x * v.z, cz = u.x * v.y - u.y * v.x;
  return std::atan2(std::sqrt(cx * cx + cy * cy + cz * cz), u.x * v.x + u.y * v.y + u.z * v.z);
}

// A square patch [i0, i1) x [j0, j1) of a face: centre direction and the
// largest angle from it to the patch (attained at a corner: the patch is
// geodesically convex and the distance to a point is convex on it).
struct Patch {
  Dir c;
  double rad, cb, sb;  // cos / sin of (rad + kLgSlack)
};
Patch make_patch(int face, int N, int i0, int i1, int j0, int j1) {
  const double a0 = -1.0 + 2.0 * i0 / N, a1 = -1.0 + 2.0 * i1 / N;
  const double b0 = -1.0 + 2.0 * j0 / N, b1 = -1.0 + 2.0 * j1 / N;
  Patch p;
  p.c = face_dir(face, 0.5 * (a0 + a1), 0.5 * (b0 + b1));
  p.rad = std::max(std::max(angle(p.c, face_dir(face, a0, b0)), angle(p.c, face_dir(face, a1, b0))),
                   std::max(angle(p.c, face_dir(face, a0, b1)), angle(p.c, face_dir(face, a1, b1))));
  p.cb = std::cos(p.rad + kLgSlack);
  p.sb = std::sin(p.rad + kLgSlack);
  return p;
}

// angle(v, patch centre) <= alpha + rad + slack, with ca/sa = cos/sin(alpha):
// dot(v, c) >= cos(alpha + beta) = ca cb - sa sb (alpha + beta < pi), the
// threshold lowered by 1e-12 so rounding can only add cells.
inline bool meets(const Dir &v, double ca, double sa, double alpha, const Patch &p) {
  if (alpha + p.rad + kLgSlack >= 3.14159) return true;
  return v.x * p.c.x + v.y * p.c.y + v.z * p.c.z >= ca * p.cb - sa * p.sb - 1e-12;
}

// The cell patches of an N x N face have the same angular radius on all six
// faces (the faces are permutations / reflections of each other), so the
// camera grid keeps one (cos, sin) of rad + slack per (i, j) for each N it
// has seen and forms the cell centres on the fly.
struct CellTable {
  int N = 0;
  std::vector<double> cb, sb;  // per (j * N + i)
};
const CellTable &cell_table(int N) {
  static std::mutex mu;
  static std::vector<std::unique_ptr<CellTable>> cache;
  std::lock_guard<std::mutex> lock(mu);
  for (const auto &t : cache)
    if (t->N == N) return *t;
  auto t = std::make_unique<CellTable>();
  t->N = N;
  t->cb.resize((size_t)N * N);
  t->sb.resize((size_t)N * N);
  for (int j = 0; j < N; j++)
    for (int i = 0; i < N; i++) {
      const Patch p = make_patch(0, N, i, i + 1, j, j + 1);
      t->cb[(size_t)j * N + i] = p.cb;
      t->sb[(size_t)j * N + i] = p.sb;
    }
  cache.push_back(std::move(t));
  return *cache.back();
}

// The cube map's patch hierarchy: faces, blocks of kB x kB tiles, tiles of
// kT x kT cells, cells (from the cached per-N table).  for_cells calls fn(c)
// for every cell a disk (centre v, angular radius alpha, ca/sa its cos/sin)
// meets; a tile well inside the disk gives all its cells untested (a list may
// hold extra spheres, never miss one).
struct CubeGrid {
  static constexpr int kT = 8, kB = 8;
  int N, NT, NB;
  const CellTable *ct;
  std::vector<Patch> tilep, blockp;
  Patch facep[6];
  explicit CubeGrid(int n) : N(n), NT((n + kT - 1) / kT), NB((NT + kB - 1) / kB), ct(&cell_table(n)) {
    tilep.resize((size_t)6 * NT * NT);
    for (int f = 0; f < 6; f++)
      for (int tj = 0; tj < NT; tj++)
        for (int ti = 0; ti < NT; ti++)
          tilep[(size_t)(f * NT + tj) * NT + ti] =
              make_patch(f, N, ti * kT, std::min(N, ti * kT + kT), tj * kT, std::min(N, tj * kT + kT));
    blockp.resize((size_t)6 * NB * NB);
    for (int f = 0; f < 6; f++)
      for (int bj = 0; bj < NB; bj++)
        for (int bi = 0; bi < NB; bi++)
          blockp[(size_t)(f * NB + bj) * NB + bi] = make_patch(f, N, bi * kB * kT, std::min(N, (bi + 1) * kB * kT),
                                                               bj * kB * kT, std::min(N, (bj + 1) * kB * kT));
    for (int f = 0; f < 6; f++) facep[f] = make_patch(f, N, 0, N, 0, N);
  }
  template <class F>
  void for_cells(const Dir &v, double ca, double sa, double alpha, F &&fn) const {
    const bool wide = alpha + kLgSlack >= 3.0;  // meets() takes every patch then
    for (int f = 0; f < 6; f++) {
      if (!meets(v, ca, sa, alpha, facep[f])) continue;
      for (int bj = 0; bj < NB; bj++)
        for (int bi = 0; bi < NB; bi++) {
          if (!meets(v, ca, sa, alpha, blockp[(size_t)(f * NB + bj) * NB + bi])) continue;
          for (int tj = bj * kB; tj < std::min(NT, (bj + 1) * kB); tj++)
            for (int ti = bi * kB; ti < std::min(NT, (bi + 1) * kB); ti++) {
              const Patch &tp = tilep[(size_t)(f * NT + tj) * NT + ti];
              if (!meets(v, ca, sa, alpha, tp)) continue;
              const bool inside = alpha < 3.0 && alpha > tp.rad + 1e-3 &&
                                  v.x * tp.c.x + v.y * tp.c.y + v.z * tp.c.z >= std::cos(alpha - tp.rad - 1e-3);
              for (int j = tj * kT; j < std::min(N, tj * kT + kT); j++) {
                const double b = -1.0 + (2.0 * j + 1.0) / N;
                for (int i = ti * kT; i < std::min(N, ti * kT + kT); i++) {
                  const size_t ij = (size_t)j * N + i;
                  if (!inside) {
                    Patch p;
                    p.c = face_dir(f, -1.0 + (2.0 * i + 1.0) / N, b);
                    p.rad = wide ? 3.2 : 0.0;  // only meets()'s "whole sphere" shortcut reads it
                    p.cb = ct->cb[ij];
                    p.sb = ct->sb[ij];
                    if (!meets(v, ca, sa, alpha, p)) continue;
                  }
                  fn((size_t)f * N * N + ij);
                }
              }
            }
        }
    }
  }
};

}  // namespace

void build_light_grid(const double *cx, const double *cy, const double *cz, const double *r, int n,
                      const double *lx, const double *ly, const double *lz, int nl, double diam, int N,
                      std::vector<int32_t> &start, std::vector<int32_t> &ids) {
  const int cells = 6 * N * N;
  const size_t stride = (size_t)cells + 2;
  start.assign(stride * (size_t)nl, 0);
  ids.clear();
  const CubeGrid G(N);
  const double dm = std::isfinite(diam) ? diam : 0.0;
  // one thread per light (its lists, then concatenated in light order)
  std::vector<std::vector<int32_t>> lid((size_t)nl);
  auto build_one = [&](int l) {
    std::vector<std::vector<int32_t>> lists((size_t)cells);
    std::vector<int32_t> global;
    const bool light_ok = std::isfinite(lx[l]) && std::isfinite(ly[l]) && std::isfinite(lz[l]);
    for (int s = 0; s < n; s++) {
      const double vx = cx[s] - lx[l], vy = cy[s] - ly[l], vz = cz[s] - lz[l];
      const double D = std::sqrt(vx * vx + vy * vy + vz * vz);
      const double R = std::fabs(r[s]) * (1.0 + 1e-6) + 1e-6 * (D + dm);  // >= r + max_off + rounding
      if (!light_ok || !std::isfinite(D) || !std::isfinite(R) || !(D > R + kLgOvershoot) || !std::isfinite(dm)) {
        global.push_back(s);  // contains the light or comes within the overshoot of it, or non-finite: every direction
        continue;
      }
      const Dir v{vx / D, vy / D, vz / D};
      const double alpha = std::asin(R / D) + kLgSlack;
      const double ca = std::cos(alpha), sa = std::sin(alpha);
      G.for_cells(v, ca, sa, alpha, [&](size_t c) { lists[c].push_back(s); });
    }
    int32_t *st = start.data() + stride * (size_t)l;  // offsets within this light's ids for now
    std::vector<int32_t> &out = lid[(size_t)l];
    for (int c = 0; c < cells; c++) {
      st[c] = (int32_t)out.size();
      out.insert(out.end(), lists[c].begin(), lists[c].end());
    }
    st[cells] = (int32_t)out.size();
    out.insert(out.end(), global.begin(), global.end());
    st[cells + 1] = (int32_t)out.size();
  };
  std::vector<std::thread> th;
  for (int l = 1; l < nl; l++) th.emplace_back(build_one, l);
  if (nl > 0) build_one(0);
  for (auto &t : th) t.join();
  for (int l = 0; l < nl; l++) {
    const int32_t base = (int32_t)ids.size();
    int32_t *st = start.data() + stride * (size_t)l;
    for (size_t c = 0; c < stride; c++) st[c] += base;
    ids.insert(ids.end(), lid[(size_t)l].begin(), lid[(size_t)l].end());
  }
}

namespace {

// build_point_grid for origins anywhere in the ball B(P, rho) (rho = 0: the
// point itself), its disk-binning spread over `nthreads` workers;
// `total_recs` (shared by concurrent builds) counts the records of all of
// them against max_entries.
bool point_grid(const CubeGrid &G, const double *cx, const double *cy, const double *cz, const double *r, int n,
                double px, double py, double pz, double rho, double diam, int max_global, size_t max_entries,
                int nthreads, std::atomic<size_t> &total_recs, std::vector<int32_t> &start,
                std::vector<int32_t> &ent) {
  start.clear();
  ent.clear();
  const int N = G.N;
  if (!std::isfinite(px) || !std::isfinite(py) || !std::isfinite(pz) || !std::isfinite(diam) || !std::isfinite(rho) ||
      !(rho >= 0.0))
    return false;
  const int cells = 6 * N * N;
  // records (cell, tlo, sphere)
  struct Rec {
    int32_t cell;
    float tlo;
    int32_t s;
  };
  struct Disk {
    Dir v;
    double ca, sa, alpha;
    float tlo;
    int32_t s;
  };
  // fp32 bound at or below x (float(x) rounds to nearest)
  auto down = [](double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
  };
  std::vector<Disk> disks;
  std::vector<int32_t> global;
  disks.reserve(2 * (size_t)n);
  for (int s = 0; s < n; s++) {
    const double vx = cx[s] - px, vy = cy[s] - py, vz = cz[s] - pz;
    const double D = std::sqrt(vx * vx + vy * vy + vz * vz);
    // the light grid's radius: >= |r| + the rounding of the reference's test,
    // grown by rho: a ray from any origin p in B(P, rho) that meets the
    // sphere has its direction in the disk of B(C - P, R) (the Minkowski sum)
    // and every root at least D - R from p
    const double R = std::fabs(r[s]) * (1.0 + 1e-6) + 1e-6 * (D + diam) + rho;
    if (!std::isfinite(D) || !std::isfinite(R) || !(D > R)) {
      global.push_back(s);  // contains (or nearly) P, or non-finite: every direction, tlo = -inf
      if ((int)global.size() > max_global) return false;
      continue;
    }
    const Dir v{vx / D, vy / D, vz / D};
    const double alpha = std::asin(R / D) + kLgSlack;
    const double ca = std::cos(alpha), sa = std::sin(alpha);
    // ahead: every root is >= (D - R) / |d| (|d| = 1 within a few ulps; the
    // rounding of the computed root is inside R's margin); behind: only the
    // disc == 0 root, >= -(D + R)
    disks.push_back(Disk{v, ca, sa, alpha, down((D - R) * (1.0 - 1e-9)), s});
    disks.push_back(Disk{Dir{-v.x, -v.y, -v.z}, ca, sa, alpha, down(-(D + R) * (1.0 + 1e-9)), s});
  }
  const size_t fcells = (size_t)N * N;
  // kThreads workers over slices of the spheres, records per worker.  A
  // sphere whose two disks (very wide ones) both meet a cell is listed there
  // twice: the second test of it changes nothing (same t, same index)
  const int kThreads = nthreads;
  std::vector<std::vector<Rec>> recs((size_t)kThreads);
  std::unique_ptr<bool[]> over(new bool[(size_t)kThreads]());
  // records of all workers together: a worker stops (and the build is
  // refused) as soon as the total passes max_entries, so the host memory held
  // is bounded by max_entries records plus one disk per worker, not
  // kThreads * max_entries
  if (total_recs.fetch_add((size_t)cells * global.size()) + (size_t)cells * global.size() > max_entries) return false;
  auto build_slice = [&](int w) {
    std::vector<Rec> &out = recs[w];
    const size_t pairs = disks.size() / 2, lo = pairs * w / kThreads, hi = pairs * (w + 1) / kThreads;
    for (size_t di = 2 * lo; di < 2 * hi; di++) {
      const Disk &k = disks[di];
      const Dir &v = k.v;
      const double ca = k.ca, sa = k.sa, alpha = k.alpha;
      const size_t before = out.size();
      G.for_cells(v, ca, sa, alpha, [&](size_t c) { out.push_back(Rec{(int32_t)c, k.tlo, k.s}); });
      if (total_recs.fetch_add(out.size() - before, std::memory_order_relaxed) + (out.size() - before) > max_entries) {
        over[w] = true;
        return;
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int w = 1; w < kThreads; w++) th.emplace_back(build_slice, w);
    build_slice(0);
    for (auto &t : th) t.join();
  }
  size_t nrec = 0;
  for (int w = 0; w < kThreads; w++) {
    if (over[w]) return false;
    nrec += recs[w].size();
  }
  const size_t total = nrec + (size_t)cells * global.size();
  if (total > max_entries || total > (size_t)INT32_MAX) return false;
  // counting sort by cell, then each cell's list by (tlo, index)
  start.assign((size_t)cells + 1, 0);
  for (int w = 0; w < kThreads; w++)
    for (const Rec &e : recs[w]) start[(size_t)e.cell + 1]++;
  for (int c = 0; c < cells; c++) start[(size_t)c + 1] += start[c] + (int32_t)global.size();
  ent.resize(2 * total);
  auto emit_face = [&](int f) {
    std::vector<std::pair<float, int32_t>> L;
    std::vector<size_t> fill(fcells);
    std::vector<std::pair<float, int32_t>> flat(
        (size_t)(start[(size_t)(f + 1) * fcells] - start[(size_t)f * fcells]));
    const size_t base = (size_t)start[(size_t)f * fcells];
    for (size_t ij = 0; ij < fcells; ij++) {
      fill[ij] = (size_t)start[f * fcells + ij] - base;
      for (int32_t s : global) flat[fill[ij]++] = {-INFINITY, s};
    }
    for (int w = 0; w < kThreads; w++)
      for (const Rec &e : recs[w])
        if ((size_t)e.cell / fcells == (size_t)f) flat[fill[(size_t)e.cell - f * fcells]++] = {e.tlo, e.s};
    for (size_t ij = 0; ij < fcells; ij++) {
      const size_t b = (size_t)start[f * fcells + ij] - base, e = (size_t)start[f * fcells + ij + 1] - base;
      if (e - b > 1) std::sort(flat.begin() + (long)b, flat.begin() + (long)e);
      for (size_t k = b; k < e; k++) {
        ent[2 * (base + k)] = flat[k].second;
        std::memcpy(&ent[2 * (base + k) + 1], &flat[k].first, sizeof(int32_t));
      }
    }
  };
  if (kThreads == 1) {  // one worker: no face threads either (concurrent builds run one per thread)
    for (int f = 0; f < 6; f++) emit_face(f);
  } else {
    std::vector<std::thread> th;
    for (int f = 1; f < 6; f++) th.emplace_back(emit_face, f);
    emit_face(0);
    for (auto &t : th) t.join();
  }
  return true;
}

}  // namespace

void cube_tables(int N, std::vector<CubePatch> &faces, std::vector<CubePatch> &blocks, std::vector<CubePatch> &tiles,
                 std::vector<double> &cell_cbsb, int &NT, int &NB) {
  static_assert(CubeGrid::kT == kCubeT && CubeGrid::kB == kCubeB, "one patch hierarchy");
  const CubeGrid G(N);
  auto put = [](const Patch &p) { return CubePatch{p.c.x, p.c.y, p.c.z, p.rad, p.cb, p.sb}; };
  NT = G.NT;
  NB = G.NB;
  faces.clear();
  for (int f = 0; f < 6; f++) faces.push_back(put(G.facep[f]));
  blocks.clear();
  for (const Patch &p : G.blockp) blocks.push_back(put(p));
  tiles.clear();
  for (const Patch &p : G.tilep) tiles.push_back(put(p));
  cell_cbsb.resize(2 * (size_t)N * N);
  for (size_t ij = 0; ij < (size_t)N * N; ij++) {
    cell_cbsb[2 * ij] = G.ct->cb[ij];
    cell_cbsb[2 * ij + 1] = G.ct->sb[ij];
  }
}

bool build_point_grid(const double *cx, const double *cy, const double *cz, const double *r, int n, double px,
                      double py, double pz, double diam, int N, int max_global, size_t max_entries,
                      std::vector<int32_t> &start, std::vector<int32_t> &ent) {
  start.clear();
  ent.clear();
  if (N < 1 || N > 4096) return false;
  const CubeGrid G(N);
  std::atomic<size_t> total{0};
  return point_grid(G, cx, cy, cz, r, n, px, py, pz, 0.0, diam, max_global, max_entries, 8, total, start, ent);
}

size_t build_sphere_grids(const double *cx, const double *cy, const double *cz, const double *r, int n,
                          const double *rho, double diam, int N, int max_global, size_t max_entries,
                          std::vector<int32_t> &start, std::vector<int32_t> &ent, std::vector<uint8_t> &ok) {
  start.clear();
  ent.clear();
  ok.assign((size_t)std::max(n, 0), 0);
  if (N < 1 || N > 1024 || n <= 0) return 0;
  const int cells = 6 * N * N;
  const size_t stride = (size_t)cells + 1;
  const CubeGrid G(N);
  std::vector<std::vector<int32_t>> st((size_t)n), en((size_t)n);
  std::atomic<size_t> total{0};
  std::atomic<int> next{0};
  std::atomic<bool> over{false};
  // one sphere's grid per worker at a time (single-threaded builds)
  auto worker = [&]() {
    for (int s; (s = next.fetch_add(1)) < n && !over.load(std::memory_order_relaxed);) {
      ok[(size_t)s] = point_grid(G, cx, cy, cz, r, n, cx[s], cy[s], cz[s], rho[s], diam, max_global, max_entries, 1,
                                 total, st[(size_t)s], en[(size_t)s])
                          ? 1
                          : 0;
      if (total.load(std::memory_order_relaxed) > max_entries) over = true;
    }
  };
  {
    const unsigned hw = std::thread::hardware_concurrency();
    const int nw = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
    std::vector<std::thread> th;
    for (int w = 1; w < nw; w++) th.emplace_back(worker);
    worker();
    for (auto &t : th) t.join();
  }
  if (over) {
    ok.assign((size_t)n, 0);
    return 0;
  }
  size_t entries = 0;
  for (int s = 0; s < n; s++)
    if (ok[(size_t)s]) entries += en[(size_t)s].size() / 2;
  if (entries > (size_t)INT32_MAX) {
    ok.assign((size_t)n, 0);
    return 0;
  }
  start.assign(stride * (size_t)n, 0);
  ent.resize(2 * entries);
  size_t base = 0;
  for (int s = 0; s < n; s++) {
    int32_t *so = start.data() + stride * (size_t)s;
    if (!ok[(size_t)s]) {  // refused (too many spheres overlap its origin ball): empty lists, never used
      for (size_t c = 0; c < stride; c++) so[c] = (int32_t)base;
      continue;
    }
    for (size_t c = 0; c < stride; c++) so[c] = (int32_t)(base + (size_t)st[(size_t)s][c]);
    std::memcpy(ent.data() + 2 * base, en[(size_t)s].data(), en[(size_t)s].size() * sizeof(int32_t));
    base += en[(size_t)s].size() / 2;
    std::vector<int32_t>().swap(st[(size_t)s]);
    std::vector<int32_t>().swap(en[(size_t)s]);
  }
  return entries;
}

}  // namespace rtk
