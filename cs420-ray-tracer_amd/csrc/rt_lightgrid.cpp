// rt_lightgrid.cpp -- host builder of the per-light direction grids (see rt_lightgrid.h).
#include "rt_lightgrid.h"

#include <algorithm>
#include <cmath>
#include <cstring>
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

}  // namespace

void build_light_grid(const double *cx, const double *cy, const double *cz, const double *r, int n,
                      const double *lx, const double *ly, const double *lz, int nl, double diam, int N,
                      std::vector<int32_t> &start, std::vector<int32_t> &ids) {
  const int cells = 6 * N * N;
  const size_t stride = (size_t)cells + 2;
  start.assign(stride * (size_t)nl, 0);
  ids.clear();
  constexpr int kT = 8;  // patches of kT x kT cells for the coarse pass
  const int NT = (N + kT - 1) / kT;
  std::vector<Patch> cellp((size_t)cells), tilep((size_t)6 * NT * NT);
  for (int f = 0; f < 6; f++)
    for (int j = 0; j < N; j++)
      for (int i = 0; i < N; i++) cellp[(size_t)(f * N + j) * N + i] = make_patch(f, N, i, i + 1, j, j + 1);
  for (int f = 0; f < 6; f++)
    for (int tj = 0; tj < NT; tj++)
      for (int ti = 0; ti < NT; ti++)
        tilep[(size_t)(f * NT + tj) * NT + ti] =
            make_patch(f, N, ti * kT, std::min(N, ti * kT + kT), tj * kT, std::min(N, tj * kT + kT));
  Patch facep[6];
  for (int f = 0; f < 6; f++) facep[f] = make_patch(f, N, 0, N, 0, N);
  const double dm = std::isfinite(diam) ? diam : 0.0;
  std::vector<std::vector<int32_t>> lists((size_t)cells);
  std::vector<int32_t> global;
  for (int l = 0; l < nl; l++) {
    for (auto &v : lists) v.clear();
    global.clear();
    const bool light_ok = std::isfinite(lx[l]) && std::isfinite(ly[l]) && std::isfinite(lz[l]);
    for (int s = 0; s < n; s++) {
      const double vx = cx[s] - lx[l], vy = cy[s] - ly[l], vz = cz[s] - lz[l];
      const double D = std::sqrt(vx * vx + vy * vy + vz * vz);
      const double R = std::fabs(r[s]) * (1.0 + 1e-6) + 1e-6 * (D + dm);  // >= r + max_off + rounding
      if (!light_ok || !std::isfinite(D) || !std::isfinite(R) || !(D > R) || !std::isfinite(dm)) {
        global.push_back(s);  // contains (or nearly) the light, or non-finite: every direction
        continue;
      }
      const Dir v{vx / D, vy / D, vz / D};
      const double alpha = std::asin(R / D) + kLgSlack;
      const double ca = std::cos(alpha), sa = std::sin(alpha);
      for (int f = 0; f < 6; f++) {
        if (!meets(v, ca, sa, alpha, facep[f])) continue;
        for (int tj = 0; tj < NT; tj++)
          for (int ti = 0; ti < NT; ti++) {
            if (!meets(v, ca, sa, alpha, tilep[(size_t)(f * NT + tj) * NT + ti])) continue;
            for (int j = tj * kT; j < std::min(N, tj * kT + kT); j++)
              for (int i = ti * kT; i < std::min(N, ti * kT + kT); i++) {
                const size_t c = (size_t)(f * N + j) * N + i;
                if (meets(v, ca, sa, alpha, cellp[c])) lists[c].push_back(s);
              }
          }
      }
    }
    int32_t *st = start.data() + stride * (size_t)l;
    for (int c = 0; c < cells; c++) {
      st[c] = (int32_t)ids.size();
      ids.insert(ids.end(), lists[c].begin(), lists[c].end());
    }
    st[cells] = (int32_t)ids.size();
    ids.insert(ids.end(), global.begin(), global.end());
    st[cells + 1] = (int32_t)ids.size();
  }
}

bool build_point_grid(const double *cx, const double *cy, const double *cz, const double *r, int n, double px,
                      double py, double pz, double diam, int N, int max_global, size_t max_entries,
                      std::vector<int32_t> &start, std::vector<int32_t> &ent) {
  start.clear();
  ent.clear();
  if (N < 1 || !std::isfinite(px) || !std::isfinite(py) || !std::isfinite(pz) || !std::isfinite(diam)) return false;
  const int cells = 6 * N * N;
  constexpr int kT = 8;
  const int NT = (N + kT - 1) / kT;
  std::vector<Patch> cellp((size_t)cells), tilep((size_t)6 * NT * NT);
  for (int f = 0; f < 6; f++)
    for (int j = 0; j < N; j++)
      for (int i = 0; i < N; i++) cellp[(size_t)(f * N + j) * N + i] = make_patch(f, N, i, i + 1, j, j + 1);
  for (int f = 0; f < 6; f++)
    for (int tj = 0; tj < NT; tj++)
      for (int ti = 0; ti < NT; ti++)
        tilep[(size_t)(f * NT + tj) * NT + ti] =
            make_patch(f, N, ti * kT, std::min(N, ti * kT + kT), tj * kT, std::min(N, tj * kT + kT));
  Patch facep[6];
  for (int f = 0; f < 6; f++) facep[f] = make_patch(f, N, 0, N, 0, N);
  // (tlo, sphere) per cell; a sphere met both ways keeps its smaller bound
  std::vector<std::vector<std::pair<float, int32_t>>> lists((size_t)cells);
  std::vector<int32_t> global;
  size_t total = 0;
  auto mark = [&](const Dir &v, double ca, double sa, double alpha, float tlo, int32_t s) {
    for (int f = 0; f < 6; f++) {
      if (!meets(v, ca, sa, alpha, facep[f])) continue;
      for (int tj = 0; tj < NT; tj++)
        for (int ti = 0; ti < NT; ti++) {
          if (!meets(v, ca, sa, alpha, tilep[(size_t)(f * NT + tj) * NT + ti])) continue;
          for (int j = tj * kT; j < std::min(N, tj * kT + kT); j++)
            for (int i = ti * kT; i < std::min(N, ti * kT + kT); i++) {
              const size_t c = (size_t)(f * N + j) * N + i;
              if (!meets(v, ca, sa, alpha, cellp[c])) continue;
              auto &L = lists[c];
              if (!L.empty() && L.back().second == s) {
                L.back().first = std::min(L.back().first, tlo);
              } else {
                L.emplace_back(tlo, s);
                ++total;
              }
            }
        }
    }
  };
  // fp32 bound at or below x (float(x) rounds to nearest)
  auto down = [](double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
  };
  for (int s = 0; s < n; s++) {
    const double vx = cx[s] - px, vy = cy[s] - py, vz = cz[s] - pz;
    const double D = std::sqrt(vx * vx + vy * vy + vz * vz);
    // the light grid's radius: >= |r| + the rounding of the reference's test
    const double R = std::fabs(r[s]) * (1.0 + 1e-6) + 1e-6 * (D + diam);
    if (!std::isfinite(D) || !std::isfinite(R) || !(D > R)) {
      global.push_back(s);  // contains (or nearly) P, or non-finite: every direction, tlo = -inf
      if ((int)global.size() > max_global) return false;
      continue;
    }
    const Dir v{vx / D, vy / D, vz / D}, w{-v.x, -v.y, -v.z};
    const double alpha = std::asin(R / D) + kLgSlack;
    const double ca = std::cos(alpha), sa = std::sin(alpha);
    // ahead: every root is >= (D - R) / |d| (|d| = 1 within a few ulps; the
    // rounding of the computed root is inside R's margin); behind: only the
    // disc == 0 root, >= -(D + R)
    mark(v, ca, sa, alpha, down((D - R) * (1.0 - 1e-9)), s);
    mark(w, ca, sa, alpha, down(-(D + R) * (1.0 + 1e-9)), s);
    if (total > max_entries) return false;
  }
  if (total + (size_t)cells * global.size() > max_entries) return false;
  start.assign((size_t)cells + 1, 0);
  ent.reserve(2 * (total + (size_t)cells * global.size()));
  for (int c = 0; c < cells; c++) {
    auto &L = lists[c];
    for (int32_t s : global) L.emplace_back(-INFINITY, s);
    std::sort(L.begin(), L.end());  // (tlo, index) ascending
    start[c] = (int32_t)(ent.size() / 2);
    for (const auto &e : L) {
      int32_t bits;
      std::memcpy(&bits, &e.first, sizeof bits);
      ent.push_back(e.second);
      ent.push_back(bits);
    }
    if (ent.size() / 2 > (size_t)INT32_MAX) return false;
  }
  start[cells] = (int32_t)(ent.size() / 2);
  return true;
}

}  // namespace rtk
