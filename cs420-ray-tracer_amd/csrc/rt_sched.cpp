// rt_sched.cpp -- see rt_sched.h.
#include "rt_sched.h"

#include <algorithm>
#include <cmath>

#ifndef RT_SCHED_BLOCKS
#define RT_SCHED_BLOCKS 1
#endif

namespace rtk {

namespace {

constexpr int kClasses = kSchedClasses;

// Image position of point (qx,qy,qz) for the reference camera: the ray
// P + t (f + r su + u sv) through it has su = (w.r)/(w.f), sv = (w.u)/(w.f)
// (w = Q - P; f, r, u orthonormal), su = (x/(W-1) - 0.5) scale and
// sv = ((H-1-y)/(H-1) - 0.5) scale.  False when Q is not in front of P.
bool project(const SchedView &v, double qx, double qy, double qz, double &x, double &y) {
  const double wx = qx - v.px, wy = qy - v.py, wz = qz - v.pz;
  const double a = wx * v.fx + wy * v.fy + wz * v.fz;
  const double len = std::sqrt(wx * wx + wy * wy + wz * wz);
  if (!(a > 1e-9 * len) || !(v.scale > 0.0)) return false;
  const double su = (wx * v.rx + wy * v.ry + wz * v.rz) / (a * v.scale);
  const double sv = (wx * v.ux + wy * v.uy + wz * v.uz) / (a * v.scale);
  x = (su + 0.5) * (v.W - 1);
  y = (v.H - 1) - (sv + 0.5) * (v.H - 1);
  return std::isfinite(x) && std::isfinite(y);
}

}  // namespace

void tile_order(const SchedView &v, const std::vector<SchedSphere> &refl, std::vector<int> &perm,
                long long *class_count) {
  const int ntx = (v.xw + v.tw - 1) / v.tw, nty = (v.count + v.th - 1) / v.th;
  const long long ntiles = (long long)ntx * nty;
  perm.resize((size_t)ntiles);
  // image-row span of each tile row (a shard's launch rows map to cyclic bands)
  std::vector<double> ylo(nty), yhi(nty);
  for (int ty = 0; ty < nty; ++ty) {
    double lo = 1e300, hi = -1e300;
    for (int k = ty * v.th; k < std::min(v.count, (ty + 1) * v.th); ++k) {
      const long long y = (long long)(k / v.band) * v.band * v.stride + (long long)v.first * v.band + k % v.band;
      if (y >= v.H) continue;
      lo = std::min(lo, (double)y);
      hi = std::max(hi, (double)y);
    }
    ylo[ty] = lo;
    yhi[ty] = hi;
  }
  std::vector<unsigned char> cls((size_t)ntiles, 0);
  auto bump = [&](int ty, int tx0, int tx1) {
    for (int tx = std::max(0, tx0); tx <= std::min(ntx - 1, tx1); ++tx) {
      unsigned char &c = cls[(size_t)ty * ntx + tx];
      if (c + 1 < kClasses) ++c;
    }
  };
  for (const SchedSphere &s : refl) {
    const double r = std::fabs(s.r);
    double xmin = 1e300, xmax = -1e300, ymin = 1e300, ymax = -1e300;
    bool whole = !(std::isfinite(s.cx + s.cy + s.cz + r));
    for (int c = 0; c < 8 && !whole; ++c) {
      double x, y;
      if (!project(v, s.cx + ((c & 1) ? r : -r), s.cy + ((c & 2) ? r : -r), s.cz + ((c & 4) ? r : -r), x, y)) {
        whole = true;  // straddles the camera plane: its image is unbounded
        break;
      }
      xmin = std::min(xmin, x);
      xmax = std::max(xmax, x);
      ymin = std::min(ymin, y);
      ymax = std::max(ymax, y);
    }
    if (whole) {
      for (int ty = 0; ty < nty; ++ty) bump(ty, 0, ntx - 1);
      continue;
    }
    // the projected box of the sphere's bounding box holds its image (all
    // corners in front of the camera); one pixel of slack
    xmin -= 1.0;
    xmax += 1.0;
    ymin -= 1.0;
    ymax += 1.0;
    if (xmax < v.x0 || xmin > v.x0 + v.xw - 1) continue;
    const int tx0 = (int)std::floor((std::max(xmin, (double)v.x0) - v.x0) / v.tw);
    const int tx1 = (int)std::floor((std::min(xmax, (double)(v.x0 + v.xw - 1)) - v.x0) / v.tw);
    for (int ty = 0; ty < nty; ++ty)
      if (yhi[ty] >= ymin && ylo[ty] <= ymax) bump(ty, tx0, tx1);
  }
  // counting sort, heaviest class first; within a class the tiles follow 2x2
  // blocks in scanline order of the blocks, so the consecutive slots one
  // merged wave takes (kMergeTiles = 4) are a 16x16-pixel square, whose
  // reflection rays are more alike than those of a 32x8 strip
  std::vector<int> order;
  order.reserve((size_t)ntiles);
#if RT_SCHED_BLOCKS == 2
  // Z order over the whole tile grid: 2x2 blocks of 2x2 blocks, ...
  for (long long t = 0; t < ntiles; ++t) order.push_back((int)t);
  auto morton = [ntx](int t) {
    const unsigned x = (unsigned)(t % ntx), y = (unsigned)(t / ntx);
    unsigned long long m = 0;
    for (int b = 0; b < 16; ++b)
      m |= (unsigned long long)((x >> b) & 1u) << (2 * b) | (unsigned long long)((y >> b) & 1u) << (2 * b + 1);
    return m;
  };
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return morton(a) < morton(b); });
#elif RT_SCHED_BLOCKS
  for (int by = 0; by < nty; by += 2)
    for (int bx = 0; bx < ntx; bx += 2)
      for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 2; ++i)
          if (by + j < nty && bx + i < ntx) order.push_back((by + j) * ntx + bx + i);
#else
  for (long long t = 0; t < ntiles; ++t) order.push_back((int)t);
#endif
  long long start[kClasses + 1] = {};
  for (long long t = 0; t < ntiles; ++t) ++start[kClasses - 1 - cls[(size_t)t] + 1];
  if (class_count)
    for (int k = 0; k < kClasses; ++k) class_count[k] = start[kClasses - k];
  for (int k = 0; k < kClasses; ++k) start[k + 1] += start[k];
  for (const int t : order) perm[(size_t)start[kClasses - 1 - cls[(size_t)t]]++] = t;
}

}  // namespace rtk
