// The camera grid's device builder (rt_kernel.hip cg_disk_kernel /
// cg_bin_kernel), per lane: the sphere's disks seen from the grid's point P,
// and the block / tile / cell tests of the host builder (rt_lightgrid.cpp
// build_point_grid: the same cube-map patch hierarchy, margins and slack).
// Host-callable too: tests/native/cg_device_check.cpp runs these same
// functions, lane by lane, in the kernels' pass structure on the CPU.
#pragma once

#include <cmath>
#include <cstdint>

#include "rt_lightgrid.h"

#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rtk {

struct CgDisk {  // one side of a sphere seen from a grid's point
  double ux, uy, uz, alpha, ca, sa;
  float tlo;
  int s;
};

RT_HD inline float cg_float_down(double x) {  // x rounded down to fp32
  float f = (float)x;
  if ((double)f > x) {
    const int b = __builtin_bit_cast(int, f);
    f = f == 0.0f ? -0x1p-149f : __builtin_bit_cast(float, f > 0.0f ? b - 1 : b + 1);
  }
  return f;
}

// angle(u, patch centre) <= alpha + rad + slack (the host builder's meets())
RT_HD inline bool cg_meets(const CgDisk &k, double cx, double cy, double cz, double rad, double cb, double sb) {
  if (k.alpha + rad + kLgSlack >= 3.14159) return true;
  return k.ux * cx + k.uy * cy + k.uz * cz >= k.ca * cb - k.sa * sb - 1e-12;
}
RT_HD inline bool cg_meets(const CgDisk &k, const CubePatch &p) { return cg_meets(k, p.cx, p.cy, p.cz, p.rad, p.cb, p.sb); }

// A sphere (centre c, |radius| r) seen from P: its direction v = c - P,
// distance D and the light grids' grown radius R; `global` -- P inside (or
// nearly inside) it, or non-finite data -- makes it one disk of every
// direction (alpha >= pi meets every patch) with tlo = -inf.  rho > 0: seen
// from anywhere in the ball B(P, rho) (the sphere grids, build_sphere_grids:
// R grows by rho, the Minkowski sum).
struct CgView {
  double vx, vy, vz, D, R, alpha, ca, sa;
  bool global;
};
RT_HD inline CgView cg_view(double cx, double cy, double cz, double r, double px, double py, double pz, double diam,
                            double rho = 0.0, double gextra = 0.0) {
  CgView v;
  v.vx = cx - px, v.vy = cy - py, v.vz = cz - pz;
  v.D = __builtin_sqrt(v.vx * v.vx + v.vy * v.vy + v.vz * v.vz);
  v.R = r * (1.0 + 1e-6) + 1e-6 * (v.D + diam) + rho;
  // gextra (light grids: kLgOvershoot): spheres within it of the point go global too
  v.global = !__builtin_isfinite(v.D) || !__builtin_isfinite(v.R) || !(v.D > v.R + gextra);
  v.alpha = v.global ? 4.0 : asin(v.R / v.D) + kLgSlack;
  v.ca = cos(v.alpha);
  v.sa = sin(v.alpha);
  return v;
}
// Its disk along +u (side 0: roots ahead, tlo = (D - R)(1 - 1e-9)) or -u
// (side 1: the negative tangent root behind P, sphere.h:43-47, tlo =
// -(D + R)(1 + 1e-9)), tlo rounded down to fp32.
RT_HD inline CgDisk cg_side(const CgView &v, int side, int s) {
  const double sg = side ? -1.0 : 1.0;
  CgDisk k;
  k.ux = v.global ? 1.0 : sg * (v.vx / v.D), k.uy = v.global ? 0.0 : sg * (v.vy / v.D),
  k.uz = v.global ? 0.0 : sg * (v.vz / v.D);
  k.alpha = v.alpha, k.ca = v.ca, k.sa = v.sa;
  k.tlo = v.global ? -__builtin_inff()
                   : (side ? cg_float_down(-(v.D + v.R) * (1.0 + 1e-9)) : cg_float_down((v.D - v.R) * (1.0 - 1e-9)));
  k.s = s;
  return k;
}

// Pass 1, lane b: does the disk meet block b's face and block patches?
RT_HD inline bool cg_block(const CgDisk &k, const CubePatch *faces, const CubePatch *blocks, int NB, int b) {
  return cg_meets(k, faces[b / (NB * NB)]) && cg_meets(k, blocks[b]);
}

// Pass 2, lane = tile (lane & 7, lane >> 3) of block (f, bi, bj): meets the
// disk (tm); lies well inside it (inside: all its cells listed untested).
RT_HD inline void cg_tile(const CgDisk &k, const CubePatch *tiles, int NT, int f, int bi, int bj, int lane, bool &tm,
                          bool &inside) {
  const int ti = bi * kCubeB + (lane & 7), tj = bj * kCubeB + (lane >> 3);
  tm = false, inside = false;
  if (ti < NT && tj < NT) {
    const CubePatch tp = tiles[((size_t)f * NT + tj) * NT + ti];
    tm = cg_meets(k, tp);
    inside = tm && k.alpha < 3.0 && k.alpha > tp.rad + 1e-3 &&
             k.ux * tp.cx + k.uy * tp.cy + k.uz * tp.cz >= cos(k.alpha - tp.rad - 1e-3);
  }
}

// Pass 2, lane = cell (lane & 7, lane >> 3) of tile tl of block (f, bi, bj)
// (tin: the tile is inside the disk): the face-major cell index (f N + j) N
// + i when the disk lists it, else -1 (wide = cg_wide(k)).  The cell's patch: its centre formed
// as face_dir does, cos / sin of its rad + slack from the per-(i, j) table.
RT_HD inline bool cg_wide(const CgDisk &k) { return k.alpha + kLgSlack >= 3.0; }
RT_HD inline int cg_cell(const CgDisk &k, bool wide, const double *cell_cbsb, int N, int f, int bi, int bj, int tl,
                         int lane, bool tin) {
  const int i = (bi * kCubeB + (tl & 7)) * kCubeT + (lane & 7), j = (bj * kCubeB + (tl >> 3)) * kCubeT + (lane >> 3);
  bool cm = false;
  if (i < N && j < N) {
    if (tin) {
      cm = true;
    } else {
      const double fa = -1.0 + (2.0 * i + 1.0) / N, fb = -1.0 + (2.0 * j + 1.0) / N;
      double dx, dy, dz;
      switch (f) {
        case 0: dx = 1.0, dy = fa, dz = fb; break;
        case 1: dx = -1.0, dy = fa, dz = fb; break;
        case 2: dx = fa, dy = 1.0, dz = fb; break;
        case 3: dx = fa, dy = -1.0, dz = fb; break;
        case 4: dx = fa, dy = fb, dz = 1.0; break;
        default: dx = fa, dy = fb, dz = -1.0; break;
      }
      const double l = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
      const size_t ij = (size_t)j * N + i;
      cm = cg_meets(k, dx / l, dy / l, dz / l, wide ? 3.2 : 0.0, cell_cbsb[2 * ij], cell_cbsb[2 * ij + 1]);
    }
  }
  return cm ? (f * N + j) * N + i : -1;
}

// Pass 3's order of a cell's list: ascending (tlo, sphere index).
RT_HD inline bool cg_before(float ta, int ia, float tb, int ib) { return ta < tb || (ta == tb && ia < ib); }

}  // namespace rtk
