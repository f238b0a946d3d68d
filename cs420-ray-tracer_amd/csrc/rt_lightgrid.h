// rt_lightgrid.h -- per-light direction grids ("light buffers") for shadow rays.
//
// Every shadow ray of light L runs (up to rounding) along the line through L
// and the shaded point p, and only spheres that meet the half-line
// {L + s*u : s >= 0}, u = (p - L)/|p - L|, can report a root t < |L - p| on
// it (scene.h:65-86 / sphere.h:26-59; negative tangent roots behind p lie on
// the same half-line).  Seen from L such a sphere covers a disk of directions
// around (C - L) of angular radius asin(R/|C - L|), R = radius + margin.
//
// Directions from L are binned on a cube map (6 faces x N x N cells).  A cell
// lists every sphere whose grown disk meets the cell; spheres that contain L
// (or come within R of it) and spheres with non-finite data are on a "global"
// list tested for every direction.  A shadow query tests the global list and
// its cell's list with the reference's exact intersection; the candidate set
// is a superset of the spheres that can occlude, so the result is the
// reference's.  Margins: R = |r|(1 + 1e-6) + 1e-6 (|C - L| + scene diameter)
// covers the line's offset from L and the rounding of the reference's test
// (same argument as the cull bound in rt_device.h) as long as the line passes
// within max_off = 1e-7 * diameter of L, which the device checks per ray
// (falling back to testing every sphere); directions are binned in fp32
// (angle error < 1e-6 rad) and every disk is grown by kLgSlack = 4e-6 rad.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rtk {

constexpr double kLgSlack = 4e-6;
// A shadow ray starts EPSILON (0.001, ray_math_constants.h:22) past its point
// and its t is compared with the point's distance to the light (scene.h:72-82),
// so it runs up to EPSILON PAST the light: a sphere whose surface comes within
// that of the light can occlude a ray from any direction (the overshoot enters
// it behind the light) -- such spheres go on the light's global list.  The
// slack here is absolute (~1e-9) and covers the overshoot only: the rounding
// of the shadow ray's origin hp + EPSILON * ldir, of dist and of t grows with
// |coordinates|, and it is covered by R's relative term 1e-6 (|C - L| +
// diameter) as long as the line passes within max_off = 1e-7 * diameter of
// the light (the device checks that per ray unless the host bounds it for the
// whole scene, off_free; otherwise the ray tests every sphere).
// tests/native/lg_check.cpp pins it with half its lights just outside spheres,
// scenes at scales 0.1 .. 1000 up to 1e8 from the origin, and small scenes
// (diameters 0.2 .. 20) 1e6 .. 1e10 from it: 0 missed occluders.
constexpr double kLgOvershoot = 0.001 * (1.0 + 1e-6);

// Cell of direction (ux, uy, uz) on an N x N cube map: face 0..5 = +X -X +Y -Y
// +Z -Z, (a, b) = the two minor coordinates divided by the major one, in
// [-1, 1].  Returns -1 for a zero or non-finite direction.  Shared by the host
// builder and the device lookup so both bin identically.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int lg_cell(float ux, float uy, float uz, int N, float rel = 0.0f) {
  const float ax = ux < 0 ? -ux : ux, ay = uy < 0 ? -uy : uy, az = uz < 0 ? -uz : uz;
  int face;
  float m, p, q;
  if (ax >= ay && ax >= az) {
    face = ux >= 0 ? 0 : 1;
    m = ax, p = uy, q = uz;
  } else if (ay >= az) {
    face = uy >= 0 ? 2 : 3;
    m = ay, p = ux, q = uz;
  } else {
    face = uz >= 0 ? 4 : 5;
    m = az, p = ux, q = uy;
  }
  if (!(m > 1e-30f) || !(m <= 3.4e38f) || p != p || q != q) return -1;
  // rel: a relative error of the quotients (0 here; tests/native/lg_check.cpp
  // bins with +-2^-22 too, the device's rcp-based quotients, lg_cell_rcp)
  const float fa = ((p / m) * (1.0f + rel) + 1.0f) * 0.5f * (float)N,
              fb = ((q / m) * (1.0f + rel) + 1.0f) * 0.5f * (float)N;
  int i = (int)(fa < 0.f ? 0.f : fa), j = (int)(fb < 0.f ? 0.f : fb);
  i = i > N - 1 ? N - 1 : i;
  j = j > N - 1 ? N - 1 : j;
  return (face * N + j) * N + i;
}

// Host builder.  For light l the lists are at
//   cell c (0 <= c < 6N^2): ids[start[l*stride + c] .. start[l*stride + c + 1])
//   global list:           ids[start[l*stride + 6N^2] .. start[l*stride + 6N^2 + 1])
// with stride = 6N^2 + 2; ids within a list ascend (sphere order).
void build_light_grid(const double *cx, const double *cy, const double *cz, const double *r, int n,
                      const double *lx, const double *ly, const double *lz, int nl, double diam, int N,
                      std::vector<int32_t> &start, std::vector<int32_t> &ids);

// Camera grid: the same cube map around the camera position P, for the
// closest hit of camera rays (origin exactly P, camera.h:17-25).  A cell lists
// every sphere whose grown disk meets it seen along +u (roots t >= 0) or along
// -u (the negative tangent root that sphere.h:43-47 keeps at disc == 0), each
// entry with a lower bound `tlo` of any t the reference's test can return for
// it (D - R ahead, -(D + R) behind, -inf for spheres that contain or nearly
// contain P, which are on every list), entries ascending by (tlo, index): a
// closest-hit scan may stop at the first entry whose tlo exceeds its best t.
// Entry k of cell c is ent[2k] = sphere index, ent[2k + 1] = tlo as fp32 bits
// (rounded down), k in [start[c], start[c + 1]).  Returns false (no grid) when
// more than max_global spheres contain P or the lists exceed max_entries.
bool build_point_grid(const double *cx, const double *cy, const double *cz, const double *r, int n, double px,
                      double py, double pz, double diam, int N, int max_global, size_t max_entries,
                      std::vector<int32_t> &start, std::vector<int32_t> &ent);

// Sphere grids: one such grid per sphere s, for the closest hit of rays that
// leave s (reflection rays, main.cpp:46: origin hit point + normal * 0.001),
// built for origins anywhere in the ball B(C_s, rho[s]): every disk grows by
// rho (the directions from B(C_s, rho) to a sphere of radius R around C are
// those of B(C - C_s, R + rho)) and every bound by rho (tlo = D - R - rho
// ahead, -(D + R + rho) behind); s itself and the spheres within R + rho of
// C_s are on every list.  The device uses grid s only for a ray whose origin
// it has checked to lie in B(C_s, rho[s]).  Sphere s's cell c is
// ent[2k], ent[2k + 1] for k in [start[s * (6N^2 + 1) + c], start[... + c + 1]);
// ok[s] = 0 where that grid was refused (more than max_global spheres overlap
// the ball; its lists are empty).  Returns the number of entries, 0 (and
// every ok[s] = 0) when they would exceed max_entries.
size_t build_sphere_grids(const double *cx, const double *cy, const double *cz, const double *r, int n,
                          const double *rho, double diam, int N, int max_global, size_t max_entries,
                          std::vector<int32_t> &start, std::vector<int32_t> &ent, std::vector<uint8_t> &ok);

// The cube map's patch hierarchy for the device-side camera-grid builder
// (rt_kernel.hip cg_bin_kernel): faces, blocks of kCubeB x kCubeB tiles, tiles of
// kCubeT x kCubeT cells, each with its centre direction c and rad = the largest
// angle from c to the patch, cb / sb = cos / sin(rad + kLgSlack) (the host
// builder's Patch); cells from a per-(i, j) table (cb, sb) shared by the six
// faces, their centres formed on the fly.  Same values as build_point_grid's.
constexpr int kCubeT = 8, kCubeB = 8;
struct CubePatch {
  double cx, cy, cz, rad, cb, sb;
};
void cube_tables(int N, std::vector<CubePatch> &faces, std::vector<CubePatch> &blocks, std::vector<CubePatch> &tiles,
                 std::vector<double> &cell_cbsb, int &NT, int &NB);

}  // namespace rtk
