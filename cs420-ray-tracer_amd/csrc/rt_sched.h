// rt_sched.h -- host-side launch order of the render kernel's tiles.
//
// A wave's cost is set mostly by the reflection chains its pixels start: a
// tile whose camera rays land on reflective spheres traces up to depth-1
// more levels of incoherent rays (3-10x a ground or sky tile on synth200).
// Workgroups are dispatched in blockIdx order, so with tiles in scanline
// order the expensive band of the image starts mid-kernel and its slowest
// waves end long after the rest (the tail).  tile_order() predicts each
// tile's class from the projections of the reflective spheres onto the image
// (the reference's camera model, camera.h:17-25 / main.cpp:151-154) and
// returns the tiles heaviest class first, scanline order within a class
// (longest-processing-time-first list scheduling).  Only the order of the
// launch changes; every pixel is traced exactly as before.
#pragma once
#include <vector>

namespace rtk {

struct SchedSphere {
  double cx, cy, cz, r;
};

struct SchedView {
  double px, py, pz, fx, fy, fz, rx, ry, rz, ux, uy, uz, scale;  // Cam
  int W, H;
  int band, first, stride, count;  // Rows: launch row k -> image row y
  int x0, xw;                      // pixel columns [x0, x0 + xw)
  int tw, th;                      // tile size in pixels
};

// perm[b] = tile index (ty * ntx + tx) dispatched b-th; ntx = ceil(xw / tw),
// nty = ceil(count / th).  `refl` holds the reflective spheres only.
// class_count (optional, kSchedClasses entries): tiles per class; perm lists
// class kSchedClasses-1 first, then the lower classes in turn.
constexpr int kSchedClasses = 4;  // 0 .. 3 reflective spheres over a tile (capped)
void tile_order(const SchedView &v, const std::vector<SchedSphere> &refl, std::vector<int> &perm,
                long long *class_count = nullptr);

}  // namespace rtk
