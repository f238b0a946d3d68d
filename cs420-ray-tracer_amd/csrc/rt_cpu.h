// rt_cpu.h -- the CPU tile worker of the hybrid CPU+GPU scheduler (ray_hybrid,
// SURVEY 8(f) row 4).  It is linked into ray_hybrid only, never into
// librt_hip.so: the library has no CPU render path, and ray_hybrid refuses to
// run without a GPU, as the reference's does (src/main_hybrid.cpp:755-761).
//
// The reference's hybrid CPU path is trace_ray_cpu + process_tile_cpu
// (src/main_hybrid.cpp:115-167), the serial fp64 trace_ray of src/main.cpp:16-58
// over Scene (include/scene.h:41-121), Sphere (include/sphere.h:26-64), Camera
// (include/camera.h:10-25) and Vec3 (include/vec3.h).  This worker evaluates
// the same expressions in the same order (compiled with -ffp-contract=off), so
// a CPU tile is byte-identical to the GPU's tile of the same pixels.
#pragma once
#include <cstdint>
#include <vector>

#include "rt_hip.h"

namespace rtc {

struct V3 {
  double x, y, z;
};

class CpuTracer {
 public:
  CpuTracer(const rt_scene &scene, const rt_camera &cam);

  // Camera::get_ray (camera.h:17-25): the direction (normalised twice: get_ray
  // and the Ray constructor, ray.h:12) of the camera ray through (u, v).
  V3 camera_dir(double u, double v) const;
  // trace_ray / trace_ray_cpu (main.cpp:16-58, main_hybrid.cpp:115-160) for a
  // ray whose direction is already normalised.
  V3 trace(V3 o, V3 d, int depth) const;
  // process_tile_cpu (main_hybrid.cpp:162-173): pixels x0 <= x < x1,
  // y0 <= y < y1 (y = 0 the bottom row, v = y / (H - 1)) into fb[y * W + x].
  void render_tile(int x0, int y0, int x1, int y1, int W, int H, int depth, V3 *fb) const;
  // estimate_tile_complexity (main_hybrid.cpp:323-347): 5 camera rays at the
  // tile's corners and centre, u = x / img_w, v = y / img_h (the reference's
  // IMG_WIDTH / IMG_HEIGHT, not W - 1), weights 1,1,2,1,1, summed over every
  // sphere whose Sphere::intersect reports a hit.
  int tile_complexity(int x0, int y0, int x1, int y1, int img_w, int img_h) const;

 private:
  struct Sph {
    V3 c;
    double r;
    V3 col;
    double refl, shin;
  };
  struct Light {
    V3 p, col;
  };
  bool intersect(const Sph &s, V3 o, V3 d, double &t) const;
  bool closest(V3 o, V3 d, double &t, int &idx) const;
  bool in_shadow(V3 p, const Light &l) const;
  V3 shade(V3 p, V3 n, const Sph &s, V3 view) const;

  std::vector<Sph> sph_;
  std::vector<Light> lights_;
  V3 amb_;
  V3 pos_, fwd_, right_, up_;
  double scale_;
};

}  // namespace rtc
