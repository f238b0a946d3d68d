// rt_cpu.cpp -- CPU tile worker of ray_hybrid (see rt_cpu.h).  Every
// expression keeps the reference's operand order; build with
// -ffp-contract=off (no FMA contraction) so the rounding is the reference's.
#include "rt_cpu.h"

#include <cmath>

namespace rtc {
namespace {

constexpr double kEps = 0.001;  // ray_math_constants.h:22
constexpr double kInf = 1e20;   // ray_math_constants.h:23
constexpr double kSpec = 0.5;   // scene.h:38

// include/vec3.h:13-33
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator*(V3 a, double t) { return {a.x * t, a.y * t, a.z * t}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 unit(V3 a) {
  const double len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return {a.x / len, a.y / len, a.z / len};
}
inline double max0(double x) { return 0.0 < x ? x : 0.0; }  // std::max(0.0, x)

}  // namespace

CpuTracer::CpuTracer(const rt_scene &s, const rt_camera &cam) {
  sph_.reserve((size_t)s.num_spheres);
  for (int i = 0; i < s.num_spheres; ++i) {
    const rt_sphere &q = s.spheres[i];
    sph_.push_back(Sph{{q.center[0], q.center[1], q.center[2]}, q.radius, {q.color[0], q.color[1], q.color[2]},
                       q.reflectivity, q.shininess});
  }
  for (int i = 0; i < s.num_lights; ++i) {
    const rt_light &l = s.lights[i];
    lights_.push_back(Light{{l.position[0], l.position[1], l.position[2]}, {l.color[0], l.color[1], l.color[2]}});
  }
  amb_ = {s.ambient[0], s.ambient[1], s.ambient[2]};
  pos_ = {cam.position[0], cam.position[1], cam.position[2]};
  fwd_ = {cam.forward[0], cam.forward[1], cam.forward[2]};
  right_ = {cam.right[0], cam.right[1], cam.right[2]};
  up_ = {cam.up[0], cam.up[1], cam.up[2]};
  scale_ = cam.scale;
}

V3 CpuTracer::camera_dir(double u, double v) const {
  const double aspect = 1.0;  // camera.h:18 (the image aspect is ignored upstream)
  const V3 dir = fwd_ + right_ * ((u - 0.5) * scale_ * aspect) + up_ * ((v - 0.5) * scale_);
  return unit(unit(dir));  // get_ray normalises, Ray() normalises again
}

// Sphere::intersect, sphere.h:26-59
bool CpuTracer::intersect(const Sph &s, V3 o, V3 d, double &t) const {
  const V3 oc = o - s.c;
  const double a = dot(d, d);
  const double b = 2.0 * dot(oc, d);
  const double c = dot(oc, oc) - s.r * s.r;
  const double disc = b * b - 4 * a * c;
  if (disc < 0) return false;
  if (disc == 0) {
    t = -b / (2 * a);  // kept even when negative
    return true;
  }
  const double t1 = (-b - std::sqrt(disc)) / (2 * a);
  const double t2 = (-b + std::sqrt(disc)) / (2 * a);
  const double tmax = (t1 < t2) ? t2 : t1;  // std::max
  if (tmax < 0) return false;
  t = (t2 < t1) ? t2 : t1;  // std::min
  if (t < 0) t = tmax;
  return true;
}

// Scene::find_intersection, scene.h:41-61
bool CpuTracer::closest(V3 o, V3 d, double &t, int &idx) const {
  t = kInf;
  idx = -1;
  for (int i = 0; i < (int)sph_.size(); ++i) {
    double ti = 0;
    if (intersect(sph_[(size_t)i], o, d, ti) && ti < t) {
      idx = i;
      t = ti;
    }
  }
  return idx >= 0;
}

// Scene::in_shadow, scene.h:65-86
bool CpuTracer::in_shadow(V3 p, const Light &l) const {
  const V3 to_light = l.p - p;
  const double dist = std::sqrt(to_light.x * to_light.x + to_light.y * to_light.y + to_light.z * to_light.z);
  const V3 ldir = unit(to_light);
  double t;
  int idx;
  if (closest(p + ldir * kEps, unit(ldir), t, idx)) return t < dist;
  return false;
}

// Scene::shade, scene.h:89-121
V3 CpuTracer::shade(V3 p, V3 n, const Sph &s, V3 view) const {
  V3 color = amb_ * s.col;
  for (const Light &l : lights_) {
    if (in_shadow(p, l)) continue;
    const V3 ldir = unit(l.p - p);
    const double ndl = max0(dot(n, ldir));
    const V3 diffuse = s.col * (1.0 - s.refl) * ndl;
    const V3 v = ldir * -1;
    const V3 rdir = v - n * 2.0 * dot(v, n);  // reflect(), vec3.h:31-33
    const double rdv = max0(dot(rdir, view));
    const double spec = std::pow(rdv, s.shin);
    const V3 specular = l.col * kSpec * spec;
    color = specular + diffuse + color;
  }
  return color;
}

// trace_ray, main.cpp:16-58 (= trace_ray_cpu, main_hybrid.cpp:115-160)
V3 CpuTracer::trace(V3 o, V3 d, int depth) const {
  if (depth <= 0) return {0, 0, 0};
  double t;
  int idx;
  if (!closest(o, d, t, idx)) {
    const double st = 0.5 * (d.y + 1.0);
    return V3{1, 1, 1} * (1.0 - st) + V3{0.5, 0.7, 1.0} * st;
  }
  const Sph &s = sph_[(size_t)idx];
  const V3 hit = o + d * t;
  const V3 n = unit(hit - s.c);
  const V3 view = unit(o - hit);
  V3 c = shade(hit, n, s, view);
  if (s.refl > 0) {
    const V3 rd = d - n * 2.0 * dot(d, n);
    const V3 rc = trace(hit + n * kEps, unit(rd), depth - 1);
    c = c * (1.0 - s.refl) + rc * s.refl;
  }
  return c;
}

void CpuTracer::render_tile(int x0, int y0, int x1, int y1, int W, int H, int depth, V3 *fb) const {
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) {
      const double u = double(x) / (W - 1);
      const double v = double(y) / (H - 1);
      fb[(size_t)y * W + x] = trace(pos_, camera_dir(u, v), depth);
    }
}

int CpuTracer::tile_complexity(int x0, int y0, int x1, int y1, int img_w, int img_h) const {
  const int sx[5] = {x0, x1 - 1, (x0 + x1) / 2, x0, x1 - 1};
  const int sy[5] = {y0, y0, (y0 + y1) / 2, y1 - 1, y1 - 1};
  const int w[5] = {1, 1, 2, 1, 1};  // the centre ray counts twice
  int cplx = 0;
  for (int i = 0; i < 5; ++i) {
    const V3 d = camera_dir(double(sx[i]) / float(img_w), double(sy[i]) / float(img_h));
    for (const Sph &s : sph_) {
      double t;
      if (intersect(s, pos_, d, t)) cplx += w[i];
    }
  }
  return cplx;
}

}  // namespace rtc
