// rt_compat.cpp -- launch_gpu_kernel / upload_lights_and_ambience with the
// reference's C ABI (include/rt_hip_compat.h; src/kernel.cu:185-207 as
// src/main_hybrid.cpp:104-109,170-171 declares them), mapped onto one default
// rt_ctx per device and rt_render_tile (RT_FB_F32X3: the reference's float3
// framebuffer layout).  Host code only; every device step goes through the
// public C-ABI of rt_hip.h.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "rt_hip.h"
#include "rt_hip_compat.h"

namespace {

// The reference keeps the lights and the ambient colour in __constant__
// module state of the current device (kernel.cu:7-9); here: per device.
struct DevState {
  rt_ctx *ctx = nullptr;
  std::vector<rt_gpu_light> lights;
  rt_float3 ambient{0.f, 0.f, 0.f};
  unsigned long long lights_gen = 0;
  // what the context holds: the spheres and lights it was uploaded with
  std::vector<rt_gpu_sphere> spheres;
  int used_lights = -1;
  unsigned long long used_gen = ~0ull;
};

std::mutex g_mu;
std::vector<DevState> g_dev;
thread_local int t_status = RT_OK;

DevState *state_of_current_device(int &dev) {
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  if ((size_t)dev >= g_dev.size()) g_dev.resize((size_t)dev + 1);
  return &g_dev[(size_t)dev];
}

// Uploads the caller's fp32 scene (promoted to double) to the device context.
int upload(DevState &s, int nl) {
  std::vector<rt_sphere> sp(s.spheres.size());
  for (size_t i = 0; i < s.spheres.size(); i++) {
    const rt_gpu_sphere &g = s.spheres[i];
    sp[i] = rt_sphere{{g.center.x, g.center.y, g.center.z}, g.radius,
                      {g.material.albedo.x, g.material.albedo.y, g.material.albedo.z},
                      g.material.metallic, g.material.shininess};
  }
  std::vector<rt_light> li((size_t)nl);
  for (int i = 0; i < nl; i++) {
    const rt_gpu_light &g = s.lights[(size_t)i];
    li[(size_t)i] = rt_light{{g.position.x, g.position.y, g.position.z}, {g.color.x, g.color.y, g.color.z},
                             g.intensity};
  }
  rt_scene sc{};
  sc.num_spheres = (int32_t)sp.size();
  sc.num_lights = nl;
  sc.spheres = sp.empty() ? nullptr : sp.data();
  sc.lights = li.empty() ? nullptr : li.data();
  sc.ambient[0] = s.ambient.x, sc.ambient[1] = s.ambient.y, sc.ambient[2] = s.ambient.z;
  return rt_upload_scene(s.ctx, &sc);
}

}  // namespace

extern "C" {

void upload_lights_and_ambience(rt_gpu_light *lights, int count, rt_float3 ambience) {
  std::lock_guard<std::mutex> lock(g_mu);
  int dev = 0;
  DevState *s = state_of_current_device(dev);
  if (!s) {
    t_status = RT_ERR_NO_DEVICE;
    return;
  }
  if (count < 0 || (count > 0 && !lights)) {
    t_status = RT_ERR_INVALID_ARG;
    return;
  }
  s->lights.assign(lights, lights + count);
  s->ambient = ambience;
  s->lights_gen++;
  t_status = RT_OK;
}

void launch_gpu_kernel(rt_float3 *d_framebuffer, rt_gpu_sphere *d_spheres, int num_spheres, int num_lights,
                       rt_gpu_camera *camera, int tile_x, int tile_y, int tile_width, int tile_height,
                       int image_width, int image_height, int max_depth, void *stream) {
  std::lock_guard<std::mutex> lock(g_mu);
  int dev = 0;
  DevState *s = state_of_current_device(dev);
  if (!s) {
    t_status = RT_ERR_NO_DEVICE;
    return;
  }
  if (!d_framebuffer || !camera || num_spheres < 0 || (num_spheres > 0 && !d_spheres) || num_lights < 0 ||
      num_lights > (int)s->lights.size()) {
    t_status = RT_ERR_INVALID_ARG;
    return;
  }
  if (!s->ctx) {
    const int rc = rt_create(dev, &s->ctx);
    if (rc != RT_OK) {
      s->ctx = nullptr;
      t_status = rc;
      return;
    }
  }
  hipStream_t hs = static_cast<hipStream_t>(stream);
  // The scene and the camera live in the caller's device memory: read them
  // on the caller's stream, after the work it already enqueued there.
  std::vector<rt_gpu_sphere> sph((size_t)num_spheres);
  rt_gpu_camera cam{};
  if ((num_spheres > 0 &&
       hipMemcpyAsync(sph.data(), d_spheres, sizeof(rt_gpu_sphere) * (size_t)num_spheres, hipMemcpyDeviceToHost,
                      hs) != hipSuccess) ||
      hipMemcpyAsync(&cam, camera, sizeof cam, hipMemcpyDeviceToHost, hs) != hipSuccess ||
      hipStreamSynchronize(hs) != hipSuccess) {
    t_status = RT_ERR_HIP;
    return;
  }
  const bool same = s->used_gen == s->lights_gen && s->used_lights == num_lights &&
                    sph.size() == s->spheres.size() &&
                    (sph.empty() || std::memcmp(sph.data(), s->spheres.data(), sizeof(rt_gpu_sphere) * sph.size()) == 0);
  if (!same) {
    s->spheres.swap(sph);
    const int rc = upload(*s, num_lights);
    if (rc != RT_OK) {
      s->used_gen = ~0ull;
      t_status = rc;
      return;
    }
    s->used_gen = s->lights_gen;
    s->used_lights = num_lights;
  }
  // camera.h:10-25 from the caller's origin, view direction and fov (fp64)
  rt_scene cs{};
  cs.cam_look_at[0] = cam.forward.x, cs.cam_look_at[1] = cam.forward.y, cs.cam_look_at[2] = cam.forward.z;
  cs.cam_fov = cam.fov;
  rt_camera c{};
  int rc = rt_camera_from_scene(&cs, &c);  // position (0,0,0): look_at - position == forward exactly
  if (rc == RT_OK) {
    c.position[0] = cam.origin.x, c.position[1] = cam.origin.y, c.position[2] = cam.origin.z;
    rc = rt_set_stream(s->ctx, stream);
  }
  if (rc == RT_OK)
    rc = rt_render_tile(s->ctx, &c, image_width, image_height, max_depth, tile_x, tile_y, tile_width, tile_height,
                        RT_FB_F32X3, d_framebuffer);
  // The caller owns its streams and may destroy them between calls (the
  // reference's render_hybrid creates and destroys three per call,
  // main_hybrid.cpp:407-409, 489-491): the context must not keep the handle.
  // Switching back to its own stream orders that stream after the tile
  // (rt_set_stream records an event on the caller's stream, which is still
  // alive here), so a later call on any stream also waits for it.
  const int rs = rt_set_stream(s->ctx, nullptr);
  t_status = rc != RT_OK ? rc : rs;
}

int rt_compat_status(void) { return t_status; }

}  // extern "C"
