// rt_host.cpp -- host half of librt_hip.so: scene text parser, camera basis,
// PPM writer, status strings.  No device code here.
//
// The parser keeps the reference loader's record grammar and its quirks
// (include/scene_loader.h:27-135): '#' comments (also after leading
// spaces/tabs), `sphere x y z r  R G B  metallic roughness shininess`,
// `light x y z R G B intensity`, `ambient R G B`, `camera px py pz lx ly lz fov`;
// last ambient/camera wins; malformed records are skipped with a warning;
// trailing tokens are ignored.  Numbers go through std::istream >> double, the
// same extractor the reference uses, so parsed doubles are identical.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>

#include <fcntl.h>
#include <unistd.h>

#include "rt_hip.h"

namespace {

struct Grow {
  std::vector<rt_sphere> spheres;
  std::vector<rt_light> lights;
};

void set3(double *d, double x, double y, double z) {
  d[0] = x;
  d[1] = y;
  d[2] = z;
}

int parse_stream(std::istream &in, rt_scene *out, int verbose) {
  std::memset(out, 0, sizeof(*out));
  set3(out->cam_look_at, 0, 0, -1);  // CameraConfig() defaults, scene.h:22
  out->cam_fov = 60.0;
  Grow g;
  std::string line;
  int line_number = 0;
  while (std::getline(in, line)) {
    line_number++;
    if (line.empty() || line[0] == '#') continue;
    size_t start = line.find_first_not_of(" \t");
    if (start == std::string::npos) continue;
    if (line[start] == '#') continue;
    std::istringstream iss(line.substr(start));
    std::string type;
    iss >> type;
    double v[10];
    auto read = [&](int n) {
      for (int i = 0; i < n; i++)
        if (!(iss >> v[i])) return false;
      return true;
    };
    auto warn = [&](const char *what) {
      out->warnings++;
      if (verbose) std::cerr << "Warning: Invalid " << what << " at line " << line_number << ", skipping\n";
    };
    if (type == "sphere") {
      if (!read(10)) { warn("sphere"); continue; }
      rt_sphere s;
      set3(s.center, v[0], v[1], v[2]);
      s.radius = v[3];
      set3(s.color, v[4], v[5], v[6]);
      s.reflectivity = v[7];  // "metallic"; v[8] (roughness) is dropped as upstream
      s.shininess = v[9];
      g.spheres.push_back(s);
    } else if (type == "light") {
      if (!read(7)) { warn("light"); continue; }
      rt_light l;
      set3(l.position, v[0], v[1], v[2]);
      set3(l.color, v[3], v[4], v[5]);
      l.intensity = v[6];
      g.lights.push_back(l);
    } else if (type == "ambient") {
      if (!read(3)) { warn("ambient"); continue; }
      set3(out->ambient, v[0], v[1], v[2]);
    } else if (type == "camera") {
      if (!read(7)) { warn("camera"); continue; }
      set3(out->cam_position, v[0], v[1], v[2]);
      set3(out->cam_look_at, v[3], v[4], v[5]);
      out->cam_fov = v[6];
      out->has_camera = 1;
    } else {
      out->warnings++;
      if (verbose) std::cerr << "Warning: Unknown type '" << type << "' at line " << line_number << ", skipping\n";
    }
  }
  out->num_spheres = (int32_t)g.spheres.size();
  out->num_lights = (int32_t)g.lights.size();
  out->spheres = (rt_sphere *)std::malloc(sizeof(rt_sphere) * (g.spheres.size() + 1));
  out->lights = (rt_light *)std::malloc(sizeof(rt_light) * (g.lights.size() + 1));
  if (!out->spheres || !out->lights) return RT_ERR_OUT_OF_MEMORY;
  if (!g.spheres.empty()) std::memcpy(out->spheres, g.spheres.data(), sizeof(rt_sphere) * g.spheres.size());
  if (!g.lights.empty()) std::memcpy(out->lights, g.lights.data(), sizeof(rt_light) * g.lights.size());
  if (verbose)
    std::cout << "Loaded scene: " << out->num_spheres << " spheres, " << out->num_lights << " lights\n";
  return RT_OK;
}

// Vec3 algebra of include/vec3.h:13-29, used only for the per-frame camera basis.
struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V normalized(V a) {
  double len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return {a.x / len, a.y / len, a.z / len};
}
void put(double *d, V v) { set3(d, v.x, v.y, v.z); }

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_HIP_ABI_VERSION; }

int rt_rows_for_shard(int height, int band, int rank, int num_shards, rt_rows *out) {
  if (!out || height < 0 || band < 1 || num_shards < 1 || rank < 0 || rank >= num_shards) return RT_ERR_INVALID_ARG;
  const long long nb = ((long long)height + band - 1) / band;          // bands of the image
  const long long per = (nb + num_shards - 1) / num_shards;           // bands per rank
  if (per * band > 0x7fffffffLL) return RT_ERR_INVALID_ARG;
  *out = rt_rows{band, rank, num_shards, (int32_t)(per * band)};
  return RT_OK;
}

const char *rt_error_string(int status) {
  switch (status) {
    case RT_OK: return "ok";
    case RT_ERR_INVALID_ARG: return "invalid argument";
    case RT_ERR_NO_DEVICE: return "no HIP device";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_OUT_OF_MEMORY: return "out of memory";
    case RT_ERR_NO_SCENE: return "no scene uploaded";
    case RT_ERR_IO: return "I/O error";
    case RT_ERR_DEPTH: return "depth exceeds RT_MAX_DEPTH";
    case RT_ERR_CHECK: return "device index out of range (bounds-checked build)";
    default: return "unknown status";
  }
}

int rt_scene_parse(const char *text, rt_scene *out, int verbose) {
  if (!text || !out) return RT_ERR_INVALID_ARG;
  std::istringstream in{std::string(text)};
  return parse_stream(in, out, verbose);
}

int rt_scene_load(const char *path, rt_scene *out, int verbose) {
  if (!path || !out) return RT_ERR_INVALID_ARG;
  std::ifstream f(path);
  if (!f.is_open()) {  // the reference throws "Could not open scene file: ..." (scene_loader.h:33-35)
    std::memset(out, 0, sizeof(*out));
    if (verbose) std::cerr << "Could not open scene file: " << path << "\n";
    return RT_ERR_IO;
  }
  return parse_stream(f, out, verbose);
}

void rt_scene_free(rt_scene *scene) {
  if (!scene) return;
  std::free(scene->spheres);
  std::free(scene->lights);
  scene->spheres = nullptr;
  scene->lights = nullptr;
  scene->num_spheres = scene->num_lights = 0;
}

int rt_camera_from_scene(const rt_scene *s, rt_camera *c) {
  if (!s || !c) return RT_ERR_INVALID_ARG;
  V pos{s->cam_position[0], s->cam_position[1], s->cam_position[2]};
  V look{s->cam_look_at[0], s->cam_look_at[1], s->cam_look_at[2]};
  V fwd = normalized(sub(look, pos));        // camera.h:12
  V right = normalized(cross(fwd, {0, 1, 0}));  // camera.h:13
  V up = normalized(cross(right, fwd));      // camera.h:14
  put(c->position, pos);
  put(c->forward, fwd);
  put(c->right, right);
  put(c->up, up);
  c->scale = std::tan(s->cam_fov * 0.5 * M_PI / 180.0);  // camera.h:19 (glibc tan, host)
  return RT_OK;
}

// P3 text identical to write_ppm (src/main.cpp:69-91) -- "r g b\n" per pixel,
// top row first -- formatted from a 256-entry table (1.85 s at 1080p upstream
// with ostream double formatting): pixel ranges are formatted on up to 16
// threads into their own buffers and written with write(2) in order as they
// complete, so the formatting hides under the writes.  On the GPU box's
// overlay file system the writes are the floor (~0.22 ms per MB into the page
// cache: 5.3-6 ms for 1080p); ordered write(2) beat fwrite (6.7-7.2 ms),
// pwrite from every thread (5.8-7.0) and a mapped file (13-14 ms)
// (scripts/p3_write_bench.cpp, profiles/r7b/).  The calling thread formats
// too, and takes any range no helper has claimed, so the file is complete
// even when no thread can be started; every started thread is joined.
int rt_write_ppm(const char *path, const uint8_t *rgb, int width, int height, int binary) {
  if (!path || !rgb || width < 0 || height < 0) return RT_ERR_INVALID_ARG;
  const size_t n = (size_t)width * (size_t)height;
  char hdr[64];
  const int hn = std::snprintf(hdr, sizeof hdr, "%s\n%d %d\n255\n", binary ? "P6" : "P3", width, height);
  const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return RT_ERR_IO;
  int rc = RT_OK;
  auto put = [&](const char *p, size_t len) {
    while (rc == RT_OK && len > 0) {
      const ssize_t w = ::write(fd, p, len);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) rc = RT_ERR_IO;
      else p += w, len -= (size_t)w;
    }
  };
  put(hdr, (size_t)hn);
  if (binary) {
    put(reinterpret_cast<const char *>(rgb), n * 3);
  } else {
    // "0".."255" and their lengths, built once (a function-local static: safe
    // when several threads write images at the same time)
    struct Tab {
      char s[256][4];
      unsigned char n[256];
      Tab() {
        for (int v = 0; v < 256; v++) n[v] = (unsigned char)std::snprintf(s[v], 4, "%d", v);
      }
    };
    static const Tab T;
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t nthr = n < ((size_t)1 << 16) ? 1 : std::max<size_t>(1, std::min<size_t>(hw ? hw : 1, 16));
    const size_t nchunk = nthr == 1 ? 1 : nthr * 4;
    std::vector<std::unique_ptr<char[]>> bufs(nchunk);
    std::vector<size_t> len(nchunk, 0);
    std::vector<unsigned char> done(nchunk, 0);  // under mu
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<size_t> next{0};
    // claims and formats the next unclaimed range (false: none left); at most
    // 12 bytes per pixel, each number as its 4-byte table slot (the next
    // write overwrites the slot's tail; the buffer has 4 bytes of room)
    auto format_next = [&]() {
      const size_t k = next.fetch_add(1);
      if (k >= nchunk) return false;
      const size_t p0 = n * k / nchunk, p1 = n * (k + 1) / nchunk;
      char *o = new (std::nothrow) char[(p1 - p0) * 12 + 4];
      if (o) {
        char *const b = o;
        for (size_t p = p0; p < p1; p++) {
          for (int c = 0; c < 3; c++) {
            const unsigned v = rgb[3 * p + c];
            std::memcpy(o, T.s[v], 4);
            o += T.n[v];
            *o++ = c == 2 ? '\n' : ' ';
          }
        }
        bufs[k].reset(b);
        len[k] = (size_t)(o - b);
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        done[k] = 1;
      }
      cv.notify_all();
      return true;
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < nthr; t++) {
      try {
        th.emplace_back([&] {
          while (format_next()) {
          }
        });
      } catch (...) {
        break;  // the started threads and this one format the rest
      }
    }
    for (size_t k = 0; k < nchunk; k++) {
      for (;;) {
        {
          std::unique_lock<std::mutex> lk(mu);
          if (done[k]) break;
          if (next.load() >= nchunk) {  // claimed by a helper: wait for it
            cv.wait(lk, [&] { return done[k] != 0; });
            break;
          }
        }
        format_next();  // nothing finished yet: format an unclaimed range here
      }
      if (!bufs[k]) rc = RT_ERR_IO;  // (allocation failed)
      else put(bufs[k].get(), len[k]);
      bufs[k].reset();
    }
    for (auto &t : th) t.join();
  }
  if (::close(fd) != 0) rc = RT_ERR_IO;
  return rc;
}

}  // extern "C"
